// K3 / K3b at the reference's precision: fp32 embedding gather -> dropout -> Conv1D(3, 4) ->
// global max-pool -> ReLU, and its sparse backward.  Keras/Theano trains the CDSSM towers in
// fp32 (dssm_cnn_v2/cnn_dssm_th.py:182); this is the native path of `dtype="fp32"`.
//
// Forward: v_mfma_f32_16x16x4_f32 (exact fp32 products and sums, 1/16 of the bf16 rate).  A
// persistent workgroup owns one FILTER GROUP (32 filters of both widths = 2 MFMA tiles each,
// 5 groups cover 150 -> 160) whose weights (7E x 32 fp32, 89.6 KB at E = 100) it stages into
// LDS once, then walks (sample, window-segment) items in chunks of 128 windows: the chunk's
// 131 table rows are gathered (with the counter-hash dropout mask of ops/reference.py) into
// LDS while the previous chunk computes.  Each of the 4 waves (one per SIMD) takes 32 windows
// = 2 row blocks and runs 8 independent accumulators (2 blocks x 2 widths x 2 tiles): one
// A read per block and one B pair read per width feed 8 MFMAs of 32 cycles.  The k = 3 and
// k = 4 windows share their first 3E reduction indices, so their A fragments are the same
// reads.  Per-segment max / argmax -> `part`; a finalize kernel merges segments in window
// order (first maximum wins), adds the bias, applies ReLU.
//
// Backward (same algebra as conv_pool_bwd.hip, fp32 operands): the gradient of filter f of
// sample n reaches only its argmax window.  dW / db: one workgroup per (filter, sample
// split), partial sums per split (summed in order on the host side: deterministic).  dTable:
// one wave per (sample, filter) pair, fp32 row atomics (E per window row).
#include "common.h"

namespace pv {
namespace convf32 {

constexpr int FW = 150;                  // filters per width
constexpr int FG = 32;                   // filters per group: two 16-wide MFMA tiles
constexpr int NG = (FW + FG - 1) / FG;   // 5 groups
constexpr int EMAX = 112;                // LDS sized for E <= EMAX, E % 4 == 0
constexpr int CW = 128;                  // windows per chunk: 4 waves x 2 blocks x 16
constexpr int CR = CW + 3;               // table rows per chunk
constexpr int NTH = 256;
constexpr int PPT = (CR * (EMAX / 4) + NTH - 1) / NTH;  // 16-byte row pieces per thread

struct Params {
  const int* ids;
  const float* table;
  const float* w3;
  const float* w4;
  float2* part;  // (N * nseg, 2 * FW): {segment max, argmax bits}
  int N, L, V, E, nseg, sw;
  unsigned seed;
  const unsigned* seed_ptr;
  unsigned row_offset;
  int thr, token_mode;
};

// keep masks of fp32 columns 4pc .. 4pc+3 of a row with row hash hr (ops/reference.py
// dropout_keep_mask: nibble mode for thr % 16 == 0, byte mode otherwise, token mode)
__device__ __forceinline__ u32x4 keep4(unsigned hr, int pc, int thr, int token_mode) {
  if (token_mode) {
    const unsigned m = ((int)(hr & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
    return u32x4{m, m, m, m};
  }
  u32x4 k;
  if ((thr & 15) == 0) {
    const unsigned h = dropout_group_hash(hr, (unsigned)(pc >> 1)) >> (16 * (pc & 1));
    const unsigned t = (unsigned)thr >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = ((h >> (4 * i)) & 0xFu) >= t ? 0xFFFFFFFFu : 0u;
  } else {
    const unsigned h = dropout_group_hash(hr, (unsigned)pc);
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = (int)((h >> (8 * i)) & 0xFFu) >= thr ? 0xFFFFFFFFu : 0u;
  }
  return k;
}

// keep bit of column e (the same specification, one element)
__device__ __forceinline__ bool keep1(unsigned hr, int e, int thr, int token_mode) {
  if (token_mode) return (int)(hr & 0xFFu) >= thr;
  if ((thr & 15) == 0) {
    const unsigned h = dropout_group_hash(hr, (unsigned)(e >> 3));
    return ((h >> (4 * (e & 7))) & 0xFu) >= ((unsigned)thr >> 4);
  }
  const unsigned h = dropout_group_hash(hr, (unsigned)(e >> 2));
  return (int)((h >> (8 * (e & 3))) & 0xFFu) >= thr;
}

__device__ __forceinline__ bool better(float v, int i, float bv, int bi) {
  return v > bv || (v == bv && i < bi);
}

// EC > 0: E fixed at compile time (the reference's 100): the K loops unroll completely, every
// LDS read takes a constant offset and no loop / address VALU sits between the MFMAs (the
// fp32 MFMA runs on the SIMD's vector ALUs, so every VALU instruction in the stream costs
// MFMA time: SQ_VALU_MFMA_COEXEC_CYCLES = 0); EC = 0: any E % 4 == 0 <= EMAX.
template <int EC>
__global__ __launch_bounds__(NTH, 1) void conv_f32_fwd_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) float wl[7 * EMAX * FG];  // [kk][16][2 tiles]
  __shared__ __attribute__((aligned(16))) float xl[CR * EMAX];      // [row][E]
  __shared__ float2 red[4][2][FG];
  const unsigned seed = p.seed + (p.seed_ptr ? *p.seed_ptr : 0u);
  const int E = EC > 0 ? EC : p.E, E4 = E >> 2;
  const int g = blockIdx.x % NG, slot = blockIdx.x / NG, nslots = gridDim.x / NG;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int items = p.N * p.nseg;
  if (slot >= items) return;  // whole workgroup: uniform
  // this group's weights -> LDS once: wl[kk * 32 + 2 * f16 + t] = W[g*32 + 16t + f16][kk],
  // kk < 3E the k = 3 window's (tap, column) index, then 4E of the k = 4 window's
  for (int x = threadIdx.x; x < 7 * E * FG; x += NTH) {
    const int kk = x / FG, r = x - kk * FG;
    const int f = g * FG + (r & 1) * 16 + (r >> 1);
    float v = 0.f;
    if (f < FW) v = kk < 3 * E ? p.w3[(size_t)f * 3 * E + kk] : p.w4[(size_t)f * 4 * E + (kk - 3 * E)];
    wl[x] = v;
  }
  const int nw3 = p.L - 2, nw4 = p.L - 3;
  auto seg_end = [&](int seg) { return min((seg + 1) * p.sw, nw3); };
  auto nch = [&](int it) {
    const int seg = it % p.nseg;
    return (seg_end(seg) - seg * p.sw + CW - 1) / CW;
  };
  // Row staging, two loads deep: the token ids of chunk k + 2 and the table rows of chunk
  // k + 1 (addressed by the ids loaded one iteration earlier) are issued before chunk k's
  // MFMAs and waited for only when chunk k + 1 is stored to LDS (an id -> row chain per
  // piece inside one iteration exposed two global latencies per chunk).
  // (the validity selects wait for their loads, so they are kept as bit masks and applied
  // only where the loaded values are consumed)
  int tk[PPT];
  u32x4 v[PPT];
  unsigned idok = 0u, rowok = 0u;
  auto ids_load = [&](int it, int c) {
    const int n = it / p.nseg, t0 = (it % p.nseg) * p.sw + c * CW;
    idok = 0u;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int q = threadIdx.x + i * NTH;
      const int r = q / E4, t = t0 + r;
      const bool ok = r < CR && t < p.L;
      tk[i] = p.ids[(size_t)n * p.L + (ok ? t : 0)];
      idok |= (ok ? 1u : 0u) << i;
    }
  };
  auto rows_load = [&]() {
    rowok = 0u;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int q = threadIdx.x + i * NTH;
      const int pc = q % E4, tok = tk[i];
      const bool ok = ((idok >> i) & 1u) && tok >= 0 && tok < p.V;
      v[i] = *reinterpret_cast<const u32x4*>(p.table + (size_t)(ok ? tok : 0) * E + 4 * pc);
      rowok |= (ok ? 1u : 0u) << i;
    }
  };
  auto stage_store = [&](int it, int c) {
    const int n = it / p.nseg, t0 = (it % p.nseg) * p.sw + c * CW;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int q = threadIdx.x + i * NTH;
      const int r = q / E4, pc = q - r * E4;
      if (r < CR) {
        u32x4 x = v[i];
        const unsigned m = ((rowok >> i) & 1u) ? 0xFFFFFFFFu : 0u;
        x &= u32x4{m, m, m, m};
        if (p.thr > 0) x &= keep4(dropout_row_hash(seed, p.row_offset + (unsigned)(n * p.L + t0 + r)), pc, p.thr,
                                  p.token_mode);
        *reinterpret_cast<u32x4*>(xl + r * E + 4 * pc) = x;
      }
    }
  };
  auto next = [&](int& it, int& c) {
    if (++c >= nch(it)) {
      c = 0;
      it += nslots;
    }
  };
  f32x4 m[2][2];  // running max [width][tile]: rows 4*(lane/16)+r, filter 16t + lane%16
  int ix[2][2][4];
  auto reset = [&]() {
#pragma unroll
    for (int w = 0; w < 2; ++w)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        m[w][t] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
        for (int r = 0; r < 4; ++r) ix[w][t][r] = 0x7FFFFFFF;
      }
  };
  reset();
  const int a_off = (wave * 32 + (lane & 15)) * E + (lane >> 4);  // block 0's A element of step 0
  const int b_off = (lane >> 4) * FG + 2 * (lane & 15);
  const int S3 = 3 * E / 4, S4 = E;
  constexpr int U3 = EC > 0 ? 3 * EC / 4 : 1, U4 = EC > 0 ? EC / 4 : 1;  // full unroll at fixed E

  int it = slot, c = 0;
  ids_load(it, c);
  rows_load();
  int it2 = it, c2 = c;
  next(it2, c2);
  __syncthreads();  // wl complete (xl unused so far)
  stage_store(it, c);
  if (it2 < items) ids_load(it2, c2);
  __syncthreads();
  while (it < items) {
    // (it2, c2): the next chunk, whose ids are in tk; (it3, c3): the one after it
    if (it2 < items) rows_load();
    int it3 = it2, c3 = c2;
    next(it3, c3);
    if (it3 < items) ids_load(it3, c3);
    // ---- MFMAs of this chunk
    f32x4 acc[2][2][2];  // [block][width][tile]
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int w = 0; w < 2; ++w)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[b][w][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    // operands of step s + 1 are read before step s's MFMAs (LDS latency behind 8 x 32 cycles)
    const float* xa = xl + a_off;
    const float* wb3 = wl + b_off;
    const float* wb4 = wl + 3 * E * FG + b_off;
    float a0n = xa[0], a1n = xa[16 * E];
    float2 b3n = *reinterpret_cast<const float2*>(wb3), b4n = *reinterpret_cast<const float2*>(wb4);
#pragma unroll U3
    for (int s = 0; s < S3; ++s) {
      const float a0 = a0n, a1 = a1n;
      const float2 b3 = b3n, b4 = b4n;
      const int sn = s + 1;  // < S4: step S3's k = 3 operand read is unused (k = 4 region, in bounds)
      a0n = xa[4 * sn];
      a1n = xa[16 * E + 4 * sn];
      b3n = *reinterpret_cast<const float2*>(wb3 + 4 * sn * FG);
      b4n = *reinterpret_cast<const float2*>(wb4 + 4 * sn * FG);
      // keep the reads ahead of the MFMAs: left alone, hipcc sinks each read to its use and
      // waits for it at once (two exposed LDS latencies per step)
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // the 4 LDS reads
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // then the 8 MFMAs
      acc[0][0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b3.x, acc[0][0][0], 0, 0, 0);
      acc[0][0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b3.y, acc[0][0][1], 0, 0, 0);
      acc[0][1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b4.x, acc[0][1][0], 0, 0, 0);
      acc[0][1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b4.y, acc[0][1][1], 0, 0, 0);
      acc[1][0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b3.x, acc[1][0][0], 0, 0, 0);
      acc[1][0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b3.y, acc[1][0][1], 0, 0, 0);
      acc[1][1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b4.x, acc[1][1][0], 0, 0, 0);
      acc[1][1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b4.y, acc[1][1][1], 0, 0, 0);
    }
#pragma unroll U4
    for (int s = S3; s < S4; ++s) {  // the k = 4 window's 4th tap
      const float a0 = a0n, a1 = a1n;
      const float2 b4 = b4n;
      const int sn = s + 1 < S4 ? s + 1 : s;
      a0n = xa[4 * sn];
      a1n = xa[16 * E + 4 * sn];
      b4n = *reinterpret_cast<const float2*>(wb4 + 4 * sn * FG);
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      acc[0][1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b4.x, acc[0][1][0], 0, 0, 0);
      acc[0][1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b4.y, acc[0][1][1], 0, 0, 0);
      acc[1][1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b4.x, acc[1][1][0], 0, 0, 0);
      acc[1][1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b4.y, acc[1][1][1], 0, 0, 0);
    }
    // ---- running max / argmax (windows ascend per lane position: strict > keeps the first)
    const int seg = it % p.nseg;
    const int wend = seg_end(seg);
    const int t0 = seg * p.sw + c * CW;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int win = t0 + wave * 32 + b * 16 + 4 * (lane >> 4) + r;
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          const bool ok = win < min(wend, w == 0 ? nw3 : nw4);
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const float y = acc[b][w][t][r];
            if (ok && y > m[w][t][r]) {
              m[w][t][r] = y;
              ix[w][t][r] = win;
            }
          }
        }
      }
    __syncthreads();  // every wave is done reading xl
    if (it2 < items) stage_store(it2, c2);
    if (it2 != it) {  // this item's last chunk: merge rows, lanes, waves -> part
#pragma unroll
      for (int w = 0; w < 2; ++w)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float bv = m[w][t][0];
          int bi = ix[w][t][0];
#pragma unroll
          for (int r = 1; r < 4; ++r)
            if (better(m[w][t][r], ix[w][t][r], bv, bi)) {
              bv = m[w][t][r];
              bi = ix[w][t][r];
            }
#pragma unroll
          for (int o = 16; o < 64; o <<= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (better(ov, oi, bv, bi)) {
              bv = ov;
              bi = oi;
            }
          }
          if (lane < 16) red[wave][w][t * 16 + lane] = make_float2(bv, __int_as_float(bi));
        }
      __syncthreads();
      if (threadIdx.x < 2 * FG) {
        const int w = threadIdx.x / FG, fl = threadIdx.x % FG;
        float2 best = red[0][w][fl];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float2 o = red[q][w][fl];
          if (better(o.x, __float_as_int(o.y), best.x, __float_as_int(best.y))) best = o;
        }
        const int f = g * FG + fl;  // red column 16t + f16 = the filter's offset in the group
        if (f < FW) p.part[(size_t)it * (2 * FW) + w * FW + f] = best;
      }
      reset();
    }
    __syncthreads();  // xl holds the next chunk; red free again
    it = it2;
    c = c2;
    it2 = it3;
    c2 = c3;
  }
}

// segments in window order (strict >: the earliest maximum wins), bias, ReLU
__global__ __launch_bounds__(256) void conv_f32_finalize_kernel(const float2* __restrict__ part,
                                                                const float* __restrict__ b3,
                                                                const float* __restrict__ b4, float* pooled,
                                                                int* argmax, int N, int nseg, float scale) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * 2 * FW) return;
  const int n = i / (2 * FW), f = i - n * (2 * FW);
  float bv = -INFINITY;
  int bi = 0;
  for (int s = 0; s < nseg; ++s) {
    const float2 q = part[((size_t)n * nseg + s) * (2 * FW) + f];
    if (q.x > bv || s == 0) {
      bv = q.x;
      bi = __float_as_int(q.y);
    }
  }
  const float y = bv * scale + (f < FW ? b3[f] : b4[f - FW]);
  pooled[i] = y > 0.f ? y : 0.f;
  argmax[i] = bi;
}

// ---- dW, db: grid (2 * FW, nsplit); each wave takes 4 samples per round (their id and table
// loads in flight together); lane l owns window elements l + 64 m (tap j = x / E, column
// e = x % E, fixed per lane)
constexpr int DW_M = (4 * EMAX + 63) / 64;  // 7
constexpr int DW_U = 4;
__global__ __launch_bounds__(256) void conv_f32_dw_kernel(const float* __restrict__ gpool,
                                                          const float* __restrict__ pooled,
                                                          const int* __restrict__ argmax, const int* __restrict__ ids,
                                                          const float* __restrict__ table, float* dwpart,
                                                          float* dbpart, int N, int L, int E, int V, int per,
                                                          unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                                                          int thr, int token_mode, float scale) {
  __shared__ float red[4][4 * EMAX];
  __shared__ float gs[4];
  if (seed_ptr) seed += *seed_ptr;
  const int f = blockIdx.x, split = blockIdx.y, K = f < FW ? 3 : 4, KE = K * E;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = split * per, n1 = min(N, n0 + per);
  int jq[DW_M], eq[DW_M];
#pragma unroll
  for (int q = 0; q < DW_M; ++q) {
    const int x = lane + 64 * q;
    jq[q] = x < KE ? x / E : -1;
    eq[q] = x < KE ? x - jq[q] * E : 0;
  }
  float acc[DW_M];
#pragma unroll
  for (int q = 0; q < DW_M; ++q) acc[q] = 0.f;
  float gsum = 0.f;
  for (int nb = n0 + wave * DW_U; nb < n1; nb += 4 * DW_U) {
    float g[DW_U];
    int a[DW_U];
#pragma unroll
    for (int u = 0; u < DW_U; ++u) {
      const int n = nb + u;
      g[u] = 0.f;
      a[u] = 0;
      if (n < n1) {
        const size_t o = (size_t)n * (2 * FW) + f;
        const float gv = gpool[o];
        const bool live = pooled[o] > 0.f && gv != 0.f;
        g[u] = live ? gv : 0.f;
        a[u] = live ? argmax[o] : 0;
      }
      gsum += g[u];
    }
    int tok[DW_U][DW_M];
#pragma unroll
    for (int u = 0; u < DW_U; ++u)
#pragma unroll
      for (int q = 0; q < DW_M; ++q)
        tok[u][q] = (g[u] != 0.f && jq[q] >= 0) ? ids[(size_t)(nb + u) * L + a[u] + jq[q]] : -1;
#pragma unroll
    for (int u = 0; u < DW_U; ++u)
#pragma unroll
      for (int q = 0; q < DW_M; ++q) {
        const int t = tok[u][q];
        float xv = (t >= 0 && t < V) ? table[(size_t)t * E + eq[q]] : 0.f;
        if (thr > 0 && xv != 0.f &&
            !keep1(dropout_row_hash(seed, row_offset + (unsigned)((nb + u) * L + a[u] + jq[q])), eq[q], thr,
                   token_mode))
          xv = 0.f;
        acc[q] = fmaf(g[u], xv, acc[q]);
      }
  }
#pragma unroll
  for (int q = 0; q < DW_M; ++q) {
    const int x = lane + 64 * q;
    if (x < 4 * EMAX) red[wave][x] = acc[q];
  }
  if (lane == 0) gs[wave] = gsum;  // the same in every lane
  __syncthreads();
  float* out = dwpart + ((size_t)split * (2 * FW) + f) * (4 * E);
  for (int x = threadIdx.x; x < KE; x += 256) out[x] = scale * (((red[0][x] + red[1][x]) + red[2][x]) + red[3][x]);
  if (threadIdx.x == 0) dbpart[(size_t)split * (2 * FW) + f] = ((gs[0] + gs[1]) + gs[2]) + gs[3];
}

// ---- dTable: one wave per (sample, filter) pair; fp32 row atomics
__global__ __launch_bounds__(256) void conv_f32_dx_kernel(const float* __restrict__ gpool,
                                                          const float* __restrict__ pooled,
                                                          const int* __restrict__ argmax, const int* __restrict__ ids,
                                                          const float* __restrict__ w3, const float* __restrict__ w4,
                                                          float* dtable, int N, int L, int E, int V, unsigned seed,
                                                          const unsigned* seed_ptr, unsigned row_offset, int thr,
                                                          int token_mode, float scale) {
  if (seed_ptr) seed += *seed_ptr;
  const int lane = threadIdx.x & 63;
  const long pair = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= (long)N * 2 * FW) return;
  const int n = (int)(pair / (2 * FW)), f = (int)(pair - (long)n * 2 * FW);
  const float g = gpool[pair];
  if (!(pooled[pair] > 0.f) || g == 0.f) return;
  const int a = argmax[pair], K = f < FW ? 3 : 4;
  const float* w = f < FW ? w3 + (size_t)f * 3 * E : w4 + (size_t)(f - FW) * 4 * E;
  const float gs = g * scale;
  for (int j = 0; j < K; ++j) {
    const int t = a + j;
    const int tok = ids[(size_t)n * L + t];
    if (!PV_OK(tok >= 0 && tok < V, PV_ERR_ID) || tok < 0 || tok >= V) continue;
    const unsigned hr = thr > 0 ? dropout_row_hash(seed, row_offset + (unsigned)(n * L + t)) : 0u;
    for (int e = lane; e < E; e += 64) {
      if (thr > 0 && !keep1(hr, e, thr, token_mode)) continue;
      atomicAdd(dtable + (size_t)tok * E + e, gs * w[j * E + e]);
    }
  }
}

// ---- dTable for small vocabularies (V * E * 4 B <= DXP_LDS: the char-level tables): the
// global-atomic kernel above sends every (pair, row, column) add of the ~100-row table to the
// same few thousand L2 addresses.  Here each workgroup accumulates its pairs in an LDS copy of
// the table (LDS atomics), then writes it as one partial table; a second kernel sums the
// partials in workgroup order into dtable.
constexpr int DXP_LDS = 64 * 1024;
__global__ __launch_bounds__(256) void conv_f32_dx_lds_kernel(const float* __restrict__ gpool,
                                                              const float* __restrict__ pooled,
                                                              const int* __restrict__ argmax,
                                                              const int* __restrict__ ids,
                                                              const float* __restrict__ w3,
                                                              const float* __restrict__ w4, float* partial, int N,
                                                              int L, int E, int V, unsigned seed,
                                                              const unsigned* seed_ptr, unsigned row_offset, int thr,
                                                              int token_mode, float scale) {
  __shared__ float tab[DXP_LDS / 4];
  if (seed_ptr) seed += *seed_ptr;
  const int VE = V * E;
  for (int x = threadIdx.x; x < VE; x += 256) tab[x] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long pairs = (long)N * 2 * FW;
  for (long pair = (long)blockIdx.x * 4 + (threadIdx.x >> 6); pair < pairs; pair += (long)gridDim.x * 4) {
    const float g = gpool[pair];
    if (!(pooled[pair] > 0.f) || g == 0.f) continue;  // wave-uniform
    const int n = (int)(pair / (2 * FW)), f = (int)(pair - (long)n * 2 * FW);
    const int a = argmax[pair], K = f < FW ? 3 : 4;
    const float* w = f < FW ? w3 + (size_t)f * 3 * E : w4 + (size_t)(f - FW) * 4 * E;
    const float gs = g * scale;
    for (int j = 0; j < K; ++j) {
      const int t = a + j;
      const int tok = ids[(size_t)n * L + t];
      if (tok < 0 || tok >= V) continue;
      const unsigned hr = thr > 0 ? dropout_row_hash(seed, row_offset + (unsigned)(n * L + t)) : 0u;
      for (int e = lane; e < E; e += 64) {
        if (thr > 0 && !keep1(hr, e, thr, token_mode)) continue;
        atomicAdd(tab + tok * E + e, gs * w[j * E + e]);
      }
    }
  }
  __syncthreads();
  float* out = partial + (size_t)blockIdx.x * VE;
  for (int x = threadIdx.x; x < VE; x += 256) out[x] = tab[x];
}

__global__ __launch_bounds__(256) void conv_f32_dx_sum_kernel(const float* __restrict__ partial, float* dtable,
                                                              int VE, int nparts) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= VE) return;
  float s = 0.f;
  for (int b = 0; b < nparts; ++b) s += partial[(size_t)b * VE + x];
  dtable[x] += s;
}

PV_DEBUG_EXPORT(convf32)
}  // namespace convf32
}  // namespace pv

using namespace pv::convf32;

PV_API int pv_conv_f32_groups() { return NG; }
PV_API int pv_conv_f32_chunk() { return CW; }
PV_API int pv_conv_f32_emax() { return EMAX; }

PV_API int pv_conv_f32_fwd(const int* ids, const float* table, const float* w3, const float* w4, const float* b3,
                           const float* b4, void* part, float* pooled, int* argmax, int N, int L, int V, int E,
                           int nseg, int sw, int nslots, unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                           int thr, int token_mode, float scale, void* stream) {
  if (N <= 0) return 0;
  const int nw3 = L - 2;
  if (L < 4 || E < 4 || E > EMAX || (E & 3) || nseg < 1 || sw < CW || sw % CW || (long)nseg * sw < nw3 ||
      (long)(nseg - 1) * sw >= nw3 || nslots < 1)
    return -1;
  hipStream_t st = (hipStream_t)stream;
  Params p{ids, table, w3, w4, (float2*)part, N, L, V, E, nseg, sw, seed, seed_ptr, row_offset, thr, token_mode};
  if (E == 100)
    hipLaunchKernelGGL(conv_f32_fwd_kernel<100>, dim3(nslots * NG), dim3(NTH), 0, st, p);
  else
    hipLaunchKernelGGL(conv_f32_fwd_kernel<0>, dim3(nslots * NG), dim3(NTH), 0, st, p);
  PV_LAUNCH_CHECK();
  const int tot = N * 2 * FW;
  hipLaunchKernelGGL(conv_f32_finalize_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, (const float2*)part, b3, b4,
                     pooled, argmax, N, nseg, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_conv_f32_bwd_dw(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                              const float* table, float* dwpart, float* dbpart, int N, int L, int E, int V, int nsplit,
                              unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                              float scale, void* stream) {
  if (E < 1 || E > EMAX || nsplit < 1) return -1;
  if (N <= 0) return 0;
  const int per = (N + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(conv_f32_dw_kernel, dim3(2 * FW, nsplit), dim3(256), 0, (hipStream_t)stream, gpool, pooled,
                     argmax, ids, table, dwpart, dbpart, N, L, E, V, per, seed, seed_ptr, row_offset, thr, token_mode,
                     scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// LDS-privatised dTable: partial tables per workgroup (nparts x V x E fp32 scratch)
PV_API int pv_conv_f32_dx_lds_max() { return DXP_LDS / 4; }

PV_API int pv_conv_f32_bwd_dx_lds(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                  const float* w3, const float* w4, float* partial, float* dtable, int N, int L, int E,
                                  int V, int nparts, unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                                  int thr, int token_mode, float scale, void* stream) {
  if (E < 1 || V < 1 || (long)V * E > DXP_LDS / 4 || nparts < 1) return -1;
  if (N <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(conv_f32_dx_lds_kernel, dim3(nparts), dim3(256), 0, st, gpool, pooled, argmax, ids, w3, w4,
                     partial, N, L, E, V, seed, seed_ptr, row_offset, thr, token_mode, scale);
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv_f32_dx_sum_kernel, dim3((V * E + 255) / 256), dim3(256), 0, st, (const float*)partial,
                     dtable, V * E, nparts);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_conv_f32_bwd_dx(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                              const float* w3, const float* w4, float* dtable, int N, int L, int E, int V,
                              unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                              float scale, void* stream) {
  if (E < 1) return -1;
  if (N <= 0) return 0;
  const long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_f32_dx_kernel, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, (hipStream_t)stream, gpool,
                     pooled, argmax, ids, w3, w4, dtable, N, L, E, V, seed, seed_ptr, row_offset, thr, token_mode,
                     scale);
  PV_LAUNCH_CHECK();
  return 0;
}
