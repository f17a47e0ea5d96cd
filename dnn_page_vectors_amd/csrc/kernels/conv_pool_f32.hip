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
// order (first maximum wins), adds the bias, applies ReLU.  That is v1 (any E % 4 == 0 up to
// EMAX; fully unrolled at E = 100).  At E = 100 the production kernel is v2: the same MFMA
// stream in 4 waves over 64-window chunks while 4 loader waves stage the next chunk into a
// second LDS buffer.  With dropout, a keep-bit plane (conv_f32_mask_kernel, one u32 per 32
// columns per row) is computed once and read by all five filter groups.
//
// Backward (same algebra as conv_pool_bwd.hip, fp32 operands): the gradient of filter f of
// sample n reaches only its argmax window.  dW / db: one workgroup per (filter, sample
// split), partial sums per split (summed in order on the host side: deterministic).  dTable:
// wave-private LDS tables for V x E <= 10 K (the char vocabularies; deterministic), a shared
// LDS table with float atomics up to 16 K, fp32 row atomics above (deterministic mode replaces
// those two with an ordered index_add_ in ops/conv_pool.py).
#include "common.h"

namespace pv {
namespace convf32 {
PV_DEBUG_FLAG

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
  const unsigned* mask;  // keep-bit plane (conv_f32_mask_kernel) or nullptr: hash inline
  int wpr;               // mask words per row
};

// keep bits of the 4 fp32 columns 4pc .. 4pc+3 from their row's mask word -> AND masks
__device__ __forceinline__ u32x4 bits4(unsigned word, int pc) {
  const unsigned nib = word >> (4 * (pc & 7));
  return u32x4{0u - (nib & 1u), 0u - ((nib >> 1) & 1u), 0u - ((nib >> 2) & 1u), 0u - ((nib >> 3) & 1u)};
}

// keep masks of fp32 columns 4pc .. 4pc+3 of a row with row hash hr (ops/reference.py
// dropout_keep_mask: nibble mode for thr % 16 == 0, byte mode otherwise, token mode)
__device__ __forceinline__ u32x4 keep4(unsigned hr, int pc, int thr, int token_mode) {
  if (token_mode) {
    const unsigned m = ((int)(hr & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
    return u32x4{m, m, m, m};
  }
  u32x4 k;
  if ((thr & 15) == 0) {
    const unsigned b = dropout_keep_bits8(dropout_group_hash(hr, (unsigned)(pc >> 1)), thr >> 4) >> (4 * (pc & 1));
#pragma unroll
    for (int i = 0; i < 4; ++i) k[i] = 0u - ((b >> i) & 1u);
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
  if ((thr & 15) == 0) return dropout_nibble(dropout_group_hash(hr, (unsigned)(e >> 3)), e & 7) >= ((unsigned)thr >> 4);
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
  unsigned mk[PPT], mk1[PPT];  // mask words of the chunk whose ids are in tk / whose rows are in v
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
      const size_t row = (size_t)n * p.L + (ok ? t : 0);
      tk[i] = p.ids[row];
      if (p.mask) mk[i] = p.mask[row * p.wpr + ((q - r * E4) >> 3)];
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
      mk1[i] = mk[i];
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
        if (p.mask) x &= bits4(mk1[i], pc);
        else if (p.thr > 0)
          x &= keep4(dropout_row_hash(seed, p.row_offset + (unsigned)(n * p.L + t0 + r)), pc, p.thr, p.token_mode);
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

// ---- v2: role-split workgroup (the bf16 forward's v7 pattern) ----------------------------
// 512 threads: waves 0-3 (one per SIMD) run the MFMAs of a 64-window chunk (one 16-window
// block each) from LDS buffer k % 2 while waves 4-7 gather, mask and store chunk k + 1 into the
// other buffer; one workgroup barrier per chunk.  The loaders also merge the MFMA waves'
// per-item maxima (written to red[k % 2] before the barrier) into `part`.  E is fixed at 100
// (LDS: 89.6 KB weights + 2 x 26.8 KB rows).
constexpr int NTH2 = 512, CW2 = 64, CR2 = CW2 + 3, E2 = 100;
constexpr int PPT2 = (CR2 * (E2 / 4) + 255) / 256;  // 16-byte pieces per loader thread (7)

// MM: the loader's mask source at compile time (0 no dropout, 1 keep-bit plane, 2 inline
// hashes): no per-piece runtime branches in the staging code
template <int MM>
__global__ __launch_bounds__(NTH2, 1) void conv_f32_fwd2_kernel(Params p) {
  constexpr int E = E2, E4 = E / 4;
  __shared__ __attribute__((aligned(16))) float wl[7 * E * FG];
  __shared__ __attribute__((aligned(16))) float xl[2][CR2 * E];
  __shared__ float2 red[2][4][2][FG];
  const unsigned seed = p.seed + (p.seed_ptr ? *p.seed_ptr : 0u);
  const int g = blockIdx.x % NG, slot = blockIdx.x / NG, nslots = gridDim.x / NG;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int items = p.N * p.nseg;
  if (slot >= items) return;
  for (int x = threadIdx.x; x < 7 * E * FG; x += NTH2) {
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
    return (seg_end(seg) - seg * p.sw + CW2 - 1) / CW2;
  };
  auto next = [&](int& it, int& c) {
    if (++c >= nch(it)) {
      c = 0;
      it += nslots;
    }
  };
  if (wave >= 4) {
    // ---------------- loader role
    const int lt = threadIdx.x - 256;
    int tk[PPT2];
    unsigned mk[PPT2], mk1[PPT2];
    u32x4 v[PPT2];
    unsigned idok = 0u, rowok = 0u;
    auto ids_load = [&](int it, int c) {
      const int n = it / p.nseg, t0 = (it % p.nseg) * p.sw + c * CW2;
      idok = 0u;
#pragma unroll
      for (int i = 0; i < PPT2; ++i) {
        const int q = lt + i * 256;
        const int r = q / E4, t = t0 + r;
        const bool ok = r < CR2 && t < p.L;
        const size_t row = (size_t)n * p.L + (ok ? t : 0);
        tk[i] = p.ids[row];
        if constexpr (MM == 1) mk[i] = p.mask[row * 4 + ((q - r * E4) >> 3)];  // wpr = 4 at E = 100
        idok |= (ok ? 1u : 0u) << i;
      }
    };
    auto rows_load = [&]() {
      rowok = 0u;
#pragma unroll
      for (int i = 0; i < PPT2; ++i) {
        const int q = lt + i * 256;
        const int pc = q % E4, tok = tk[i];
        const bool ok = ((idok >> i) & 1u) && tok >= 0 && tok < p.V;
        v[i] = *reinterpret_cast<const u32x4*>(p.table + (size_t)(ok ? tok : 0) * E + 4 * pc);
        if constexpr (MM == 1) mk1[i] = mk[i];
        rowok |= (ok ? 1u : 0u) << i;
      }
    };
    auto stage_store = [&](int it, int c, float* dst) {
      const int n = it / p.nseg, t0 = (it % p.nseg) * p.sw + c * CW2;
#pragma unroll
      for (int i = 0; i < PPT2; ++i) {
        const int q = lt + i * 256;
        const int r = q / E4, pc = q - r * E4;
        if (r < CR2) {
          u32x4 x = v[i];
          const unsigned m = ((rowok >> i) & 1u) ? 0xFFFFFFFFu : 0u;
          x &= u32x4{m, m, m, m};
          if constexpr (MM == 1) x &= bits4(mk1[i], pc);
          else if constexpr (MM == 2)
            x &= keep4(dropout_row_hash(seed, p.row_offset + (unsigned)(n * p.L + t0 + r)), pc, p.thr,
                       p.token_mode);
          *reinterpret_cast<u32x4*>(dst + r * E + 4 * pc) = x;
        }
      }
    };
    // the item whose maxima the MFMA waves left in red[par] before the barrier just passed
    auto merge = [&](int it, int par) {
      if (lt < 2 * FG) {
        const int w = lt / FG, fl = lt % FG;
        float2 best = red[par][0][w][fl];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float2 o = red[par][q][w][fl];
          if (better(o.x, __float_as_int(o.y), best.x, __float_as_int(best.y))) best = o;
        }
        const int f = g * FG + fl;
        if (f < FW) p.part[(size_t)it * (2 * FW) + w * FW + f] = best;
      }
    };
    int it = slot, c = 0;
    ids_load(it, c);
    rows_load();
    stage_store(it, c, xl[0]);
    int it1 = it, c1 = c;
    next(it1, c1);
    if (it1 < items) ids_load(it1, c1);
    int par = 0, done_it = -1;
    __syncthreads();  // S0: weights + chunk 0
    while (it < items) {
      // chunk k = (it, c) is being computed from xl[par]; stage chunk k + 1 into xl[par ^ 1]
      if (it1 < items) {
        rows_load();
        int it2 = it1, c2 = c1;
        next(it2, c2);
        if (it2 < items) ids_load(it2, c2);
        stage_store(it1, c1, xl[par ^ 1]);
      }
      if (done_it >= 0) merge(done_it, par ^ 1);
      done_it = (it1 != it) ? it : -1;  // chunk k ends its item: red[par] after the barrier
      __syncthreads();  // B_{k+1}
      it = it1;
      c = c1;
      next(it1, c1);
      par ^= 1;
    }
    if (done_it >= 0) merge(done_it, par ^ 1);
    return;
  }
  // ---------------- MFMA role
  f32x4 m[2][2];
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
  const int a_off = (wave * 16 + (lane & 15)) * E + (lane >> 4);
  const int b_off = (lane >> 4) * FG + 2 * (lane & 15);
  constexpr int S3 = 3 * E / 4, S4 = E;
  int it = slot, c = 0, par = 0;
  __syncthreads();  // S0
  while (it < items) {
    const float* xa = xl[par] + a_off;
    const float* wb3 = wl + b_off;
    const float* wb4 = wl + 3 * E * FG + b_off;
    f32x4 acc[2][2];
#pragma unroll
    for (int w = 0; w < 2; ++w)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[w][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float an = xa[0];
    float2 b3n = *reinterpret_cast<const float2*>(wb3), b4n = *reinterpret_cast<const float2*>(wb4);
#pragma unroll
    for (int s = 0; s < S3; ++s) {
      const float a = an;
      const float2 b3 = b3n, b4 = b4n;
      an = xa[4 * (s + 1)];
      b3n = *reinterpret_cast<const float2*>(wb3 + 4 * (s + 1) * FG);
      b4n = *reinterpret_cast<const float2*>(wb4 + 4 * (s + 1) * FG);
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b3.x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b3.y, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b4.x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b4.y, acc[1][1], 0, 0, 0);
    }
#pragma unroll
    for (int s = S3; s < S4; ++s) {
      const float a = an;
      const float2 b4 = b4n;
      const int sn = s + 1 < S4 ? s + 1 : s;
      an = xa[4 * sn];
      b4n = *reinterpret_cast<const float2*>(wb4 + 4 * sn * FG);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b4.x, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b4.y, acc[1][1], 0, 0, 0);
    }
    const int seg = it % p.nseg;
    const int wend = seg_end(seg);
    const int t0 = seg * p.sw + c * CW2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int win = t0 + wave * 16 + 4 * (lane >> 4) + r;
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const bool ok = win < min(wend, w == 0 ? nw3 : nw4);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const float y = acc[w][t][r];
          if (ok && y > m[w][t][r]) {
            m[w][t][r] = y;
            ix[w][t][r] = win;
          }
        }
      }
    }
    int it1 = it, c1 = c;
    next(it1, c1);
    if (it1 != it) {  // item end: rows and lanes -> red[par] (the loaders merge the waves)
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
          if (lane < 16) red[par][wave][w][t * 16 + lane] = make_float2(bv, __int_as_float(bi));
        }
      reset();
    }
    __syncthreads();  // B_{k+1}
    it = it1;
    c = c1;
    par ^= 1;
  }
}

// ---- dropout keep-bit plane: bit j of word w of local row R = keep(column 32w + j) of flat row
// row_offset + R (ops/reference.py dropout_keep_mask).  The forward's five filter-group
// workgroups of a chunk, dW and dTable read one u32 per 32 columns instead of recomputing the
// hashes (the fp32 MFMA shares the SIMD's vector issue: every hash instruction cost MFMA time).
__global__ __launch_bounds__(256) void conv_f32_mask_kernel(unsigned* __restrict__ mask, long rows, int wpr,
                                                            unsigned seed, const unsigned* seed_ptr,
                                                            unsigned row_offset, int thr, int token_mode) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * wpr) return;
  if (seed_ptr) seed += *seed_ptr;
  const long R = i / wpr;
  const int w = (int)(i - R * wpr);
  const unsigned hr = dropout_row_hash(seed, row_offset + (unsigned)R);
  unsigned bits = 0u;
  if (token_mode) {
    bits = ((int)(hr & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
  } else if ((thr & 15) == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bits |= dropout_keep_bits8(dropout_group_hash(hr, (unsigned)(4 * w + q)), thr >> 4) << (8 * q);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const unsigned h = dropout_group_hash(hr, (unsigned)(8 * w + q));
#pragma unroll
      for (int j = 0; j < 4; ++j) bits |= ((int)((h >> (8 * j)) & 0xFFu) >= thr ? 1u : 0u) << (4 * q + j);
    }
  }
  mask[i] = bits;
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
                                                          int thr, int token_mode, float scale,
                                                          const unsigned* __restrict__ mask, int wpr) {
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
        if (thr > 0 && xv != 0.f) {
          const unsigned R = (unsigned)((nb + u) * L + a[u] + jq[q]);
          const bool keep = mask ? ((mask[(size_t)R * wpr + (eq[q] >> 5)] >> (eq[q] & 31)) & 1u) != 0u
                                 : keep1(dropout_row_hash(seed, row_offset + R), eq[q], thr, token_mode);
          if (!keep) xv = 0.f;
        }
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
                                                          int token_mode, float scale, const unsigned* __restrict__ mask, int wpr) {
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
    const unsigned hr = thr > 0 && !mask ? dropout_row_hash(seed, row_offset + (unsigned)(n * L + t)) : 0u;
    const unsigned* mrow = mask ? mask + (size_t)(n * L + t) * wpr : nullptr;
    for (int e = lane; e < E; e += 64) {
      if (thr > 0 && !(mrow ? ((mrow[e >> 5] >> (e & 31)) & 1u) != 0u : keep1(hr, e, thr, token_mode))) continue;
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
constexpr int DXP_NTH = 256;  // (1024 measured slower: 0.68 -> 0.82 ms per step)
__global__ __launch_bounds__(DXP_NTH) void conv_f32_dx_lds_kernel(const float* __restrict__ gpool,
                                                              const float* __restrict__ pooled,
                                                              const int* __restrict__ argmax,
                                                              const int* __restrict__ ids,
                                                              const float* __restrict__ w3,
                                                              const float* __restrict__ w4, float* partial, int N,
                                                              int L, int E, int V, unsigned seed,
                                                              const unsigned* seed_ptr, unsigned row_offset, int thr,
                                                              int token_mode, float scale, const unsigned* __restrict__ mask, int wpr) {
  __shared__ float tab[DXP_LDS / 4];
  if (seed_ptr) seed += *seed_ptr;
  const int VE = V * E;
  for (int x = threadIdx.x; x < VE; x += DXP_NTH) tab[x] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long pairs = (long)N * 2 * FW;
  for (long pair = (long)blockIdx.x * (DXP_NTH / 64) + (threadIdx.x >> 6); pair < pairs;
       pair += (long)gridDim.x * (DXP_NTH / 64)) {
    const float g = gpool[pair];
    if (!(pooled[pair] > 0.f) || g == 0.f) continue;  // wave-uniform
    const int n = (int)(pair / (2 * FW)), f = (int)(pair - (long)n * 2 * FW);
    const int a = argmax[pair], K = f < FW ? 3 : 4;
    const float* w = f < FW ? w3 + (size_t)f * 3 * E : w4 + (size_t)(f - FW) * 4 * E;
    const float gs = g * scale;
    // the window's token ids and weight rows loaded together (one latency per pair, not per row)
    int tok[4];
    float wv[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tok[j] = j < K ? ids[(size_t)n * L + a + j] : -1;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int e = lane + 64 * c;
        wv[j][c] = (j < K && e < E) ? w[j * E + e] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (tok[j] < 0 || tok[j] >= V) continue;
      const int t = a + j;
      const unsigned hr = thr > 0 && !mask ? dropout_row_hash(seed, row_offset + (unsigned)(n * L + t)) : 0u;
      const unsigned* mrow = mask ? mask + (size_t)(n * L + t) * wpr : nullptr;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int e = lane + 64 * c;
        if (e >= E) continue;
        if (thr > 0 && !(mrow ? ((mrow[e >> 5] >> (e & 31)) & 1u) != 0u : keep1(hr, e, thr, token_mode))) continue;
        atomicAdd(tab + tok[j] * E + e, gs * wv[j][c]);
      }
    }
  }
  __syncthreads();
  float* out = partial + (size_t)blockIdx.x * VE;
  for (int x = threadIdx.x; x < VE; x += DXP_NTH) out[x] = tab[x];
}

// V x E <= DXW_MAX (the ~100-symbol char tables): one PRIVATE LDS table per wave (4 x 40 KB),
// updated by plain read-add-write (a wave's LDS operations complete in order and its lanes
// hold distinct columns) instead of ds_add_f32, whose float-atomic unit retires ~0.3 lanes per
// clock per CU and serialised this kernel (0.6-0.7 ms per step); the four tables are summed
// into the workgroup's partial.
constexpr int DXW_MAX = 10240;
// 8 waves: waves w and w + 4 share table w % 4 and walk the same pairs, wave w adding columns
// 0..63 and wave w + 4 columns 64..127 (each address still has one writer), so twice as many
// waves hide the pairs' dependent loads
__global__ __launch_bounds__(512, 1) void conv_f32_dx_wave_kernel(const float* __restrict__ gpool,
                                                                  const float* __restrict__ pooled,
                                                                  const int* __restrict__ argmax,
                                                                  const int* __restrict__ ids,
                                                                  const float* __restrict__ w3,
                                                                  const float* __restrict__ w4, float* partial,
                                                                  int N, int L, int E, int V, unsigned seed,
                                                                  const unsigned* seed_ptr, unsigned row_offset,
                                                                  int thr, int token_mode, float scale) {
  __shared__ float tabs[4 * DXW_MAX];
  if (seed_ptr) seed += *seed_ptr;
  const int VE = V * E;
  for (int x = threadIdx.x; x < 4 * VE; x += 512) tabs[x] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = wave & 3;
  const int e = lane + 64 * (wave >> 2);
  float* tab = tabs + grp * VE;
  const long pairs = (long)N * 2 * FW;
  if (e - lane < E) {  // wave-uniform: the upper half has columns
    for (long pair = (long)blockIdx.x * 4 + grp; pair < pairs; pair += (long)gridDim.x * 4) {
      const float g = gpool[pair];
      if (!(pooled[pair] > 0.f) || g == 0.f) continue;  // wave-uniform
      const int n = (int)(pair / (2 * FW)), f = (int)(pair - (long)n * 2 * FW);
      const int a = argmax[pair], K = f < FW ? 3 : 4;
      const float* w = f < FW ? w3 + (size_t)f * 3 * E : w4 + (size_t)(f - FW) * 4 * E;
      const float gs = g * scale;
      int tok[4];
      float wv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tok[j] = j < K ? ids[(size_t)n * L + a + j] : -1;
        wv[j] = (j < K && e < E) ? w[j * E + e] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (tok[j] < 0 || tok[j] >= V) continue;
        const unsigned hr = thr > 0 ? dropout_row_hash(seed, row_offset + (unsigned)(n * L + a + j)) : 0u;
        if (e < E && (thr <= 0 || keep1(hr, e, thr, token_mode))) tab[tok[j] * E + e] += gs * wv[j];
      }
    }
  }
  __syncthreads();
  float* out = partial + (size_t)blockIdx.x * VE;
  for (int x = threadIdx.x; x < VE; x += 512) out[x] = ((tabs[x] + tabs[VE + x]) + tabs[2 * VE + x]) + tabs[3 * VE + x];
}

// partial tables -> dtable in a fixed order, in two levels (one thread per element walking all
// 256 partials was latency-bound at 40-60 us): level 1, thread (x, gy) sums its group's
// partials into the group's first partial row; level 2 adds the DXS_G group sums in order
constexpr int DXS_G = 16;
__global__ __launch_bounds__(256) void conv_f32_dx_sum1_kernel(float* __restrict__ partial, int VE, int nparts) {
  const int x = blockIdx.x * 256 + threadIdx.x, gy = blockIdx.y;
  const int chunk = (nparts + DXS_G - 1) / DXS_G, b0 = gy * chunk, b1 = min(nparts, b0 + chunk);
  if (x >= VE || b0 >= b1) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int b = b0;
  for (; b + 4 <= b1; b += 4)
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += partial[(size_t)(b + k) * VE + x];
  for (; b < b1; ++b) s[0] += partial[(size_t)b * VE + x];
  partial[(size_t)b0 * VE + x] = (s[0] + s[1]) + (s[2] + s[3]);
}

__global__ __launch_bounds__(256) void conv_f32_dx_sum2_kernel(const float* __restrict__ partial, float* dtable,
                                                               int VE, int nparts) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= VE) return;
  const int chunk = (nparts + DXS_G - 1) / DXS_G;
  float t = 0.f;
  for (int gy = 0; gy * chunk < nparts; ++gy) t += partial[(size_t)gy * chunk * VE + x];
  dtable[x] += t;
}

PV_DEBUG_EXPORT(convf32)
}  // namespace convf32
}  // namespace pv

using namespace pv::convf32;

static int g_fwd2 = 1;  // 1: role-split forward (v2) at E = 100; 0: v1 (A/B)
static int g_dxw = 1;   // 1: wave-private LDS dTable for V x E <= DXW_MAX; 0: shared table + ds_add_f32 (A/B)
PV_API void pv_conv_f32_set_dxw(int on) { g_dxw = on; }
PV_API void pv_conv_f32_set_v2(int on) { g_fwd2 = on; }
PV_API int pv_conv_f32_groups() { return NG; }

// keep-bit plane of rows local rows 0 .. rows-1 (flat rows row_offset + R), wpr words per row
PV_API int pv_conv_f32_mask(unsigned* mask, long rows, int wpr, unsigned seed, const unsigned* seed_ptr,
                            unsigned row_offset, int thr, int token_mode, void* stream) {
  if (rows < 0 || wpr < 1 || thr <= 0) return -1;
  if (rows == 0) return 0;
  const long n = rows * wpr;
  hipLaunchKernelGGL(conv_f32_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mask,
                     rows, wpr, seed, seed_ptr, row_offset, thr, token_mode);
  PV_LAUNCH_CHECK();
  return 0;
}
PV_API int pv_conv_f32_chunk() { return CW; }
PV_API int pv_conv_f32_emax() { return EMAX; }

PV_API int pv_conv_f32_fwd(const int* ids, const float* table, const float* w3, const float* w4, const float* b3,
                           const float* b4, void* part, float* pooled, int* argmax, int N, int L, int V, int E,
                           int nseg, int sw, int nslots, unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                           int thr, int token_mode, float scale, const unsigned* mask, int wpr, void* stream) {
  if (N <= 0) return 0;
  const int nw3 = L - 2;
  const bool v2 = E == E2 && g_fwd2;
  const int cw = v2 ? CW2 : CW;
  if (L < 4 || E < 4 || E > EMAX || (E & 3) || nseg < 1 || sw < cw || sw % cw || (long)nseg * sw < nw3 ||
      (long)(nseg - 1) * sw >= nw3 || nslots < 1)
    return -1;
  hipStream_t st = (hipStream_t)stream;
  if (mask && wpr < (E + 31) / 32) return -1;
  Params p{ids,  table,    w3,         w4,  (float2*)part, N,          L,    V,   E, nseg, sw,
           seed, seed_ptr, row_offset, thr, token_mode,    thr > 0 ? mask : nullptr, wpr};
  if (v2 && p.thr <= 0)
    hipLaunchKernelGGL(conv_f32_fwd2_kernel<0>, dim3(nslots * NG), dim3(NTH2), 0, st, p);
  else if (v2 && p.mask)
    hipLaunchKernelGGL(conv_f32_fwd2_kernel<1>, dim3(nslots * NG), dim3(NTH2), 0, st, p);
  else if (v2)
    hipLaunchKernelGGL(conv_f32_fwd2_kernel<2>, dim3(nslots * NG), dim3(NTH2), 0, st, p);
  else if (E == 100)
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
                              float scale, const unsigned* mask, int wpr, void* stream) {
  if (E < 1 || E > EMAX || nsplit < 1 || (mask && wpr < (E + 31) / 32)) return -1;
  if (N <= 0) return 0;
  const int per = (N + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(conv_f32_dw_kernel, dim3(2 * FW, nsplit), dim3(256), 0, (hipStream_t)stream, gpool, pooled,
                     argmax, ids, table, dwpart, dbpart, N, L, E, V, per, seed, seed_ptr, row_offset, thr, token_mode,
                     scale, mask, wpr);
  PV_LAUNCH_CHECK();
  return 0;
}

// LDS-privatised dTable: partial tables per workgroup (nparts x V x E fp32 scratch)
PV_API int pv_conv_f32_dx_lds_max() { return DXP_LDS / 4; }

PV_API int pv_conv_f32_bwd_dx_lds(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                  const float* w3, const float* w4, float* partial, float* dtable, int N, int L, int E,
                                  int V, int nparts, unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                                  int thr, int token_mode, float scale, const unsigned* mask, int wpr, void* stream) {
  if (E < 1 || E > 128 || V < 1 || (long)V * E > DXP_LDS / 4 || nparts < 1 || (mask && wpr < (E + 31) / 32))
    return -1;
  if (N <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (V * E <= DXW_MAX && E <= 128 && g_dxw)
    hipLaunchKernelGGL(conv_f32_dx_wave_kernel, dim3(nparts), dim3(512), 0, st, gpool, pooled, argmax, ids, w3, w4,
                       partial, N, L, E, V, seed, seed_ptr, row_offset, thr, token_mode, scale);
  else
    hipLaunchKernelGGL(conv_f32_dx_lds_kernel, dim3(nparts), dim3(DXP_NTH), 0, st, gpool, pooled, argmax, ids, w3, w4,
                     partial, N, L, E, V, seed, seed_ptr, row_offset, thr, token_mode, scale, mask, wpr);
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv_f32_dx_sum1_kernel, dim3((V * E + 255) / 256, DXS_G), dim3(256), 0, st, partial, V * E,
                     nparts);
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(conv_f32_dx_sum2_kernel, dim3((V * E + 255) / 256), dim3(256), 0, st, (const float*)partial,
                     dtable, V * E, nparts);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_conv_f32_bwd_dx(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                              const float* w3, const float* w4, float* dtable, int N, int L, int E, int V,
                              unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                              float scale, const unsigned* mask, int wpr, void* stream) {
  if (E < 1 || (mask && wpr < (E + 31) / 32)) return -1;
  if (N <= 0) return 0;
  const long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_f32_dx_kernel, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, (hipStream_t)stream, gpool,
                     pooled, argmax, ids, w3, w4, dtable, N, L, E, V, seed, seed_ptr, row_offset, thr, token_mode,
                     scale, mask, wpr);
  PV_LAUNCH_CHECK();
  return 0;
}
