// K5-K7: cosine relevance + gamma-softmax + cross-entropy, fused.
//
// Reference head (dssm_cnn_v2/cnn_dssm_th.py:159-182): R = clip(cos(q, d), 0, 1),
// P(D+|Q) = exp(gR+) / sum_j exp(gR_j), loss = BCE(y=1, P) = -log clip(P, 1e-7, 1-1e-7).
//
// (1) explicit mode (reference parity, 1 positive + J negatives per row):
//     dssm_explicit_kernel computes loss, P and the gradients w.r.t. the L2-normalised
//     vectors in ONE pass (one wave per row) — forward and backward fused.
//
// (2) in-batch / cross-GPU mode (new): every query is scored against all M gathered
//     documents, S = g*clip(Qn.Dn^T) (B x M) with bf16 MFMA, never materialised:
//       ib_fwd      : per (query block, doc split) partial sum_j exp(S_ij - g), summed
//                     over the splits in a fixed order (ib_rowsum: no atomics)
//                     (no running max needed: clip bounds S to [0, g] (or [-g, g]), so
//                     exp(S - g) <= 1 and the sum cannot overflow)
//       ib_bwd<ROW> : recompute the S tile, G = gscale*g*P*clip' (bf16, in registers),
//                     then dQ = G.Dn  (ROW=true, rows=queries)  or
//                          dD = G^T.Qn (ROW=false, rows=docs) with MFMA; per-split
//                     partials are summed by ib_split_reduce.
//       ib_pos      : the positive logit (same bf16 inputs) and the one-hot term of
//                     the gradient, -gscale*g*clip' * {d_pos, q}.
#include "common.h"
#include <stdlib.h>
#include <algorithm>
#include <type_traits>

namespace pv {
namespace loss {
PV_DEBUG_FLAG

constexpr float BCE_EPS = 1e-7f;

// sum over the ns split planes of a partial-sum buffer at float4 index i (plane stride `plane`
// float4s), in plane order — the loads issued eight at a time (a plane-at-a-time loop keeps one
// load per lane in flight: the split sums of the loss glue ran at ~1.3 TB/s, latency-bound);
// out-of-range loads read as zero, and x + 0 == x, so the sum is the sequential one bit for bit
__device__ __forceinline__ f32x4 split_sum4(const f32x4* __restrict__ ws, size_t plane, size_t i, int ns) {
  f32x4 a = ws[i];
  for (int sp = 1; sp < ns; sp += 8) {
    f32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = sp + k < ns ? ws[(size_t)(sp + k) * plane + i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) a += v[k];
  }
  return a;
}

// q: (B, D) normalised, d: (B, 1+J, D) normalised (positive first).  One wave per row; the
// query row lives in registers (MAXD floats per lane: D <= 64 MAXD), the 1+J raw cosines in
// wave-uniform registers (J1 <= MAXJ); compile-time (MAXD, MAXJ) in {2, 4, 8, 16} x {16, 64}
// (BERT towers without projection: D = 768).
template <int MAXD, int MAXJ>
__global__ __launch_bounds__(256) void dssm_explicit_kernel(const float* __restrict__ q, const float* __restrict__ d,
                                                            float* __restrict__ loss, float* __restrict__ prob,
                                                            float* __restrict__ dq, float* __restrict__ dd, int B,
                                                            int J1, int D, float gamma, float gscale, int clip) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float qv[MAXD];
  const float* qr = q + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < MAXD; ++i) {
    int c = lane + 64 * i;
    qv[i] = c < D ? qr[c] : 0.f;
  }
  float cs[MAXJ];  // raw cosines (the clip pass-through needs them in the backward)
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j >= J1) break;
    const float* dr = d + ((size_t)row * J1 + j) * D;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      int c = lane + 64 * i;
      if (c < D) s += qv[i] * dr[c];
    }
    cs[j] = wave_sum(s);
    const float R = clip ? fminf(fmaxf(cs[j], 0.f), 1.f) : cs[j];
    mx = fmaxf(mx, gamma * R);
  }
  auto S_of = [&](int j) { return gamma * (clip ? fminf(fmaxf(cs[j], 0.f), 1.f) : cs[j]); };
  float den = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j >= J1) break;
    den += __expf(S_of(j) - mx);
  }
  const float P0 = __expf(S_of(0) - mx) / den;
  const float Pc = fminf(fmaxf(P0, BCE_EPS), 1.f - BCE_EPS);
  if (lane == 0) {
    loss[row] = -__logf(Pc);
    prob[row] = P0;
  }
  // d(-log P0)/dS_j = P_j - [j==0]  (zero when the BCE clip is active)
  const bool live = P0 > BCE_EPS && P0 < 1.f - BCE_EPS;
  float gq[MAXD];
#pragma unroll
  for (int i = 0; i < MAXD; ++i) gq[i] = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j >= J1) break;
    const float Pj = __expf(S_of(j) - mx) / den;
    const float dS = live ? (Pj - (j == 0 ? 1.f : 0.f)) * gscale : 0.f;
    // clip pass-through with inclusive bounds, as T.clip
    const float dR = (clip && (cs[j] < 0.f || cs[j] > 1.f)) ? 0.f : dS * gamma;
    const float* dr = d + ((size_t)row * J1 + j) * D;
    float* ddr = dd + ((size_t)row * J1 + j) * D;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      int c = lane + 64 * i;
      if (c < D) {
        gq[i] += dR * dr[c];
        ddr[c] = dR * qv[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXD; ++i) {
    int c = lane + 64 * i;
    if (c < D) dq[(size_t)row * D + c] = gq[i];
  }
}

// ---------------------------------------------------------------- in-batch --------
constexpr int TQ = 128;   // rows per block (4 waves x 32)
constexpr int TD = 64;    // columns per tile
constexpr int PADK = 8;   // LDS row padding (bf16 elements)

// ---- swapped orientation, G never leaves registers ---------------------------
// The S tile is computed transposed, S^T = Yt . X^T (A = 16 staged rows of Y from LDS,
// B = 16 register-resident rows of X), so each lane owns ONE X row (lane & 15) and four
// consecutive Y rows 4g..4g+3 of each 16-row subtile.  Two such subtiles, converted to
// bf16, are exactly the B operand of the next product  out^T[feat][x] += Y^T[feat][y] .
// G^T[y][x]  with the k (= y) order permuted as j -> 16*(j>>2) + 4g + (j&3); the matching
// A operand (Y^T) is read from the SAME row-major LDS image with ds_read_b64_tr_b16
// (a transposed LDS read), so neither a transposed copy of Y nor a G round trip through
// LDS is needed.  Y tiles are double-buffered (register prefetch of tile t+1 during the
// MFMAs of tile t, one barrier per tile).  LDS row stride DP+16 elements puts the 8 rows
// of a transposed read on disjoint 8-bank groups.
typedef short v4s __attribute__((ext_vector_type(4)));

template <int KS>
struct IbTile {
  static constexpr int DP = KS * 32, LDY = DP + 16, CH = DP / 8;
  static constexpr int NLD = (TD * CH + 255) / 256;  // 16-byte chunks per thread per tile
};

template <int KS>
__device__ __forceinline__ void ib_load(const unsigned short* __restrict__ Y, int c0, int c_end, u32x4 (&v)[IbTile<KS>::NLD]) {
  using T = IbTile<KS>;
#pragma unroll
  for (int u = 0; u < T::NLD; ++u) {
    const int q = threadIdx.x + 256 * u;
    const int r = q / T::CH, cc = (q % T::CH) * 8;
    v[u] = (q < TD * T::CH && c0 + r < c_end) ? *reinterpret_cast<const u32x4*>(Y + (size_t)(c0 + r) * T::DP + cc)
                                              : u32x4{0, 0, 0, 0};
  }
}

template <int KS>
__device__ __forceinline__ void ib_store(unsigned short* yt, const u32x4 (&v)[IbTile<KS>::NLD]) {
  using T = IbTile<KS>;
#pragma unroll
  for (int u = 0; u < T::NLD; ++u) {
    const int q = threadIdx.x + 256 * u;
    if (q < TD * T::CH) *reinterpret_cast<u32x4*>(yt + (q / T::CH) * T::LDY + (q % T::CH) * 8) = v[u];
  }
}

// acc[c][i][r] = X[row i*16 + (lane&15)] . Y[tile row c*16 + 4g + r]
template <int KS>
__device__ __forceinline__ void st_tile(const bf16x8 (&xb)[2][KS], const unsigned short* yt, f32x4 (&acc)[4][2]) {
  using T = IbTile<KS>;
  const int lane = threadIdx.x & 63;
  // k-step 0 takes the inline-constant 0 as its C operand (no per-tile zeroing moves)
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(yt + (c * 16 + (lane & 15)) * T::LDY + s * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        acc[c][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, xb[i][s], s == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[c][i],
                                                            0, 0, 0);
    }
}

template <int KS>
__device__ __forceinline__ void load_xb(const unsigned short* __restrict__ X, int r0, int nx, bf16x8 (&xb)[2][KS]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = r0 + i * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      xb[i][s] = r < nx ? *reinterpret_cast<const bf16x8*>(X + (size_t)r * KS * 32 + s * 32 + (lane >> 4) * 8)
                        : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}

// CLIP (compile time) and FULL (a uniform branch per tile: only a split's last tile can be
// partial) keep the per-element epilogue to fmed3 + fma + exp2 + add: the exp epilogue, not
// the MFMAs, bounds these kernels (one exp per 320 MFMA FLOPs at D = 160).
template <int KS, bool CLIP>
__global__ __launch_bounds__(256, 2) void ib_fwd_kernel(const unsigned short* __restrict__ X,
                                                         const unsigned short* __restrict__ Y,
                                                         float* __restrict__ part, int nx, int ny, int per_split,
                                                         float gamma) {
  using T = IbTile<KS>;
  __shared__ __attribute__((aligned(16))) unsigned short yt[2][TD * T::LDY];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int r0 = blockIdx.x * TQ + wave * 32;
  const int c_begin = blockIdx.y * per_split, c_end = min(ny, c_begin + per_split);
  bf16x8 xb[2][KS];
  load_xb<KS>(X, r0, nx, xb);
  u32x4 st[T::NLD];
  ib_load<KS>(Y, c_begin, c_end, st);
  ib_store<KS>(yt[0], st);
  __syncthreads();
  float rs[2] = {0.f, 0.f};
  const float gl = gamma * 1.4426950408889634f;
  int buf = 0;
  for (int c0 = c_begin; c0 < c_end; c0 += TD, buf ^= 1) {
    const bool more = c0 + TD < c_end;
    if (more) ib_load<KS>(Y, c0 + TD, c_end, st);
    f32x4 acc[4][2];
    st_tile<KS>(xb, yt[buf], acc);
    auto epi = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool yv = FULL || c0 + c * 16 + 4 * g + r < c_end;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            float v = acc[c][i][r];
            if constexpr (CLIP) v = __builtin_amdgcn_fmed3f(v, 0.f, 1.f);
            float x = __builtin_fmaf(v, gl, -gl);
            if constexpr (!FULL) x = yv ? x : -INFINITY;
            rs[i] += __builtin_amdgcn_exp2f(x);
          }
        }
    };
    if (c0 + TD <= c_end) epi(std::true_type{});
    else epi(std::false_type{});
    if (more) ib_store<KS>(yt[buf ^ 1], st);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float v = rs[i];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const int r = r0 + i * 16 + (lane & 15);
    if (g == 0 && r < nx) part[(size_t)blockIdx.y * nx + r] = v;  // summed in split order by ib_rowsum
  }
}

// sumexp[r] = sum_s part[s][r] in a fixed order (the forward loss is bit-reproducible);
// with spos (the positive logit g*clip(cos+), ib_pos) also the per-row loss
// g + log(sumexp) - spos (= -log P+ of the softmax over exp(g*(S-1))) and P+ = exp(-loss).
__global__ void ib_rowsum_kernel(const float* __restrict__ part, float* __restrict__ out, int nx, int ns,
                                 const float* __restrict__ spos = nullptr, float* __restrict__ loss = nullptr,
                                 float* __restrict__ prob = nullptr, float gamma = 0.f) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nx) return;
  float a = 0.f;
  for (int s = 0; s < ns; ++s) a += part[(size_t)s * nx + r];
  out[r] = a;
  if (spos) {
    const float l = gamma + __logf(a) - spos[r];
    loss[r] = l;
    prob[r] = __expf(-l);
  }
}

// The S-tile epilogue variants (ROW / CLIP / FWD) of the ib3 and ib5 kernels below:
// ROW = true : X = queries, Y = docs,    out = dQ, scale indexed by X row
// ROW = false: X = docs,    Y = queries, out = dD, scale indexed by Y row
// Each split writes its partial product with plain stores into out (a single split) or
// into its slice of the workspace ws[split][nx][DP]; ib_split_reduce sums the slices
// (fp32 atomics from 16-32 splits cost ~4x more than the extra write + read).
// FWD (with ROW, X = queries): the forward pass that also produces the query gradient's
// normaliser-free part U = sum_j exp(g*(S_ij - 1)) * clip'_ij * Y_j, and the row sums
// sum_j exp(g*(S_ij - 1)) into `part` like ib_fwd.  dQ_i is a per-row multiple of U_i
// (scale_i = g_up_i * gamma / sumexp_i, known only in backward, is a row scalar), so the
// backward's dQ pass — a third recomputation of S — disappears: dQ = scale * U.
// (The round-2 256-thread generation of these kernels and a 4-wave-workgroup variant of
// ib3 / ib5 were measured slower and removed: docs/PERF.md "In-batch loss generations".)

// ---- ib3: 512-thread workgroups, Y tiles by LDS-DMA into a 3-slot ring --------------------
// The per-tile math above (S^T tile -> G^T in registers -> out^T += Y^T G^T), with
// the three costs that kept that kernel at ~0.75 PF/s at the W = 8 shape removed:
//  * 8 waves x 32 X rows = 256 rows per workgroup (one per CU, 2 waves per SIMD): each
//    staged Y tile feeds twice the MFMAs, half the Y bytes per FLOP;
//  * Y tiles land in LDS by global_load_lds_dwordx4 (no staging VGPRs: the old kernel sat at
//    256 VGPRs and spilled), issued two tiles ahead into a 3-slot ring, one barrier per tile,
//    each wave waiting only for its own pieces of the next tile (counted vmcnt);
//  * the workgroups of one Y split are consecutive after the XCD remap, so they share an
//    XCD's L2 (the split's Y tiles come from the Infinity Cache / HBM once per XCD).
// The LDS image keeps the old row stride (DP + 16 elements, 4 KS + 2 chunks of 16 B): the
// two pad chunks per row take part in the DMA (each re-reads chunk 0 of its row) so every
// wave-instruction writes 1 KB of consecutive LDS, and the conflict-free read patterns of
// st_tile / the transposed reads are unchanged.  !ROW: the 64 per-row scales of a tile ride
// along as one 4-byte-per-lane DMA (wave 7).
constexpr int TQ3 = 256;

template <int KS>
struct Ib3 {
  static constexpr int DP = KS * 32, LDY = DP + 16;
  static constexpr int CPR = LDY / 8;           // 16-byte chunks per LDS row
  static constexpr int PIECES = TD * CPR / 64;  // 1 KB wave-instructions per tile (= CPR)
  static constexpr int TILE_B = TD * LDY * 2;
};

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// wave-uniform n: wait until at most n of this wave's vector-memory operations are in flight
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}

// DMA instructions one wave issues per staged tile
template <int KS, bool ROW, int NW = 8>
__device__ __forceinline__ int ib3_pieces(int wave) {
  constexpr int P = Ib3<KS>::PIECES;
  const int n = wave < P ? (P - wave + NW - 1) / NW : 0;
  return n + ((!ROW && wave == NW - 1) ? 1 : 0);
}

template <int KS, bool ROW, int NW = 8>
__device__ __forceinline__ void ib3_stage(const unsigned short* __restrict__ Y, const float* __restrict__ scale,
                                          int c0, int c_end, char* dst, float* sdst) {
  using T = Ib3<KS>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < (T::PIECES + NW - 1) / NW; ++u) {
    const int p = wave + NW * u;
    if (p < T::PIECES) {
      const int q = p * 64 + lane;
      const int r = q / T::CPR, c = q - r * T::CPR;
      const int row = min(c0 + r, c_end - 1);  // rows past the split: valid bytes, masked by the epilogue
      const int cc = c < 4 * KS ? c : 0;
      glds16(Y + (size_t)row * T::DP + cc * 8, dst + p * 1024);
    }
  }
  if (!ROW && wave == NW - 1) glds4(scale + min(c0 + lane, c_end - 1), sdst);
}

template <int KS, bool ROW, bool CLIP, bool FWD = false, int NW = 8>
__global__ __launch_bounds__(NW * 64, 2) void ib3_kernel(const unsigned short* __restrict__ X,
                                                      const unsigned short* __restrict__ Y,
                                                      const float* __restrict__ scale, float* __restrict__ out,
                                                      float* __restrict__ ws, int nx, int ny, int per_split,
                                                      int nrb, float gamma, float* __restrict__ part = nullptr) {
  static_assert(!FWD || ROW, "the fused forward runs over query rows");
  using T = Ib3<KS>;
  constexpr int NC = T::DP / 16;
  constexpr int NB = 3;  // ring slots
  __shared__ __attribute__((aligned(1024))) char ring[NB * T::TILE_B];
  __shared__ __attribute__((aligned(16))) float ysc[NB][TD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  // XCD remap: the consecutive ids of one XCD cover the row blocks of one split first
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / nrb, rb = bid - split * nrb;
  const int r0 = rb * (NW * 32) + wave * 32;
  const int c_begin = split * per_split, c_end = min(ny, c_begin + per_split);
  const int ntiles = (c_end - c_begin + TD - 1) / TD;
  const float gl = gamma * 1.4426950408889634f;
  const int np = ib3_pieces<KS, ROW, NW>(wave);
  bf16x8 xb[2][KS];
  load_xb<KS>(X, r0, nx, xb);
  float rsc[2] = {0.f, 0.f};
  float rs[2] = {0.f, 0.f};
  if (ROW && !FWD) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = r0 + i * 16 + (lane & 15);
      rsc[i] = r < nx ? scale[r] : 0.f;
    }
  }
  f32x4 o[NC][2];
#pragma unroll
  for (int n = 0; n < NC; ++n)
#pragma unroll
    for (int i = 0; i < 2; ++i) o[n][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  ib3_stage<KS, ROW, NW>(Y, scale, c_begin, c_end, ring, ysc[0]);
  if (ntiles > 1) ib3_stage<KS, ROW, NW>(Y, scale, c_begin + TD, c_end, ring + T::TILE_B, ysc[1]);
  wait_vm(ntiles > 1 ? np : 0);
  __builtin_amdgcn_s_barrier();
  const int trow = 4 * g + ((lane & 15) >> 2), tcol = 4 * (lane & 3);
  f32x4 acc[4][2];
  // epilogue of the S tile in `acc` (tile slot sb, first Y row c0) + out^T += Y^T . G^T
  auto epi_out = [&](int sb, int c0) {
    const unsigned short* yb = reinterpret_cast<const unsigned short*>(ring + sb * T::TILE_B);
    u32x4 gp[2][2];
    auto epi = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 ysv;
        if constexpr (!ROW) ysv = *reinterpret_cast<const f32x4*>(&ysc[sb][c * 16 + 4 * g]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float gv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int yr = c * 16 + 4 * g + r;
            const float v = acc[c][i][r];
            float x;
            if constexpr (FWD) {
              const float vc = CLIP ? __builtin_amdgcn_fmed3f(v, 0.f, 1.f) : v;
              x = __builtin_fmaf(vc, gl, -gl);
              if constexpr (!FULL) x = c0 + yr < c_end ? x : -INFINITY;
              const float e = __builtin_amdgcn_exp2f(x);
              rs[i] += e;
              gv[r] = (!CLIP || vc == v) ? e : 0.f;
              continue;
            }
            if constexpr (CLIP) {
              const float vc = __builtin_amdgcn_fmed3f(v, 0.f, 1.f);
              x = vc == v ? __builtin_fmaf(vc, gl, -gl) : -INFINITY;
            } else {
              x = __builtin_fmaf(v, gl, -gl);
            }
            if constexpr (!FULL) x = c0 + yr < c_end ? x : -INFINITY;
            gv[r] = (ROW ? rsc[i] : ysv[r]) * __builtin_amdgcn_exp2f(x);
          }
          gp[c >> 1][i][(c & 1) * 2] = pack_bf16x2(gv[0], gv[1]);
          gp[c >> 1][i][(c & 1) * 2 + 1] = pack_bf16x2(gv[2], gv[3]);
        }
      }
    };
    if (c0 + TD <= c_end) epi(std::true_type{});
    else epi(std::false_type{});
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int n = 0; n < NC; ++n) {
        typedef __attribute__((address_space(3))) v4s lds_v4s;
        const unsigned short* p0 = yb + (s2 * 32 + trow) * T::LDY + n * 16 + tcol;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p0));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p0 + 16 * T::LDY));
        const bf16x8 a = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 2; ++i)
          o[n][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, gp[s2][i]), o[n][i], 0, 0, 0);
      }
  };
  int buf = 0;
#pragma unroll 1
  for (int t = 0; t < ntiles; ++t) {
    const int c0 = c_begin + t * TD;
    const bool ahead = t + 2 < ntiles;
    if (ahead) {  // slot (t + 2) % 3 = (t - 1) % 3: every wave left it at the last barrier
      const int sb = buf + 2 >= NB ? buf + 2 - NB : buf + 2;
      ib3_stage<KS, ROW, NW>(Y, scale, c0 + 2 * TD, c_end, ring + sb * T::TILE_B, ysc[sb]);
    }
    st_tile<KS>(xb, reinterpret_cast<const unsigned short*>(ring + buf * T::TILE_B), acc);
    epi_out(buf, c0);
    // tile t + 1 must have landed (this wave's pieces; the barrier covers the others');
    // tile t + 2's pieces may stay in flight
    wait_vm(ahead ? np : 0);
    __builtin_amdgcn_s_barrier();
    buf = buf + 1 == NB ? 0 : buf + 1;
  }
  if constexpr (FWD) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int r = r0 + i * 16 + (lane & 15);
      if (g == 0 && r < nx) part[(size_t)split * nx + r] = v;
    }
  }
  float* dst = (gridDim.x == (unsigned)nrb) ? out : ws + (size_t)split * nx * T::DP;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int x = r0 + i * 16 + (lane & 15);
    if (x >= nx) continue;
    float* orow = dst + (size_t)x * T::DP;
#pragma unroll
    for (int n = 0; n < NC; ++n) *reinterpret_cast<f32x4*>(orow + n * 16 + 4 * g) = o[n][i];
  }
}

// ---- ib5: the ib3 pipeline on v_mfma_f32_32x32x16_bf16 --------------------------------------
// The epilogue (clip, exp, mask, row sums: ~6 VALU per S element) is as long as the matrix
// work, and a 16x16x32 MFMA holds its SIMD's vector issue for 8 of its 16 cycles; a
// 32x32x16 MFMA holds it for 8 of 32, so the partner wave's exp epilogue fits beside the
// matrix phases (MI355X_MICROARCH.md, per-instruction constants).  Per wave: 32 X rows = the
// N side of every product; per 64-row Y tile:
//   S^T[y][x] (two 32x32 tiles, 10 k-steps of 16 over DP)   A = Y rows (ds_read_b128), B = X (registers)
//   G^T = epilogue(S^T) in registers, and as 32x32 accumulators its rows (y) are exactly the
//   k index of the next product's B operand (cdna_hip_programming.md "An accumulator tile as
//   the next MFMA's operand": element j of lane half h is row 16s + 8(j>>2) + 4h + (j&3));
//   out^T[feat][x] += Y^T[feat][y] G^T[y][x]  (5 feature tiles x 4 k-steps), A = two
//   ds_read_b64_tr_b16 per fragment (rows 16s + 4h + 0..3 and + 8..11 of the y tile).
// LDS image: unpadded 320-byte rows (DP = 160), 16-byte chunk c of row y stored at
// c ^ ((y >> 2) & 3): conflict-free for the b128 reads (16 rows of one chunk per lane group)
// and the transposed reads (4 consecutive rows x 64 bytes per half-wave).  Y tiles by LDS-DMA
// into a 3-slot ring as in ib3 (pieces = whole 1 KB wave-instructions: TD * DP * 2 / 1024).
template <int KS>
struct Ib5 {
  static constexpr int DP = KS * 32, ROWB = DP * 2, CPR = DP / 8;
  static constexpr int PIECES = TD * CPR / 64;  // 20 at DP = 160
  static constexpr int TILE_B = TD * ROWB;
  static constexpr int K16 = DP / 16;           // k-steps of the S product
  static constexpr int FT = DP / 32;            // feature tiles of the out product
};

// chunk swizzle of row y: DP = 160 (80-dword rows, 16 mod 64): (y >> 2) & 3 within aligned
// groups of 4 chunks; DP = 128 (64-dword rows, every row on bank 0): a bijection of y mod 16
// whose high two bits are y & 3 (16 rows of one chunk -> 16 slots for the b128 reads, the
// 4 rows of a transposed read -> 4 different 64-byte groups)
template <int KS>
__device__ __forceinline__ int ib5_swz(int y) {
  if constexpr (KS == 4) return ((y & 3) << 2) | ((y >> 2) & 3);
  else return (y >> 2) & 3;
}

template <int KS, bool ROW, int NW = 8>
__device__ __forceinline__ int ib5_pieces(int wave) {
  constexpr int P = Ib5<KS>::PIECES;
  const int n = wave < P ? (P - wave + NW - 1) / NW : 0;
  return n + ((!ROW && wave == NW - 1) ? 1 : 0);
}

template <int KS, bool ROW, int NW = 8>
__device__ __forceinline__ void ib5_stage(const unsigned short* __restrict__ Y, const float* __restrict__ scale,
                                          int c0, int c_end, char* dst, float* sdst) {
  using T = Ib5<KS>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < (T::PIECES + NW - 1) / NW; ++u) {
    const int p = wave + NW * u;
    if (p < T::PIECES) {
      const int q = p * 64 + lane;
      const int r = q / T::CPR, pc = q - r * T::CPR;
      const int c = pc ^ ib5_swz<KS>(r);           // logical chunk stored at physical chunk pc
      const int row = min(c0 + r, c_end - 1);  // rows past the split: valid bytes, masked by the epilogue
      glds16(Y + (size_t)row * T::DP + c * 8, dst + p * 1024);
    }
  }
  if (!ROW && wave == NW - 1) glds4(scale + min(c0 + lane, c_end - 1), sdst);
}

template <int KS, bool ROW, bool CLIP, bool FWD = false, int NW = 8>
__global__ __launch_bounds__(NW * 64, 2) void ib5_kernel(const unsigned short* __restrict__ X,
                                                      const unsigned short* __restrict__ Y,
                                                      const float* __restrict__ scale, float* __restrict__ out,
                                                      float* __restrict__ ws, int nx, int ny, int per_split,
                                                      int nrb, float gamma, float* __restrict__ part = nullptr) {
  static_assert(!FWD || ROW, "the fused forward runs over query rows");
  static_assert(KS == 4 || KS == 5, "ib5: chunk swizzles exist for DP = 128 and 160");
  using T = Ib5<KS>;
  constexpr int NB = 3;
  __shared__ __attribute__((aligned(1024))) char ring[NB * T::TILE_B];
  __shared__ __attribute__((aligned(16))) float ysc[NB][TD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / nrb, rb = bid - split * nrb;
  const int r0 = rb * (NW * 32) + wave * 32;
  const int x = r0 + l32;  // this lane's X row
  const int c_begin = split * per_split, c_end = min(ny, c_begin + per_split);
  const int ntiles = (c_end - c_begin + TD - 1) / TD;
  const float gl = gamma * 1.4426950408889634f;
  const int np = ib5_pieces<KS, ROW, NW>(wave);
  // B operand of the S product: X[x][16 ks + 8 h .. + 7]
  bf16x8 xb[T::K16];
#pragma unroll
  for (int ks = 0; ks < T::K16; ++ks)
    xb[ks] = x < nx ? *reinterpret_cast<const bf16x8*>(X + (size_t)x * T::DP + 16 * ks + 8 * h)
                    : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  const float rsc = (ROW && !FWD && x < nx) ? scale[x] : 0.f;
  float rs = 0.f;
  f32x16 o[T::FT];
#pragma unroll
  for (int f = 0; f < T::FT; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[f][r] = 0.f;
  ib5_stage<KS, ROW, NW>(Y, scale, c_begin, c_end, ring, ysc[0]);
  if (ntiles > 1) ib5_stage<KS, ROW, NW>(Y, scale, c_begin + TD, c_end, ring + T::TILE_B, ysc[1]);
  wait_vm(ntiles > 1 ? np : 0);
  __builtin_amdgcn_s_barrier();
  // transposed-read lane address inside a (4-row x 16-feature) block: row q = (lane & 15) >> 2,
  // features 4p .. 4p+3 (p = lane & 3); lane group g = lane >> 4 -> half h = g >> 1 (rows + 4h),
  // feature half (g & 1) (+16)
  const int tq = (lane & 15) >> 2, tf = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  int buf = 0;
#pragma unroll 1
  for (int t = 0; t < ntiles; ++t) {
    const int c0 = c_begin + t * TD;
    const bool ahead = t + 2 < ntiles;
    if (ahead) {
      const int sb = buf + 2 >= NB ? buf + 2 - NB : buf + 2;
      ib5_stage<KS, ROW, NW>(Y, scale, c0 + 2 * TD, c_end, ring + sb * T::TILE_B, ysc[sb]);
    }
    const char* yb = ring + buf * T::TILE_B;
    // S^T tiles: acc[yt][r] = S^T[y = 32 yt + 8 (r >> 2) + 4 h + (r & 3)][x]
    f32x16 acc[2];
#pragma unroll
    for (int ks = 0; ks < T::K16; ++ks)
#pragma unroll
      for (int yt = 0; yt < 2; ++yt) {
        const int y = 32 * yt + l32, c = 2 * ks + h;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(yb + y * T::ROWB + ((c ^ ib5_swz<KS>(y)) << 4));
        acc[yt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xb[ks], ks == 0 ? f32x16{} : acc[yt], 0, 0, 0);
      }
    // epilogue -> G^T as bf16 B fragments gp[yt][s] (registers 8s .. 8s+7 of acc[yt])
    u32x4 gp[2][2];
    auto epi = [&](auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
      for (int yt = 0; yt < 2; ++yt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // rows y = 32 yt + 8 j + 4 h + (0..3)
          f32x4 ysv;
          if constexpr (!ROW) ysv = *reinterpret_cast<const f32x4*>(&ysc[buf][32 * yt + 8 * j + 4 * h]);
          float gv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int yr = 32 * yt + 8 * j + 4 * h + r;
            const float v = acc[yt][4 * j + r];
            float xx;
            if constexpr (FWD) {
              const float vc = CLIP ? __builtin_amdgcn_fmed3f(v, 0.f, 1.f) : v;
              xx = __builtin_fmaf(vc, gl, -gl);
              if constexpr (!FULL) xx = c0 + yr < c_end ? xx : -INFINITY;
              const float e = __builtin_amdgcn_exp2f(xx);
              rs += e;
              gv[r] = (!CLIP || vc == v) ? e : 0.f;
              continue;
            }
            if constexpr (CLIP) {
              const float vc = __builtin_amdgcn_fmed3f(v, 0.f, 1.f);
              xx = vc == v ? __builtin_fmaf(vc, gl, -gl) : -INFINITY;
            } else {
              xx = __builtin_fmaf(v, gl, -gl);
            }
            if constexpr (!FULL) xx = c0 + yr < c_end ? xx : -INFINITY;
            gv[r] = (ROW ? rsc : ysv[r]) * __builtin_amdgcn_exp2f(xx);
          }
          gp[yt][j >> 1][(j & 1) * 2] = pack_bf16x2(gv[0], gv[1]);
          gp[yt][j >> 1][(j & 1) * 2 + 1] = pack_bf16x2(gv[2], gv[3]);
        }
    };
    if (c0 + TD <= c_end) epi(std::true_type{});
    else epi(std::false_type{});
    // out^T[feat][x] += Y^T[feat][y] . G^T[y][x]; k-step (yt, s) = rows 32 yt + 16 s + {4h + 0..3, 8 + 4h + 0..3}
#pragma unroll
    for (int yt = 0; yt < 2; ++yt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int f = 0; f < T::FT; ++f) {
          typedef __attribute__((address_space(3))) v4s lds_v4s;
          const int ylo = 32 * yt + 16 * s2 + 4 * h + tq, yhi = ylo + 8;
          const int fe = 32 * f + tf;  // feature of this lane's 8-byte piece (chunk fe >> 3, half (fe & 7))
          const char* plo = yb + ylo * T::ROWB + ((((fe >> 3) ^ ib5_swz<KS>(ylo))) << 4) + (fe & 7) * 2;
          const char* phi = yb + yhi * T::ROWB + ((((fe >> 3) ^ ib5_swz<KS>(yhi))) << 4) + (fe & 7) * 2;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plo));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(phi));
          const bf16x8 a = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, __builtin_bit_cast(bf16x8, gp[yt][s2]), o[f], 0, 0, 0);
        }
    wait_vm(ahead ? np : 0);
    __builtin_amdgcn_s_barrier();
    buf = buf + 1 == NB ? 0 : buf + 1;
  }
  if constexpr (FWD) {
    rs += __shfl_xor(rs, 32, 64);
    if (h == 0 && x < nx) part[(size_t)split * nx + x] = rs;
  }
  float* dst = (gridDim.x == (unsigned)nrb) ? out : ws + (size_t)split * nx * T::DP;
  if (x < nx) {
    float* orow = dst + (size_t)x * T::DP;
#pragma unroll
    for (int f = 0; f < T::FT; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(orow + 32 * f + 8 * j + 4 * h) =
            f32x4{o[f][4 * j], o[f][4 * j + 1], o[f][4 * j + 2], o[f][4 * j + 3]};
  }
}

// ---- ib7: ib5 software-pipelined ------------------------------------------------------------
// ib5 runs each tile as S product -> epilogue -> out product, and the one-barrier-per-tile ring
// keeps the 8 waves of a workgroup in phase: both waves of a SIMD sit in their MFMA phase or in
// their VALU epilogue (~27 issue cycles per S element: clamp, compare, fma, select, v_exp,
// scale, cvt) at the same time, so matrix and vector work barely co-execute (~1.0 PF/s on the
// 344 GFLOP passes at the W = 8 shape, docs/PERF.md).  ib7 computes the NEXT tile's S product
// in the same basic block as this tile's epilogue (independent instructions the scheduler
// interleaves: each 32x32x16 MFMA holds vector issue for 8 of its 32 cycles), so one wave's
// epilogue hides behind its own matrix work.  The next tile must be resident one iteration
// earlier: a 4-slot ring (80 KB at DP = 160) staged three tiles ahead, each iteration waiting for
// tile t + 2.  Per tile, three phases keep the live registers at ib5's: (1) S rows 32..63
// beside the epilogue of rows 0..31, (2) the next tile's S rows 0..31 and the out product over
// rows 0..31 beside the epilogue of rows 32..63, (3) the out product over rows 32..63 —
// scheduling barriers hold that order.  Same arithmetic as ib5 (the out product's k-steps in
// the same order): bit-identical results.
template <int KS, bool ROW, bool CLIP, bool FWD = false, int NW = 8>
__global__ __launch_bounds__(NW * 64, 2) void ib7_kernel(const unsigned short* __restrict__ X,
                                                      const unsigned short* __restrict__ Y,
                                                      const float* __restrict__ scale, float* __restrict__ out,
                                                      float* __restrict__ ws, int nx, int ny, int per_split,
                                                      int nrb, float gamma, float* __restrict__ part = nullptr) {
  static_assert(!FWD || ROW, "the fused forward runs over query rows");
  static_assert(KS == 4 || KS == 5, "ib7: chunk swizzles exist for DP = 128 and 160");
  static_assert(Ib5<KS>::K16 >= 8, "ib7: one epilogue group per S k-step");
  using T = Ib5<KS>;
  constexpr int NB = 4;
  __shared__ __attribute__((aligned(1024))) char ring[NB * T::TILE_B];
  __shared__ __attribute__((aligned(16))) float ysc[NB][TD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / nrb, rb = bid - split * nrb;
  const int r0 = rb * (NW * 32) + wave * 32;
  const int x = r0 + l32;
  const int c_begin = split * per_split, c_end = min(ny, c_begin + per_split);
  const int ntiles = (c_end - c_begin + TD - 1) / TD;
  const float gl = gamma * 1.4426950408889634f;
  const int np = ib5_pieces<KS, ROW, NW>(wave);
  bf16x8 xb[T::K16];
#pragma unroll
  for (int ks = 0; ks < T::K16; ++ks)
    xb[ks] = x < nx ? *reinterpret_cast<const bf16x8*>(X + (size_t)x * T::DP + 16 * ks + 8 * h)
                    : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  const float rsc = (ROW && !FWD && x < nx) ? scale[x] : 0.f;
  float rs = 0.f;
  f32x16 o[T::FT];
#pragma unroll
  for (int f = 0; f < T::FT; ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[f][r] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < ntiles) ib5_stage<KS, ROW, NW>(Y, scale, c_begin + i * TD, c_end, ring + i * T::TILE_B, ysc[i]);
  // tiles 0 and 1 landed; tile 2's pieces may stay in flight
  wait_vm(ntiles > 2 ? np : 0);
  __builtin_amdgcn_s_barrier();
  const int tq = (lane & 15) >> 2, tf = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  // Fragment addresses (DP = 160) as a lane base + compile-time offsets (ds_read immediates).  S product,
  // A = Y row y = 32 yt + l32, 16-byte chunk c = 2 ks + h stored at c ^ swz(y); swz(y) =
  // ib5_swz(l32) for both yt (32 yt keeps y >> 2 & 3 and y & 3), and it flips only the chunk's
  // low two bits: c ^ swz = 4 (ks >> 1) + ((2 (ks & 1) + h) ^ swz) -> two lane bases (ks parity)
  // plus 64 (ks >> 1) + 32 yt * ROWB.  Out product, A = rows ylo = 32 yt + 16 s2 + 4 h + tq and
  // ylo + 8, feature fe = 32 f + tf: chunk (fe >> 3) ^ swz(ylo) = 4 f + ((tf >> 3) ^ swz(ylo)),
  // and swz(ylo) = swz(4 h + tq), swz(ylo + 8) = swz(4 h + tq + 8) -> two lane bases plus
  // (32 yt + 16 s2) * ROWB + 64 f.
  const int swzA = ib5_swz<KS>(l32);
  const int offA0 = l32 * T::ROWB + ((h ^ swzA) << 4), offA1 = l32 * T::ROWB + (((2 + h) ^ swzA) << 4);
  const int ylo0 = 4 * h + tq;
  const int offTlo = ylo0 * T::ROWB + (((tf >> 3) ^ ib5_swz<KS>(ylo0)) << 4) + (tf & 7) * 2;
  const int offThi = (ylo0 + 8) * T::ROWB + (((tf >> 3) ^ ib5_swz<KS>(ylo0 + 8)) << 4) + (tf & 7) * 2;
  // (DP = 128: the swizzle is 4 bits wide and permutes whole rows of chunks — the generic
  // per-fragment address, as in ib5)
  auto ldA = [&](const char* base, int ks, int yt) {
    if constexpr (KS == 5) {
      const char* p = base + ((ks & 1) ? offA1 : offA0) + 64 * (ks >> 1) + 32 * yt * T::ROWB;
      return *reinterpret_cast<const bf16x8*>(p);
    } else {
      const int y = 32 * yt + l32, c = 2 * ks + h;
      return *reinterpret_cast<const bf16x8*>(base + y * T::ROWB + ((c ^ ib5_swz<KS>(y)) << 4));
    }
  };
  auto ldT = [&](const char* base, int yt, int s2, int f) {
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const char *plo, *phi;
    if constexpr (KS == 5) {
      const int c = (32 * yt + 16 * s2) * T::ROWB + 64 * f;
      plo = base + offTlo + c;
      phi = base + offThi + c;
    } else {
      const int ylo = 32 * yt + 16 * s2 + 4 * h + tq, yhi = ylo + 8;
      const int fe = 32 * f + tf;
      plo = base + ylo * T::ROWB + ((((fe >> 3) ^ ib5_swz<KS>(ylo))) << 4) + (fe & 7) * 2;
      phi = base + yhi * T::ROWB + ((((fe >> 3) ^ ib5_swz<KS>(yhi))) << 4) + (fe & 7) * 2;
    }
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plo));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(phi));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  // acc[yt][r] = S^T[y = 32 yt + 8 (r >> 2) + 4 h + (r & 3)][x] of the current tile
  f32x16 acc[2];
  {
    bf16x8 a = ldA(ring, 0, 0);
#pragma unroll
    for (int ks = 0; ks < T::K16; ++ks) {
      const bf16x8 b = a;
      if (ks + 1 < T::K16) a = ldA(ring, ks + 1, 0);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, xb[ks], ks == 0 ? f32x16{} : acc[0], 0, 0, 0);
    }
  }
  // one tile; FULL (compile time): every Y row of the tile is inside the split (all tiles but
  // possibly the last, which is peeled off so the steady-state loop body is one basic block)
  auto tile = [&](int t, auto full_c) {
    constexpr bool FULL = decltype(full_c)::value;
    const int c0 = c_begin + t * TD;
    const int sb = t & (NB - 1);
    const bool ahead = t + 3 < ntiles;
    if (ahead) {  // slot (t + 3) % 4 = (t - 1) % 4: every wave left it at the last barrier
      const int nb = (t + 3) & (NB - 1);
      ib5_stage<KS, ROW, NW>(Y, scale, c0 + 3 * TD, c_end, ring + nb * T::TILE_B, ysc[nb]);
    }
    const char* cb = ring + sb * T::TILE_B;
    const char* nbp = ring + ((t + 1) & (NB - 1)) * T::TILE_B;
    u32x4 gp[2][2];
    // epilogue of the 4 S^T rows y = 32 yt + 8 j + 4 h + (0..3) of this tile -> G^T fragment
    auto epi4 = [&](int yt, int j) {
      f32x4 ysv;
      if constexpr (!ROW) ysv = *reinterpret_cast<const f32x4*>(&ysc[sb][32 * yt + 8 * j + 4 * h]);
      float gv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int yr = 32 * yt + 8 * j + 4 * h + r;
        const float v = acc[yt][4 * j + r];
        float xx;
        if constexpr (FWD) {
          const float vc = CLIP ? __builtin_amdgcn_fmed3f(v, 0.f, 1.f) : v;
          xx = __builtin_fmaf(vc, gl, -gl);
          if constexpr (!FULL) xx = c0 + yr < c_end ? xx : -INFINITY;
          const float e = __builtin_amdgcn_exp2f(xx);
          rs += e;
          gv[r] = (!CLIP || vc == v) ? e : 0.f;
          continue;
        }
        if constexpr (CLIP) {
          const float vc = __builtin_amdgcn_fmed3f(v, 0.f, 1.f);
          xx = vc == v ? __builtin_fmaf(vc, gl, -gl) : -INFINITY;
        } else {
          xx = __builtin_fmaf(v, gl, -gl);
        }
        if constexpr (!FULL) xx = c0 + yr < c_end ? xx : -INFINITY;
        gv[r] = (ROW ? rsc : ysv[r]) * __builtin_amdgcn_exp2f(xx);
      }
      gp[yt][j >> 1][(j & 1) * 2] = pack_bf16x2(gv[0], gv[1]);
      gp[yt][j >> 1][(j & 1) * 2 + 1] = pack_bf16x2(gv[2], gv[3]);
    };
    // phase 1: this tile's S rows 32..63 (acc[1]) beside the epilogue of rows 0..31
    {
      bf16x8 a = ldA(cb, 0, 1);
#pragma unroll
      for (int ks = 0; ks < T::K16; ++ks) {
        const bf16x8 b = a;
        if (ks + 1 < T::K16) a = ldA(cb, ks + 1, 1);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, xb[ks], ks == 0 ? f32x16{} : acc[1], 0, 0, 0);
        if ((ks & 1) == 0 && ks < 8) epi4(0, ks >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // phase 2: the NEXT tile's S rows 0..31 (acc[0], slot t + 1: stale rows past the last tile
    // are computed and unused) and out^T += Y^T G^T over rows 0..31, beside the epilogue of
    // rows 32..63
    {
      bf16x8 a = ldA(nbp, 0, 0);
      bf16x8 at = ldT(cb, 0, 0, 0);
#pragma unroll
      for (int ks = 0; ks < T::K16; ++ks) {
        const bf16x8 b = a, bt = at;
        if (ks + 1 < T::K16) {
          a = ldA(nbp, ks + 1, 0);
          at = ldT(cb, 0, (ks + 1) / T::FT, (ks + 1) % T::FT);
        }
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, xb[ks], ks == 0 ? f32x16{} : acc[0], 0, 0, 0);
        const int s2 = ks / T::FT, f = ks % T::FT;  // 2 FT = K16 out-product steps over rows 0..31
        o[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bt, __builtin_bit_cast(bf16x8, gp[0][s2]), o[f], 0, 0, 0);
        if ((ks & 1) == 0 && ks < 8) epi4(1, ks >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // phase 3: out^T += Y^T G^T over rows 32..63
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int f = 0; f < T::FT; ++f)
        o[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ldT(cb, 1, s2, f), __builtin_bit_cast(bf16x8, gp[1][s2]), o[f],
                                                       0, 0, 0);
    // tile t + 2 landed (this wave's pieces; the barrier covers the others'); t + 3 may stay in flight
    wait_vm(ahead ? np : 0);
    __builtin_amdgcn_s_barrier();
  };
  const int nfull = (c_end - c_begin) / TD;
#pragma unroll 1
  for (int t = 0; t < nfull; ++t) tile(t, std::true_type{});
  if (nfull < ntiles) tile(nfull, std::false_type{});
  if constexpr (FWD) {
    rs += __shfl_xor(rs, 32, 64);
    if (h == 0 && x < nx) part[(size_t)split * nx + x] = rs;
  }
  float* dst = (gridDim.x == (unsigned)nrb) ? out : ws + (size_t)split * nx * T::DP;
  if (x < nx) {
    float* orow = dst + (size_t)x * T::DP;
#pragma unroll
    for (int f = 0; f < T::FT; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(orow + 32 * f + 8 * j + 4 * h) =
            f32x4{o[f][4 * j], o[f][4 * j + 1], o[f][4 * j + 2], o[f][4 * j + 3]};
  }
}

// out[i] = sum_s ws[s][i], n4 = nx*DP/4
__global__ __launch_bounds__(256) void ib_split_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                              long n4, int ns) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    reinterpret_cast<f32x4*>(out)[i] = split_sum4(reinterpret_cast<const f32x4*>(ws), (size_t)n4, (size_t)i, ns);
  }
}

// ---- ibw: wide vectors (D = 768 BERT towers, DP % 128 == 0) ----------------------------------
// The flash structure of ib3 / ib5 for vectors too wide to keep a query row's D accumulators
// in one wave: the S tile's reduction over D AND the gradient product's output columns are
// split across the workgroup's 4 waves (wave w owns the d-slice [w DP/4, (w+1) DP/4)).
//   * a workgroup owns 16 "owner" rows (their bf16 d-slice fragments in registers) and walks
//     32-row tiles of the "iterated" matrix (staged once in LDS, shared by the 4 waves);
//   * each wave computes its d-slice's partial S^T (32 iter rows x 16 owner rows, 2 KS
//     MFMAs), the partials meet in LDS and every wave sums the full tile;
//   * FWD : per owner row sum_j exp(g (clip(S) - 1)) -> part[split][row] (ib_rowsum);
//     ROW : out_owner += sum_j G_oj It_j with G = scale[owner] exp(..) clip'  (dQ);
//     COL : out_owner += sum_j G_jo It_j with G = scale[iter row] exp(..) clip' (dD);
//     G^T stays in registers as the B operand of out^T += It^T G^T (the S^T C-layout is the
//     B layout with the k order of pack_b), It^T through ds_read_b64_tr_b16 (ib3's trick);
//   * no S / dS block reaches HBM and no library GEMM runs (the round-4 path materialised
//     fp32 S blocks through torch.mm and ran two more GEMMs on a bf16 dS per block).
// Partial outputs per split go to ws[split][owner][DP] (ib_split_reduce), part[split][owner].
constexpr int IBW_T = 32;  // iterated rows per staged tile

template <int KS, int MODE, int CLIPV>  // KS = DP / 128 k-steps of 32 per wave; MODE 0 FWD, 1 ROW, 2 COL
__global__ __launch_bounds__(256, 2) void ibw_kernel(const unsigned short* __restrict__ O, int no,
                                                     const unsigned short* __restrict__ It, int ni,
                                                     const float* __restrict__ scale, float gamma,
                                                     float* __restrict__ out, int tiles_per_split) {
  constexpr int DP = KS * 128, LDW = DP + 8;  // LDS row stride (elements): 16-B aligned, staggered banks
  extern __shared__ __attribute__((aligned(16))) unsigned short ibw_lds[];
  unsigned short* it = ibw_lds;                                      // [IBW_T][LDW]
  f32x4* sp = reinterpret_cast<f32x4*>(ibw_lds + IBW_T * LDW);       // [4 waves][2][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int o0 = blockIdx.x * 16, split = blockIdx.y;
  const int orow = o0 + (lane & 15);
  const int dw = wave * KS * 32;  // this wave's d-slice
  bf16x8 ob[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k)
    ob[k] = orow < no ? *reinterpret_cast<const bf16x8*>(O + (size_t)orow * DP + dw + k * 32 + g * 8)
                      : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  const float osc = (MODE == 1 && orow < no) ? scale[orow] : 0.f;
  f32x4 acc[MODE == 0 ? 1 : 2 * KS];
#pragma unroll
  for (int i = 0; i < (MODE == 0 ? 1 : 2 * KS); ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsum = 0.f;
  const int ntiles = (ni + IBW_T - 1) / IBW_T;
  const int t_lo = split * tiles_per_split, t_hi = min(ntiles, t_lo + tiles_per_split);
  for (int t = t_lo; t < t_hi; ++t) {
    const int i0 = t * IBW_T;
    // stage the tile: IBW_T x DP bf16, 16-byte pieces
    for (int q = threadIdx.x; q < IBW_T * (DP / 8); q += 256) {
      const int r = q / (DP / 8), c = (q % (DP / 8)) * 8;
      *reinterpret_cast<u32x4*>(it + r * LDW + c) =
          i0 + r < ni ? *reinterpret_cast<const u32x4*>(It + (size_t)(i0 + r) * DP + c) : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    // this wave's d-slice of S^T: rows = iter rows (2 subtiles of 16), cols = owner rows
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(it + (c * 16 + (lane & 15)) * LDW + dw + k * 32 + g * 8);
        s4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ob[k], s4, 0, 0, 0);
      }
      sp[(wave * 2 + c) * 64 + lane] = s4;
    }
    __syncthreads();
    f32x4 sv[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      sv[c] = sp[c * 64 + lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) sv[c] += sp[(w * 2 + c) * 64 + lane];
    }
    // epilogue: element (iter row i0 + 16c + 4g + r, owner row orow)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ir = i0 + c * 16 + 4 * g + r;
        const float raw = sv[c][r];
        const float x = CLIPV ? fminf(fmaxf(raw, 0.f), 1.f) : raw;
        const float e = ir < ni ? __expf(gamma * (x - 1.f)) : 0.f;
        if (MODE == 0) {
          rsum += e;
        } else {
          const bool pass = !CLIPV || (raw >= 0.f && raw <= 1.f);
          const float sc = MODE == 1 ? osc : (ir < ni ? scale[ir] : 0.f);
          sv[c][r] = pass ? sc * e : 0.f;
        }
      }
    if (MODE != 0) {
      // G^T as the B operand of one k-step of 32 iter rows (k order 16 (j >> 2) + 4g + (j & 3))
      u32x4 w4;
      w4[0] = pack_bf16x2(sv[0][0], sv[0][1]);
      w4[1] = pack_bf16x2(sv[0][2], sv[0][3]);
      w4[2] = pack_bf16x2(sv[1][0], sv[1][1]);
      w4[3] = pack_bf16x2(sv[1][2], sv[1][3]);
      const bf16x8 gb = __builtin_bit_cast(bf16x8, w4);
#pragma unroll
      for (int i = 0; i < 2 * KS; ++i) {
        // It^T fragment: A[m = d (dw + 16 i + lane & 15)][k = the permuted iter rows]
        const unsigned short* p = it + (4 * g + ((lane & 15) >> 2)) * LDW + dw + i * 16 + 4 * (lane & 3);
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p + 16 * LDW));
        const bf16x8 a = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, gb, acc[i], 0, 0, 0);
      }
    }
    __syncthreads();  // the tile and the partials are rewritten next iteration
  }
  if (MODE == 0) {
    rsum += __shfl_xor(rsum, 16, 64);
    rsum += __shfl_xor(rsum, 32, 64);
    if (wave == 0 && g == 0 && orow < no) out[(size_t)split * no + orow] = rsum;
    return;
  }
  if (orow >= no) return;
  // acc[i] C layout: lane holds out^T[d = dw + 16 i + 4g + r][owner = orow]
  float* dst = out + ((size_t)split * no + orow) * DP + dw;
#pragma unroll
  for (int i = 0; i < 2 * KS; ++i) *reinterpret_cast<f32x4*>(dst + i * 16 + 4 * g) = acc[i];
}

// tiles per split so that (owner blocks x splits) >= ~512 workgroups (2 per CU)
inline void ibw_plan(int no, int ni, int& ns, int& per) {
  const int ob = (no + 15) / 16, nt = (ni + IBW_T - 1) / IBW_T;
  ns = std::max(1, std::min(nt, (512 + ob - 1) / ob));
  per = (nt + ns - 1) / ns;
  ns = (nt + per - 1) / per;
}

// Positive logit + one-hot gradient term; one wave per query row.
// spos[i] = g*clip(qn_i . dn_pos), and when gscale != null:
//   h = -gscale_i*g*clip'; dQ_i += h*dn_pos ; dD_pos += h*qn_i
__global__ __launch_bounds__(256) void ib_pos_kernel(const unsigned short* __restrict__ X,
                                                     const unsigned short* __restrict__ Y, const int* __restrict__ pos,
                                                     float* __restrict__ spos, const float* __restrict__ gscale,
                                                     float* __restrict__ dX, float* __restrict__ dY, int nx, int DP,
                                                     float gamma, int clip) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nx) return;
  const int p = pos[row];
  float s = 0.f;
  for (int f = lane; f < DP; f += 64)
    s += bf16_to_f32(X[(size_t)row * DP + f]) * bf16_to_f32(Y[(size_t)p * DP + f]);
  s = wave_sum(s);
  const float rc = clip ? fminf(fmaxf(s, 0.f), 1.f) : s;
  if (spos && lane == 0) spos[row] = gamma * rc;
  if (gscale) {
    const bool pass = !clip || (s >= 0.f && s <= 1.f);
    const float h = pass ? -gscale[row] * gamma : 0.f;
    if (h != 0.f)
      for (int f = lane; f < DP; f += 64) {
        atomicAdd(&dX[(size_t)row * DP + f], h * bf16_to_f32(Y[(size_t)p * DP + f]));
        atomicAdd(&dY[(size_t)p * DP + f], h * bf16_to_f32(X[(size_t)row * DP + f]));
      }
  }
}

// Wide vectors, fallback path (D > 192 that ibw_kernel does not cover, e.g. DP = 640 / 896):
// the narrow flash kernels keep a query row's D accumulators in registers, which D = 768 does
// not fit, so the logits are tiled at the GEMM level instead — S is produced one column block (B x Mb, bounded memory) at a time by
// a bf16 x bf16 -> fp32 library GEMM and never exists whole.  Per block, one wave per row:
//  * forward (scale == nullptr): part[row] = sum_c exp(g * (clip(S_rc) - 1)) (the logits are
//    shifted by the largest possible one, as in the flash kernels, so block partial sums
//    simply add: ib_rowsum sums them in block order and finalises loss / P+);
//  * backward: S_rc <- scale_r * exp(g * (clip(S_rc) - 1)) * clip'(S_rc) in place (the
//    negative part of dS; ib_pos adds the positive pair), the block's dQ += dS . D_blk and
//    dD_blk = dS^T . Q are library GEMMs again.
__global__ __launch_bounds__(256) void ib_rows_blk_kernel(float* __restrict__ S, int ld, int B, int Mb,
                                                          const float* __restrict__ scale, float* __restrict__ part,
                                                          float gamma, int clip) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float* s = S + (size_t)row * ld;
  if (!scale) {
    float sum = 0.f;
    for (int c = lane; c < Mb; c += 64) {
      float r = s[c];
      if (clip) r = fminf(fmaxf(r, 0.f), 1.f);
      sum += __expf(gamma * (r - 1.f));
    }
    sum = wave_sum(sum);
    if (lane == 0) part[row] = sum;
    return;
  }
  const float sc = scale[row];
  for (int c = lane; c < Mb; c += 64) {
    const float raw = s[c];
    const bool pass = !clip || (raw >= 0.f && raw <= 1.f);
    const float r = clip ? fminf(fmaxf(raw, 0.f), 1.f) : raw;
    s[c] = pass ? sc * __expf(gamma * (r - 1.f)) : 0.f;
  }
}

// Batch statistics of the per-row loss in one workgroup: mean loss and accuracy
// (fraction of rows with P+ > 0.5) -- the training step's scalar loss and metric without
// torch's mean / compare / cast / mean launches.
__global__ __launch_bounds__(256) void loss_stats_kernel(const float* __restrict__ loss,
                                                         const float* __restrict__ prob, int B,
                                                         float* __restrict__ out_loss, float* __restrict__ out_acc) {
  float s = 0.f, a = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    s += loss[i];
    a += prob[i] > 0.5f ? 1.f : 0.f;
  }
  s = wave_sum(s);
  a = wave_sum(a);
  __shared__ float ws[4], wa[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    ws[w] = s;
    wa[w] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float inv = 1.f / (float)B;
    *out_loss = (ws[0] + ws[1] + ws[2] + ws[3]) * inv;
    if (out_acc) *out_acc = (wa[0] + wa[1] + wa[2] + wa[3]) * inv;
  }
}

// Backward prologue of the in-batch / cross-GPU loss: per-row upstream gradient g (a scalar
// mean-loss gradient broadcast as g0 * invB, or a (B,) vector), the softmax scale
// gamma * g / sumexp, and (when the forward kept U) dQ = scale * U -- one launch instead of
// the fill / copy / mul / div / mul of the eager expression.  Thread = one (row, 4 columns).
__global__ __launch_bounds__(256) void ib_grad_scale_kernel(const float* __restrict__ gl, int scalar, float invB,
                                                            const float* __restrict__ sumexp, int B, float gamma,
                                                            const float* __restrict__ U, int DP,
                                                            float* __restrict__ dq, float* __restrict__ scale,
                                                            float* __restrict__ grow) {
  const int per = U ? DP / 4 : 1;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)B * per) return;
  const int i = (int)(t / per), c4 = (int)(t - (long)i * per);
  const float g = scalar ? gl[0] * invB : gl[i];
  const float sc = g * gamma / sumexp[i];
  if (c4 == 0) {
    scale[i] = sc;
    grow[i] = g;
  }
  if (U) {
    const f32x4 u = *reinterpret_cast<const f32x4*>(U + (size_t)i * DP + 4 * c4);
    *reinterpret_cast<f32x4*>(dq + (size_t)i * DP + 4 * c4) = u * sc;
  }
}

// ---- fused glue of the in-batch loss (round 6) ------------------------------------------------
// Forward finish, one wave per query row, after the fused ib7 forward + dQ-part pass:
//   the positive logit (ib_pos's forward half: raw cosine s -> sraw, g*clip(s)), the split
//   partial sums -> sumexp -> loss = g + log(sumexp) - g*clip(s) and P+ (ib_rowsum), the split
//   partials of U -> U (ib_split_reduce), and each workgroup's partial sums of the batch mean
//   loss / accuracy, which ib_stats_final_kernel (one workgroup) adds in workgroup order
//   (deterministic, capturable).  Four launches -> two.  (A first version finished the batch sums
//   in the workgroup that took the last ticket of an agent-scope counter: the release fence each
//   workgroup needs before its ticket writes back its XCD's L2 — 74 vs 25 us per launch on the
//   headline shape, step 7.007 vs 6.948 ms, profiles/r6/glue3/.)
__global__ __launch_bounds__(256) void ib_fin_fwd_kernel(const unsigned short* __restrict__ X,
                                                         const unsigned short* __restrict__ Y,
                                                         const int* __restrict__ pos,
                                                         const float* __restrict__ part, int ns,
                                                         const float* __restrict__ ws_u, float* __restrict__ U,
                                                         int nx, int DP, float gamma, int clip,
                                                         float* __restrict__ sumexp, float* __restrict__ loss,
                                                         float* __restrict__ prob, float* __restrict__ sraw,
                                                         float* __restrict__ bpart) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  __shared__ float sl[4], sa[4];
  float lrow = 0.f, arow = 0.f;
  if (row < nx) {
    const int p = pos[row];
    float d = 0.f;
    for (int f = lane; f < DP; f += 64) d += bf16_to_f32(X[(size_t)row * DP + f]) * bf16_to_f32(Y[(size_t)p * DP + f]);
    d = wave_sum(d);
    float a = lane < ns ? part[(size_t)lane * nx + row] : 0.f;  // ns <= 64 (ib3_splits)
    a = wave_sum(a);
    const float spos = gamma * (clip ? fminf(fmaxf(d, 0.f), 1.f) : d);
    const float l = gamma + __logf(a) - spos;
    const float pr = __expf(-l);
    if (lane == 0) {
      sumexp[row] = a;
      loss[row] = l;
      prob[row] = pr;
      sraw[row] = d;
    }
    lrow = l;
    arow = pr > 0.5f ? 1.f : 0.f;
    if (ws_u && ns > 1) {
      const size_t plane4 = (size_t)nx * DP / 4;
      for (int c = lane; c < DP / 4; c += 64) {
        const size_t o4 = (size_t)row * (DP / 4) + c;
        reinterpret_cast<f32x4*>(U)[o4] = split_sum4(reinterpret_cast<const f32x4*>(ws_u), plane4, o4, ns);
      }
    }
  }
  if (!bpart) return;
  if (lane == 0) {
    sl[w] = lrow;
    sa[w] = arow;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    *reinterpret_cast<f32x2*>(bpart + 2 * blockIdx.x) = f32x2{(sl[0] + sl[1]) + (sl[2] + sl[3]),
                                                              (sa[0] + sa[1]) + (sa[2] + sa[3])};
}

// batch mean loss / accuracy from ib_fin_fwd_kernel's per-workgroup partials, summed in
// workgroup order (thread i: workgroups i, i + 256, ...; then the 256 sums in thread order)
__global__ __launch_bounds__(256) void ib_stats_final_kernel(const float* __restrict__ bpart, int nb, int nx,
                                                             float* __restrict__ out_loss, float* __restrict__ out_acc) {
  float s = 0.f, a = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256) {
    const f32x2 v = *reinterpret_cast<const f32x2*>(bpart + 2 * b);
    s += v[0];
    a += v[1];
  }
  __shared__ float ts[256], ta[256];
  ts[threadIdx.x] = s;
  ta[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, A = 0.f;
    for (int i = 0; i < 256; ++i) {
      S += ts[i];
      A += ta[i];
    }
    const float inv = 1.f / (float)nx;
    *out_loss = S * inv;
    if (out_acc) *out_acc = A * inv;
  }
}

// dD finish, thread = (page row, 4 columns): the split partials of the dD pass (ib_split_reduce;
// ns = 1: in place) plus the positive pair's one-hot term for the rows that are some query's
// positive (ib_pos's backward half on the page side): dD_m += h_b X_b with b = inv[m],
// h_b = -grow_b * gamma where clip(s_b) passes its gradient.
__global__ __launch_bounds__(256) void ib_fin_dd_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                        int nrows, int DP, int ns, const int* __restrict__ inv,
                                                        const unsigned short* __restrict__ Q,
                                                        const float* __restrict__ grow, const float* __restrict__ sraw,
                                                        float gamma, int clip) {
  const int per = DP / 4;
  const long n4 = (long)nrows * per;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 a = split_sum4(reinterpret_cast<const f32x4*>(ws), (size_t)n4, (size_t)i, ns);
    const int m = (int)(i / per), c = 4 * (int)(i - (long)m * per);
    const int b = inv[m];
    if (b >= 0) {
      const float sb = sraw[b];
      if (!clip || (sb >= 0.f && sb <= 1.f)) {
        const float h = -grow[b] * gamma;
        const unsigned short* q = Q + (size_t)b * DP + c;
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += h * bf16_to_f32(q[k]);
      }
    }
    reinterpret_cast<f32x4*>(out)[i] = a;
  }
}

// Backward prologue with the query side of the positive pair folded in: ib_grad_scale's scale /
// per-row gradient / dQ = scale * U, plus dQ_i += h_i * Y_pos(i) (h_i as in ib_fin_dd_kernel).
__global__ __launch_bounds__(256) void ib_grad_scale_pos_kernel(const float* __restrict__ gl, int scalar, float invB,
                                                                const float* __restrict__ sumexp, int B, float gamma,
                                                                const float* __restrict__ U, int DP,
                                                                float* __restrict__ dq, float* __restrict__ scale,
                                                                float* __restrict__ grow,
                                                                const unsigned short* __restrict__ Y,
                                                                const int* __restrict__ pos,
                                                                const float* __restrict__ sraw, int clip) {
  const int per = DP / 4;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)B * per) return;
  const int i = (int)(t / per), c4 = (int)(t - (long)i * per);
  const float g = scalar ? gl[0] * invB : gl[i];
  const float sc = g * gamma / sumexp[i];
  if (c4 == 0) {
    scale[i] = sc;
    grow[i] = g;
  }
  f32x4 u = *reinterpret_cast<const f32x4*>(U + (size_t)i * DP + 4 * c4) * sc;
  const float sb = sraw[i];
  if (!clip || (sb >= 0.f && sb <= 1.f)) {
    const float h = -g * gamma;
    const unsigned short* y = Y + (size_t)pos[i] * DP + 4 * c4;
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] += h * bf16_to_f32(y[k]);
  }
  *reinterpret_cast<f32x4*>(dq + (size_t)i * DP + 4 * c4) = u;
}

PV_DEBUG_EXPORT(loss)
}  // namespace loss
}  // namespace pv

using namespace pv;

PV_API int pv_dssm_explicit(const float* q, const float* d, float* loss, float* prob, float* dq, float* dd, int B,
                            int J1, int D, float gamma, float gscale, int clip, void* stream) {
  if (J1 < 1 || J1 > 64 || D < 1 || D > 1024) return -1;
  const dim3 grid((B + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
#define PV_EXPL(MD, MJ)                                                                                  \
  hipLaunchKernelGGL((pv::loss::dssm_explicit_kernel<MD, MJ>), grid, dim3(256), 0, st, q, d, loss, prob, dq, dd, \
                     B, J1, D, gamma, gscale, clip)
  const int md = D <= 128 ? 2 : D <= 256 ? 4 : D <= 512 ? 8 : 16;
  if (J1 <= 16) {
    if (md == 2) PV_EXPL(2, 16); else if (md == 4) PV_EXPL(4, 16); else if (md == 8) PV_EXPL(8, 16); else PV_EXPL(16, 16);
  } else {
    if (md == 2) PV_EXPL(2, 64); else if (md == 4) PV_EXPL(4, 64); else if (md == 8) PV_EXPL(8, 64); else PV_EXPL(16, 64);
  }
#undef PV_EXPL
  PV_LAUNCH_CHECK();
  return 0;
}

static int ib_splits(int nx, int ny, int per_min) {
  int rb = (nx + pv::loss::TQ - 1) / pv::loss::TQ;
  int want = (1024 + rb - 1) / rb;  // ~1024 workgroups
  int maxs = (ny + per_min - 1) / per_min;
  if (want > maxs) want = maxs;
  return want < 1 ? 1 : want;
}

#define IB_DISPATCH(KSV, ...)           \
  switch (KSV) {                         \
    case 1: { constexpr int KS = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int KS = 2; __VA_ARGS__; break; } \
    case 3: { constexpr int KS = 3; __VA_ARGS__; break; } \
    case 4: { constexpr int KS = 4; __VA_ARGS__; break; } \
    case 5: { constexpr int KS = 5; __VA_ARGS__; break; } \
    case 6: { constexpr int KS = 6; __VA_ARGS__; break; } \
    case 8: { constexpr int KS = 8; __VA_ARGS__; break; } \
    default: return -1;                  \
  }

static int ib_fwd_splits(int nx, int ny) {
  int ns = ib_splits(nx, ny, 256);
  const int per = ((ny + ns - 1) / ns + pv::loss::TD - 1) / pv::loss::TD * pv::loss::TD;
  return (ny + per - 1) / per;
}

// floats of workspace pv_ib_fwd needs
PV_API long pv_ib_fwd_ws(int nx, int ny, int DP) {
  (void)DP;
  return (long)ib_fwd_splits(nx, ny) * nx;
}

PV_API int pv_ib_fwd(const void* X, const void* Y, float* sumexp, float* ws, int nx, int ny, int DP, float gamma,
                     int clip, const float* spos, float* loss, float* prob, void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192) return -2;
  const int ns = ib_fwd_splits(nx, ny);
  const int per = ((ny + ns - 1) / ns + TD - 1) / TD * TD;
  dim3 grid((nx + TQ - 1) / TQ, ns);
  if (clip) {
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib_fwd_kernel<KS, true>), grid, dim3(256), 0, (hipStream_t)stream,
                                            (const unsigned short*)X, (const unsigned short*)Y, ws, nx, ny, per,
                                            gamma));
  } else {
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib_fwd_kernel<KS, false>), grid, dim3(256), 0, (hipStream_t)stream,
                                            (const unsigned short*)X, (const unsigned short*)Y, ws, nx, ny, per,
                                            gamma));
  }
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ib_rowsum_kernel, dim3((nx + 255) / 256), dim3(256), 0, (hipStream_t)stream, ws, sumexp, nx, ns,
                     spos, loss, prob, gamma);
  PV_LAUNCH_CHECK();
  return 0;
}

// Kernel generation (pv_ib_set_version; the production generation is 7):
//   7: ib7 (ib5 software-pipelined) for every pass at DP = 160 / 128, ib3 for the other widths
//      (fused forward -15 %, dD pass -3 % vs gens 5 / 3: profiles/r5_ib7/)
//   5, 3: the earlier generations, kept as the numerics oracles of the ib7 tests (ib7 is
//      bit-identical to ib5) and for tools/ib_micro.py; no environment switch selects them
static int g_ib_version = 7;
static int ib_version() { return g_ib_version; }

PV_API int pv_ib_version() { return ib_version(); }
// A/B and tests: switch the kernel version (between steps only: workspaces are sized per version)
PV_API int pv_ib_set_version(int v) {
  if (v != 3 && v != 5 && v != 7) return -1;
  g_ib_version = v;
  return 0;
}

static int ib3_splits(int nx, int ny) {
  // 256 workgroups of 8 waves fill the chip (one per CU); keep >= 16 tiles per split
  const int rb = (nx + 255) / 256;
  int ns = (256 + rb - 1) / rb;
  const int maxs = (ny + 16 * pv::loss::TD - 1) / (16 * pv::loss::TD);
  if (ns > maxs) ns = maxs;
  return ns < 1 ? 1 : ns;
}

// (splits, Y rows per split) of the current kernel version, every split non-empty
static void ib_split_plan(int nx, int ny, int& ns, int& per) {
  ns = ib3_splits(nx, ny);
  per = ((ny + ns - 1) / ns + pv::loss::TD - 1) / pv::loss::TD * pv::loss::TD;
  ns = (ny + per - 1) / per;
}

// floats of workspace pv_ib_bwd needs for (nx, ny, DP) (0 = writes out directly)
PV_API long pv_ib_bwd_ws(int nx, int ny, int DP) {
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  return ns > 1 ? (long)ns * nx * DP : 0;
}

// out (nx, DP) fp32 is fully written (no zeroing needed).
PV_API int pv_ib_bwd(const void* X, const void* Y, const float* scale, float* out, float* ws, int nx, int ny, int DP,
                      float gamma, int clip, int row_scale, void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192) return -2;
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  if (ns > 1 && !ws) return -3;
  hipStream_t s = (hipStream_t)stream;
  const int nrb = (nx + 255) / 256;
  const dim3 grid3(nrb * ns);
#define PV_IB_BWD(ROWV, CLIPV)                                                                                  \
  if (ib_version() == 7 && DP == 160) {                                                                         \
    hipLaunchKernelGGL((ib7_kernel<5, ROWV, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,          \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else if (ib_version() == 7 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib7_kernel<4, ROWV, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,          \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else if (ib_version() == 5 && ROWV && DP == 160) {                                                                 \
    hipLaunchKernelGGL((ib5_kernel<5, ROWV, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,          \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else if (ib_version() == 5 && ROWV && DP == 128) {                                                          \
    hipLaunchKernelGGL((ib5_kernel<4, ROWV, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,          \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else {                                                                                                      \
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib3_kernel<KS, ROWV, CLIPV>), grid3, dim3(512), 0, s,              \
                                            (const unsigned short*)X, (const unsigned short*)Y, scale, out, ws, \
                                            nx, ny, per, nrb, gamma));                                          \
  }
  if (row_scale) {
    if (clip) { PV_IB_BWD(true, true); } else { PV_IB_BWD(true, false); }
  } else {
    if (clip) { PV_IB_BWD(false, true); } else { PV_IB_BWD(false, false); }
  }
#undef PV_IB_BWD
  PV_LAUNCH_CHECK();
  if (ns > 1) {
    const long n4 = (long)nx * DP / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(ib_split_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, out, n4, ns);
    PV_LAUNCH_CHECK();
  }
  return 0;
}

// Fused forward + dQ part (ib5 / ib3 with FWD = true): sumexp (nx), U (nx, DP) fp32 fully
// written; ws_u = pv_ib_bwd_ws(nx, ny, DP) floats, part = pv_ib_fwd_dq_parts(nx, ny) floats.
PV_API long pv_ib_fwd_dq_parts(int nx, int ny) {
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  return (long)ns * nx;
}

PV_API int pv_ib_fwd_dq(const void* X, const void* Y, float* sumexp, float* U, float* ws_u, float* part, int nx,
                        int ny, int DP, float gamma, int clip, const float* spos, float* loss, float* prob,
                        void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192) return -2;
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  if (ns > 1 && !ws_u) return -3;
  hipStream_t s = (hipStream_t)stream;
  const int nrb = (nx + 255) / 256;
  const dim3 grid3(nrb * ns);
#define PV_IB_FWDDQ(CLIPV)                                                                                      \
  if (ib_version() == 7 && DP == 160) {                                                                         \
    hipLaunchKernelGGL((ib7_kernel<5, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 7 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib7_kernel<4, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 5 && DP == 160) {                                                                         \
    hipLaunchKernelGGL((ib5_kernel<5, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 5 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib5_kernel<4, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else {                                                                                                      \
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib3_kernel<KS, true, CLIPV, true>), grid3, dim3(512), 0, s,        \
                                            (const unsigned short*)X, (const unsigned short*)Y, nullptr, U,     \
                                            ws_u, nx, ny, per, nrb, gamma, part));                              \
  }
  if (clip) { PV_IB_FWDDQ(true); } else { PV_IB_FWDDQ(false); }
#undef PV_IB_FWDDQ
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(ib_rowsum_kernel, dim3((nx + 255) / 256), dim3(256), 0, s, part, sumexp, nx, ns, spos, loss,
                     prob, gamma);
  PV_LAUNCH_CHECK();
  if (ns > 1) {
    const long n4 = (long)nx * DP / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(ib_split_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws_u, U, n4, ns);
    PV_LAUNCH_CHECK();
  }
  return 0;
}

PV_API int pv_ib_pos(const void* X, const void* Y, const int* pos, float* spos, const float* gscale, float* dX,
                     float* dY, int nx, int DP, float gamma, int clip, void* stream) {
  hipLaunchKernelGGL(pv::loss::ib_pos_kernel, dim3((nx + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)X, (const unsigned short*)Y, pos, spos, gscale, dX, dY, nx, DP, gamma,
                     clip);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_ib_rows_blk(float* S, int ld, int B, int Mb, const float* scale, float* part, float gamma, int clip,
                          void* stream) {
  if (B <= 0 || Mb <= 0 || ld < Mb || (!scale && !part)) return -1;
  hipLaunchKernelGGL(pv::loss::ib_rows_blk_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, ld, B, Mb,
                     scale, part, gamma, clip);
  PV_LAUNCH_CHECK();
  return 0;
}

// sumexp = sum of the ns block partials (part[s][row], fixed order); loss = spos-based
// g + log(sumexp) - spos, P+ = exp(-loss)
PV_API int pv_ib_rowsum(const float* part, float* sumexp, int B, int ns, const float* spos, float* loss, float* prob,
                        float gamma, void* stream) {
  if (B <= 0 || ns <= 0) return -1;
  hipLaunchKernelGGL(pv::loss::ib_rowsum_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, part,
                     sumexp, B, ns, spos, loss, prob, gamma);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_loss_stats(const float* loss, const float* prob, int B, float* out_loss, float* out_acc, void* stream) {
  if (B < 1) return -1;
  hipLaunchKernelGGL(pv::loss::loss_stats_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, loss, prob, B, out_loss,
                     out_acc);
  PV_LAUNCH_CHECK();
  return 0;
}

// gl: scalar (scalar = 1, gradient of the mean: g = gl[0] * invB) or (B,) per-row gradient.
PV_API int pv_ib_grad_scale(const float* gl, int scalar, float invB, const float* sumexp, int B, float gamma,
                            const float* U, int DP, float* dq, float* scale, float* grow, void* stream) {
  if (B < 1 || (U && (DP % 4 || !dq))) return -1;
  const long n = (long)B * (U ? DP / 4 : 1);
  hipLaunchKernelGGL(pv::loss::ib_grad_scale_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gl, scalar, invB, sumexp, B, gamma, U, DP, dq, scale, grow);
  PV_LAUNCH_CHECK();
  return 0;
}

// Wide-vector in-batch loss passes (ibw_kernel), DP % 128 == 0, 256 <= DP <= 1024.
// mode 0: part (ns x no) row partial sums of exp(g (clip(S) - 1)), S = O . It^T;
// mode 1 / 2: out (no x DP) fp32 = sum_j G . It_j with the scale indexed by the owner row (1) or
// the iterated row (2); ws >= pv_ibw_ws(no, ni, DP) floats when ns > 1.  pv_ibw_splits -> ns.
PV_API int pv_ibw_splits(int no, int ni) {
  int ns, per;
  pv::loss::ibw_plan(no, ni, ns, per);
  return ns;
}

PV_API long pv_ibw_ws(int no, int ni, int DP) {
  int ns, per;
  pv::loss::ibw_plan(no, ni, ns, per);
  return ns > 1 ? (long)ns * no * DP : 0;
}

PV_API int pv_ibw(const void* O, int no, const void* It, int ni, int DP, const float* scale, float gamma, int clip,
                  int mode, float* out, float* ws, void* stream) {
  using namespace pv::loss;
  if (no <= 0 || ni <= 0 || DP % 128 || DP < 256 || DP > 1024 || mode < 0 || mode > 2) return -1;
  if (mode > 0 && !scale) return -2;
  int ns, per;
  ibw_plan(no, ni, ns, per);
  if (mode > 0 && ns > 1 && !ws) return -3;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((no + 15) / 16, ns);
  float* dst = (mode == 0 || ns == 1) ? out : ws;
  const size_t lds = (size_t)IBW_T * (DP + 8) * 2 + 4 * 2 * 64 * sizeof(f32x4);
  const unsigned short* o16 = (const unsigned short*)O;
  const unsigned short* i16 = (const unsigned short*)It;
  bool done = false;
#define PV_IBW(KSV, MODEV, CLIPV)                                                                          \
  if (!done && DP == KSV * 128 && mode == MODEV && clip == CLIPV) {                                       \
    static bool attr = false;                                                                              \
    if (!attr) {                                                                                           \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&ibw_kernel<KSV, MODEV, CLIPV>),               \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)         \
        return -5;                                                                                         \
      attr = true;                                                                                         \
    }                                                                                                      \
    hipLaunchKernelGGL((ibw_kernel<KSV, MODEV, CLIPV>), grid, dim3(256), lds, s, o16, no, i16, ni, scale,  \
                       gamma, dst, per);                                                                   \
    done = true;                                                                                           \
  }
#define PV_IBW_KS(KSV) \
  PV_IBW(KSV, 0, 0) PV_IBW(KSV, 0, 1) PV_IBW(KSV, 1, 0) PV_IBW(KSV, 1, 1) PV_IBW(KSV, 2, 0) PV_IBW(KSV, 2, 1)
  PV_IBW_KS(2) PV_IBW_KS(3) PV_IBW_KS(4) PV_IBW_KS(6) PV_IBW_KS(8)
#undef PV_IBW_KS
#undef PV_IBW
  if (!done) return -4;  // DP = 640, 896: no instantiation
  PV_LAUNCH_CHECK();
  if (mode > 0 && ns > 1) {
    const long n4 = (long)no * DP / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ib_split_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ws, out, n4, ns);
    PV_LAUNCH_CHECK();
  }
  return 0;
}

// ---- fused in-batch loss glue (round 6): see ib_fin_fwd_kernel / ib_fin_dd_kernel ----------
// Forward: the ib7 (or ib5 / ib3) forward + dQ-part pass, then ONE finish launch.  pos (nx)
// positive page per query; sraw (nx) receives the raw positive cosines the backward needs;
// bpart: 2 * ceil(nx / 4) floats of workgroup partials; out_loss / out_acc: 0-dim outputs (null
// bpart / out_loss: no batch statistics).
PV_API int pv_ib_fwd_dq2(const void* X, const void* Y, const int* pos, float* sumexp, float* U, float* ws_u,
                         float* part, int nx, int ny, int DP, float gamma, int clip, float* sraw, float* loss,
                         float* prob, float* bpart, float* out_loss, float* out_acc, void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192 || nx < 1) return -2;
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  if ((ns > 1 && !ws_u) || ns > 64) return -3;
  hipStream_t s = (hipStream_t)stream;
  const int nrb = (nx + 255) / 256;
  const dim3 grid3(nrb * ns);
#define PV_IB_FWDDQ2(CLIPV)                                                                                     \
  if (ib_version() == 7 && DP == 160) {                                                                         \
    hipLaunchKernelGGL((ib7_kernel<5, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 7 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib7_kernel<4, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 5 && DP == 160) {                                                                  \
    hipLaunchKernelGGL((ib5_kernel<5, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else if (ib_version() == 5 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib5_kernel<4, true, CLIPV, true>), grid3, dim3(512), 0, s, (const unsigned short*)X,    \
                       (const unsigned short*)Y, nullptr, U, ws_u, nx, ny, per, nrb, gamma, part);              \
  } else {                                                                                                      \
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib3_kernel<KS, true, CLIPV, true>), grid3, dim3(512), 0, s,        \
                                            (const unsigned short*)X, (const unsigned short*)Y, nullptr, U,     \
                                            ws_u, nx, ny, per, nrb, gamma, part));                              \
  }
  if (clip) { PV_IB_FWDDQ2(true); } else { PV_IB_FWDDQ2(false); }
#undef PV_IB_FWDDQ2
  PV_LAUNCH_CHECK();
  const int nb = (nx + 3) / 4;
  const bool stats = bpart && out_loss;
  hipLaunchKernelGGL(ib_fin_fwd_kernel, dim3(nb), dim3(256), 0, s, (const unsigned short*)X,
                     (const unsigned short*)Y, pos, part, ns, ns > 1 ? ws_u : nullptr, U, nx, DP, gamma, clip, sumexp,
                     loss, prob, sraw, stats ? bpart : nullptr);
  PV_LAUNCH_CHECK();
  if (stats) {
    hipLaunchKernelGGL(ib_stats_final_kernel, dim3(1), dim3(256), 0, s, (const float*)bpart, nb, nx, out_loss, out_acc);
    PV_LAUNCH_CHECK();
  }
  return 0;
}

// Backward prologue (dQ = scale * U + the positive pair's query term), see ib_grad_scale_pos_kernel.
PV_API int pv_ib_grad_scale_pos(const float* gl, int scalar, float invB, const float* sumexp, int B, float gamma,
                                const float* U, int DP, float* dq, float* scale, float* grow, const void* Y,
                                const int* pos, const float* sraw, int clip, void* stream) {
  if (B < 1 || DP % 4 || !U || !dq) return -1;
  const long n = (long)B * (DP / 4);
  hipLaunchKernelGGL(pv::loss::ib_grad_scale_pos_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gl, scalar, invB, sumexp, B, gamma, U, DP, dq, scale, grow,
                     (const unsigned short*)Y, pos, sraw, clip);
  PV_LAUNCH_CHECK();
  return 0;
}

// dD pass (X = pages, Y = queries, scale indexed by the query) + ONE finish launch that sums the
// split partials and adds the positive pair's page term: inv (nx) = the query whose positive
// page row m is (-1: none).
PV_API int pv_ib_bwd_dd_pos(const void* X, const void* Y, const float* scale, float* out, float* ws, int nx, int ny,
                            int DP, float gamma, int clip, const int* inv, const float* grow, const float* sraw,
                            void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192) return -2;
  int ns, per;
  ib_split_plan(nx, ny, ns, per);
  if (ns > 1 && !ws) return -3;
  hipStream_t s = (hipStream_t)stream;
  const int nrb = (nx + 255) / 256;
  const dim3 grid3(nrb * ns);
#define PV_IB_DD(CLIPV)                                                                                         \
  if (ib_version() == 7 && DP == 160) {                                                                         \
    hipLaunchKernelGGL((ib7_kernel<5, false, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,         \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else if (ib_version() == 7 && DP == 128) {                                                                  \
    hipLaunchKernelGGL((ib7_kernel<4, false, CLIPV>), grid3, dim3(512), 0, s, (const unsigned short*)X,         \
                       (const unsigned short*)Y, scale, out, ws, nx, ny, per, nrb, gamma);                      \
  } else {                                                                                                      \
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib3_kernel<KS, false, CLIPV>), grid3, dim3(512), 0, s,             \
                                            (const unsigned short*)X, (const unsigned short*)Y, scale, out, ws, \
                                            nx, ny, per, nrb, gamma));                                          \
  }
  if (clip) { PV_IB_DD(true); } else { PV_IB_DD(false); }
#undef PV_IB_DD
  PV_LAUNCH_CHECK();
  const long n4 = (long)nx * DP / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(ib_fin_dd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ns > 1 ? ws : out, out, nx, DP,
                     ns > 1 ? ns : 1, inv, (const unsigned short*)Y, grow, sraw, gamma, clip);
  PV_LAUNCH_CHECK();
  return 0;
}

