// bf16 GEMM engine for the dense layers (K4 backward, the MLP bag GEMMs, the BERT
// projections): C[M][N] = epilogue( A[M][K] . B[N][K]^T ), fp32 accumulation on
// v_mfma_f32_16x16x32_bf16.
//
// Operand storage (compile time), so every GEMM of a linear layer runs without a transpose:
//   ROW: K contiguous  (A: [M][K], B: [N][K])      -- forward  y = x W^T
//   COL: M / N contiguous (A: [K][M], B: [K][N])   -- dgrad dx = dy W (B COL), wgrad
//                                                     dW = dy^T x (A and B COL), counts bag
//                                                     C W (B COL) and C^T G (both COL)
// Workgroup tile 256 x 256 x 64, 8 waves (2 x 4), each wave 128 x 64 = 8 x 4 accumulators.
// Staging: direct-to-LDS loads (global_load_lds_dwordx4, no VGPR round trip), double-
// buffered K tiles; the LDS image is lane-linear per wave instruction, so the bank-conflict
// swizzle is applied to the per-lane SOURCE address and the same XOR on the reads
// (cdna_hip_programming.md rule 21):
//   ROW tile [256 rows][64 k], 128-B rows: 16-B chunk c of row r stored at c ^ (r & 7);
//        A/B fragments by ds_read_b128 (conflict-free for the 16-lane read groups);
//   COL tile [64 k][256 m], 512-B rows: 16-B chunk c of k-row r stored at c ^ 2h(r),
//        h(r) = (r & 3) | ((r >> 3) & 1) << 2; fragments by two ds_read_b64_tr_b16 (the
//        hardware transpose read) per 8 k-values, natural k order.
// Epilogue (fused): alpha scale, per-column bias, activation (relu / gelu-tanh / tanh),
// beta = 1 accumulation into C (residual / flat-gradient accumulate), fp32 or bf16 output,
// and split-K: each K slice writes its fp32 partial tile into its slab of a workspace that
// dense.hip::colsum_kernel reduces (with the same epilogue) — the (M/256)(N/256) output tiles
// of a weight gradient are far fewer than the 256 CUs.
// Edges: rows / columns beyond M / N are loaded from a clamped (valid) address and never
// stored; K must be a multiple of 64 (callers pad — the operands here all are).
#include "common.h"
#include <stdlib.h>

namespace pv {
namespace gemm {
PV_DEBUG_FLAG

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTH = 512;
constexpr int TILE_BYTES = 256 * 64 * 2;  // one operand tile (32 KB)
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

enum Layout { ROW = 0, COL = 1 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_TANH = 3 };

struct Params {
  const unsigned short* A;
  const unsigned short* B;
  long lda, ldb;        // elements between consecutive rows of the STORED matrices
  void* C;
  long ldc;
  int M, N, K;
  int ksplit;           // K slices (1: direct epilogue; > 1: fp32 partial slabs into C)
  long slab;            // elements between the partial slabs (ksplit > 1)
  const float* bias;    // (N) or null
  float alpha;
  int act;
  int beta;             // 1: C += result (fp32 or bf16 C)
  int out_bf16;
  int tiles_m, tiles_n;
  int n_fastest;        // tile order: 1 = N-fastest (A panel shared by consecutive tiles)
  int group;            // > 0: tiles in column-major groups of `group` tile rows (L2 reuse of both panels)
};

// Output tile of (per-split) tile id t.  Consecutive ids run on one XCD (xcd_remap), ~32 of
// them at a time: with group = G they cover G tile rows x (32 / G) tile columns, so each K
// step brings G A-slices and 32 / G B-slices into that XCD's L2 instead of 1 + 32 (a row of
// tiles) — the difference between an L2-resident and an HBM-streamed square GEMM.
__device__ __forceinline__ void tile_of(const Params& p, int t, int& tm, int& tn) {
  if (p.group > 0) {
    const int per_group = p.group * p.tiles_n;
    const int g = t / per_group, first = g * p.group;
    const int gm = min(p.tiles_m - first, p.group);
    const int r = t - g * per_group;
    tm = first + r % gm;
    tn = r / gm;
    return;
  }
  tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
}

__device__ __forceinline__ int h_of(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ void glds16(const unsigned short* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Stage one operand tile (rows [r0, r0 + 256) of the logical operand, k [k0, k0 + 64)) into
// `dst` (32 KB).  4 wave-instructions of 1 KB per wave.
template <int LAY>
__device__ __forceinline__ void stage(const unsigned short* __restrict__ X, long ld, int r0, int rmax, int k0,
                                      char* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int piece = wave * 4 + u;  // 0..31
    if constexpr (LAY == ROW) {
      const int r = piece * 8 + (lane >> 3);           // tile row 0..255
      const int c = (lane & 7) ^ (r & 7);              // logical 16-byte chunk of the row
      const int gr = min(r0 + r, rmax);                // clamped (never stored)
      glds16(X + (size_t)gr * ld + k0 + c * 8, dst + piece * 1024);
    } else {
      const int kr = piece * 2 + (lane >> 5);          // tile k-row 0..63
      const int c = (lane & 31) ^ (2 * h_of(kr));      // logical 16-byte chunk (8 rows of the operand)
      int col = r0 + c * 8;
      col = col <= rmax ? col : 0;                     // groups past the edge (M % 8 == 0): never stored
      glds16(X + (size_t)(k0 + kr) * ld + col, dst + piece * 1024);
    }
  }
}

// A/B fragment of rows [rb, rb + 16) (tile-local), k-step s (32 k) from a staged tile
template <int LAY>
__device__ __forceinline__ bf16x8 frag(const char* t, int rb, int s) {
  const int lane = threadIdx.x & 63;
  if constexpr (LAY == ROW) {
    const int r = rb + (lane & 15);
    const int c = (4 * s + (lane >> 4)) ^ (r & 7);
    return *reinterpret_cast<const bf16x8*>(t + r * 128 + c * 16);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int klo = 32 * s + 8 * g + q, khi = klo + 4;
    const int col = rb + 4 * p;                 // operand row index (tile-local), 4 of them
    const int c = col >> 3, half = (col & 7) * 2;  // chunk and byte offset in it
    const char* plo = t + klo * 512 + ((c ^ (2 * h_of(klo))) * 16) + half;
    const char* phi = t + khi * 512 + ((c ^ (2 * h_of(khi))) * 16) + half;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)plo);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)phi);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

__device__ __forceinline__ float act_f(float x, int act) {
  if (act == ACT_RELU) return x > 0.f ? x : 0.f;
  if (act == ACT_GELU) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + (1.f - 2.f / (__expf(2.f * u) + 1.f)));
  }
  if (act == ACT_TANH) return 1.f - 2.f / (__expf(2.f * x) + 1.f);
  return x;
}

__device__ __forceinline__ void epilogue(const Params& p, f32x4 (&acc)[8][4], int split, int m0, int n0, int wr,
                                         int wc, int lane) {
  // acc[i][j][r] is C[m0 + wr*128 + 16i + 4(lane>>4) + r][n0 + wc*64 + 16j + (lane&15)]
  const int colb = n0 + wc * 64 + (lane & 15);
  const int rowb = m0 + wr * 128 + 4 * (lane >> 4);
  if (p.ksplit > 1) {  // fp32 partial slab of this K slice
    float* Cs = reinterpret_cast<float*>(p.C) + (size_t)split * p.slab;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rowb + 16 * i + r;
        if (row >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = colb + 16 * j;
          if (col < p.N) Cs[(size_t)row * p.ldc + col] = acc[i][j][r] * p.alpha;
        }
      }
    return;
  }
  float bj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = colb + 16 * j;
    bj[j] = (p.bias && col < p.N) ? p.bias[col] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rowb + 16 * i + r;
      if (row >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = colb + 16 * j;
        if (col >= p.N) continue;
        float v = act_f(acc[i][j][r] * p.alpha + bj[j], p.act);
        const size_t o = (size_t)row * p.ldc + col;
        if (p.out_bf16) {
          unsigned short* Cb = reinterpret_cast<unsigned short*>(p.C);
          if (p.beta) v += bf16_to_f32(Cb[o]);
          Cb[o] = f32_to_bf16(v);
        } else {
          float* Cf = reinterpret_cast<float*>(p.C);
          Cf[o] = p.beta ? Cf[o] + v : v;
        }
      }
    }
}

// ---- v2 schedule: fragment reads software-pipelined one sub-step ahead --------------------
// A K tile is 4 sub-steps of 16 MFMAs (k-step s x half h of the wave's 8 A row tiles); the
// fragments of sub-step u+1 are read while the MFMAs of u run (two register sets), and the
// tile switch is placed INSIDE the last sub-step: wait for the next tile (staged one tile
// ahead), barrier, issue its first fragment reads, THEN the last 16 MFMAs of the current
// tile, then stage the tile after next into the buffer everyone has finished reading.  One
// barrier per K tile and no fragment-read bubble at the tile boundary.
template <int LAY, int H>
__device__ __forceinline__ void read_a4(const char* t, int rb, int s, bf16x8 (&a)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = frag<LAY>(t, rb + 64 * H + 16 * i, s);
}

template <int ALAY, int BLAY>
__global__ __launch_bounds__(NTH, 2) void gemm2_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // [buf][A, B]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 2, wc = wave & 3;
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int ntile = p.tiles_m * p.tiles_n;
  const int split = bid / ntile, t = bid - split * ntile;
  int tm, tn;
  tile_of(p, t, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * per, kt1 = min(ktiles, kt0 + per);
  const int arb = wr * 128, brb = wc * 64;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    stage<ALAY>(p.A, p.lda, m0, p.M - 1, kt0 * BK, smem);
    stage<BLAY>(p.B, p.ldb, n0, p.N - 1, kt0 * BK, smem + TILE_BYTES);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt0 + 1 < kt1) {
      stage<ALAY>(p.A, p.lda, m0, p.M - 1, (kt0 + 1) * BK, smem + 2 * TILE_BYTES);
      stage<BLAY>(p.B, p.ldb, n0, p.N - 1, (kt0 + 1) * BK, smem + 3 * TILE_BYTES);
    }
    bf16x8 a0[4], a1[4], b0[4], b1[4];
    {
      const char* ta = smem;
      const char* tb = smem + TILE_BYTES;
#pragma unroll
      for (int j = 0; j < 4; ++j) b0[j] = frag<BLAY>(tb, brb + 16 * j, 0);
      read_a4<ALAY, 0>(ta, arb, 0, a0);
    }
    int buf = 0;
#pragma unroll 1
    for (int kt = kt0; kt < kt1; ++kt) {
      const char* ta = smem + buf * 2 * TILE_BYTES;
      const char* tb = ta + TILE_BYTES;
      // u = 0: (s0, h0) computes with a0/b0; read (s0, h1) -> a1, and s1's B -> b1
      read_a4<ALAY, 1>(ta, arb, 0, a1);
#pragma unroll
      for (int j = 0; j < 4; ++j) b1[j] = frag<BLAY>(tb, brb + 16 * j, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      // u = 1: (s0, h1) with a1/b0; read (s1, h0) -> a0
      read_a4<ALAY, 0>(ta, arb, 1, a0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b0[j], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      // u = 2: (s1, h0) with a0/b1; read (s1, h1) -> a1
      read_a4<ALAY, 1>(ta, arb, 1, a1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b1[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      // u = 3: (s1, h1) with a1/b1; tile switch: next tile landed -> barrier -> its first reads
      const bool more = kt + 1 < kt1;
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
      if (more) {
        const char* na = smem + (buf ^ 1) * 2 * TILE_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) b0[j] = frag<BLAY>(na + TILE_BYTES, brb + 16 * j, 0);
        read_a4<ALAY, 0>(na, arb, 0, a0);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (kt + 2 < kt1) {  // everyone passed the barrier: this buffer is free
        char* sa = smem + buf * 2 * TILE_BYTES;
        stage<ALAY>(p.A, p.lda, m0, p.M - 1, (kt + 2) * BK, sa);
        stage<BLAY>(p.B, p.ldb, n0, p.N - 1, (kt + 2) * BK, sa + TILE_BYTES);
      }
      buf ^= 1;
    }
  }
  epilogue(p, acc, split, m0, n0, wr, wc, lane);
}


PV_DEBUG_EXPORT(gemm)
}  // namespace gemm
}  // namespace pv

using namespace pv;

// tile grouping (Params::group); 0 = the row / column panel order
static int g_gemm_group = getenv("PAGEVEC_GEMM_GROUP") ? atoi(getenv("PAGEVEC_GEMM_GROUP")) : 4;
PV_API void pv_gemm_set_group(int g) { g_gemm_group = g; }

// C = epi(alpha * A . B^T); a_col / b_col select the COL storage of A ([K][M]) / B ([K][N]).
// ksplit > 1: C is a workspace of ksplit fp32 slabs (slab = elements per slab), reduced by
// the caller (pv_colsum); bias / act / beta / bf16 apply only with ksplit == 1.
PV_API int pv_gemm_bf16(const void* A, long lda, int a_col, const void* B, long ldb, int b_col, void* C, long ldc,
                        int M, int N, int K, int ksplit, long slab, const float* bias, float alpha, int act, int beta,
                        int out_bf16, void* stream) {
  using namespace pv::gemm;
  if (M <= 0 || N <= 0 || K <= 0 || K % BK) return -1;
  if (ksplit < 1) ksplit = 1;
  if (ksplit > 1 && (out_bf16 || beta || bias || act)) return -2;  // split-K: the caller's reduce does the epilogue
  if (((size_t)A & 15) || ((size_t)B & 15)) return -3;           // 16-byte source vectors
  if (lda % 8 || ldb % 8) return -4;                            // rows start 16-byte aligned
  if ((a_col && M % 8) || (b_col && N % 8)) return -5;           // whole 8-column groups of COL operands
  Params p{(const unsigned short*)A, (const unsigned short*)B, lda, ldb, C, ldc, M, N, K, ksplit, slab,
           bias, alpha, act, beta, out_bf16, (M + BM - 1) / BM, (N + BN - 1) / BN, N <= M ? 1 : 0,
           g_gemm_group};
  const int grid = p.tiles_m * p.tiles_n * ksplit;
  hipStream_t st = (hipStream_t)stream;
#define PV_GEMM_LAUNCH(KER)                                                                        \
  do {                                                                                            \
    if (!a_col && !b_col) hipLaunchKernelGGL((KER<ROW, ROW>), dim3(grid), dim3(NTH), 0, st, p);    \
    else if (!a_col && b_col) hipLaunchKernelGGL((KER<ROW, COL>), dim3(grid), dim3(NTH), 0, st, p); \
    else if (a_col && !b_col) hipLaunchKernelGGL((KER<COL, ROW>), dim3(grid), dim3(NTH), 0, st, p); \
    else hipLaunchKernelGGL((KER<COL, COL>), dim3(grid), dim3(NTH), 0, st, p);                     \
  } while (0)
  PV_GEMM_LAUNCH(gemm2_kernel);
#undef PV_GEMM_LAUNCH
  PV_LAUNCH_CHECK();
  return 0;
}
