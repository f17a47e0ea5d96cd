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
#include <type_traits>

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
};

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

template <int ALAY, int BLAY>
__global__ __launch_bounds__(NTH, 2) void gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // [buf][A, B]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  // tile id: XCD-aware (tiles of one K slice and neighbouring tiles share an XCD's L2)
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int ntile = p.tiles_m * p.tiles_n;
  const int split = bid / ntile, t = bid - split * ntile;
  // consecutive tile ids (one XCD under the remap) share the panel of the LARGER operand,
  // so it is read from HBM once and re-served from that XCD's L2 (tall-skinny GEMMs: the
  // whole small operand stays L2-resident anyway)
  const int tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  const int tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * per, kt1 = min(ktiles, kt0 + per);

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
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const char* ta = smem + buf * 2 * TILE_BYTES;
      const char* tb = ta + TILE_BYTES;
      if (kt + 1 < kt1) {  // prefetch the next K tile into the other buffer (overlaps the MFMAs)
        char* na = smem + (buf ^ 1) * 2 * TILE_BYTES;
        stage<ALAY>(p.A, p.lda, m0, p.M - 1, (kt + 1) * BK, na);
        stage<BLAY>(p.B, p.ldb, n0, p.N - 1, (kt + 1) * BK, na + TILE_BYTES);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag<BLAY>(tb, wc * 64 + 16 * j, s);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bf16x8 afr = frag<ALAY>(ta, wr * 128 + 16 * i, s);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      buf ^= 1;
    }
  }

  epilogue(p, acc, split, m0, n0, wr, wc, lane);
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
  const int tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  const int tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
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


// v3 accumulator map: acc[i][j][r] = C[m0 + 128 (i >> 2) + 64 wr + 16 (i & 3) + 4 (lane >> 4) + r]
//                                       [n0 + 128 (j >> 1) + 32 wc + 16 (j & 1) + (lane & 15)]
__device__ __forceinline__ void epilogue3(const Params& p, f32x4 (&acc)[8][4], int split, int m0, int n0, int wr,
                                          int wc, int lane) {
  const bool part = p.ksplit > 1;
  float* Cs = reinterpret_cast<float*>(p.C) + (part ? (size_t)split * p.slab : 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + 128 * (j >> 1) + 32 * wc + 16 * (j & 1) + (lane & 15);
    if (col >= p.N) continue;
    const float bj = (!part && p.bias) ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + 128 * (i >> 2) + 64 * wr + 16 * (i & 3) + 4 * (lane >> 4) + r;
        if (row >= p.M) continue;
        const size_t o = (size_t)row * p.ldc + col;
        if (part) {
          Cs[o] = acc[i][j][r] * p.alpha;
          continue;
        }
        float v = act_f(acc[i][j][r] * p.alpha + bj, p.act);
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

// ---- v3 schedule: 8 waves in two staggered groups, 4 phases per K tile ------------------
// (cdna_hip_programming.md §5 "The 256² 8-phase template" / MI355X_MICROARCH "two waves per
// SIMD": waves w and w + 4 share a SIMD; group 1 (waves 4-7) runs one barrier behind group 0,
// so on every SIMD one wave's MFMA segment coincides with its partner's load segment.)
// Each operand tile is staged as two 128-row HALVES; a wave owns rows {64 wr + [0, 64)} of
// BOTH A halves and columns {32 wc + [0, 32)} of BOTH B halves, so its 128 x 64 output is 4
// quadrants and the K tile's phases run (A0, B0) (A0, B1) (A1, B0) (A1, B1), B fragments
// of both halves kept in registers: the LDS of a tile is read only in phases 0 (A0, B0),
// 1 (B1) and 2 (A1).  Its buffer is therefore free from phase 3 on, and the halves of tile
// T are staged 4-5 phases before their first read: A0 in phase 3 of tile T - 2, B0 / B1 / A1
// in phases 0 / 1 / 2 of tile T - 1 (2 glds per thread each).  WAR: every half is re-staged
// >= 2 phases after its last read (reads retire by lgkmcnt(0) at the start of the MFMA
// segment).  RAW: each load segment ends with vmcnt(6) (the 3 newest phases' glds may fly),
// and the next load segment (2 barriers later) reads only halves staged >= 4 phases ago.
// Raw s_barrier only: __syncthreads() would drain the in-flight glds (vmcnt(0)).
// Segment = ds_reads + glds + vmcnt | barrier | lgkmcnt(0) setprio(1) 16 MFMAs setprio(0) | barrier.
constexpr int HALF_BYTES = 128 * 64 * 2;  // 16 KB: 128 rows x 64 k bf16

// Half tile = 128 operand rows x 64 k.  ROW: [128][64] (128-B rows, chunk c of row r at
// c ^ (r & 7)); COL: [64 k][128] (256-B k-rows, chunk c of k-row r at c ^ 2h(r): the 4 k-rows
// x 32 bytes of a 16-lane transposed read land on 4 disjoint bank groups, and the two
// 16-lane groups of a 32-lane half on different ones through bit 3 of r).
template <int LAY>
__device__ __forceinline__ void stage_half(const unsigned short* __restrict__ X, long ld, int r0, int rmax, int k0,
                                           char* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int piece = wave * 2 + u;                  // 0..15, 1 KB each
    if constexpr (LAY == ROW) {
      const int r = piece * 8 + (lane >> 3);         // half row 0..127
      const int c = (lane & 7) ^ (r & 7);
      const int gr = min(r0 + r, rmax);
      glds16(X + (size_t)gr * ld + k0 + c * 8, dst + piece * 1024);
    } else {
      const int kr = piece * 4 + (lane >> 4);        // k-row 0..63
      const int c = (lane & 15) ^ (2 * h_of(kr));    // logical chunk (8 operand rows)
      int col = r0 + c * 8;
      col = col <= rmax ? col : 0;                   // groups past the edge: never stored
      glds16(X + (size_t)(k0 + kr) * ld + col, dst + piece * 1024);
    }
  }
}

// fragment of operand rows [rb, rb + 16) (half-local), k-step s from a staged half tile
template <int LAY>
__device__ __forceinline__ bf16x8 frag_h(const char* t, int rb, int s) {
  if constexpr (LAY == ROW) {
    return frag<ROW>(t, rb, s);
  } else {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int klo = 32 * s + 8 * g + q, khi = klo + 4;
    const int col = rb + 4 * p;
    const int c = col >> 3, half = (col & 7) * 2;
    const char* plo = t + klo * 256 + ((c ^ (2 * h_of(klo))) * 16) + half;
    const char* phi = t + khi * 256 + ((c ^ (2 * h_of(khi))) * 16) + half;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)plo);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)phi);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <int ALAY, int BLAY>
__global__ __launch_bounds__(NTH, 1) void gemm3_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * HALF_BYTES];  // [buf][A0 B0 B1 A1]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int grp = wave >> 2, wr = wave >> 2, wc = wave & 3;
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int ntile = p.tiles_m * p.tiles_n;
  const int split = bid / ntile, t = bid - split * ntile;
  const int tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  const int tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * per, kt1 = min(ktiles, kt0 + per);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    // half q (0 A0, 1 B0, 2 B1, 3 A1) of tile kt into its buffer ((kt - kt0) & 1); past the
    // split's end a clamped reload (same timing as a real one, so WAR-safe; never read)
    auto stage_q = [&](int q, int kt) {
      char* dst = smem + ((kt - kt0) & 1) * 4 * HALF_BYTES + q * HALF_BYTES;
      const int kk = min(kt, kt1 - 1) * BK;
      if (q == 0) stage_half<ALAY>(p.A, p.lda, m0, p.M - 1, kk, dst);
      else if (q == 3) stage_half<ALAY>(p.A, p.lda, m0 + 128, p.M - 1, kk, dst);
      else stage_half<BLAY>(p.B, p.ldb, n0 + 128 * (q - 1), p.N - 1, kk, dst);
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) stage_q(q, kt0);
    stage_q(0, kt0 + 1);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // tile kt0 landed; kt0 + 1's A0 may fly
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 one barrier behind
    bf16x8 a[4][2], b0[2][2], b1[2][2];
    const int arow = wr * 64, bcol = wc * 32;
#pragma unroll 1
    for (int kt = kt0; kt < kt1; ++kt) {
      const char* cur = smem + ((kt - kt0) & 1) * 4 * HALF_BYTES;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        const int ah = ph >> 1;  // A half (0: phases 0, 1; 1: phases 2, 3)
        // ---- load segment
        if (ph == 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) b0[j][s2] = frag<BLAY>(cur + 1 * HALF_BYTES, bcol + 16 * j, s2);
        }
        if (ph == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) b1[j][s2] = frag<BLAY>(cur + 2 * HALF_BYTES, bcol + 16 * j, s2);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ph == 0 || ph == 2) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
              a[i][s2] = frag<ALAY>(cur + (ah ? 3 : 0) * HALF_BYTES, arow + 16 * i, s2);
        }
        if (ph < 3) stage_q(ph + 1, kt + 1);
        else stage_q(0, kt + 2);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA segment: quadrant (ah, bh = ph & 1), K = 64
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const bf16x8 bb = (ph & 1) ? b1[j][s2] : b0[j][s2];
              acc[4 * ah + i][2 * (ph & 1) + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], bb, acc[4 * ah + i][2 * (ph & 1) + j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  epilogue3(p, acc, split, m0, n0, wr, wc, lane);
}

// ---- v4: the 8-phase schedule, two K tiles per iteration ---------------------------------
// (cdna_hip_programming.md §5 "The 256² 8-phase template".)  Same wave / quadrant / half-tile
// decomposition as v3 (a wave owns rows {64 wr + [0, 64)} of both A halves and columns
// {32 wc + [0, 32)} of both B halves; epilogue3's accumulator map), but the K loop covers two
// K tiles per iteration — tile T in buffer E (phases 1-4), tile T + 1 in buffer O (phases
// 5-8) — so every LDS address is a compile-time offset, and the loads wait only twice per
// iteration (vmcnt(6) in phases 4 and 8: three half-tiles stay in flight, each load gets 4-6
// phases of latency instead of v3's per-phase 3).  Per phase: fragment reads, one half-tile
// staged (2 glds per thread), barrier, lgkmcnt(0), 16 MFMAs at priority 1, barrier; waves 4-7
// run one barrier behind waves 0-3 (on every SIMD an MFMA segment meets a load segment).
//
//   phase  reads            MFMAs (A, B)  stages (half -> buffer, tile)      waits
//   1      B0_E, A0_E       A0 B0         A1 -> O, T+1                      lgkmcnt(8) (B0_E reads)
//   2      B1_E             A0 B1         B0 -> E, T+2
//   3      A1_E             A1 B0         A0 -> E, T+2
//   4      -                A1 B1         B1 -> E, T+2                      vmcnt(6): O complete
//   5      B0_O, A0_O       A0 B0         A1 -> E, T+2                      lgkmcnt(8)
//   6      B1_O             A0 B1         B0 -> O, T+3
//   7      A1_O             A1 B0         A0 -> O, T+3
//   8      -                A1 B1         B1 -> O, T+3                      vmcnt(6): E complete
// WAR: every half is restaged >= 2 phases after its last read, or 1 phase after when the
// reading phase retired those reads (the B reads are issued first and lgkmcnt(8) retires
// them before that phase's first barrier).  RAW: a buffer is read one phase after the wait
// that retires it (the staggered group passes that wait's barrier before its reads).
// Prologue: E = tile kt0 and B0 / A0 / B1 of kt0 + 1 issued, vmcnt(6) -> the steady state
// at phase 1.  Past the split's end a stage reloads the last tile (uniform counts, never
// read); an odd tile count skips the MFMAs of the missing tile T + 1 (uniform branch).
template <int ALAY, int BLAY>
__global__ __launch_bounds__(NTH, 1) void gemm4_kernel(Params p) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 4 * HALF_BYTES];  // [E, O][A0 B0 B1 A1]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int grp = wave >> 2, wr = wave >> 2, wc = wave & 3;
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int ntile = p.tiles_m * p.tiles_n;
  const int split = bid / ntile, t = bid - split * ntile;
  const int tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  const int tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * per, kt1 = min(ktiles, kt0 + per);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    // half q (0 A0, 1 B0, 2 B1, 3 A1) of tile kt into buffer b (0 E, 1 O)
    auto stg = [&](int b, int q, int kt) {
      char* dst = smem + b * 4 * HALF_BYTES + q * HALF_BYTES;
      const int kk = min(kt, kt1 - 1) * BK;
      if (q == 0) stage_half<ALAY>(p.A, p.lda, m0, p.M - 1, kk, dst);
      else if (q == 3) stage_half<ALAY>(p.A, p.lda, m0 + 128, p.M - 1, kk, dst);
      else stage_half<BLAY>(p.B, p.ldb, n0 + 128 * (q - 1), p.N - 1, kk, dst);
    };
    bf16x8 a[4][2], b0[2][2], b1[2][2];
    const int arow = wr * 64, bcol = wc * 32;
    auto rd_b = [&](const char* half, bf16x8 (&b)[2][2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) b[j][s2] = frag_h<BLAY>(half, bcol + 16 * j, s2);
    };
    auto rd_a = [&](const char* half) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = frag_h<ALAY>(half, arow + 16 * i, s2);
    };
    // the B reads (issued first) retired, the A reads (8 ds_read_b128 or 16 transposed
    // reads) may stay in flight
    auto wait_b = [&]() {
      if constexpr (ALAY == ROW) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
    };
    // barrier, reads retired, 16 MFMAs of quadrant (AH, BH), barrier
    auto mma = [&](auto ah_c, auto bh_c, bf16x8 (&b)[2][2], bool live) {
      constexpr int AH = decltype(ah_c)::value, BH = decltype(bh_c)::value;
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (live) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[4 * AH + i][2 * BH + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s2], b[j][s2], acc[4 * AH + i][2 * BH + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    const char* E = smem;
    const char* O = smem + 4 * HALF_BYTES;
    // prologue
#pragma unroll
    for (int q = 0; q < 4; ++q) stg(0, q, kt0);
    stg(1, 1, kt0 + 1);
    stg(1, 0, kt0 + 1);
    stg(1, 2, kt0 + 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: group 1 one barrier behind
#pragma unroll 1
    for (int kt = kt0; kt < kt1; kt += 2) {
      const bool two = kt + 1 < kt1;
      // phase 1
      rd_b(E + 1 * HALF_BYTES, b0);
      __builtin_amdgcn_sched_barrier(0);
      rd_a(E + 0 * HALF_BYTES);
      stg(1, 3, kt + 1);
      wait_b();
      mma(I0{}, I0{}, b0, true);
      // phase 2
      rd_b(E + 2 * HALF_BYTES, b1);
      stg(0, 1, kt + 2);
      mma(I0{}, I1{}, b1, true);
      // phase 3
      rd_a(E + 3 * HALF_BYTES);
      stg(0, 0, kt + 2);
      mma(I1{}, I0{}, b0, true);
      // phase 4
      stg(0, 2, kt + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      mma(I1{}, I1{}, b1, true);
      // phase 5
      rd_b(O + 1 * HALF_BYTES, b0);
      __builtin_amdgcn_sched_barrier(0);
      rd_a(O + 0 * HALF_BYTES);
      stg(0, 3, kt + 2);
      wait_b();
      mma(I0{}, I0{}, b0, two);
      // phase 6
      rd_b(O + 2 * HALF_BYTES, b1);
      stg(1, 1, kt + 3);
      mma(I0{}, I1{}, b1, two);
      // phase 7
      rd_a(O + 3 * HALF_BYTES);
      stg(1, 0, kt + 3);
      mma(I1{}, I0{}, b0, two);
      // phase 8
      stg(1, 2, kt + 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      mma(I1{}, I1{}, b1, two);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  epilogue3(p, acc, split, m0, n0, wr, wc, lane);
}

PV_DEBUG_EXPORT(gemm)
}  // namespace gemm
}  // namespace pv

using namespace pv;

// schedule: 2 = fragment reads pipelined one sub-step ahead (gemm2_kernel, default);
// 1 = the plain double-buffered loop (gemm_kernel) — A/B arm for tools/gemm_engine_micro.py
static int g_gemm_sched = getenv("PAGEVEC_GEMM_SCHED") ? atoi(getenv("PAGEVEC_GEMM_SCHED")) : 2;
PV_API void pv_gemm_set_sched(int s) { g_gemm_sched = s; }

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
           bias, alpha, act, beta, out_bf16, (M + BM - 1) / BM, (N + BN - 1) / BN, N <= M ? 1 : 0};
  const int grid = p.tiles_m * p.tiles_n * ksplit;
  hipStream_t st = (hipStream_t)stream;
#define PV_GEMM_LAUNCH(KER)                                                                        \
  do {                                                                                            \
    if (!a_col && !b_col) hipLaunchKernelGGL((KER<ROW, ROW>), dim3(grid), dim3(NTH), 0, st, p);    \
    else if (!a_col && b_col) hipLaunchKernelGGL((KER<ROW, COL>), dim3(grid), dim3(NTH), 0, st, p); \
    else if (a_col && !b_col) hipLaunchKernelGGL((KER<COL, ROW>), dim3(grid), dim3(NTH), 0, st, p); \
    else hipLaunchKernelGGL((KER<COL, COL>), dim3(grid), dim3(NTH), 0, st, p);                     \
  } while (0)
  if (g_gemm_sched == 4) PV_GEMM_LAUNCH(gemm4_kernel);
  else if (g_gemm_sched == 3 && !a_col && !b_col)
    hipLaunchKernelGGL((gemm3_kernel<ROW, ROW>), dim3(grid), dim3(NTH), 0, st, p);
  else if (g_gemm_sched == 1) PV_GEMM_LAUNCH(gemm_kernel);
  else PV_GEMM_LAUNCH(gemm2_kernel);
#undef PV_GEMM_LAUNCH
  PV_LAUNCH_CHECK();
  return 0;
}
