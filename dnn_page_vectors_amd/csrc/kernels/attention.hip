// Fused multi-head attention for the BERT dual encoder (BASELINE config 4), head dim 64,
// key-padding mask, straight from / into the PACKED projection layouts:
//   qkv  (N, L, 3, H, 64) bf16   (the QKV GEMM output, no permute/contiguous copies)
//   out  (N, L, H, 64)    bf16   (= (N, L, H*64), the input of the output projection)
//   dqkv (N, L, 3, H, 64) bf16   (the backward writes dQ, dK, dV into their slots — no cat)
//
// Every product uses the swapped orientation of loss.hip: scores are computed TRANSPOSED
// (A = the 16 key rows staged in LDS, B = the 16 query rows held in registers), so one
// lane owns one query column and 4 keys of each 16-key subtile.  The softmax statistics
// are then lane-local (+ two xor shuffles across the 4 lane groups), and the bf16 P^T
// registers are directly the B operand of O^T += V^T . P^T, whose A operand (V^T) comes
// from the row-major V tile through ds_read_b64_tr_b16 (k order j -> 16*(j>>2)+4g+(j&3)).
//
//   attn_fwd      : online softmax over 64-key blocks (exp2 domain), O and the per-row
//                   log-sum-exp (for the backward)
//   attn_bwd_prep : D = rowsum(dO * O)
//   attn_bwd_dkdv : one workgroup per 64-key block, loops over query blocks; dV = P^T dO,
//                   dK = dS^T Q with P recomputed from the saved log-sum-exp
//   attn_bwd_dq   : one workgroup per 64-query block, loops over key blocks; dQ = dS K
// No atomics: every output element is owned by exactly one workgroup.
#include "common.h"

namespace pv {
namespace attn {

constexpr int HD = 64;         // head dim
constexpr int TB = 64;         // rows per staged tile (keys or queries)
constexpr int LDT = HD + 8;    // LDS row stride (elements): 144 B, 16-B aligned
constexpr float LOG2E = 1.4426950408889634f;

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// Stage rows [r0, r0+64) of one head slot (slot 0/1/2 of qkv, or the dO / O layout with
// stride ld) into an LDS tile [64][LDT]; rows >= L are zero.  256 threads x 2 x 16 B.
__device__ __forceinline__ void load_tile(const unsigned short* __restrict__ base, size_t ld, int r0, int L,
                                          u32x4 (&v)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = threadIdx.x + 256 * u;
    const int r = q >> 3, c = (q & 7) * 8;
    v[u] = (r0 + r < L) ? *reinterpret_cast<const u32x4*>(base + (size_t)(r0 + r) * ld + c) : u32x4{0, 0, 0, 0};
  }
}

__device__ __forceinline__ void store_tile(unsigned short* t, const u32x4 (&v)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = threadIdx.x + 256 * u;
    *reinterpret_cast<u32x4*>(t + (q >> 3) * LDT + (q & 7) * 8) = v[u];
  }
}

// fragment of 16 rows (r0 + lane&15) x 8 columns (8g + 32s) from a row-major tile
__device__ __forceinline__ bf16x8 row_frag(const unsigned short* t, int r0, int s) {
  const int lane = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(t + (r0 + (lane & 15)) * LDT + s * 32 + (lane >> 4) * 8);
}

// transposed fragment: A[col = c0 + lane&15][k = rows permuted] from a row-major tile [row][col]:
// rows 32*s2 + 4g + q (q = 0..3) and +16, columns c0 .. c0+15
__device__ __forceinline__ bf16x8 tr_frag(const unsigned short* t, int s2, int c0) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const unsigned short* p = t + (s2 * 32 + 4 * g + ((lane & 15) >> 2)) * LDT + c0 + 4 * (lane & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + 16 * LDT));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// 16 rows (row0 + lane&15) x 64 d of a global row-major matrix as two B/A fragments (d-steps)
__device__ __forceinline__ void glob_frag(const unsigned short* __restrict__ base, size_t ld, int row, int L,
                                          bf16x8 (&f)[2]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < 2; ++s)
    f[s] = row < L ? *reinterpret_cast<const bf16x8*>(base + (size_t)row * ld + s * 32 + (lane >> 4) * 8)
                   : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
}

// 4 C-layout accumulators (16 rows each, rows 4g+r) -> bf16 B fragments of 2 k-steps of 32
__device__ __forceinline__ void pack_b(const f32x4 (&x)[4], bf16x8 (&b)[2]) {
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    u32x4 w;
    w[0] = pack_bf16x2(x[2 * s2][0], x[2 * s2][1]);
    w[1] = pack_bf16x2(x[2 * s2][2], x[2 * s2][3]);
    w[2] = pack_bf16x2(x[2 * s2 + 1][0], x[2 * s2 + 1][1]);
    w[3] = pack_bf16x2(x[2 * s2 + 1][2], x[2 * s2 + 1][3]);
    b[s2] = __builtin_bit_cast(bf16x8, w);
  }
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// Column sums of a wave's QG x 4 output accumulators (rows d = 16 i + 4 g + r, columns = the
// wave's 16 QG tokens) over its tokens: the sum of rows 16 i + 4 g + r lands in lane 15 of
// lane group g (an inclusive row_shr 1 / 2 / 4 / 8 DPP scan inside each 16-lane row: four
// VALU adds per value, no LDS traffic).
template <int CTRL>
__device__ __forceinline__ float row_shr_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int QG>
__device__ __forceinline__ void token_colsum(const f32x4 (&a)[QG][4], float (&out)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < QG; ++j) v += a[j][i][r];
      v = row_shr_add<0x111>(v);
      v = row_shr_add<0x112>(v);
      v = row_shr_add<0x114>(v);
      v = row_shr_add<0x118>(v);
      out[i][r] = v;
    }
}



// ---------------------------------------------------------------------------- forward
// QG = 16-query groups per wave: every staged K / V fragment feeds QG MFMAs (LDS reads and
// tile stores per FLOP / QG).  grid (ceil(L / (64 QG)), H, N), 256 threads; wave w owns
// queries q0 + 16 (w QG + j) .. +15, j < QG.
template <int QG>
__global__ __launch_bounds__(256, QG >= 4 ? 1 : 2) void attn_fwd_kernel(const unsigned short* __restrict__ qkv,
                                                                        const int* __restrict__ mask,
                                                                        unsigned short* __restrict__ out,
                                                                        float* __restrict__ lse, int L, int H,
                                                                        float scale) {
  __shared__ __attribute__((aligned(16))) unsigned short kt[2][TB * LDT];
  __shared__ __attribute__((aligned(16))) unsigned short vt[2][TB * LDT];
  __shared__ float mk[2][TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int n = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * TB * QG + wave * 16 * QG;
  const size_t ld = (size_t)3 * H * HD;
  const unsigned short* Q = qkv + (size_t)n * L * ld + (size_t)h * HD;
  const unsigned short* K = Q + (size_t)H * HD;
  const unsigned short* V = Q + (size_t)2 * H * HD;
  const int* mrow = mask ? mask + (size_t)n * L : nullptr;
  const float sl = scale * LOG2E;
  bf16x8 qb[QG][2];
  f32x4 o[QG][4];
  float m[QG], l[QG];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    glob_frag(Q, ld, q0 + 16 * j + (lane & 15), L, qb[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  u32x4 sk[2], sv[2];
  float smk = 0.f;
  load_tile(K, ld, 0, L, sk);
  load_tile(V, ld, 0, L, sv);
  if (threadIdx.x < TB) smk = (threadIdx.x < L && (!mrow || mrow[threadIdx.x])) ? 1.f : 0.f;
  store_tile(kt[0], sk);
  store_tile(vt[0], sv);
  if (threadIdx.x < TB) mk[0][threadIdx.x] = smk;
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < L; k0 += TB, buf ^= 1) {
    const bool more = k0 + TB < L;
    if (more) {
      load_tile(K, ld, k0 + TB, L, sk);
      load_tile(V, ld, k0 + TB, L, sv);
      if (threadIdx.x < TB) {
        const int kk = k0 + TB + threadIdx.x;
        smk = (kk < L && (!mrow || mrow[kk])) ? 1.f : 0.f;
      }
    }
    // S^T (keys x queries), 4 key subtiles per query group; one K fragment read per QG MFMAs
    f32x4 s[QG][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int j = 0; j < QG; ++j) s[j][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 a = row_frag(kt[buf], c * 16, st);
#pragma unroll
        for (int j = 0; j < QG; ++j) s[j][c] = MFMA(a, qb[j][st], s[j][c]);
      }
    }
    bf16x8 pb[QG][2];
#pragma unroll
    for (int j = 0; j < QG; ++j) {
      float bm = -INFINITY;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float keep = mk[buf][c * 16 + 4 * g + r];
          s[j][c][r] = keep != 0.f ? s[j][c][r] * sl : -INFINITY;
          bm = fmaxf(bm, s[j][c][r]);
        }
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m[j], bm);
      const float corr = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m[j] - mn);
      m[j] = mn;
      l[j] *= corr;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[j][i] *= corr;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = s[j][c][r] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[j][c][r] - mn);
          s[j][c][r] = pv;
          l[j] += pv;
        }
      pack_b(s[j], pb[j]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = tr_frag(vt[buf], s2, i * 16);
#pragma unroll
        for (int j = 0; j < QG; ++j) o[j][i] = MFMA(a, pb[j][s2], o[j][i]);
      }
    if (more) {
      store_tile(kt[buf ^ 1], sk);
      store_tile(vt[buf ^ 1], sv);
      if (threadIdx.x < TB) mk[buf ^ 1][threadIdx.x] = smk;
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    float lj = l[j];
    lj += __shfl_xor(lj, 16, 64);
    lj += __shfl_xor(lj, 32, 64);
    const int q = q0 + 16 * j + (lane & 15);
    if (q < L) {
      const float inv = lj > 0.f ? 1.f / lj : 0.f;
      unsigned short* orow = out + ((size_t)n * L + q) * H * HD + (size_t)h * HD;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint2*>(orow + i * 16 + 4 * g) =
            uint2{pack_bf16x2(o[j][i][0] * inv, o[j][i][1] * inv), pack_bf16x2(o[j][i][2] * inv, o[j][i][3] * inv)};
      if (g == 0) lse[((size_t)n * H + h) * L + q] = m[j] + __log2f(lj);  // log2 domain, includes scale
    }
  }
}

// DMA variant of the forward (pv_attn_set_fwd_dma): K / V tiles land in LDS by
// global_load_lds_dwordx4 instead of global loads into staging VGPRs + ds_write_b128.  The
// [64][LDT] tile image is 576 consecutive 16-byte chunks (LDT = 72 elements = 9 chunks), so
// piece p (one wave-instruction, 1 KB) writes chunks 64p .. 64p + 63: chunk q -> row q / 9,
// column chunk q % 9 (the pad chunk 8 re-reads chunk 0); rows >= L re-read row L - 1 (finite
// data, masked by mk).  Tile k + 1's pieces are issued before tile k's math and waited for
// (own vmcnt) + one barrier after it.
__device__ __forceinline__ void attn_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void dma_tile(const unsigned short* __restrict__ base, size_t ld, int r0, int L,
                                         unsigned short* t) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int pc = wave + 4 * u;  // pieces 0..8
    if (pc < 9) {
      const int q = pc * 64 + lane;
      const int r = q / 9, c = q - 9 * (q / 9);
      const int row = min(r0 + r, L - 1);
      attn_glds16(base + (size_t)row * ld + (c < 8 ? c : 0) * 8, reinterpret_cast<char*>(t) + pc * 1024);
    }
  }
}

template <int QG>
__global__ __launch_bounds__(256, QG >= 4 ? 1 : 2) void attn_fwd_dma_kernel(const unsigned short* __restrict__ qkv,
                                                                            const int* __restrict__ mask,
                                                                            unsigned short* __restrict__ out,
                                                                            float* __restrict__ lse, int L, int H,
                                                                            float scale) {
  __shared__ __attribute__((aligned(1024))) unsigned short kt[2][TB * LDT];
  __shared__ __attribute__((aligned(1024))) unsigned short vt[2][TB * LDT];
  __shared__ float mk[2][TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int n = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * TB * QG + wave * 16 * QG;
  const size_t ld = (size_t)3 * H * HD;
  const unsigned short* Q = qkv + (size_t)n * L * ld + (size_t)h * HD;
  const unsigned short* K = Q + (size_t)H * HD;
  const unsigned short* V = Q + (size_t)2 * H * HD;
  const int* mrow = mask ? mask + (size_t)n * L : nullptr;
  const float sl = scale * LOG2E;
  bf16x8 qb[QG][2];
  f32x4 o[QG][4];
  float m[QG], l[QG];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    glob_frag(Q, ld, q0 + 16 * j + (lane & 15), L, qb[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    l[j] = 0.f;
  }
  dma_tile(K, ld, 0, L, kt[0]);
  dma_tile(V, ld, 0, L, vt[0]);
  float smk = 0.f;
  if (threadIdx.x < TB) mk[0][threadIdx.x] = (threadIdx.x < L && (!mrow || mrow[threadIdx.x])) ? 1.f : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < L; k0 += TB, buf ^= 1) {
    const bool more = k0 + TB < L;
    if (more) {  // the other buffer was released by the previous iteration's barrier
      dma_tile(K, ld, k0 + TB, L, kt[buf ^ 1]);
      dma_tile(V, ld, k0 + TB, L, vt[buf ^ 1]);
      if (threadIdx.x < TB) {
        const int kk = k0 + TB + threadIdx.x;
        smk = (kk < L && (!mrow || mrow[kk])) ? 1.f : 0.f;
      }
    }
    f32x4 s[QG][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int j = 0; j < QG; ++j) s[j][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 a = row_frag(kt[buf], c * 16, st);
#pragma unroll
        for (int j = 0; j < QG; ++j) s[j][c] = MFMA(a, qb[j][st], s[j][c]);
      }
    }
    bf16x8 pb[QG][2];
#pragma unroll
    for (int j = 0; j < QG; ++j) {
      float bm = -INFINITY;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float keep = mk[buf][c * 16 + 4 * g + r];
          s[j][c][r] = keep != 0.f ? s[j][c][r] * sl : -INFINITY;
          bm = fmaxf(bm, s[j][c][r]);
        }
      bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m[j], bm);
      const float corr = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m[j] - mn);
      m[j] = mn;
      l[j] *= corr;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[j][i] *= corr;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = s[j][c][r] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(s[j][c][r] - mn);
          s[j][c][r] = pv;
          l[j] += pv;
        }
      pack_b(s[j], pb[j]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = tr_frag(vt[buf], s2, i * 16);
#pragma unroll
        for (int j = 0; j < QG; ++j) o[j][i] = MFMA(a, pb[j][s2], o[j][i]);
      }
    if (more && threadIdx.x < TB) mk[buf ^ 1][threadIdx.x] = smk;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of the next tile
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    float lj = l[j];
    lj += __shfl_xor(lj, 16, 64);
    lj += __shfl_xor(lj, 32, 64);
    const int q = q0 + 16 * j + (lane & 15);
    if (q < L) {
      const float inv = lj > 0.f ? 1.f / lj : 0.f;
      unsigned short* orow = out + ((size_t)n * L + q) * H * HD + (size_t)h * HD;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint2*>(orow + i * 16 + 4 * g) =
            uint2{pack_bf16x2(o[j][i][0] * inv, o[j][i][1] * inv), pack_bf16x2(o[j][i][2] * inv, o[j][i][3] * inv)};
      if (g == 0) lse[((size_t)n * H + h) * L + q] = m[j] + __log2f(lj);
    }
  }
}

// ---------------------------------------------------------------------------- backward
// D[n,h,q] = sum_d dO * O ; one wave per (n, q), lanes over heads x 16 pieces
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const unsigned short* __restrict__ dout,
                                                            const unsigned short* __restrict__ out,
                                                            float* __restrict__ Dv, int NL, int L, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // n*L + q
  const int lane = threadIdx.x & 63;
  if (row >= NL) return;
  const int n = row / L, q = row - n * L;
  const unsigned short* a = dout + (size_t)row * H * HD;
  const unsigned short* b = out + (size_t)row * H * HD;
  for (int h = 0; h < H; ++h) {
    // lane covers one element pair of the head's 64 (32 lanes) -> use all 64 lanes on 2 heads
    float acc = 0.f;
    if (lane < 32) {
      const unsigned x = reinterpret_cast<const unsigned*>(a + h * HD)[lane];
      const unsigned y = reinterpret_cast<const unsigned*>(b + h * HD)[lane];
      acc = __uint_as_float(x << 16) * __uint_as_float(y << 16) +
            __uint_as_float(x & 0xFFFF0000u) * __uint_as_float(y & 0xFFFF0000u);
    }
    acc = wave_sum(acc);
    if (lane == 0) Dv[((size_t)n * H + h) * L + q] = acc;
  }
}

// Same D with all 64 lanes busy: a wave per row (n, q), lane l loads 4 consecutive columns
// of each 256-column chunk c (head 4c + l/16), the per-head sums are 16-lane xor reductions
// (4 shuffles per chunk) — for H = 12: 3 chunks, 12 shuffles per row instead of 12 full wave
// reductions with half the lanes idle.  Requires H % 4 == 0 (H * 64 a multiple of 256).
__global__ __launch_bounds__(256) void attn_bwd_prep4_kernel(const unsigned short* __restrict__ dout,
                                                             const unsigned short* __restrict__ out,
                                                             float* __restrict__ Dv, int NL, int L, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // n*L + q
  const int lane = threadIdx.x & 63;
  if (row >= NL) return;
  const int n = row / L, q = row - n * L;
  const unsigned short* a = dout + (size_t)row * H * HD;
  const unsigned short* b = out + (size_t)row * H * HD;
  for (int c = 0; c < H / 4; ++c) {
    const int col = c * 256 + lane * 4;
    const uint2 x = *reinterpret_cast<const uint2*>(a + col);
    const uint2 y = *reinterpret_cast<const uint2*>(b + col);
    float acc = __uint_as_float(x.x << 16) * __uint_as_float(y.x << 16) +
                __uint_as_float(x.x & 0xFFFF0000u) * __uint_as_float(y.x & 0xFFFF0000u) +
                __uint_as_float(x.y << 16) * __uint_as_float(y.y << 16) +
                __uint_as_float(x.y & 0xFFFF0000u) * __uint_as_float(y.y & 0xFFFF0000u);
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if ((lane & 15) == 15) Dv[((size_t)n * H + 4 * c + (lane >> 4)) * L + q] = acc;
  }
}

// grid (ceil(L / (64 QG)) key blocks, H, N); wave w owns keys kw + 16 j .. +15 (lane column),
// kw = block + 16 QG w, j < QG
template <int QG>
__global__ __launch_bounds__(256, QG >= 4 ? 1 : 2) void attn_bwd_dkdv_kernel(const unsigned short* __restrict__ qkv,
                                                               const int* __restrict__ mask,
                                                               const unsigned short* __restrict__ dout,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ Dv,
                                                               unsigned short* __restrict__ dqkv, int L, int H,
                                                               float scale, float* __restrict__ bpart, int nb64) {
  __shared__ __attribute__((aligned(16))) unsigned short qt[2][TB * LDT];
  __shared__ __attribute__((aligned(16))) unsigned short dt[2][TB * LDT];
  __shared__ float sl_[2][TB], sd_[2][TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int n = blockIdx.z, h = blockIdx.y, kw = blockIdx.x * TB * QG + wave * 16 * QG;
  const size_t ld = (size_t)3 * H * HD, ldo = (size_t)H * HD;
  const unsigned short* Q = qkv + (size_t)n * L * ld + (size_t)h * HD;
  const unsigned short* K = Q + (size_t)H * HD;
  const unsigned short* V = Q + (size_t)2 * H * HD;
  const unsigned short* dO = dout + (size_t)n * L * ldo + (size_t)h * HD;
  const float* LS = lse + ((size_t)n * H + h) * L;
  const float* DD = Dv + ((size_t)n * H + h) * L;
  const float sl = scale * LOG2E;
  bf16x8 kb[QG][2], vb[QG][2];
  bool kvalid[QG];
  f32x4 dk[QG][4], dv[QG][4];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    const int key = kw + 16 * j + (lane & 15);
    kvalid[j] = key < L && (!mask || mask[(size_t)n * L + key]);
    glob_frag(K, ld, key, L, kb[j]);
    glob_frag(V, ld, key, L, vb[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) dk[j][i] = dv[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  u32x4 sq[2], sdo[2];
  float slv = 0.f, sdv = 0.f;
  load_tile(Q, ld, 0, L, sq);
  load_tile(dO, ldo, 0, L, sdo);
  if (threadIdx.x < TB) {
    slv = threadIdx.x < L ? LS[threadIdx.x] : 0.f;
    sdv = threadIdx.x < L ? DD[threadIdx.x] : 0.f;
  }
  store_tile(qt[0], sq);
  store_tile(dt[0], sdo);
  if (threadIdx.x < TB) {
    sl_[0][threadIdx.x] = slv;
    sd_[0][threadIdx.x] = sdv;
  }
  __syncthreads();
  int buf = 0;
  for (int q0 = 0; q0 < L; q0 += TB, buf ^= 1) {
    const bool more = q0 + TB < L;
    if (more) {
      load_tile(Q, ld, q0 + TB, L, sq);
      load_tile(dO, ldo, q0 + TB, L, sdo);
      if (threadIdx.x < TB) {
        const int qq = q0 + TB + threadIdx.x;
        slv = qq < L ? LS[qq] : 0.f;
        sdv = qq < L ? DD[qq] : 0.f;
      }
    }
    // S (queries x keys) and dP = dO . V^T, 4 query subtiles: rows q = c*16 + 4g + r, col = key
    f32x4 p[QG][4], dp[QG][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int j = 0; j < QG; ++j) p[j][c] = dp[j][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 aq = row_frag(qt[buf], c * 16, st);
        const bf16x8 ad = row_frag(dt[buf], c * 16, st);
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          p[j][c] = MFMA(aq, kb[j][st], p[j][c]);
          dp[j][c] = MFMA(ad, vb[j][st], dp[j][c]);
        }
      }
    }
    bf16x8 pb[QG][2], db[QG][2];
#pragma unroll
    for (int j = 0; j < QG; ++j) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = c * 16 + 4 * g + r;
          const bool ok = kvalid[j] && q0 + qi < L;
          const float pv = ok ? __builtin_amdgcn_exp2f(p[j][c][r] * sl - sl_[buf][qi]) : 0.f;
          p[j][c][r] = pv;
          dp[j][c][r] = pv * (dp[j][c][r] - sd_[buf][qi]);  // dS (without the softmax scale)
        }
      pack_b(p[j], pb[j]);
      pack_b(dp[j], db[j]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 ad = tr_frag(dt[buf], s2, i * 16);
        const bf16x8 aq = tr_frag(qt[buf], s2, i * 16);
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          dv[j][i] = MFMA(ad, pb[j][s2], dv[j][i]);
          dk[j][i] = MFMA(aq, db[j][s2], dk[j][i]);
        }
      }
    if (more) {
      store_tile(qt[buf ^ 1], sq);
      store_tile(dt[buf ^ 1], sdo);
      if (threadIdx.x < TB) {
        sl_[buf ^ 1][threadIdx.x] = slv;
        sd_[buf ^ 1][threadIdx.x] = sdv;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    const int key = kw + 16 * j + (lane & 15);
    if (key < L) {
      unsigned short* row = dqkv + ((size_t)n * L + key) * ld + (size_t)h * HD;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *reinterpret_cast<uint2*>(row + (size_t)H * HD + i * 16 + 4 * g) =
            uint2{pack_bf16x2(dk[j][i][0] * scale, dk[j][i][1] * scale),
                  pack_bf16x2(dk[j][i][2] * scale, dk[j][i][3] * scale)};
        *reinterpret_cast<uint2*>(row + (size_t)2 * H * HD + i * 16 + 4 * g) =
            uint2{pack_bf16x2(dv[j][i][0], dv[j][i][1]), pack_bf16x2(dv[j][i][2], dv[j][i][3])};
      }
    }
  }
  if (bpart) {  // the qkv bias gradient's K / V parts: this workgroup's column sums over its keys
    float sk[4][4], sv[4][4];
    token_colsum<QG>(dk, sk);
    token_colsum<QG>(dv, sv);
    __shared__ float bred[4][2 * HD];
    if ((lane & 15) == 15)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bred[wave][i * 16 + 4 * g + r] = sk[i][r] * scale;
          bred[wave][HD + i * 16 + 4 * g + r] = sv[i][r];
        }
    __syncthreads();
    if (threadIdx.x < 2 * HD) {
      const int c = threadIdx.x;
      const float v = bred[0][c] + bred[1][c] + bred[2][c] + bred[3][c];
      const int slot = 1 + c / HD, d = c % HD;
      bpart[((size_t)n * nb64 + blockIdx.x) * (3 * H * HD) + (size_t)slot * H * HD + (size_t)h * HD + d] = v;
    }
  }
}

// grid (ceil(L / (64 QG)) query blocks, H, N); wave w owns queries qw + 16 j .. +15, j < QG
template <int QG>
__global__ __launch_bounds__(256, QG >= 4 ? 1 : 2) void attn_bwd_dq_kernel(const unsigned short* __restrict__ qkv,
                                                             const int* __restrict__ mask,
                                                             const unsigned short* __restrict__ dout,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ Dv,
                                                             unsigned short* __restrict__ dqkv, int L, int H,
                                                             float scale, float* __restrict__ bpart, int nb64) {
  __shared__ __attribute__((aligned(16))) unsigned short kt[2][TB * LDT];
  __shared__ __attribute__((aligned(16))) unsigned short vt[2][TB * LDT];
  __shared__ float mk[2][TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int n = blockIdx.z, h = blockIdx.y, qw = blockIdx.x * TB * QG + wave * 16 * QG;
  const size_t ld = (size_t)3 * H * HD, ldo = (size_t)H * HD;
  const unsigned short* Q = qkv + (size_t)n * L * ld + (size_t)h * HD;
  const unsigned short* K = Q + (size_t)H * HD;
  const unsigned short* V = Q + (size_t)2 * H * HD;
  const unsigned short* dO = dout + (size_t)n * L * ldo + (size_t)h * HD;
  const int* mrow = mask ? mask + (size_t)n * L : nullptr;
  const float sl = scale * LOG2E;
  float lq[QG], dq_[QG];
  bf16x8 qb[QG][2], ob[QG][2];
  f32x4 acc[QG][4];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    const int q = qw + 16 * j + (lane & 15);
    lq[j] = q < L ? lse[((size_t)n * H + h) * L + q] : 0.f;
    dq_[j] = q < L ? Dv[((size_t)n * H + h) * L + q] : 0.f;
    glob_frag(Q, ld, q, L, qb[j]);
    glob_frag(dO, ldo, q, L, ob[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  u32x4 sk[2], sv[2];
  float smk = 0.f;
  load_tile(K, ld, 0, L, sk);
  load_tile(V, ld, 0, L, sv);
  if (threadIdx.x < TB) smk = (threadIdx.x < L && (!mrow || mrow[threadIdx.x])) ? 1.f : 0.f;
  store_tile(kt[0], sk);
  store_tile(vt[0], sv);
  if (threadIdx.x < TB) mk[0][threadIdx.x] = smk;
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < L; k0 += TB, buf ^= 1) {
    const bool more = k0 + TB < L;
    if (more) {
      load_tile(K, ld, k0 + TB, L, sk);
      load_tile(V, ld, k0 + TB, L, sv);
      if (threadIdx.x < TB) {
        const int kk = k0 + TB + threadIdx.x;
        smk = (kk < L && (!mrow || mrow[kk])) ? 1.f : 0.f;
      }
    }
    f32x4 s[QG][4], dp[QG][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int j = 0; j < QG; ++j) s[j][c] = dp[j][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf16x8 ak = row_frag(kt[buf], c * 16, st);
        const bf16x8 av = row_frag(vt[buf], c * 16, st);
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          s[j][c] = MFMA(ak, qb[j][st], s[j][c]);
          dp[j][c] = MFMA(av, ob[j][st], dp[j][c]);
        }
      }
    }
    bf16x8 db[QG][2];
#pragma unroll
    for (int j = 0; j < QG; ++j) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float keep = mk[buf][c * 16 + 4 * g + r];
          const float pv = keep != 0.f ? __builtin_amdgcn_exp2f(s[j][c][r] * sl - lq[j]) : 0.f;
          s[j][c][r] = pv * (dp[j][c][r] - dq_[j]);  // dS^T
        }
      pack_b(s[j], db[j]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 a = tr_frag(kt[buf], s2, i * 16);
#pragma unroll
        for (int j = 0; j < QG; ++j) acc[j][i] = MFMA(a, db[j][s2], acc[j][i]);
      }
    if (more) {
      store_tile(kt[buf ^ 1], sk);
      store_tile(vt[buf ^ 1], sv);
      if (threadIdx.x < TB) mk[buf ^ 1][threadIdx.x] = smk;
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    const int q = qw + 16 * j + (lane & 15);
    if (q < L) {
      unsigned short* row = dqkv + ((size_t)n * L + q) * ld + (size_t)h * HD;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint2*>(row + i * 16 + 4 * g) =
            uint2{pack_bf16x2(acc[j][i][0] * scale, acc[j][i][1] * scale),
                  pack_bf16x2(acc[j][i][2] * scale, acc[j][i][3] * scale)};
    }
  }
  if (bpart) {  // the qkv bias gradient's Q part: column sums over this workgroup's queries
    float sq[4][4];
    token_colsum<QG>(acc, sq);
    __shared__ float bred[4][HD];
    if ((lane & 15) == 15)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) bred[wave][i * 16 + 4 * g + r] = sq[i][r] * scale;
    __syncthreads();
    if (threadIdx.x < HD) {
      const int d = threadIdx.x;
      bpart[((size_t)n * nb64 + blockIdx.x) * (3 * H * HD) + (size_t)h * HD + d] =
          bred[0][d] + bred[1][d] + bred[2][d] + bred[3][d];
    }
  }
}

#undef MFMA

}  // namespace attn
}  // namespace pv

using namespace pv;

namespace {
// 16-row groups per wave (template QG) of the forward / dQ and of the dK dV kernels;
// pv_attn_set_qg for the A/B (0 = the measured default: tools/attn_micro.py at the BERT
// shapes, profiles/r5_attn/: L 256 fwd 157-173 -> 124-128 us with QG 2, bwd 453 -> 435 us with
// QG 2 for dQ only (dK dV with 2: 473; QG 4: 1 wave per SIMD, slower everywhere); L 32 (the
// query segments) stays at QG 1 — a 128-row workgroup would be mostly empty)
int g_qg_fwd = 0, g_qg_dq = 0, g_qg_dkdv = 0;
int g_fwd_dma = 0;  // pv_attn_set_fwd_dma: K / V tiles by LDS-DMA in the forward (A/B)
int qg_or(int v, int def) { return (v == 1 || v == 2 || v == 4) ? v : def; }
}  // namespace

PV_API void pv_attn_set_fwd_dma(int on) { g_fwd_dma = on; }

PV_API void pv_attn_set_qg(int fwd, int dq, int dkdv) {
  g_qg_fwd = fwd;
  g_qg_dq = dq;
  g_qg_dkdv = dkdv;
}

// qkv (N, L, 3, H, 64) bf16; mask (N, L) int32 or null; out (N, L, H, 64) bf16; lse (N, H, L) f32
PV_API int pv_attn_fwd(const void* qkv, const int* mask, void* out, float* lse, int N, int L, int H, float scale,
                       void* stream) {
  using namespace pv::attn;
  if (N <= 0 || L <= 0 || H <= 0) return -1;
  const int qg = qg_or(g_qg_fwd, L >= 128 ? 2 : 1);
#define PV_AFWD(QGV)                                                                                            hipLaunchKernelGGL(attn_fwd_kernel<QGV>, dim3((L + TB * QGV - 1) / (TB * QGV), H, N), dim3(256), 0,                            (hipStream_t)stream, (const unsigned short*)qkv, mask, (unsigned short*)out, lse, L, H, scale)
  if (qg == 4) {
    PV_AFWD(4);
  } else if (qg == 2) {
    PV_AFWD(2);
  } else {
    PV_AFWD(1);
  }
#undef PV_AFWD
  PV_LAUNCH_CHECK();
  return 0;
}

// dout, out (N, L, H, 64) bf16; lse (N, H, L); D workspace (N, H, L) f32; dqkv (N, L, 3, H, 64) bf16.
// bpart (optional, zero-filled by the caller): (N * ceil(L / 64), 3 * H * 64) fp32 rows of per-
// workgroup column sums of dQ / dK / dV — their column sum is the qkv bias gradient
// (ops/transformer.py: no separate pass over dqkv).
PV_API int pv_attn_bwd2(const void* qkv, const int* mask, const void* out, const void* dout, const float* lse,
                        float* D, void* dqkv, int N, int L, int H, float scale, float* bpart, void* stream) {
  using namespace pv::attn;
  if (N <= 0 || L <= 0 || H <= 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int NL = N * L;
  if (H % 4 == 0)
    hipLaunchKernelGGL(attn_bwd_prep4_kernel, dim3((NL + 3) / 4), dim3(256), 0, s, (const unsigned short*)dout,
                       (const unsigned short*)out, D, NL, L, H);
  else
    hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((NL + 3) / 4), dim3(256), 0, s, (const unsigned short*)dout,
                       (const unsigned short*)out, D, NL, L, H);
  PV_LAUNCH_CHECK();
  const int qk = qg_or(g_qg_dkdv, 1), qq = qg_or(g_qg_dq, L >= 128 ? 2 : 1);
#define PV_ABWD(KERN, QGV)                                                                                       hipLaunchKernelGGL(KERN<QGV>, dim3((L + TB * QGV - 1) / (TB * QGV), H, N), dim3(256), 0, s,                                     (const unsigned short*)qkv, mask, (const unsigned short*)dout, lse, D, (unsigned short*)dqkv,                      L, H, scale, bpart, (L + TB - 1) / TB)
  if (qk == 4) PV_ABWD(attn_bwd_dkdv_kernel, 4);
  else if (qk == 2) PV_ABWD(attn_bwd_dkdv_kernel, 2);
  else PV_ABWD(attn_bwd_dkdv_kernel, 1);
  PV_LAUNCH_CHECK();
  if (qq == 4) PV_ABWD(attn_bwd_dq_kernel, 4);
  else if (qq == 2) PV_ABWD(attn_bwd_dq_kernel, 2);
  else PV_ABWD(attn_bwd_dq_kernel, 1);
#undef PV_ABWD
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_attn_bwd(const void* qkv, const int* mask, const void* out, const void* dout, const float* lse,
                       float* D, void* dqkv, int N, int L, int H, float scale, void* stream) {
  return pv_attn_bwd2(qkv, mask, out, dout, lse, D, dqkv, N, L, H, scale, nullptr, stream);
}
