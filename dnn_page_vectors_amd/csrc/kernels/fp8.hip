// FP8 (OCP e4m3) linear layers for the long-page chunked encoder (BASELINE config 5:
// "Long-page 4k-token chunked encoder, mean-pool, fp8 MFMA on CDNA4").
//
// * amax_kernel      : per-tensor max |x| (fp32 atomicMax on the non-negative bit pattern)
// * quant_fp8_kernel : x -> e4m3 with scale s = 448 / amax (saturating), packed 4 per dword
//                      by v_cvt_pk_fp8_f32 (gfx950: OCP e4m3fn, not MI300's fnuz)
// * fp8_linear_kernel: Y[M,N] = act(inv_sx * inv_sw * (X8[M,K] . W8[N,K]^T) + b) with
//                      v_mfma_f32_16x16x32_fp8_fp8 (2x the bf16 operand density per byte,
//                      half the staging bytes), fp32 accumulate, fused dequant + bias +
//                      activation epilogue, fp32 and/or bf16 output.
// 64x64 block tile, BK = 64 bytes, 4 waves (2x2) of 32x32; K must be a multiple of 16.
// Training uses fp8 for the forward GEMMs and bf16 hipBLASLt GEMMs for dgrad/wgrad.
#include "common.h"

namespace pv {
namespace fp8 {

constexpr int BM = 64, BN = 64, BK = 64;
constexpr int LDB = BK + 16;  // bytes per LDS row (80: 16-B aligned)

// grid-stride 16-byte loads, wave then block reduction, ONE atomic per block (a few
// hundred blocks: contention-free, unlike per-wave atomics on one address)
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long n, float* __restrict__ amax,
                                                   int aligned) {
  __shared__ float sh[4];
  const long n4 = aligned ? n / 4 : 0;
  const long stride = (long)gridDim.x * blockDim.x;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
    atomicMax(reinterpret_cast<unsigned*>(amax), __float_as_uint(m));
  }
}

// Byte transpose for the fp8 weight gradient (ops/embedding.py, config 5): dst (C x ldd) with
// dst[c][r] = src[r][c] for r < R, 0 for R <= r < ldd (the MX GEMM's K padding).  64 x 64 byte
// tiles through LDS: one 16-byte load per thread, 16 column bytes gathered per thread, one
// 16-byte store per thread.
__global__ __launch_bounds__(256) void transpose_u8_kernel(const unsigned char* __restrict__ src, long lds, int R,
                                                           int C, unsigned char* __restrict__ dst, long ldd) {
  __shared__ unsigned char tile[64][80];
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  {
    const int r = threadIdx.x >> 2, c16 = (threadIdx.x & 3) * 16;
    uint4 v = {0u, 0u, 0u, 0u};
    if (r0 + r < R && c0 + c16 < lds) v = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + r) * lds + c0 + c16);
    *reinterpret_cast<uint4*>(&tile[r][c16]) = v;
  }
  __syncthreads();
  const int c = threadIdx.x >> 2, rb = (threadIdx.x & 3) * 16;
  if (c0 + c >= C || r0 + rb >= ldd) return;
  unsigned w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w[q] = (unsigned)tile[rb + 4 * q][c] | ((unsigned)tile[rb + 4 * q + 1][c] << 8) |
           ((unsigned)tile[rb + 4 * q + 2][c] << 16) | ((unsigned)tile[rb + 4 * q + 3][c] << 24);
  }
  *reinterpret_cast<uint4*>(dst + (size_t)(c0 + c) * ldd + r0 + rb) = uint4{w[0], w[1], w[2], w[3]};
}

// out: n bytes (n % 4 == 0); scale = 448 / max(amax, tiny)
__global__ void quant_fp8_kernel(const float* __restrict__ x, const float* __restrict__ amax,
                                 unsigned* __restrict__ out, long n4) {
  const float a = fmaxf(*amax, 1e-12f);
  const float s = 448.f / a;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    unsigned w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * s, -448.f), 448.f), fminf(fmaxf(v[1] * s, -448.f), 448.f),
                                        w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * s, -448.f), 448.f), fminf(fmaxf(v[3] * s, -448.f), 448.f),
                                        w, true);
    out[i] = w;
  }
}

// Fill-free pair (quantize() in ops/fp8.py): amax_part_kernel writes one max per block
// (no atomics, so the scalar needs no zero fill launch first); quant_part_kernel reduces
// the <= AMAX_PARTS partials in every block (L2-resident, 2 KB), block 0 also stores the
// scalar amax the fp8 GEMM's dequantisation reads.
constexpr int AMAX_PARTS = 512;

__global__ __launch_bounds__(256) void amax_part_kernel(const float* __restrict__ x, long n,
                                                        float* __restrict__ parts, int aligned) {
  __shared__ float sh[4];
  const long n4 = aligned ? n / 4 : 0;
  const long stride = (long)gridDim.x * blockDim.x;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) parts[blockIdx.x] = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
}

__global__ __launch_bounds__(256) void quant_part_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ parts, int nparts,
                                                         float* __restrict__ amax_out, unsigned* __restrict__ out,
                                                         long n4, uint2* __restrict__ x16) {
  __shared__ float sh[4];
  float m = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) m = fmaxf(m, parts[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  const float amax = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  if (blockIdx.x == 0 && threadIdx.x == 0) *amax_out = amax;
  const float s = 448.f / fmaxf(amax, 1e-12f);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    unsigned w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[0] * s, -448.f), 448.f), fminf(fmaxf(v[1] * s, -448.f), 448.f),
                                        w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[2] * s, -448.f), 448.f), fminf(fmaxf(v[3] * s, -448.f), 448.f),
                                        w, true);
    out[i] = w;
    if (x16) x16[i] = uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};  // bf16 copy for the backward
  }
}

__device__ __forceinline__ float act_fn(float x, int act) {
  if (act == 1) return x > 0.f ? x : 0.f;
  if (act == 3) return tanhf(x);
  return x;
}

// X8: (M, K) e4m3 bytes, W8: (N, K) e4m3 bytes. amax_x, amax_w: device scalars.
__global__ __launch_bounds__(256) void fp8_linear_kernel(const unsigned char* __restrict__ X8,
                                                         const unsigned char* __restrict__ W8,
                                                         const float* __restrict__ amax_x,
                                                         const float* __restrict__ amax_w,
                                                         const float* __restrict__ bias, float* __restrict__ Y,
                                                         unsigned short* __restrict__ Ybf, int M, int N, int K,
                                                         int act) {
  __shared__ __attribute__((aligned(16))) unsigned char As[BM * LDB];
  __shared__ __attribute__((aligned(16))) unsigned char Bs[BN * LDB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += BK) {
    {  // 64 rows x 64 bytes per operand: 256 threads x 16 bytes
      const int r = tid >> 2, c = (tid & 3) * 16;
      const int gm = m0 + r, gn = n0 + r, gk = k0 + c;
      u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
      if (gm < M && gk + 16 <= K) a = *reinterpret_cast<const u32x4*>(X8 + (size_t)gm * K + gk);
      else if (gm < M) {
        unsigned char t[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) t[q] = (gk + q < K) ? X8[(size_t)gm * K + gk + q] : 0;
        a = *reinterpret_cast<u32x4*>(t);
      }
      if (gn < N && gk + 16 <= K) b = *reinterpret_cast<const u32x4*>(W8 + (size_t)gn * K + gk);
      else if (gn < N) {
        unsigned char t[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) t[q] = (gk + q < K) ? W8[(size_t)gn * K + gk + q] : 0;
        b = *reinterpret_cast<u32x4*>(t);
      }
      *reinterpret_cast<u32x4*>(&As[r * LDB + c]) = a;
      *reinterpret_cast<u32x4*>(&Bs[r * LDB + c]) = b;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      long a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const long*>(&As[(wm * 32 + i * 16 + (lane & 15)) * LDB + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = *reinterpret_cast<const long*>(&Bs[(wn * 32 + j * 16 + (lane & 15)) * LDB + ks * 32 + (lane >> 4) * 8]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  const float deq = (fmaxf(*amax_x, 1e-12f) / 448.f) * (fmaxf(*amax_w, 1e-12f) / 448.f);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        if (row < M) {
          const float y = act_fn(acc[i][j][r] * deq + bv, act);
          if (Y) Y[(size_t)row * N + col] = y;
          if (Ybf) Ybf[(size_t)row * N + col] = f32_to_bf16(y);
        }
      }
    }
}

}  // namespace fp8
}  // namespace pv

using namespace pv;

PV_API int pv_amax(const float* x, long n, float* amax, void* stream) {
  const int aligned = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  long blocks = ((aligned ? n / 4 : n) + 255) / 256;
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pv::fp8::amax_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, n, amax,
                     aligned);
  PV_LAUNCH_CHECK();
  return 0;
}

// x (n fp32, 16-byte aligned, n % 4 == 0) -> out (n e4m3 bytes) and *amax_out; ws: at
// least AMAX_PARTS floats of scratch (uninitialised is fine).  Two launches, no fill.
PV_API int pv_amax_quant_fp8(const float* x, long n, float* ws, float* amax_out, void* out, void* out16,
                             void* stream) {
  using namespace pv::fp8;
  if (n % 4 || (reinterpret_cast<uintptr_t>(x) & 15)) return -1;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > AMAX_PARTS) blocks = AMAX_PARTS;
  if (blocks < 1) blocks = 1;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(amax_part_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, ws, 1);
  PV_LAUNCH_CHECK();
  const long n4 = n / 4;
  long qb = (n4 + 255) / 256;
  if (qb > 4096) qb = 4096;
  if (qb < 1) qb = 1;
  hipLaunchKernelGGL(quant_part_kernel, dim3((unsigned)qb), dim3(256), 0, st, x, (const float*)ws, (int)blocks,
                     amax_out, (unsigned*)out, n4, (uint2*)out16);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_quant_fp8(const float* x, const float* amax, void* out, long n, void* stream) {
  if (n % 4) return -1;
  long n4 = n / 4;
  long blocks = (n4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(pv::fp8::quant_fp8_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, amax,
                     (unsigned*)out, n4);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_fp8_linear(const void* X8, const void* W8, const float* amax_x, const float* amax_w, const float* bias,
                         float* Y, void* Ybf, int M, int N, int K, int act, void* stream) {
  using namespace pv::fp8;
  if (K % 16) return -1;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN);
  hipLaunchKernelGGL(fp8_linear_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const unsigned char*)X8,
                     (const unsigned char*)W8, amax_x, amax_w, bias, Y, (unsigned short*)Ybf, M, N, K, act);
  PV_LAUNCH_CHECK();
  return 0;
}

// ---- transposed quantisation for the MX fp8 GEMM's K-contiguous operands ------------------
// W (V, E) fp32 row-major -> out (E, ldo) e4m3 bytes, out[e][v] = e4m3(W[v][e] * 448 / amax)
// for v < V and 0 for V <= v < ldo (the GEMM's K padding); amax from the amax_part_kernel
// partials (reduced again by every block, 2 KB L2-resident), block 0 stores it.  64 x 64
// tiles through LDS: coalesced 16-byte reads along E, 4-byte (4 x e4m3) writes along V.
__global__ __launch_bounds__(256) void quant_t_kernel(const float* __restrict__ W, int V, int E,
                                                      const float* __restrict__ parts, int nparts,
                                                      float* __restrict__ amax_out, unsigned char* __restrict__ out,
                                                      int ldo) {
  __shared__ float sh[4];
  __shared__ float tile[64][65];
  float m = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) m = fmaxf(m, parts[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  const float amax = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *amax_out = amax;
  const float s = 448.f / fmaxf(amax, 1e-12f);
  const int v0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  // load: 64 rows (v) x 64 cols (e) = 1024 float4, 4 per thread
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = threadIdx.x + 256 * u;
    const int r = q >> 4, c4 = (q & 15) * 4;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (v0 + r < V && e0 + c4 < E) x = *reinterpret_cast<const f32x4*>(W + (size_t)(v0 + r) * E + e0 + c4);
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[r][c4 + k] = x[k];
  }
  __syncthreads();
  // store: out row e (64 of them) x 64 v bytes = 16 dwords per row, 4 per thread
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = threadIdx.x + 256 * u;
    const int e = q >> 4, v4 = (q & 15) * 4;
    if (e0 + e >= E || v0 + v4 >= ldo) continue;
    float f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = fminf(fmaxf(tile[v4 + k][e] * s, -448.f), 448.f);
    unsigned w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], w, true);
    *reinterpret_cast<unsigned*>(out + (size_t)(e0 + e) * ldo + v0 + v4) = w;
  }
}

// ---- block-scaled (MX) fp8 MFMA layout probe -------------------------------------------
// One v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, e8m0 scales) by one wave: lane l
// passes its 32 A bytes a[l], 32 B bytes b[l], its A / B scale bytes sa[l] / sb[l], and
// stores its 4 accumulator floats.  tests/test_kernels_gpu.py::test_mx_fp8_mfma_layout
// checks the operand / scale mapping the MX GEMM relies on against a host reference.
typedef int v8i_t __attribute__((ext_vector_type(8)));
__global__ void mx_probe_kernel(const v8i_t* a, const v8i_t* b, const int* sa, const int* sb, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}

PV_API int pv_mx_probe(const void* a, const void* b, const int* sa, const int* sb, float* c, void* stream) {
  hipLaunchKernelGGL(mx_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const v8i_t*)a, (const v8i_t*)b, sa,
                     sb, (f32x4*)c);
  PV_LAUNCH_CHECK();
  return 0;
}

// W (V, E) fp32 (16-byte aligned, E % 4 == 0) -> out (E, ldo) e4m3, transposed and zero-padded
// to ldo (ldo % 64 == 0, ldo >= V), *amax_out = max |W|; ws >= AMAX_PARTS floats of scratch.
PV_API int pv_amax_quant_fp8_t(const float* W, int V, int E, float* ws, float* amax_out, void* out, int ldo,
                               void* stream) {
  using namespace pv::fp8;
  if (E % 4 || ldo % 64 || ldo < V || (reinterpret_cast<uintptr_t>(W) & 15)) return -1;
  const long n = (long)V * E;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > AMAX_PARTS) blocks = AMAX_PARTS;
  if (blocks < 1) blocks = 1;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(amax_part_kernel, dim3((unsigned)blocks), dim3(256), 0, st, W, n, ws, 1);
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(quant_t_kernel, dim3(ldo / 64, (E + 63) / 64), dim3(256), 0, st, W, V, E, (const float*)ws,
                     (int)blocks, amax_out, (unsigned char*)out, ldo);
  PV_LAUNCH_CHECK();
  return 0;
}

// src (R x lds bytes, lds % 16 == 0, lds >= C) -> dst (C x ldd bytes), dst[c][r] = src[r][c],
// zero for R <= r < ldd (ldd % 64 == 0, ldd >= R); 16-byte aligned rows.
PV_API int pv_transpose_u8(const void* src, long lds, int R, int C, void* dst, long ldd, void* stream) {
  using namespace pv::fp8;
  if (R <= 0 || C <= 0 || lds % 16 || ldd % 64 || ldd < R || lds < C) return -1;
  if ((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15)) return -2;
  hipLaunchKernelGGL(transpose_u8_kernel, dim3((unsigned)(ldd / 64), (unsigned)((C + 63) / 64)), dim3(256), 0,
                     (hipStream_t)stream, (const unsigned char*)src, lds, R, C, (unsigned char*)dst, ldd);
  PV_LAUNCH_CHECK();
  return 0;
}
