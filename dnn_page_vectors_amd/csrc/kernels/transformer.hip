// Transformer building blocks for the BERT-base dual encoder (BASELINE config 4).
//
// The GEMMs (QKV / output / FFN projections, Q.K^T, P.V) are plain GEMMs and run on
// hipBLASLt in bf16; everything between them is a memory-bound row operation and is
// fused here so each activation is read and written once:
//   * add_layernorm_fwd : y = LN(x + r) * gamma + beta  (bf16 in/out, fp32 stats), also
//                         writes the pre-LN sum h = x + r for the residual stream
//   * layernorm_bwd     : dx = rstd * (dy*g - mean(dy*g) - xhat * mean(dy*g*xhat)),
//                         dgamma / dbeta via per-block partials + fp32 atomics
//   * bias_gelu_fwd/bwd : GELU(tanh) fused with the FFN bias (and its derivative)
//   * softmax_fwd/bwd   : scale + key-padding mask + row softmax of the attention scores
//                         (bf16, one wave per row, vectorised 16-byte loads)
// One 256-thread block handles one row for D in {768, 3072}; rows are independent.
#include "common.h"

namespace pv {
namespace tfm {

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  return t;
}

// x, r, y, h: (M, D) bf16 ; gamma/beta fp32 ; mean/rstd fp32 (M)
__global__ __launch_bounds__(256) void add_layernorm_fwd_kernel(const unsigned short* __restrict__ x,
                                                                const unsigned short* __restrict__ r,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                unsigned short* __restrict__ y,
                                                                unsigned short* __restrict__ h,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ rstd_out, int D, float eps) {
  __shared__ float sh[8];
  const size_t row = blockIdx.x;
  const unsigned short* xr = x + row * D;
  const unsigned short* rr = r ? r + row * D : nullptr;
  constexpr int MAXV = 4;  // up to 4 x 256 x 4 = 4096 elements per row
  float v[MAXV][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (threadIdx.x + i * 256) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[i][k] = 0.f;
    if (c < D) {
      const uint2 a = *reinterpret_cast<const uint2*>(xr + c);
      v[i][0] = __uint_as_float(a.x << 16);
      v[i][1] = __uint_as_float(a.x & 0xFFFF0000u);
      v[i][2] = __uint_as_float(a.y << 16);
      v[i][3] = __uint_as_float(a.y & 0xFFFF0000u);
      if (rr) {
        const uint2 b = *reinterpret_cast<const uint2*>(rr + c);
        v[i][0] += __uint_as_float(b.x << 16);
        v[i][1] += __uint_as_float(b.x & 0xFFFF0000u);
        v[i][2] += __uint_as_float(b.y << 16);
        v[i][3] += __uint_as_float(b.y & 0xFFFF0000u);
      }
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
    }
  }
  const float mu = block_sum(s, sh) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (threadIdx.x + i * 256) * 4;
    if (c < D)
#pragma unroll
      for (int k = 0; k < 4; ++k) q += (v[i][k] - mu) * (v[i][k] - mu);
  }
  const float rstd = rsqrtf(block_sum(q, sh) / D + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (threadIdx.x + i * 256) * 4;
    if (c < D) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (v[i][k] - mu) * rstd * gamma[c + k] + beta[c + k];
      *reinterpret_cast<uint2*>(y + row * D + c) = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      if (h) *reinterpret_cast<uint2*>(h + row * D + c) =
          uint2{pack_bf16x2(v[i][0], v[i][1]), pack_bf16x2(v[i][2], v[i][3])};
    }
  }
  if (threadIdx.x == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
}

// dy (bf16), hsum = pre-LN input (bf16), gamma, mean, rstd -> dx (bf16), dgamma/dbeta (+=, fp32)
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const unsigned short* __restrict__ dy,
                                                            const unsigned short* __restrict__ hsum,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            unsigned short* __restrict__ dx,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                            int M, int D, int rows_per_block) {
  __shared__ float sh[8];
  extern __shared__ float gacc[];  // 2 * D partial dgamma / dbeta
  for (int c = threadIdx.x; c < 2 * D; c += blockDim.x) gacc[c] = 0.f;
  __syncthreads();
  const int r0 = blockIdx.x * rows_per_block;
  for (int row = r0; row < min(M, r0 + rows_per_block); ++row) {
    const float mu = mean[row], rs = rstd[row];
    float a = 0.f, b = 0.f;
    for (int c = threadIdx.x; c < D; c += 256) {
      const float g = bf16_to_f32(dy[(size_t)row * D + c]);
      const float xh = (bf16_to_f32(hsum[(size_t)row * D + c]) - mu) * rs;
      const float gg = g * gamma[c];
      a += gg;
      b += gg * xh;
      gacc[c] += g * xh;
      gacc[D + c] += g;
    }
    a = block_sum(a, sh) / D;
    b = block_sum(b, sh) / D;
    for (int c = threadIdx.x; c < D; c += 256) {
      const float g = bf16_to_f32(dy[(size_t)row * D + c]);
      const float xh = (bf16_to_f32(hsum[(size_t)row * D + c]) - mu) * rs;
      dx[(size_t)row * D + c] = f32_to_bf16(rs * (g * gamma[c] - a - xh * b));
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    atomicAdd(&dgamma[c], gacc[c]);
    atomicAdd(&dbeta[c], gacc[D + c]);
  }
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float u = 0.7978845608028654f * (x + 0.044715f * x2 * x);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * x2);
}

// x: (M, D) bf16 pre-activation (without bias); y = gelu(x + b)
__global__ void bias_gelu_fwd_kernel(const unsigned short* __restrict__ x, const float* __restrict__ b,
                                     unsigned short* __restrict__ y, long n, int D) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  const long stride = (long)gridDim.x * blockDim.x * 2;
  for (; i < n; i += stride) {
    const unsigned v = *reinterpret_cast<const unsigned*>(x + i);
    const int c = (int)(i % D);
    const float a0 = __uint_as_float(v << 16) + b[c], a1 = __uint_as_float(v & 0xFFFF0000u) + b[c + 1];
    *reinterpret_cast<unsigned*>(y + i) = pack_bf16x2(gelu_tanh(a0), gelu_tanh(a1));
  }
}

// dx = dy * gelu'(x + b); db += sum over rows (fp32 atomics from block partials)
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const unsigned short* __restrict__ x,
                                                            const float* __restrict__ b,
                                                            const unsigned short* __restrict__ dy,
                                                            unsigned short* __restrict__ dx,
                                                            float* __restrict__ db, int M, int D,
                                                            int rows_per_block) {
  const int r0 = blockIdx.x * rows_per_block;
  for (int c = threadIdx.x; c < D; c += 256) {
    float acc = 0.f;
    const float bc = b[c];
    for (int row = r0; row < min(M, r0 + rows_per_block); ++row) {
      const size_t o = (size_t)row * D + c;
      const float g = bf16_to_f32(dy[o]) * gelu_tanh_grad(bf16_to_f32(x[o]) + bc);
      dx[o] = f32_to_bf16(g);
      acc += g;
    }
    atomicAdd(&db[c], acc);
  }
}

// S: (R, L) bf16 scores rows; row r belongs to batch item r / rows_per_item; mask (B, L) int
// (1 = keep). P = softmax(scale * S + (mask ? 0 : -inf)) written in place.
__global__ __launch_bounds__(256) void softmax_fwd_kernel(unsigned short* __restrict__ S, const int* __restrict__ mask,
                                                          long R, int L, int rows_per_item, float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  unsigned short* s = S + row * L;
  const int* mk = mask ? mask + (row / rows_per_item) * L : nullptr;
  float mx = -INFINITY;
  for (int c = lane; c < L; c += 64) {
    const float v = (mk && !mk[c]) ? -INFINITY : bf16_to_f32(s[c]) * scale;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int c = lane; c < L; c += 64) {
    const float v = (mk && !mk[c]) ? 0.f : __expf(bf16_to_f32(s[c]) * scale - mx);
    sum += v;
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int c = lane; c < L; c += 64) {
    const float v = (mk && !mk[c]) ? 0.f : __expf(bf16_to_f32(s[c]) * scale - mx) * inv;
    s[c] = f32_to_bf16(v);
  }
}

// dS = scale * P * (dP - sum(dP * P)) written into dP
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const unsigned short* __restrict__ P,
                                                          unsigned short* __restrict__ dP, long R, int L, float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const unsigned short* p = P + row * L;
  unsigned short* d = dP + row * L;
  float dot = 0.f;
  for (int c = lane; c < L; c += 64) dot += bf16_to_f32(p[c]) * bf16_to_f32(d[c]);
  dot = wave_sum(dot);
  for (int c = lane; c < L; c += 64) {
    const float pv = bf16_to_f32(p[c]);
    d[c] = f32_to_bf16(scale * pv * (bf16_to_f32(d[c]) - dot));
  }
}

}  // namespace tfm
}  // namespace pv

using namespace pv;

PV_API int pv_add_layernorm_fwd(const void* x, const void* r, const float* gamma, const float* beta, void* y, void* h,
                                float* mean, float* rstd, int M, int D, float eps, void* stream) {
  if (D % 4 || D > 4096) return -1;
  hipLaunchKernelGGL(pv::tfm::add_layernorm_fwd_kernel, dim3(M), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)x, (const unsigned short*)r, gamma, beta, (unsigned short*)y,
                     (unsigned short*)h, mean, rstd, D, eps);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_layernorm_bwd(const void* dy, const void* hsum, const float* gamma, const float* mean, const float* rstd,
                            void* dx, float* dgamma, float* dbeta, int M, int D, void* stream) {
  const int rpb = 32;
  hipLaunchKernelGGL(pv::tfm::layernorm_bwd_kernel, dim3((M + rpb - 1) / rpb), dim3(256), 2 * D * sizeof(float),
                     (hipStream_t)stream, (const unsigned short*)dy, (const unsigned short*)hsum, gamma, mean, rstd,
                     (unsigned short*)dx, dgamma, dbeta, M, D, rpb);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_bias_gelu_fwd(const void* x, const float* b, void* y, long n, int D, void* stream) {
  if (D % 2) return -1;
  long blocks = (n / 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(pv::tfm::bias_gelu_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)x, b, (unsigned short*)y, n, D);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_bias_gelu_bwd(const void* x, const float* b, const void* dy, void* dx, float* db, int M, int D,
                            void* stream) {
  const int rpb = 64;
  hipLaunchKernelGGL(pv::tfm::bias_gelu_bwd_kernel, dim3((M + rpb - 1) / rpb), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)x, b, (const unsigned short*)dy, (unsigned short*)dx, db, M, D, rpb);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_softmax_fwd(void* S, const int* mask, long R, int L, int rows_per_item, float scale, void* stream) {
  hipLaunchKernelGGL(pv::tfm::softmax_fwd_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (unsigned short*)S, mask, R, L, rows_per_item, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_softmax_bwd(const void* P, void* dP, long R, int L, float scale, void* stream) {
  hipLaunchKernelGGL(pv::tfm::softmax_bwd_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)P, (unsigned short*)dP, R, L, scale);
  PV_LAUNCH_CHECK();
  return 0;
}
