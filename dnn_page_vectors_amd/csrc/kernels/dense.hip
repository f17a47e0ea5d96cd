// K4 (fused linear + bias + activation, MFMA) and K5 (L2 normalise fwd/bwd).
//
// Reference: Dense(hidden_dims) + Activation('relu') (cnn_dssm_th.py:136-138) and the
// RTH/RTF magnitude sqrt(max(sum x^2, float32 tiny)) (cnn_dssm_th.py:66-75).
//
// linear_act: Y[M,N] = act(X[M,K] . W[N,K]^T + b) with fp32 (or bf16) X/W converted to
// bf16 while staging into LDS, v_mfma_f32_16x16x32_bf16, fp32 accumulate, fused
// bias/activation epilogue, optional bf16 copy of Y.  64x64 block tile, BK=32,
// 4 waves in 2x2, each wave a 32x32 sub-tile (2x2 MFMA tiles).  Used for the CDSSM
// dense head (300->150), the MLP tower (512-512-128) and BERT projections.
#include "common.h"

namespace pv {
namespace dense {

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int LDA = BK + 8;  // bf16 elements per LDS row (80 B: 16-B aligned, staggers banks)

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_TANH = 3 };

__device__ __forceinline__ float act_fn(float x, int act) {
  if (act == ACT_RELU) return x > 0.f ? x : 0.f;
  if (act == ACT_GELU) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    float u = k0 * (x + k1 * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  }
  if (act == ACT_TANH) return tanhf(x);
  return x;
}

template <typename TX>
__device__ __forceinline__ float ldf(const TX* p, size_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, size_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<unsigned short>(const unsigned short* p, size_t i) { return bf16_to_f32(p[i]); }

template <typename TX, typename TW>
__global__ __launch_bounds__(256) void linear_act_kernel(const TX* __restrict__ X, const TW* __restrict__ W,
                                                         const float* __restrict__ bias, float* __restrict__ Y,
                                                         unsigned short* __restrict__ Ybf, int M, int N, int K,
                                                         int ldx, int ldy, int act) {
  __shared__ __attribute__((aligned(16))) unsigned short As[BM * LDA];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[BN * LDA];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += BK) {
    // stage A (BM x BK) and B (BN x BK) as bf16: 64 rows x 4 segments of 8 per operand
    {
      const int r = tid >> 2, c = (tid & 3) * 8;
      unsigned pa[4], pb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gk = k0 + c + 2 * q;
        const int gm = m0 + r, gn = n0 + r;
        float x0 = (gm < M && gk < K) ? ldf<TX>(X, (size_t)gm * ldx + gk) : 0.f;
        float x1 = (gm < M && gk + 1 < K) ? ldf<TX>(X, (size_t)gm * ldx + gk + 1) : 0.f;
        float w0 = (gn < N && gk < K) ? ldf<TW>(W, (size_t)gn * K + gk) : 0.f;
        float w1 = (gn < N && gk + 1 < K) ? ldf<TW>(W, (size_t)gn * K + gk + 1) : 0.f;
        pa[q] = pack_bf16x2(x0, x1);
        pb[q] = pack_bf16x2(w0, w1);
      }
      *reinterpret_cast<u32x4*>(&As[r * LDA + c]) = u32x4{pa[0], pa[1], pa[2], pa[3]};
      *reinterpret_cast<u32x4*>(&Bs[r * LDA + c]) = u32x4{pb[0], pb[1], pb[2], pb[3]};
    }
    __syncthreads();
    bf16x8 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * 32 + i * 16 + (lane & 15)) * LDA + (lane >> 4) * 8]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * 32 + j * 16 + (lane & 15)) * LDA + (lane >> 4) * 8]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  // epilogue: row = m0 + wm*32 + i*16 + 4*(lane>>4) + r ; col = n0 + wn*32 + j*16 + (lane&15)
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
          float y = act_fn(acc[i][j][r] + bv, act);
          if (Y) Y[(size_t)row * ldy + col] = y;
          if (Ybf) Ybf[(size_t)row * ldy + col] = f32_to_bf16(y);
        }
      }
    }
}

// Row-wise L2 normalisation: y = x / sqrt(max(|x|^2, tiny)); one wave per row.
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         float* __restrict__ inv_norm, unsigned short* __restrict__ ybf,
                                                         int M, int D, int ldbf) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* xr = x + (size_t)row * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += xr[d] * xr[d];
  s = wave_sum(s);
  const float inv = 1.0f / sqrtf(fmaxf(s, 1.17549435e-38f));
  for (int d = lane; d < D; d += 64) {
    float v = xr[d] * inv;
    y[(size_t)row * D + d] = v;
    if (ybf) ybf[(size_t)row * ldbf + d] = f32_to_bf16(v);
  }
  if (ybf)
    for (int d = D + lane; d < ldbf; d += 64) ybf[(size_t)row * ldbf + d] = 0;
  if (lane == 0) inv_norm[row] = inv;
}

// dx = (dy - y * <y, dy>) * inv   (if |x|^2 < tiny the clamp is active: dx = dy * inv)
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ y, const float* __restrict__ inv_norm,
                                                         const float* __restrict__ x, const float* __restrict__ dy,
                                                         float* __restrict__ dx, int M, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* yr = y + (size_t)row * D;
  const float* gr = dy + (size_t)row * D;
  float s = 0.f, xx = 0.f;
  for (int d = lane; d < D; d += 64) {
    s += yr[d] * gr[d];
    float xv = x[(size_t)row * D + d];
    xx += xv * xv;
  }
  s = wave_sum(s);
  xx = wave_sum(xx);
  const float inv = inv_norm[row];
  const bool clamped = xx < 1.17549435e-38f;
  for (int d = lane; d < D; d += 64) dx[(size_t)row * D + d] = clamped ? gr[d] * inv : (gr[d] - yr[d] * s) * inv;
}

// dz = dy * act'(y) (in place allowed); relu: y > 0 ; tanh: 1 - y^2 ; none: 1
__global__ void act_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy, float* __restrict__ dz,
                               long n, int act) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float g = dy[i];
    if (act == ACT_RELU) g = y[i] > 0.f ? g : 0.f;
    else if (act == ACT_TANH) g = g * (1.f - y[i] * y[i]);
    dz[i] = g;
  }
}

}  // namespace dense
}  // namespace pv

using namespace pv;

// xdt/wdt: 0 = fp32, 1 = bf16
PV_API int pv_linear_act(const void* X, int xdt, const void* W, int wdt, const float* bias, float* Y, void* Ybf, int M,
                         int N, int K, int ldx, int ldy, int act, void* stream) {
  using namespace pv::dense;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN);
  hipStream_t s = (hipStream_t)stream;
  unsigned short* yb = (unsigned short*)Ybf;
  if (xdt == 0 && wdt == 0)
    hipLaunchKernelGGL((linear_act_kernel<float, float>), grid, dim3(256), 0, s, (const float*)X, (const float*)W, bias,
                       Y, yb, M, N, K, ldx, ldy, act);
  else if (xdt == 1 && wdt == 0)
    hipLaunchKernelGGL((linear_act_kernel<unsigned short, float>), grid, dim3(256), 0, s, (const unsigned short*)X,
                       (const float*)W, bias, Y, yb, M, N, K, ldx, ldy, act);
  else if (xdt == 0 && wdt == 1)
    hipLaunchKernelGGL((linear_act_kernel<float, unsigned short>), grid, dim3(256), 0, s, (const float*)X,
                       (const unsigned short*)W, bias, Y, yb, M, N, K, ldx, ldy, act);
  else
    hipLaunchKernelGGL((linear_act_kernel<unsigned short, unsigned short>), grid, dim3(256), 0, s,
                       (const unsigned short*)X, (const unsigned short*)W, bias, Y, yb, M, N, K, ldx, ldy, act);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_l2norm_fwd(const float* x, float* y, float* inv_norm, void* ybf, int M, int D, int ldbf, void* stream) {
  using namespace pv::dense;
  hipLaunchKernelGGL(l2norm_fwd_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, y, inv_norm,
                     (unsigned short*)ybf, M, D, ldbf);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_l2norm_bwd(const float* y, const float* inv_norm, const float* x, const float* dy, float* dx, int M, int D,
                         void* stream) {
  using namespace pv::dense;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, y, inv_norm, x, dy, dx,
                     M, D);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_act_bwd(const float* y, const float* dy, float* dz, long n, int act, void* stream) {
  using namespace pv::dense;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, y, dy, dz, n, act);
  PV_LAUNCH_CHECK();
  return 0;
}
