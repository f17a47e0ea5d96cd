// K4 (fused linear + bias + activation, MFMA) and K5 (L2 normalise fwd/bwd).
//
// Reference: Dense(hidden_dims) + Activation('relu') (cnn_dssm_th.py:136-138) and the
// RTH/RTF magnitude sqrt(max(sum x^2, float32 tiny)) (cnn_dssm_th.py:66-75).
//
// linear_act: Y[M,N] = act(X[M,K] . W[N,K]^T + b) with fp32 (or bf16) X/W converted to
// bf16 while staging into LDS (16-byte vector loads), v_mfma_f32_16x16x32_bf16, fp32
// accumulate, fused bias/activation epilogue, optional bf16 copy of Y.  64x64 block
// tile, BK=64 double-buffered, 4 waves in 2x2, each wave a 32x32 sub-tile.  Used for
// the CDSSM dense head (300->150) and the MLP tower (512-512-128).
#include "common.h"

namespace pv {
namespace dense {

constexpr int BM = 64, BN = 64, BK = 64;
constexpr int LDA = BK + 8;  // bf16 elements per LDS row (144 B: 16-B aligned, staggers banks)

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

template <typename T>
__device__ __forceinline__ float ldf(const T* p, size_t i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, size_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<unsigned short>(const unsigned short* p, size_t i) { return bf16_to_f32(p[i]); }

// 16 consecutive elements of row `row` starting at column k as bf16 (two 16-byte words);
// vector loads when the run is in bounds and aligned, element loads at the edges.
template <typename T>
__device__ __forceinline__ void load16(const T* __restrict__ P, int rows, int cols, int ld, int row, int k,
                                       bool vec_ok, u32x4 (&out)[2]) {
  if (row < rows && k + 16 <= cols && vec_ok) {
    const T* q = P + (size_t)row * ld + k;
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 v0 = reinterpret_cast<const f32x4*>(q)[2 * h];
        const f32x4 v1 = reinterpret_cast<const f32x4*>(q)[2 * h + 1];
        out[h] = u32x4{pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                       pack_bf16x2(v1[2], v1[3])};
      }
    } else {
      out[0] = reinterpret_cast<const u32x4*>(q)[0];
      out[1] = reinterpret_cast<const u32x4*>(q)[1];
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = k + 8 * h + 2 * e;
        const float x0 = (row < rows && c < cols) ? ldf<T>(P, (size_t)row * ld + c) : 0.f;
        const float x1 = (row < rows && c + 1 < cols) ? ldf<T>(P, (size_t)row * ld + c + 1) : 0.f;
        w[e] = pack_bf16x2(x0, x1);
      }
      out[h] = u32x4{w[0], w[1], w[2], w[3]};
    }
  }
}

// The same 16 elements for an operand stored TRANSPOSED: element (row, k + j) of the
// logical operand is P[(k + j) * ld + row] (the dgrad's W^T read straight from W: strided
// scalar loads of a small, L2-resident matrix instead of a transposed copy per step).
template <typename T>
__device__ __forceinline__ void load16t(const T* __restrict__ P, int rows, int cols, int ld, int row, int k,
                                        u32x4 (&out)[2]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    unsigned w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = k + 8 * h + 2 * e;
      const float x0 = (row < rows && c < cols) ? ldf<T>(P, (size_t)c * ld + row) : 0.f;
      const float x1 = (row < rows && c + 1 < cols) ? ldf<T>(P, (size_t)(c + 1) * ld + row) : 0.f;
      w[e] = pack_bf16x2(x0, x1);
    }
    out[h] = u32x4{w[0], w[1], w[2], w[3]};
  }
}

// Y^T tile = W . X^T: A operand = W rows (n), B operand = X rows (m), so the C layout
// puts one m per lane and 4 CONSECUTIVE n per lane -> 16-byte fp32 / 8-byte bf16 stores.
// BK = 64 (2 MFMA k-steps per tile, 8 MFMAs per wave), tile t+1 is fetched into
// registers while tile t's MFMAs run and written to the other LDS buffer (1 barrier/tile).
// WT: W is stored as [K][N] (the dgrad dx = dz W of a layer whose weight is [N_out][K_in]).
template <typename TX, typename TW, bool WT = false>
__global__ __launch_bounds__(256) void linear_act_kernel(const TX* __restrict__ X, const TW* __restrict__ W,
                                                         const float* __restrict__ bias, float* __restrict__ Y,
                                                         unsigned short* __restrict__ Ybf, int M, int N, int K,
                                                         int ldx, int ldy, int act) {
  __shared__ __attribute__((aligned(16))) unsigned short As[2][BM * LDA];  // X rows (m)
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BN * LDA];  // W rows (n)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const bool xvec = (ldx % (16 / (int)sizeof(TX))) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  const bool wvec = (K % (16 / (int)sizeof(TW))) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0;
  const int sr = tid >> 2, sc = (tid & 3) * 16;  // staging: row, first column of 16
  f32x4 acc[2][2];  // [n-subtile][m-subtile]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 ra[2], rb[2];
  load16<TX>(X, M, K, ldx, m0 + sr, sc, xvec, ra);
  if constexpr (WT) load16t<TW>(W, N, K, N, n0 + sr, sc, rb);
  else load16<TW>(W, N, K, K, n0 + sr, sc, wvec, rb);
  *reinterpret_cast<u32x4*>(&As[0][sr * LDA + sc]) = ra[0];
  *reinterpret_cast<u32x4*>(&As[0][sr * LDA + sc + 8]) = ra[1];
  *reinterpret_cast<u32x4*>(&Bs[0][sr * LDA + sc]) = rb[0];
  *reinterpret_cast<u32x4*>(&Bs[0][sr * LDA + sc + 8]) = rb[1];
  __syncthreads();
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += BK, buf ^= 1) {
    const bool more = k0 + BK < K;
    if (more) {
      load16<TX>(X, M, K, ldx, m0 + sr, k0 + BK + sc, xvec, ra);
      if constexpr (WT) load16t<TW>(W, N, K, N, n0 + sr, k0 + BK + sc, rb);
      else load16<TW>(W, N, K, K, n0 + sr, k0 + BK + sc, wvec, rb);
    }
#pragma unroll
    for (int s2 = 0; s2 < BK / 32; ++s2) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&Bs[buf][(wn * 32 + i * 16 + (lane & 15)) * LDA + s2 * 32 + g * 8]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&As[buf][(wm * 32 + j * 16 + (lane & 15)) * LDA + s2 * 32 + g * 8]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      *reinterpret_cast<u32x4*>(&As[buf ^ 1][sr * LDA + sc]) = ra[0];
      *reinterpret_cast<u32x4*>(&As[buf ^ 1][sr * LDA + sc + 8]) = ra[1];
      *reinterpret_cast<u32x4*>(&Bs[buf ^ 1][sr * LDA + sc]) = rb[0];
      *reinterpret_cast<u32x4*>(&Bs[buf ^ 1][sr * LDA + sc + 8]) = rb[1];
    }
    __syncthreads();
  }
  // acc[i][j][r] = Y[m = m0 + wm*32 + j*16 + (lane&15)][n = n0 + wn*32 + i*16 + 4g + r]
  const bool yvec = (ldy & 3) == 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + wm * 32 + j * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int n = n0 + wn * 32 + i * 16 + 4 * g;
      if (n >= N) continue;
      float y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = act_fn(acc[i][j][r] + ((bias && n + r < N) ? bias[n + r] : 0.f), act);
      if (yvec && n + 4 <= N) {
        if (Y) *reinterpret_cast<f32x4*>(Y + (size_t)m * ldy + n) = f32x4{y[0], y[1], y[2], y[3]};
        if (Ybf) *reinterpret_cast<uint2*>(Ybf + (size_t)m * ldy + n) = uint2{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) {
            if (Y) Y[(size_t)m * ldy + n + r] = y[r];
            if (Ybf) Ybf[(size_t)m * ldy + n + r] = f32_to_bf16(y[r]);
          }
      }
    }
  }
}

// Weight gradient of linear_act: dW[n][k] = sum_m dz[m][n] x[m][k] (dz fp32 or bf16 (M, N),
// x fp32 or bf16 (M, K), both row-major as the forward left them: no transposed copies).
// The reduction runs over the ROWS of both operands, so each 64-row step is staged into LDS
// transposed ([n][m] and [k][m], bf16; one ds_write_b32 per lane and column writes a row
// pair, a half-wave covers 64 consecutive m of one LDS row: conflict-free), so the MFMA
// fragments are the same ds_read_b128 rows as linear_act's.  64 x 64 or 128 x 128 output
// tile per workgroup (4 waves, 2 x 2; the larger tile halves the operand re-reads of wide
// layers), rows split over gridDim.z: each slice writes its fp32 partial
// tile into slab z of a workspace that the column-sum kernel reduces in a fixed order
// (deterministic, no atomics).
template <typename TZ, typename TX, int T>
__global__ __launch_bounds__(256) void linear_wgrad_kernel(const TZ* __restrict__ dz, const TX* __restrict__ X,
                                                           float* __restrict__ ws, int M, int N, int K, int rows_per) {
  // T x T output tile (T = 64 or 128), 4 waves in 2 x 2, each (T/2) x (T/2)
  constexpr int SUB = T / 32;  // 16x16 accumulator tiles per wave side
  __shared__ __attribute__((aligned(16))) unsigned short As[T * LDA];  // dz^T tile [n][m]
  __shared__ __attribute__((aligned(16))) unsigned short Bs[T * LDA];  // x^T tile  [k][m]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * T, k0 = blockIdx.y * T;
  const int m_begin = blockIdx.z * rows_per, m_end = min(M, m_begin + rows_per);
  f32x4 acc[SUB][SUB];  // [k-subtile][n-subtile]
#pragma unroll
  for (int i = 0; i < SUB; ++i)
#pragma unroll
    for (int j = 0; j < SUB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staging: waves 0-1 stage dz, waves 2-3 x; lane = a row PAIR (2 * (lane & 31), + 1) and
  // column groups of 16 (group q = 4u + 2 (wave & 1) + (lane >> 5), u < T / 64): one
  // ds_write_b32 per lane and column puts the pair side by side in the transposed row
  const bool zw = wave < 2;
  const int mp = 2 * (lane & 31);
  const bool zvec = (N % (16 / (int)sizeof(TZ))) == 0 && (reinterpret_cast<uintptr_t>(dz) & 15) == 0;
  const bool xvec = (K % (16 / (int)sizeof(TX))) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  unsigned short* dst = zw ? As : Bs;
  for (int m0 = m_begin; m0 < m_end; m0 += BK) {
#pragma unroll
    for (int u = 0; u < T / 64; ++u) {
      const int c0 = 16 * (4 * u + 2 * (wave & 1) + (lane >> 5));
      u32x4 r0[2], r1[2];  // rows m0 + mp, m0 + mp + 1: 16 columns as bf16 (zeros past the edges)
      if (zw) {
        load16<TZ>(dz, m_end, N, N, m0 + mp, n0 + c0, zvec, r0);
        load16<TZ>(dz, m_end, N, N, m0 + mp + 1, n0 + c0, zvec, r1);
      } else {
        load16<TX>(X, m_end, K, K, m0 + mp, k0 + c0, xvec, r0);
        load16<TX>(X, m_end, K, K, m0 + mp + 1, k0 + c0, xvec, r1);
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned lo = (r0[c >> 3][(c >> 1) & 3] >> (16 * (c & 1))) & 0xFFFFu;
        const unsigned hi = (r1[c >> 3][(c >> 1) & 3] >> (16 * (c & 1))) & 0xFFFFu;
        *reinterpret_cast<unsigned*>(&dst[(c0 + c) * LDA + mp]) = lo | (hi << 16);
      }
    }
    __syncthreads();
#pragma unroll
    for (int s2 = 0; s2 < BK / 32; ++s2) {
      bf16x8 a[SUB], b[SUB];
#pragma unroll
      for (int i = 0; i < SUB; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&Bs[(wk * (T / 2) + i * 16 + (lane & 15)) * LDA + s2 * 32 + g * 8]);
#pragma unroll
      for (int j = 0; j < SUB; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&As[(wn * (T / 2) + j * 16 + (lane & 15)) * LDA + s2 * 32 + g * 8]);
#pragma unroll
      for (int i = 0; i < SUB; ++i)
#pragma unroll
        for (int j = 0; j < SUB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // acc[i][j][r] = dW[n = n0 + wn*T/2 + j*16 + (lane&15)][k = k0 + wk*T/2 + i*16 + 4g + r]
  float* slab = ws + (size_t)blockIdx.z * N * K;
#pragma unroll
  for (int j = 0; j < SUB; ++j) {
    const int n = n0 + wn * (T / 2) + j * 16 + (lane & 15);
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int k = k0 + wk * (T / 2) + i * 16 + 4 * g;
      if (k + 4 <= K && (K & 3) == 0) {
        *reinterpret_cast<f32x4*>(slab + (size_t)n * K + k) = acc[i][j];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (k + r < K) slab[(size_t)n * K + k + r] = acc[i][j][r];
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
                                                         float* __restrict__ dx, int M, int D, long ldy) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* yr = y + (size_t)row * D;
  const float* gr = dy + (size_t)row * ldy;  // ldy >= D: e.g. the loss kernels' padded (n, DP) gradient
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
// dz16 (optional): also a bf16 copy of dz, the operand of the bf16 backward GEMMs
__global__ void act_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy, float* __restrict__ dz,
                               long n, int act, unsigned short* __restrict__ dz16) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float g = dy[i];
    if (act == ACT_RELU) g = y[i] > 0.f ? g : 0.f;
    else if (act == ACT_TANH) g = g * (1.f - y[i] * y[i]);
    dz[i] = g;
    if (dz16) dz16[i] = f32_to_bf16(g);
  }
}

// Column sums (the bias / split-K reductions of the backward and the split-K forward):
//   s[c] = sum_{r < R} x[r * ldx + c]
// mode 0: out[c] = s[c]                      (one row split; overwrite)
// mode 1: out[c] += s[c]  (float atomics)    (row splits; out pre-zeroed or a flat-gradient
//                                             region, ops/grad_sink.py)
// mode 2: out[c] = act(scale[c / E] * s[c] + bias[c % E])  (one row split; scale / bias
//                                             optional: the counts-GEMM bag epilogue)
// Block = QB column quads (4 consecutive columns: 16-byte fp32 / 8-byte bf16 loads) x
// RG = 256 / QB row groups; the row groups meet in LDS, then one store / atomic per column
// and block (<= 64 row splits: bounded same-address atomics).  blockIdx.y = row split.
template <typename TX, int QB, int VEC>
__global__ __launch_bounds__(256) void colsum_kernel(const TX* __restrict__ x, long R, long C, long ldx,
                                                     float* __restrict__ out, long rps, int mode,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ bias, int E, int act) {
  constexpr int RG = 256 / QB;
  __shared__ f32x4 red[RG][QB];
  const int qi = threadIdx.x % QB, rg = threadIdx.x / QB;
  const long c = VEC * ((long)blockIdx.x * QB + qi);
  const bool live = c < C;
  const long r0 = (long)blockIdx.y * rps;
  const long r1 = min(R, r0 + rps);
  auto ld4 = [&](long r) -> f32x4 {
    if constexpr (VEC == 1) {
      if constexpr (sizeof(TX) == 4) return f32x4{reinterpret_cast<const float*>(x)[r * ldx + c], 0.f, 0.f, 0.f};
      else return f32x4{bf16_to_f32(reinterpret_cast<const unsigned short*>(x)[r * ldx + c]), 0.f, 0.f, 0.f};
    } else if constexpr (sizeof(TX) == 4) {
      return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + r * ldx + c);
    } else {
      const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const unsigned short*>(x) + r * ldx + c);
      return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
                   __uint_as_float(u.y & 0xFFFF0000u)};
    }
  };
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  if (live) {
    long r = r0 + rg;
    for (; r + 3 * RG < r1; r += 4 * RG) {
      a0 += ld4(r);
      a1 += ld4(r + RG);
      a2 += ld4(r + 2 * RG);
      a3 += ld4(r + 3 * RG);
    }
    for (; r < r1; r += RG) a0 += ld4(r);
  }
  red[rg][qi] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (rg != 0 || !live) return;
  f32x4 s4 = red[0][qi];
#pragma unroll 4
  for (int g = 1; g < RG; ++g) s4 += red[g][qi];
  if (mode == 1) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) atomicAdd(out + c + k, s4[k]);
    return;
  }
  if (mode >= 2) {  // 3: scale holds bag lengths, the factor is 1 / max(len, 1) (bag mean)
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const long cc = c + k;
      float y = s4[k];
      if (scale) y *= mode == 3 ? 1.f / fmaxf(scale[cc / E], 1.f) : scale[cc / E];
      if (bias) y += bias[cc % E];
      s4[k] = act_fn(y, act);
    }
  }
  if constexpr (VEC == 4) *reinterpret_cast<f32x4*>(out + c) = s4;
  else out[c] = s4[0];
}

// ---- reference precision (dtype = "fp32"): fp32-exact GEMM on the fp32 MFMA ----------------
// C (M, N) = A (M, K) . B (K, N) [+ bias[n], act] with A(m, k) = A[m sam + k sak] and
// B(k, n) = B[k sbk + n sbn]: one kernel for the forward X W^T, the dgrad dZ W and the wgrad
// dZ^T X of the dense layers (reference Dense + Activation in fp32, cnn_dssm_th.py:136-138).
// v_mfma_f32_16x16x4_f32 (fp32 products and sums; no bf16 operand anywhere), 64 x 64 tiles,
// K-steps of 16 staged k-major in LDS (a fragment read is 16 consecutive m / n per lane group:
// conflict-free), 4 waves of 32 x 32, the next K-step fetched into registers during this one's
// MFMAs (one barrier per step).  blockIdx.z = split-K slice: slice z writes its own (M, N) slab
// at C + z M ldc without the epilogue (the column-sum kernel reduces the slabs in order).
// AK: sak == 1 (an A row is contiguous in k); BN1: sbn == 1 (a B row is contiguous in n): the
// staging map puts consecutive threads on the contiguous axis.
constexpr int FB = 64, FK = 16;
template <bool AK, bool BN1>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, long sam, long sak,
                                                       const float* __restrict__ B, long sbk, long sbn,
                                                       const float* __restrict__ bias, float* __restrict__ C, long ldc,
                                                       int M, int N, int K, int kper, int act, int accumulate) {
  __shared__ float As[2][FK][FB + 4];
  __shared__ float Bs[2][FK][FB + 4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.x * FB, n0 = blockIdx.y * FB;
  const int kb = blockIdx.z * kper, ke = min(K, kb + kper);
  // staging coordinates of this thread's 4 elements per operand (tile-relative)
  const int am = AK ? t >> 2 : (t & 15) * 4, ak = AK ? (t & 3) * 4 : t >> 4;
  const int bn = BN1 ? (t & 15) * 4 : t >> 2, bk = BN1 ? t >> 4 : (t & 3) * 4;
  float ra[4], rb[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int gm = m0 + am + (AK ? 0 : e), gk = k0 + ak + (AK ? e : 0);
      ra[e] = (gm < M && gk < ke) ? A[(long)gm * sam + (long)gk * sak] : 0.f;
      const int gn = n0 + bn + (BN1 ? e : 0), gk2 = k0 + bk + (BN1 ? 0 : e);
      rb[e] = (gn < N && gk2 < ke) ? B[(long)gk2 * sbk + (long)gn * sbn] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      As[buf][ak + (AK ? e : 0)][am + (AK ? 0 : e)] = ra[e];
      Bs[buf][bk + (BN1 ? 0 : e)][bn + (BN1 ? e : 0)] = rb[e];
    }
  };
  const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32, r16 = lane & 15, kq = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (kb < ke) {
    fetch(kb);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += FK) {
    const bool more = k0 + FK < ke;
    if (more) fetch(k0 + FK);
#pragma unroll
    for (int s = 0; s < FK / 4; ++s) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[buf][4 * s + kq][wm + 16 * i + r16];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[buf][4 * s + kq][wn + 16 * j + r16];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);  // buf ^ 1 was last read before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  const bool split = gridDim.z > 1;
  float* Cz = C + (size_t)blockIdx.z * M * ldc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm + 16 * i + 4 * kq + r;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + 16 * j + r16;
        if (n >= N) continue;
        float v = acc[i][j][r];
        float* o = Cz + (size_t)m * ldc + n;
        if (!split) {
          if (bias) v += bias[n];
          v = act_fn(v, act);
          if (accumulate) v += *o;
        }
        *o = v;
      }
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

// dW (N, K) partial slabs: rows [z * rows_per, (z + 1) * rows_per) of dz / x go to slab z,
// ws holds ceil(M / rows_per) * N * K floats; rows_per a multiple of 64; tile 64 or 128.
// zdt / xdt: 0 = fp32, 1 = bf16.
PV_API int pv_linear_wgrad(const void* dz, int zdt, const void* X, int xdt, float* ws, int M, int N, int K, int rows_per,
                           int tile, void* stream) {
  using namespace pv::dense;
  if (M < 1 || N < 1 || K < 1 || rows_per < BK || rows_per % BK || (tile != 64 && tile != 128)) return -1;
  dim3 grid((N + tile - 1) / tile, (K + tile - 1) / tile, (M + rows_per - 1) / rows_per);
  hipStream_t s = (hipStream_t)stream;
#define PV_WG(TZ, TXX)                                                                                           \
  if (tile == 64)                                                                                                \
    hipLaunchKernelGGL((linear_wgrad_kernel<TZ, TXX, 64>), grid, dim3(256), 0, s, (const TZ*)dz, (const TXX*)X, ws, \
                       M, N, K, rows_per);                                                                       \
  else                                                                                                           \
    hipLaunchKernelGGL((linear_wgrad_kernel<TZ, TXX, 128>), grid, dim3(256), 0, s, (const TZ*)dz, (const TXX*)X,    \
                       ws, M, N, K, rows_per)
  if (zdt == 0 && xdt == 0) { PV_WG(float, float); }
  else if (zdt == 0) { PV_WG(float, unsigned short); }
  else if (xdt == 0) { PV_WG(unsigned short, float); }
  else { PV_WG(unsigned short, unsigned short); }
#undef PV_WG
  PV_LAUNCH_CHECK();
  return 0;
}

// dx (M, K) fp32 = dz (M, N) . W (N, K): linear_act with W read transposed in its staging.
PV_API int pv_linear_dgrad(const void* dz, int zdt, const void* W, int wdt, float* dx, int M, int N, int K,
                           void* stream) {
  using namespace pv::dense;
  // GEMM view: rows M, out columns K (= the layer input width), reduction N
  dim3 grid((M + BM - 1) / BM, (K + BN - 1) / BN);
  hipStream_t s = (hipStream_t)stream;
#define PV_DG(TZ, TWW)                                                                                           \
  hipLaunchKernelGGL((linear_act_kernel<TZ, TWW, true>), grid, dim3(256), 0, s, (const TZ*)dz, (const TWW*)W, \
                     nullptr, dx, nullptr, M, K, N, N, K, 0)
  if (zdt == 0 && wdt == 0) PV_DG(float, float);
  else if (zdt == 0) PV_DG(float, unsigned short);
  else if (wdt == 0) PV_DG(unsigned short, float);
  else PV_DG(unsigned short, unsigned short);
#undef PV_DG
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

// ldy: row stride of dy in floats (>= D)
PV_API int pv_l2norm_bwd_ld(const float* y, const float* inv_norm, const float* x, const float* dy, long ldy, float* dx,
                            int M, int D, void* stream) {
  using namespace pv::dense;
  if (ldy < D) return -1;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, y, inv_norm, x, dy, dx,
                     M, D, ldy);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_l2norm_bwd(const float* y, const float* inv_norm, const float* x, const float* dy, float* dx, int M, int D,
                         void* stream) {
  return pv_l2norm_bwd_ld(y, inv_norm, x, dy, D, dx, M, D, stream);
}

PV_API int pv_act_bwd(const float* y, const float* dy, float* dz, long n, int act, void* stream) {
  using namespace pv::dense;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, y, dy, dz, n, act,
                     (unsigned short*)nullptr);
  PV_LAUNCH_CHECK();
  return 0;
}

// Bag-mean backward prologue in one pass: dz = dy * act'(y) (fp32, for the bias column sum;
// y may be null = no activation) and dz16 = bf16(dz / max(1, lens[row])) (the per-bag 1/len
// of the mean folded in; lens null = sum bags), rows of E columns.
__global__ void act_bwd_rowscale_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                        float* __restrict__ dz, unsigned short* __restrict__ dz16,
                                        const float* __restrict__ lens, long E, long n, int act) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    float g = dy[i];
    if (y) {
      if (act == pv::dense::ACT_RELU) g = y[i] > 0.f ? g : 0.f;
      else if (act == pv::dense::ACT_TANH) g = g * (1.f - y[i] * y[i]);
    }
    if (dz) dz[i] = g;
    const float s = lens ? 1.f / fmaxf(lens[i / E], 1.f) : 1.f;
    dz16[i] = f32_to_bf16(g * s);
  }
}

PV_API int pv_act_bwd_rowscale(const float* y, const float* dy, float* dz, void* dz16, const float* lens, long E,
                               long n, int act, void* stream) {
  using namespace pv::dense;
  if (E < 1 || n < 1 || !dz16) return -1;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(act_bwd_rowscale_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, y, dy, dz,
                     (unsigned short*)dz16, lens, E, n, act);
  PV_LAUNCH_CHECK();
  return 0;
}

// act_bwd writing dz (fp32) AND its bf16 copy dz16 in one pass
PV_API int pv_act_bwd2(const float* y, const float* dy, float* dz, void* dz16, long n, int act, void* stream) {
  using namespace pv::dense;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, y, dy, dz, n, act,
                     (unsigned short*)dz16);
  PV_LAUNCH_CHECK();
  return 0;
}

// xdt: 0 fp32, 1 bf16.  mode / epilogue: see colsum_kernel.  Narrow sums (bias gradients,
// C <= 4096) use 16 quads x 16 row groups per block, wide ones (split-K partials) 64 x 4;
// mode 1 adds row splits (<= 64) until the launch covers the chip.
PV_API int pv_colsum(const void* x, int xdt, long R, long C, long ldx, float* out, int mode, const float* scale,
                     const float* bias, int E, int act, void* stream) {
  using namespace pv::dense;
  if (R < 1 || C < 1) return -1;
  if (mode >= 2 && E < 1) return -2;
  if (mode > 3) return -3;
  // 4 columns per thread when rows and pointers allow 16-byte (fp32) / 8-byte (bf16) loads
  const bool vec = C % 4 == 0 && ldx % 4 == 0 && !((uintptr_t)out & 15) && !((uintptr_t)x & (xdt ? 7 : 15));
  const int V = vec ? 4 : 1;
  const long units = C / V;
  const bool narrow = units <= 1024 || !vec;  // the element-load variant exists at 16 quads only
  const int QB = narrow ? 16 : 64, RG = 256 / QB;
  const long gx = (units + QB - 1) / QB;
  long splits = 1;
  // deterministic mode (common.h): one row split, so each column gets a single atomic add
  // per launch (order-free) instead of <= 64 same-address ones
  if (mode == 1 && !pv::det_on()) {
    splits = (1024 + gx - 1) / gx;
    const long maxs = (R + 4 * RG - 1) / (4 * RG);  // >= 4 rows per thread
    if (splits > maxs) splits = maxs;
    if (splits > 64) splits = 64;
    if (splits < 1) splits = 1;
  }
  const long rps = (R + splits - 1) / splits;
  splits = (R + rps - 1) / rps;
  const dim3 grid((unsigned)gx, (unsigned)splits);
  hipStream_t st = (hipStream_t)stream;
#define PV_COLSUM(T, Q, VV)                                                                                    \
  hipLaunchKernelGGL((colsum_kernel<T, Q, VV>), grid, dim3(256), 0, st, (const T*)x, R, C, ldx, out, rps, mode, \
                     scale, bias, E, act)
  if (xdt == 1) {
    if (!vec) PV_COLSUM(unsigned short, 16, 1);
    else if (narrow) PV_COLSUM(unsigned short, 16, 4);
    else PV_COLSUM(unsigned short, 64, 4);
  } else {
    if (!vec) PV_COLSUM(float, 16, 1);
    else if (narrow) PV_COLSUM(float, 16, 4);
    else PV_COLSUM(float, 64, 4);
  }
#undef PV_COLSUM
  PV_LAUNCH_CHECK();
  return 0;
}

// fp32-exact GEMM (gemm_f32_kernel): C = A . B [+ bias, act], element strides as above; splits
// > 1: C holds `splits` (M, ldc) slabs of partial sums over K slices (no epilogue, no
// accumulate).  Both the A and B operands: one unit stride required (sak or sam, sbn or sbk).
PV_API int pv_gemm_f32(const float* A, long sam, long sak, const float* B, long sbk, long sbn, const float* bias,
                       float* C, long ldc, int M, int N, int K, int splits, int act, int accumulate, void* stream) {
  using namespace pv::dense;
  if (M < 1 || N < 1 || K < 1 || splits < 1 || ldc < N) return -1;
  if (splits > 1 && (accumulate || bias || act)) return -2;
  if ((sak != 1 && sam != 1) || (sbn != 1 && sbk != 1)) return -3;
  const int kper = ((K + splits - 1) / splits + FK - 1) / FK * FK;
  splits = (K + kper - 1) / kper;
  const dim3 grid((M + FB - 1) / FB, (N + FB - 1) / FB, splits);
  hipStream_t s = (hipStream_t)stream;
#define PV_GF(AKV, BNV)                                                                                     \
  hipLaunchKernelGGL((gemm_f32_kernel<AKV, BNV>), grid, dim3(256), 0, s, A, sam, sak, B, sbk, sbn, bias, C, ldc, \
                     M, N, K, kper, act, accumulate)
  if (sak == 1) {
    if (sbn == 1) PV_GF(true, true); else PV_GF(true, false);
  } else {
    if (sbn == 1) PV_GF(false, true); else PV_GF(false, false);
  }
#undef PV_GF
  PV_LAUNCH_CHECK();
  return 0;
}
