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
#include <algorithm>

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

// Dropout keep decisions of columns c..c+3 (c % 4 == 0) of a row, bit k = column c+k kept:
// the same counter hash as the conv kernels and ops/reference.py::dropout_keep_mask
// (thr % 16 == 0: nibble j of the group hash of g8 decides column 8*g8+j, common.h
// dropout_nibble; otherwise byte b of the group hash of g4 decides column 4*g4+b).  thr = round(256 p), scale = 256 / (256 - thr).
__device__ __forceinline__ unsigned keep4(unsigned hrow, int c, int thr) {
  unsigned bits = 0u;
  if ((thr & 15) == 0) {
    bits = (dropout_keep_bits8(dropout_group_hash(hrow, (unsigned)(c >> 3)), thr >> 4) >> (c & 7)) & 0xFu;
  } else {
    const unsigned h = dropout_group_hash(hrow, (unsigned)(c >> 2));
#pragma unroll
    for (int k = 0; k < 4; ++k) bits |= (((h >> (8 * k)) & 0xFFu) >= (unsigned)thr ? 1u : 0u) << k;
  }
  return bits;
}

// Wave-per-row fused  h = dropout(x) + r;  y = LayerNorm(h) * gamma + beta  for D = 256 * VPT.
// Lane l owns columns (i*64 + l)*4 .. +3 of every row (coalesced 8-byte accesses), the two
// row statistics are wave reductions (no LDS, no barriers), and the dropout mask is a
// counter hash of (seed, row, column) regenerated in the backward — nothing is stored.
// thr = 0: no dropout (the plain residual add + LayerNorm).
template <int VPT>
__global__ __launch_bounds__(256) void add_ln_drop_fwd_kernel(const unsigned short* __restrict__ x,
                                                              const unsigned short* __restrict__ r,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              unsigned short* __restrict__ y,
                                                              unsigned short* __restrict__ h,
                                                              float* __restrict__ mean_out,
                                                              float* __restrict__ rstd_out, int M, float eps,
                                                              int thr, float scale, unsigned seed,
                                                              const unsigned* __restrict__ seed_ptr,
                                                              const float* __restrict__ xb) {
  constexpr int D = 256 * VPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= M) return;
  if (seed_ptr) seed += *seed_ptr;
  const unsigned hrow = thr > 0 ? dropout_row_hash(seed, (unsigned)row) : 0u;
  float v[VPT][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 4;
    const size_t o = (size_t)row * D + c;
    const uint2 a = *reinterpret_cast<const uint2*>(x + o);
    v[i][0] = __uint_as_float(a.x << 16);
    v[i][1] = __uint_as_float(a.x & 0xFFFF0000u);
    v[i][2] = __uint_as_float(a.y << 16);
    v[i][3] = __uint_as_float(a.y & 0xFFFF0000u);
    if (xb) {  // the branch's linear-layer bias (its GEMM runs without one)
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(xb + c);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] += b4[k];
    }
    if (thr > 0) {
      const unsigned kb = keep4(hrow, c, thr);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = ((kb >> k) & 1u) ? v[i][k] * scale : 0.f;
    }
    if (r) {
      const uint2 b = *reinterpret_cast<const uint2*>(r + o);
      v[i][0] += __uint_as_float(b.x << 16);
      v[i][1] += __uint_as_float(b.x & 0xFFFF0000u);
      v[i][2] += __uint_as_float(b.y << 16);
      v[i][3] += __uint_as_float(b.y & 0xFFFF0000u);
    }
    // h is stored in bf16 and the backward reads it back: normalise the bf16-rounded sum
#pragma unroll
    for (int k = 0; k < 4; ++k) v[i][k] = bf16_to_f32(f32_to_bf16(v[i][k]));
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float mu = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) q += (v[i][k] - mu) * (v[i][k] - mu);
  const float rstd = rsqrtf(wave_sum(q) * (1.f / D) + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (i * 64 + lane) * 4;
    const size_t o = (size_t)row * D + c;
    const f32x4 g4 = *reinterpret_cast<const f32x4*>(gamma + c);
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(beta + c);
    float out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = (v[i][k] - mu) * rstd * g4[k] + b4[k];
    *reinterpret_cast<uint2*>(y + o) = uint2{pack_bf16x2(out[0], out[1]), pack_bf16x2(out[2], out[3])};
    if (h) *reinterpret_cast<uint2*>(h + o) = uint2{pack_bf16x2(v[i][0], v[i][1]), pack_bf16x2(v[i][2], v[i][3])};
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
}

// v2: RPW rows per wave with every row's x / r loads issued before any row's math (v1: one
// row per wave, 2 VPT loads in flight per lane, ~4.6 TB/s at the BERT shape); same per-row
// arithmetic, so the outputs are bit-identical to v1.
template <int VPT, int RPW>
__global__ __launch_bounds__(256) void add_ln_drop_fwd2_kernel(const unsigned short* __restrict__ x,
                                                               const unsigned short* __restrict__ r,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               unsigned short* __restrict__ y,
                                                               unsigned short* __restrict__ h,
                                                               float* __restrict__ mean_out,
                                                               float* __restrict__ rstd_out, int M, float eps,
                                                               int thr, float scale, unsigned seed,
                                                               const unsigned* __restrict__ seed_ptr,
                                                               const float* __restrict__ xb) {
  constexpr int D = 256 * VPT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row0 = (blockIdx.x * 4 + wave) * RPW;
  if (row0 >= M) return;
  if (seed_ptr) seed += *seed_ptr;
  uint2 xa[RPW][VPT], ra[RPW][VPT];
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = min(row0 + q, M - 1);  // clamped re-read; only rows < M are stored
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const size_t o = (size_t)row * D + (i * 64 + lane) * 4;
      xa[q][i] = *reinterpret_cast<const uint2*>(x + o);
      if (r) ra[q][i] = *reinterpret_cast<const uint2*>(r + o);
    }
  }
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row0 + q;
    if (row >= M) break;
    const unsigned hrow = thr > 0 ? dropout_row_hash(seed, (unsigned)row) : 0u;
    float v[VPT][4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 4;
      const uint2 a = xa[q][i];
      v[i][0] = __uint_as_float(a.x << 16);
      v[i][1] = __uint_as_float(a.x & 0xFFFF0000u);
      v[i][2] = __uint_as_float(a.y << 16);
      v[i][3] = __uint_as_float(a.y & 0xFFFF0000u);
      if (xb) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(xb + c);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[i][k] += b4[k];
      }
      if (thr > 0) {
        const unsigned kb = keep4(hrow, c, thr);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[i][k] = ((kb >> k) & 1u) ? v[i][k] * scale : 0.f;
      }
      if (r) {
        const uint2 b = ra[q][i];
        v[i][0] += __uint_as_float(b.x << 16);
        v[i][1] += __uint_as_float(b.x & 0xFFFF0000u);
        v[i][2] += __uint_as_float(b.y << 16);
        v[i][3] += __uint_as_float(b.y & 0xFFFF0000u);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = bf16_to_f32(f32_to_bf16(v[i][k]));
      s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    }
    const float mu = wave_sum(s) * (1.f / D);
    float qv = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) qv += (v[i][k] - mu) * (v[i][k] - mu);
    const float rstd = rsqrtf(wave_sum(qv) * (1.f / D) + eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int c = (i * 64 + lane) * 4;
      const size_t o = (size_t)row * D + c;
      const f32x4 g4 = *reinterpret_cast<const f32x4*>(gamma + c);
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(beta + c);
      float out[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) out[k] = (v[i][k] - mu) * rstd * g4[k] + b4[k];
      *reinterpret_cast<uint2*>(y + o) = uint2{pack_bf16x2(out[0], out[1]), pack_bf16x2(out[2], out[3])};
      if (h) *reinterpret_cast<uint2*>(h + o) = uint2{pack_bf16x2(v[i][0], v[i][1]), pack_bf16x2(v[i][2], v[i][3])};
    }
    if (lane == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rstd;
    }
  }
}

// Wave-per-row LayerNorm backward for D = 256 * VPT: each lane holds VPT 4-element
// vectors of dy and x_hat in registers (one read of each), the two row means are wave
// reductions (no barriers), and dgamma/dbeta accumulate in registers over the rows this
// wave owns; the 4 waves of a block combine through LDS and issue one atomic per column.
// PF = 1: the next row's dy / h / statistics are loaded before this row's math (the rows of a
// wave are gridDim.x * 4 apart, so without it each row's loads start only after the previous
// row's stores); same per-row arithmetic and accumulation order: bit-identical to PF = 0.
template <int VPT, int PF = 0>
__global__ __launch_bounds__(256) void layernorm_bwd_rows_kernel(const unsigned short* __restrict__ dy,
                                                                 const unsigned short* __restrict__ hsum,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd,
                                                                 unsigned short* __restrict__ dx,
                                                                 float* __restrict__ part, int M,
                                                                 unsigned short* __restrict__ dxm, int thr,
                                                                 float scale, unsigned seed,
                                                                 const unsigned* __restrict__ seed_ptr, int nparts) {
  constexpr int D = 256 * VPT;
  if (thr > 0 && seed_ptr) seed += *seed_ptr;
  __shared__ float red[3][4][D];
  const bool want_db = nparts == 3;  // column sums of the branch gradient (its bias gradient)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm[VPT][4], ga[VPT][4], gb[VPT][4], gc[VPT][4];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const f32x4 g4 = *reinterpret_cast<const f32x4*>(gamma + (i * 64 + lane) * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      gm[i][k] = g4[k];
      ga[i][k] = 0.f;
      gb[i][k] = 0.f;
      gc[i][k] = 0.f;
    }
  }
  const int rstride = gridDim.x * 4;
  uint2 gvn[VPT], hvn[VPT];
  float mun = 0.f, rsn = 0.f;
  if (PF && blockIdx.x * 4 + wave < M) {
    const int r = blockIdx.x * 4 + wave;
    mun = mean[r];
    rsn = rstd[r];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const size_t o = (size_t)r * D + (i * 64 + lane) * 4;
      gvn[i] = *reinterpret_cast<const uint2*>(dy + o);
      hvn[i] = *reinterpret_cast<const uint2*>(hsum + o);
    }
  }
  for (int row = blockIdx.x * 4 + wave; row < M; row += rstride) {
    float mu, rs;
    uint2 gvc[VPT], hvc[VPT];
    if (PF) {
      mu = mun;
      rs = rsn;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        gvc[i] = gvn[i];
        hvc[i] = hvn[i];
      }
      const int nr = row + rstride;
      if (nr < M) {
        mun = mean[nr];
        rsn = rstd[nr];
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
          const size_t o = (size_t)nr * D + (i * 64 + lane) * 4;
          gvn[i] = *reinterpret_cast<const uint2*>(dy + o);
          hvn[i] = *reinterpret_cast<const uint2*>(hsum + o);
        }
      }
    } else {
      mu = mean[row];
      rs = rstd[row];
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const size_t o = (size_t)row * D + (i * 64 + lane) * 4;
        gvc[i] = *reinterpret_cast<const uint2*>(dy + o);
        hvc[i] = *reinterpret_cast<const uint2*>(hsum + o);
      }
    }
    float g[VPT][4], xh[VPT][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const uint2 gv = gvc[i];
      const uint2 hv = hvc[i];
      const unsigned gw[2] = {gv.x, gv.y}, hw[2] = {hv.x, hv.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        g[i][k] = __uint_as_float((k & 1) ? (gw[k >> 1] & 0xFFFF0000u) : (gw[k >> 1] << 16));
        xh[i][k] = (__uint_as_float((k & 1) ? (hw[k >> 1] & 0xFFFF0000u) : (hw[k >> 1] << 16)) - mu) * rs;
        const float gg = g[i][k] * gm[i][k];
        a += gg;
        b += gg * xh[i][k];
        ga[i][k] += g[i][k] * xh[i][k];
        gb[i][k] += g[i][k];
      }
    }
    a = wave_sum(a) * (1.f / D);
    b = wave_sum(b) * (1.f / D);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      float o4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o4[k] = rs * (g[i][k] * gm[i][k] - a - xh[i][k] * b);
      *reinterpret_cast<uint2*>(dx + (size_t)row * D + (i * 64 + lane) * 4) =
          uint2{pack_bf16x2(o4[0], o4[1]), pack_bf16x2(o4[2], o4[3])};
      if (thr > 0) {  // gradient of the dropout branch: dh * keep * scale (mask regenerated)
        const unsigned kb = keep4(dropout_row_hash(seed, (unsigned)row), (i * 64 + lane) * 4, thr);
#pragma unroll
        for (int k = 0; k < 4; ++k) o4[k] = ((kb >> k) & 1u) ? o4[k] * scale : 0.f;
      }
      if (dxm)
        *reinterpret_cast<uint2*>(dxm + (size_t)row * D + (i * 64 + lane) * 4) =
            uint2{pack_bf16x2(o4[0], o4[1]), pack_bf16x2(o4[2], o4[3])};
      if (want_db) {
#pragma unroll
        for (int k = 0; k < 4; ++k) gc[i][k] += o4[k];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < VPT; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[0][wave][(i * 64 + lane) * 4 + k] = ga[i][k];
      red[1][wave][(i * 64 + lane) * 4 + k] = gb[i][k];
      red[2][wave][(i * 64 + lane) * 4 + k] = gc[i][k];
    }
  __syncthreads();
  // per-block partials part[block][0:D] = dgamma, [D:2D] = dbeta, [2D:3D] = dbias (colsum_*)
  float* pb = part + (size_t)blockIdx.x * nparts * D;
  for (int c = threadIdx.x; c < D; c += 256) {
    pb[c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pb[D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
    if (want_db) pb[2 * D + c] = red[2][0][c] + red[2][1][c] + red[2][2][c] + red[2][3][c];
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

// tanh(u) = 1 - 2 / (exp(2u) + 1): one v_exp + one v_rcp instead of libm tanhf
// tanh / sigmoid through v_exp_f32 and v_rcp_f32 (1 ulp): an IEEE fdiv / __frcp_rn is a
// ~10-instruction div_scale / div_fmas / div_fixup sequence per element, and these kernels
// are VALU-bound (~20 VALU per element) at the BERT shape; the results are rounded to bf16.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);
}

// tanh-GELU through s = sigmoid(2u), u = k (x + c x^3): gelu = x s, 1 + t = 2 s,
// 1 - t^2 = 4 s (1 - s), so gelu' = s + x s (1 - s) (2k + 6kc x^2) — one exp2 and one rcp
// (v_exp_f32 / v_rcp_f32) and six FMA-class ops per element.
constexpr float kGeluK = 0.7978845608028654f, kGeluC = 0.044715f, kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float gelu_sig2u(float x, float x2) {
  // sigmoid(2u) = 1 / (1 + 2^(-2 k log2e (x + c x^3)))
  const float e = __builtin_amdgcn_exp2f(x * fmaf(x2, -2.f * kGeluK * kGeluC * kLog2e, -2.f * kGeluK * kLog2e));
  return __builtin_amdgcn_rcpf(1.f + e);
}

__device__ __forceinline__ float gelu_tanh_grad_fast(float x) {
  const float x2 = x * x;
  const float sg = gelu_sig2u(x, x2);
  const float q = x * fmaf(x2, 6.f * kGeluK * kGeluC, 2.f * kGeluK);
  return fmaf(q, fmaf(-sg, sg, sg), sg);
}

// Vectorised bias-GELU backward: a thread owns 8 consecutive columns (16-byte loads and
// stores) for RPB rows; its bias-gradient partial goes to part[blockIdx.y][col] and
// colsum_kernel adds the partials in a fixed order (no atomics, deterministic).
// grid = (ceil(D/8/256), ceil(M/RPB)).
__global__ __launch_bounds__(256) void bias_gelu_bwd_vec_kernel(const unsigned short* __restrict__ x,
                                                                const float* __restrict__ b,
                                                                const unsigned short* __restrict__ dy,
                                                                unsigned short* __restrict__ dx,
                                                                float* __restrict__ part, int M, int D, int rpb) {
  const int c8 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c8 >= D) return;
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  float bc[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    bc[k] = b[c8 + k];
    acc[k] = 0.f;
  }
  for (int row = r0; row < r1; ++row) {
    const size_t o = (size_t)row * D + c8;
    const u32x4 xv = *reinterpret_cast<const u32x4*>(x + o);
    const u32x4 gv = *reinterpret_cast<const u32x4*>(dy + o);
    u32x4 out;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float x0 = __uint_as_float(xv[w] << 16) + bc[2 * w];
      const float x1 = __uint_as_float(xv[w] & 0xFFFF0000u) + bc[2 * w + 1];
      const float g0 = __uint_as_float(gv[w] << 16) * gelu_tanh_grad_fast(x0);
      const float g1 = __uint_as_float(gv[w] & 0xFFFF0000u) * gelu_tanh_grad_fast(x1);
      acc[2 * w] += g0;
      acc[2 * w + 1] += g1;
      out[w] = pack_bf16x2(g0, g1);
    }
    *reinterpret_cast<u32x4*>(dx + o) = out;
  }
  float* pr = part + (size_t)blockIdx.y * D + c8;
  *reinterpret_cast<f32x4*>(pr) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *reinterpret_cast<f32x4*>(pr + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

// v2 of the two vector kernels: 128-thread blocks (D = 3072 is 384 column octets = 3 full
// blocks; the 256-thread v1 left half of its second block idle) and U rows' loads issued
// before any of their math (v1 kept 2 loads in flight per thread, ~4.5 TB/s at the BERT shape)
template <int U>
__global__ __launch_bounds__(128) void bias_gelu_bwd_vec2_kernel(const unsigned short* __restrict__ x,
                                                                 const float* __restrict__ b,
                                                                 const unsigned short* __restrict__ dy,
                                                                 unsigned short* __restrict__ dx,
                                                                 float* __restrict__ part, int M, int D, int rpb) {
  const int c8 = (blockIdx.x * 128 + threadIdx.x) * 8;
  if (c8 >= D) return;
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + c8), b1 = *reinterpret_cast<const f32x4*>(b + c8 + 4);
  const float bc[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  for (int row = r0; row < r1; row += U) {
    u32x4 xv[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t o = (size_t)min(row + u, r1 - 1) * D + c8;  // clamped: a re-read, never stored twice
      xv[u] = *reinterpret_cast<const u32x4*>(x + o);
      gv[u] = *reinterpret_cast<const u32x4*>(dy + o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (row + u >= r1) break;
      u32x4 out;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float x0 = __uint_as_float(xv[u][w] << 16) + bc[2 * w];
        const float x1 = __uint_as_float(xv[u][w] & 0xFFFF0000u) + bc[2 * w + 1];
        const float g0 = __uint_as_float(gv[u][w] << 16) * gelu_tanh_grad_fast(x0);
        const float g1 = __uint_as_float(gv[u][w] & 0xFFFF0000u) * gelu_tanh_grad_fast(x1);
        acc[2 * w] += g0;
        acc[2 * w + 1] += g1;
        out[w] = pack_bf16x2(g0, g1);
      }
      *reinterpret_cast<u32x4*>(dx + (size_t)(row + u) * D + c8) = out;
    }
  }
  float* pr = part + (size_t)blockIdx.y * D + c8;
  *reinterpret_cast<f32x4*>(pr) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *reinterpret_cast<f32x4*>(pr + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

// BERT embedding front end over the packed token batch (ops/transformer.py::bert_embed): token
// t of group g (rows off_g .. off_g + N_g L_g, position (t - off_g) mod L_g) gets
// bf16(word[id] + pos[l] + typ0) — one pass instead of the fp32 gather, two broadcast adds, a
// cast and a cat.  A thread owns 8 columns of a row.
struct EmbedGroups {
  int off[4], L[4], n;
};

__global__ __launch_bounds__(256) void bert_embed_fwd_kernel(const int* __restrict__ ids, const float* __restrict__ word,
                                                             const float* __restrict__ pos,
                                                             const float* __restrict__ typ0,
                                                             unsigned short* __restrict__ out, long T, int H,
                                                             EmbedGroups gr) {
  const int c8n = H / 8;
  const long total = T * c8n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long t = i / c8n;
    const int c = (int)(i - t * c8n) * 8;
    int g = 0;
    while (g + 1 < gr.n && t >= gr.off[g + 1]) ++g;
    const int l = (int)((t - gr.off[g]) % gr.L[g]);
    const float* w = word + (size_t)ids[t] * H + c;
    const float* pp = pos + (size_t)l * H + c;
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(w), w1 = *reinterpret_cast<const f32x4*>(w + 4);
    const f32x4 p0 = *reinterpret_cast<const f32x4*>(pp), p1 = *reinterpret_cast<const f32x4*>(pp + 4);
    const f32x4 y0 = *reinterpret_cast<const f32x4*>(typ0 + c), y1 = *reinterpret_cast<const f32x4*>(typ0 + c + 4);
    u32x4 o;
    o[0] = pack_bf16x2(w0[0] + p0[0] + y0[0], w0[1] + p0[1] + y0[1]);
    o[1] = pack_bf16x2(w0[2] + p0[2] + y0[2], w0[3] + p0[3] + y0[3]);
    o[2] = pack_bf16x2(w1[0] + p1[0] + y1[0], w1[1] + p1[1] + y1[1]);
    o[3] = pack_bf16x2(w1[2] + p1[2] + y1[2], w1[3] + p1[3] + y1[3]);
    *reinterpret_cast<u32x4*>(out + (size_t)t * H + c) = o;
  }
}

// word-table gradient: out[id[t]] += g[t] (fp32 atomics from the bf16 rows); an all-zero
// 8-column piece (padding tokens: masked keys and unused queries carry exactly zero
// gradient) issues no atomics, so the padding row is not a contention hot spot
__global__ __launch_bounds__(256) void bert_embed_wgrad_kernel(const int* __restrict__ ids,
                                                               const unsigned short* __restrict__ g,
                                                               float* __restrict__ out, long T, int H) {
  // one wave per token row, lanes on consecutive columns: each atomic instruction covers 64
  // consecutive floats (2 cache lines; an 8-columns-per-lane layout spreads one instruction
  // over 16 lines and measured 1.5 ms slower per BERT step)
  const int lane = threadIdx.x & 63;
  const long nw = (long)gridDim.x * (blockDim.x >> 6);
  for (long t = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < T; t += nw) {
    const unsigned short* gr = g + (size_t)t * H;
    float* o = out + (size_t)ids[t] * H;
    for (int c = lane; c < H; c += 64) {
      const unsigned short b = gr[c];
      if (b & 0x7FFF) atomicAdd(o + c, __uint_as_float((unsigned)b << 16));
    }
  }
}

// Column sums in a fixed order, two stages: colsum_part (grid (ceil(D/64), S)) reduces
// a 1/S slice of the rows of 64 columns with 4 row lanes + LDS into part2[S][D];
// colsum_final adds the S partials.
constexpr int kColSplits = 32;
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ part, float* __restrict__ part2,
                                                          int R, int D, int ld) {
  __shared__ float sh[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  part += (size_t)blockIdx.z * D;  // grid.z: several column sets of one row layout in one launch
  part2 += (size_t)blockIdx.z * gridDim.y * D;
  float a = 0.f;
  if (c < D)
    for (int r = r0 + ty; r < r1; r += 4) a += part[(size_t)r * ld + c];
  sh[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < D) part2[(size_t)blockIdx.y * D + c] = sh[0][tx] + sh[1][tx] + sh[2][tx] + sh[3][tx];
}

// final split sums of up to 3 column sets (grid.y = set) -> out0 / out1 / out2
__global__ void colsum_final3_kernel(const float* __restrict__ part2, float* __restrict__ out0,
                                     float* __restrict__ out1, float* __restrict__ out2, int S, int D) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  const int set = blockIdx.y;
  const float* p = part2 + (size_t)set * S * D;
  float a = 0.f;
  for (int s = 0; s < S; ++s) a += p[(size_t)s * D + c];
  (set == 0 ? out0 : set == 1 ? out1 : out2)[c] = a;
}

__global__ void colsum_final_kernel(const float* __restrict__ part2, float* __restrict__ out, int S, int D) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float a = 0.f;
  for (int s = 0; s < S; ++s) a += part2[(size_t)s * D + c];
  out[c] = a;
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

// x * sigmoid(2u) == 0.5 x (1 + tanh u): one v_exp + one v_rcp, no libm tanhf
__device__ __forceinline__ float gelu_tanh_fast(float x) { return x * gelu_sig2u(x, x * x); }

// Vectorised bias + GELU forward (D % 8 == 0): a thread owns 8 consecutive columns
// (16-byte loads / stores, its 8 bias values in registers) for RPB rows.  The scalar kernel
// above spent its time in a 64-bit `i % D` and libm tanhf per element pair (VALU-bound at
// ~3 TB/s); grid = (ceil(D / 8 / 128), ceil(M / RPB)), 128 threads.
constexpr int kGeluFwdRpb = 16;
__global__ __launch_bounds__(128) void bias_gelu_fwd_vec_kernel(const unsigned short* __restrict__ x,
                                                                const float* __restrict__ b,
                                                                unsigned short* __restrict__ y, int M, int D) {
  const int c8 = blockIdx.x * 128 + threadIdx.x;
  if (c8 * 8 >= D) return;
  const int col = c8 * 8;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + col), b1 = *reinterpret_cast<const f32x4*>(b + col + 4);
  const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  const int r0 = blockIdx.y * kGeluFwdRpb, r1 = min(M, r0 + kGeluFwdRpb);
  for (int r = r0; r < r1; ++r) {
    const size_t o = (size_t)r * D + col;
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + o);
    u32x4 w;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a0 = __uint_as_float(v[k] << 16) + bb[2 * k];
      const float a1 = __uint_as_float(v[k] & 0xFFFF0000u) + bb[2 * k + 1];
      w[k] = pack_bf16x2(gelu_tanh_fast(a0), gelu_tanh_fast(a1));
    }
    *reinterpret_cast<u32x4*>(y + o) = w;
  }
}

template <int U>
__global__ __launch_bounds__(128) void bias_gelu_fwd_vec2_kernel(const unsigned short* __restrict__ x,
                                                                 const float* __restrict__ b,
                                                                 unsigned short* __restrict__ y, int M, int D,
                                                                 int rpb) {
  const int col = (blockIdx.x * 128 + threadIdx.x) * 8;
  if (col >= D) return;
  const f32x4 b0 = *reinterpret_cast<const f32x4*>(b + col), b1 = *reinterpret_cast<const f32x4*>(b + col + 4);
  const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  const int r0 = blockIdx.y * rpb, r1 = min(M, r0 + rpb);
  for (int r = r0; r < r1; r += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const u32x4*>(x + (size_t)min(r + u, r1 - 1) * D + col);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r + u >= r1) break;
      u32x4 w;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a0 = __uint_as_float(v[u][k] << 16) + bb[2 * k];
        const float a1 = __uint_as_float(v[u][k] & 0xFFFF0000u) + bb[2 * k + 1];
        w[k] = pack_bf16x2(gelu_tanh_fast(a0), gelu_tanh_fast(a1));
      }
      *reinterpret_cast<u32x4*>(y + (size_t)(r + u) * D + col) = w;
    }
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

// Register-resident variant for L = 256 * NV4 / 4 ... : lane holds NV4 4-element vectors of
// its row (8-byte loads), the row is read and written exactly once.
template <int NV4>
__global__ __launch_bounds__(256) void softmax_fwd_reg_kernel(unsigned short* __restrict__ S,
                                                              const int* __restrict__ mask, long R, int L,
                                                              int rows_per_item, float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  unsigned short* s = S + row * L;
  const int* mk = mask ? mask + (row / rows_per_item) * L : nullptr;
  float v[NV4][4];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV4; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < L) {
      const uint2 a = *reinterpret_cast<const uint2*>(s + c);
      const int4 m4 = mk ? *reinterpret_cast<const int4*>(mk + c) : int4{1, 1, 1, 1};
      v[i][0] = m4.x ? __uint_as_float(a.x << 16) * scale : -INFINITY;
      v[i][1] = m4.y ? __uint_as_float(a.x & 0xFFFF0000u) * scale : -INFINITY;
      v[i][2] = m4.z ? __uint_as_float(a.y << 16) * scale : -INFINITY;
      v[i][3] = m4.w ? __uint_as_float(a.y & 0xFFFF0000u) * scale : -INFINITY;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[i][k] = -INFINITY;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) mx = fmaxf(mx, v[i][k]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < NV4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[i][k] = v[i][k] == -INFINITY ? 0.f : __expf(v[i][k] - mx);
      sum += v[i][k];
    }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int i = 0; i < NV4; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < L)
      *reinterpret_cast<uint2*>(s + c) =
          uint2{pack_bf16x2(v[i][0] * inv, v[i][1] * inv), pack_bf16x2(v[i][2] * inv, v[i][3] * inv)};
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

template <int NV4>
__global__ __launch_bounds__(256) void softmax_bwd_reg_kernel(const unsigned short* __restrict__ P,
                                                              unsigned short* __restrict__ dP, long R, int L,
                                                              float scale) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const unsigned short* p = P + row * L;
  unsigned short* d = dP + row * L;
  float pv[NV4][4], dv[NV4][4];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < NV4; ++i) {
    const int c = (i * 64 + lane) * 4;
    uint2 a = {0u, 0u}, b = {0u, 0u};
    if (c < L) {
      a = *reinterpret_cast<const uint2*>(p + c);
      b = *reinterpret_cast<const uint2*>(d + c);
    }
    pv[i][0] = __uint_as_float(a.x << 16);
    pv[i][1] = __uint_as_float(a.x & 0xFFFF0000u);
    pv[i][2] = __uint_as_float(a.y << 16);
    pv[i][3] = __uint_as_float(a.y & 0xFFFF0000u);
    dv[i][0] = __uint_as_float(b.x << 16);
    dv[i][1] = __uint_as_float(b.x & 0xFFFF0000u);
    dv[i][2] = __uint_as_float(b.y << 16);
    dv[i][3] = __uint_as_float(b.y & 0xFFFF0000u);
#pragma unroll
    for (int k = 0; k < 4; ++k) dot += pv[i][k] * dv[i][k];
  }
  dot = wave_sum(dot);
#pragma unroll
  for (int i = 0; i < NV4; ++i) {
    const int c = (i * 64 + lane) * 4;
    if (c < L) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = scale * pv[i][k] * (dv[i][k] - dot);
      *reinterpret_cast<uint2*>(d + c) = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
    }
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

static int ln_blocks(int M) { return std::min(512, std::max(1, (M + 3) / 4)); }

static bool ln_rows_ok(int D) { return D == 256 || D == 512 || D == 768 || D == 1024; }

// floats of workspace pv_layernorm_bwd needs (0: the generic kernel accumulates into
// zeroed dgamma/dbeta with atomics)
PV_API long pv_layernorm_bwd_ws(int M, int D) {
  return ln_rows_ok(D) ? (long)ln_blocks(M) * 3 * D + 3L * pv::tfm::kColSplits * D : 0;  // room for dbias
}

namespace {
int g_ln_rpw = 2;     // pv_ln_set_rpw: rows per wave of the add + LN forward (1 = the v1 kernel)
int g_ln_bwd_pf = 1;  // pv_ln_bwd_set_pf: next-row prefetch in the LN backward (0 = round-3 kernel)
}  // namespace

// dgamma/dbeta are overwritten on the wave-per-row path (D in {256,512,768,1024}, ws given)
static int layernorm_bwd_impl(const void* dy, const void* hsum, const float* gamma, const float* mean,
                              const float* rstd, void* dx, float* dgamma, float* dbeta, float* ws, int M, int D,
                              void* dxm, int thr, float scale, unsigned seed, const unsigned* seed_ptr, float* dxb,
                              void* stream) {
  const int blocks = ln_blocks(M);
  hipStream_t st = (hipStream_t)stream;
#define PV_LN_ROWS(VPT)                                                                                          \
  {                                                                                                              \
    const int np = dxb ? 3 : 2;                                                                                  \
    if (g_ln_bwd_pf)                                                                                             \
      hipLaunchKernelGGL((pv::tfm::layernorm_bwd_rows_kernel<VPT, 1>), dim3(blocks), dim3(256), 0, st,             \
                         (const unsigned short*)dy, (const unsigned short*)hsum, gamma, mean, rstd,              \
                         (unsigned short*)dx, ws, M, (unsigned short*)dxm, thr, scale, seed, seed_ptr, np);      \
    else                                                                                                         \
    hipLaunchKernelGGL(pv::tfm::layernorm_bwd_rows_kernel<VPT>, dim3(blocks), dim3(256), 0, st,                  \
                       (const unsigned short*)dy, (const unsigned short*)hsum, gamma, mean, rstd,                \
                       (unsigned short*)dx, ws, M, (unsigned short*)dxm, thr, scale, seed, seed_ptr, np);        \
    PV_LAUNCH_CHECK();                                                                                           \
    float* ws2 = ws + (size_t)blocks * np * D;                                                                   \
    hipLaunchKernelGGL(pv::tfm::colsum_part_kernel, dim3((D + 63) / 64, pv::tfm::kColSplits, np), dim3(256), 0,  \
                       st, ws, ws2, blocks, D, np * D);                                                          \
    PV_LAUNCH_CHECK();                                                                                           \
    hipLaunchKernelGGL(pv::tfm::colsum_final3_kernel, dim3((D + 255) / 256, np), dim3(256), 0, st, ws2, dgamma,  \
                       dbeta, dxb, pv::tfm::kColSplits, D);                                                      \
    PV_LAUNCH_CHECK();                                                                                           \
    return 0;                                                                                                    \
  }
  if (ws) {
    switch (D) {
      case 256: PV_LN_ROWS(1)
      case 512: PV_LN_ROWS(2)
      case 768: PV_LN_ROWS(3)
      case 1024: PV_LN_ROWS(4)
      default: break;
    }
  }
  switch (D) {
    case 256: { PV_LN_ROWS(1) }
    case 512: { PV_LN_ROWS(2) }
    case 768: { PV_LN_ROWS(3) }
    case 1024: { PV_LN_ROWS(4) }
    default: break;
  }
#undef PV_LN_ROWS
  if (dxm || dxb || thr > 0) return -1;  // the fused variants exist on the wave-per-row path only
  const int rpb = 32;
  hipLaunchKernelGGL(pv::tfm::layernorm_bwd_kernel, dim3((M + rpb - 1) / rpb), dim3(256), 2 * D * sizeof(float),
                     (hipStream_t)stream, (const unsigned short*)dy, (const unsigned short*)hsum, gamma, mean, rstd,
                     (unsigned short*)dx, dgamma, dbeta, M, D, rpb);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_layernorm_bwd(const void* dy, const void* hsum, const float* gamma, const float* mean, const float* rstd,
                            void* dx, float* dgamma, float* dbeta, float* ws, int M, int D, void* stream) {
  return layernorm_bwd_impl(dy, hsum, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, D, nullptr, 0, 1.f, 0u, nullptr,
                            nullptr, stream);
}

// dx = dL/dh (the residual input's gradient), dxm = dx * keep * scale (the dropout branch's;
// null when thr = 0: then the branch gradient IS dx), keep regenerated from (seed + *seed_ptr,
// row, column) exactly as pv_add_ln_drop_fwd drew it; dxb (optional) = column sums of the
// branch gradient = the gradient of the bias pv_add_ln_drop_fwd added to x.
PV_API int pv_layernorm_bwd_drop(const void* dy, const void* hsum, const float* gamma, const float* mean,
                                 const float* rstd, void* dx, void* dxm, float* dgamma, float* dbeta, float* dxb,
                                 float* ws, int M, int D, int thr, float scale, unsigned seed,
                                 const unsigned* seed_ptr, void* stream) {
  if (!ws || !ln_rows_ok(D) || (thr > 0 && !dxm)) return -1;
  return layernorm_bwd_impl(dy, hsum, gamma, mean, rstd, dx, dgamma, dbeta, ws, M, D, dxm, thr, scale, seed,
                            seed_ptr, dxb, stream);
}

PV_API void pv_ln_bwd_set_pf(int on) { g_ln_bwd_pf = on; }

PV_API void pv_ln_set_rpw(int rpw) { g_ln_rpw = rpw; }

// Wave-per-row residual add (+ optional dropout on x) + LayerNorm, D in {256, 512, 768, 1024}.
PV_API int pv_add_ln_drop_fwd(const void* x, const float* xb, const void* r, const float* gamma, const float* beta,
                              void* y, void* h, float* mean, float* rstd, int M, int D, float eps, int thr, float scale,
                              unsigned seed, const unsigned* seed_ptr, void* stream) {
  if (!ln_rows_ok(D) || thr < 0 || thr > 255) return -1;
  hipStream_t st = (hipStream_t)stream;
  if (g_ln_rpw == 2 || g_ln_rpw == 4) {
    const int rpw = g_ln_rpw;
    const dim3 g2((M + 4 * rpw - 1) / (4 * rpw));
#define PV_ADDLN2(VPT, RPWV)                                                                                        hipLaunchKernelGGL((pv::tfm::add_ln_drop_fwd2_kernel<VPT, RPWV>), g2, dim3(256), 0, st,                                              (const unsigned short*)x, (const unsigned short*)r, gamma, beta, (unsigned short*)y,                               (unsigned short*)h, mean, rstd, M, eps, thr, scale, seed, seed_ptr, xb)
#define PV_ADDLN2_D(RPWV)                   switch (D) {                                case 256: PV_ADDLN2(1, RPWV); break;      case 512: PV_ADDLN2(2, RPWV); break;      case 768: PV_ADDLN2(3, RPWV); break;      default: PV_ADDLN2(4, RPWV); break;     }
    if (rpw == 2) { PV_ADDLN2_D(2) } else { PV_ADDLN2_D(4) }
#undef PV_ADDLN2_D
#undef PV_ADDLN2
    PV_LAUNCH_CHECK();
    return 0;
  }
  const dim3 grid((M + 3) / 4);
#define PV_ADDLN(VPT)                                                                                          \
  hipLaunchKernelGGL(pv::tfm::add_ln_drop_fwd_kernel<VPT>, grid, dim3(256), 0, st, (const unsigned short*)x,  \
                     (const unsigned short*)r, gamma, beta, (unsigned short*)y, (unsigned short*)h, mean, rstd, \
                     M, eps, thr, scale, seed, seed_ptr, xb)
  switch (D) {
    case 256: PV_ADDLN(1); break;
    case 512: PV_ADDLN(2); break;
    case 768: PV_ADDLN(3); break;
    default: PV_ADDLN(4); break;
  }
#undef PV_ADDLN
  PV_LAUNCH_CHECK();
  return 0;
}

namespace {
// pv_gelu_set_v: 1 = the round-2 vector kernels; 2 (default) = the 128-thread unrolled backward
// (296 vs 316 us per BERT layer call) with the v1 forward; 3 = the unrolled forward too
// (183 vs 174 us: slower; tools/gelu_micro.py, profiles/r5_final/gelu_micro.log)
int g_gelu_v = 2;
constexpr int kGelu2Rpb = 32;
}  // namespace

PV_API void pv_gelu_set_v(int v) { g_gelu_v = v; }

PV_API int pv_bias_gelu_fwd(const void* x, const float* b, void* y, long n, int D, void* stream) {
  if (D % 2) return -1;
  if (g_gelu_v == 3 && D % 8 == 0 && n / D <= 0x7FFFFFFFL) {  // measured slower than v1 (183 vs 174 us)
    const int M = (int)(n / D);
    dim3 grid((D / 8 + 127) / 128, (M + kGelu2Rpb - 1) / kGelu2Rpb);
    hipLaunchKernelGGL(pv::tfm::bias_gelu_fwd_vec2_kernel<4>, grid, dim3(128), 0, (hipStream_t)stream,
                       (const unsigned short*)x, b, (unsigned short*)y, M, D, kGelu2Rpb);
    PV_LAUNCH_CHECK();
    return 0;
  }
  if (D % 8 == 0 && n / D <= 0x7FFFFFFFL) {
    const int M = (int)(n / D);
    dim3 grid((D / 8 + 127) / 128, (M + pv::tfm::kGeluFwdRpb - 1) / pv::tfm::kGeluFwdRpb);
    hipLaunchKernelGGL(pv::tfm::bias_gelu_fwd_vec_kernel, grid, dim3(128), 0, (hipStream_t)stream,
                       (const unsigned short*)x, b, (unsigned short*)y, M, D);
    PV_LAUNCH_CHECK();
    return 0;
  }
  long blocks = (n / 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(pv::tfm::bias_gelu_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)x, b, (unsigned short*)y, n, D);
  PV_LAUNCH_CHECK();
  return 0;
}

static constexpr int kGeluRpb = 16;

// floats of workspace pv_bias_gelu_bwd needs (vector path)
PV_API long pv_bias_gelu_bwd_ws(int M, int D) {
  return (long)((M + kGeluRpb - 1) / kGeluRpb + pv::tfm::kColSplits) * D;
}

// db is overwritten on the vector path (D % 8 == 0, ws != null), accumulated otherwise.
PV_API int pv_bias_gelu_bwd(const void* x, const float* b, const void* dy, void* dx, float* db, float* ws, int M,
                            int D, void* stream) {
  if (D % 8 == 0 && ws) {
    const int rpb = g_gelu_v >= 2 ? kGelu2Rpb : kGeluRpb, R = (M + rpb - 1) / rpb;  // kGelu2Rpb >= kGeluRpb
    if (g_gelu_v >= 2) {
      dim3 grid((D / 8 + 127) / 128, R);
      hipLaunchKernelGGL(pv::tfm::bias_gelu_bwd_vec2_kernel<4>, grid, dim3(128), 0, (hipStream_t)stream,
                         (const unsigned short*)x, b, (const unsigned short*)dy, (unsigned short*)dx, ws, M, D, rpb);
    } else {
      dim3 grid((D / 8 + 255) / 256, R);
      hipLaunchKernelGGL(pv::tfm::bias_gelu_bwd_vec_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)x, b, (const unsigned short*)dy, (unsigned short*)dx, ws, M, D, rpb);
    }
    PV_LAUNCH_CHECK();
    float* ws2 = ws + (size_t)R * D;
    hipLaunchKernelGGL(pv::tfm::colsum_part_kernel, dim3((D + 63) / 64, pv::tfm::kColSplits), dim3(256), 0,
                       (hipStream_t)stream, ws, ws2, R, D, D);
    PV_LAUNCH_CHECK();
    hipLaunchKernelGGL(pv::tfm::colsum_final_kernel, dim3((D + 255) / 256), dim3(256), 0, (hipStream_t)stream, ws2, db,
                       pv::tfm::kColSplits, D);
    PV_LAUNCH_CHECK();
    return 0;
  }
  const int rpb = 64;
  hipLaunchKernelGGL(pv::tfm::bias_gelu_bwd_kernel, dim3((M + rpb - 1) / rpb), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)x, b, (const unsigned short*)dy, (unsigned short*)dx, db, M, D, rpb);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_softmax_fwd(void* S, const int* mask, long R, int L, int rows_per_item, float scale, void* stream) {
  const dim3 grid((unsigned)((R + 3) / 4));
  if (L % 4 == 0 && L <= 512) {
    if (L <= 256)
      hipLaunchKernelGGL(pv::tfm::softmax_fwd_reg_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream,
                         (unsigned short*)S, mask, R, L, rows_per_item, scale);
    else
      hipLaunchKernelGGL(pv::tfm::softmax_fwd_reg_kernel<2>, grid, dim3(256), 0, (hipStream_t)stream,
                         (unsigned short*)S, mask, R, L, rows_per_item, scale);
    PV_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(pv::tfm::softmax_fwd_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (unsigned short*)S, mask, R, L, rows_per_item, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_softmax_bwd(const void* P, void* dP, long R, int L, float scale, void* stream) {
  if (L % 4 == 0 && L <= 512) {
    const dim3 grid((unsigned)((R + 3) / 4));
    if (L <= 256)
      hipLaunchKernelGGL(pv::tfm::softmax_bwd_reg_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)P, (unsigned short*)dP, R, L, scale);
    else
      hipLaunchKernelGGL(pv::tfm::softmax_bwd_reg_kernel<2>, grid, dim3(256), 0, (hipStream_t)stream,
                         (const unsigned short*)P, (unsigned short*)dP, R, L, scale);
    PV_LAUNCH_CHECK();
    return 0;
  }
  hipLaunchKernelGGL(pv::tfm::softmax_bwd_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)P, (unsigned short*)dP, R, L, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// Packed BERT embedding front end (bert_embed_fwd_kernel): ids (T) int32, word (V, H) / pos
// (Lmax, H) / typ0 (H) fp32, out (T, H) bf16; groups: ng <= 4 (offset, L) pairs, offsets
// ascending from 0.  H % 8 == 0.
PV_API int pv_bert_embed_fwd(const int* ids, const float* word, const float* pos, const float* typ0, void* out, long T,
                             int H, const int* offs, const int* lens, int ng, void* stream) {
  if (T <= 0 || H % 8 || ng < 1 || ng > 4) return -1;
  pv::tfm::EmbedGroups gr{};
  for (int i = 0; i < ng; ++i) {
    gr.off[i] = offs[i];
    gr.L[i] = lens[i];
    if (lens[i] <= 0) return -2;
  }
  gr.n = ng;
  const long total = T * (H / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pv::tfm::bert_embed_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ids,
                     word, pos, typ0, (unsigned short*)out, T, H, gr);
  PV_LAUNCH_CHECK();
  return 0;
}

// out (V, H) fp32 += rows of g (T, H) bf16 at ids (atomics; all-zero pieces skipped)
PV_API int pv_bert_embed_wgrad(const int* ids, const void* g, float* out, long T, int H, void* stream) {
  if (T <= 0 || H % 8) return -1;
  long blocks = (T + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pv::tfm::bert_embed_wgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ids,
                     (const unsigned short*)g, out, T, H);
  PV_LAUNCH_CHECK();
  return 0;
}
