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
//       ib_fwd      : per (query block, doc split) partial sum_j exp(S_ij - g)  -> atomics
//                     (no running max needed: clip bounds S to [0, g] (or [-g, g]), so
//                     exp(S - g) <= 1 and the sum cannot overflow)
//       ib_bwd<ROW> : recompute the S tile, G = gscale*g*P*clip'  (bf16, via LDS),
//                     then dQ += G.Dn  (ROW=true, rows=queries)  or
//                          dD += G^T.Qn (ROW=false, rows=docs) with MFMA; partial
//                     results of each split are added with fp32 atomics.
//       ib_pos      : the positive logit (same bf16 inputs) and the one-hot term of
//                     the gradient, -gscale*g*clip' * {d_pos, q}.
#include "common.h"

namespace pv {
namespace loss {

constexpr float BCE_EPS = 1e-7f;

// q: (B, D) normalised, d: (B, 1+J, D) normalised (positive first).
__global__ __launch_bounds__(256) void dssm_explicit_kernel(const float* __restrict__ q, const float* __restrict__ d,
                                                            float* __restrict__ loss, float* __restrict__ prob,
                                                            float* __restrict__ dq, float* __restrict__ dd, int B,
                                                            int J1, int D, float gamma, float gscale, int clip) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  constexpr int MAXJ = 16, MAXD = 8;  // J+1 <= 16, D <= 512
  float qv[MAXD];
  const float* qr = q + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < MAXD; ++i) {
    int c = lane + 64 * i;
    qv[i] = c < D ? qr[c] : 0.f;
  }
  float R[MAXJ], S[MAXJ];
  float mx = -INFINITY;
  for (int j = 0; j < J1; ++j) {
    const float* dr = d + ((size_t)row * J1 + j) * D;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
      int c = lane + 64 * i;
      if (c < D) s += qv[i] * dr[c];
    }
    s = wave_sum(s);
    R[j] = clip ? fminf(fmaxf(s, 0.f), 1.f) : s;
    S[j] = gamma * R[j];
    mx = fmaxf(mx, S[j]);
  }
  float den = 0.f;
  for (int j = 0; j < J1; ++j) den += __expf(S[j] - mx);
  const float P0 = __expf(S[0] - mx) / den;
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
  for (int j = 0; j < J1; ++j) {
    const float Pj = __expf(S[j] - mx) / den;
    float dS = live ? (Pj - (j == 0 ? 1.f : 0.f)) * gscale : 0.f;
    float r = R[j];
    float dR = dS * gamma;
    if (clip) {
      // recompute the raw cosine to decide the clip pass-through (inclusive bounds, as T.clip)
      const float* dr = d + ((size_t)row * J1 + j) * D;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < MAXD; ++i) {
        int c = lane + 64 * i;
        if (c < D) s += qv[i] * dr[c];
      }
      s = wave_sum(s);
      (void)r;
      if (s < 0.f || s > 1.f) dR = 0.f;
    }
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

// S tile for one wave: rows r0..r0+31 (2 subtiles), cols 0..63 of the LDS tile (4 subtiles).
// a: row fragments [2][KS] (registers); ytile: [TD][DP+PADK] bf16 in LDS.
template <int KS>
__device__ __forceinline__ void s_tile(const bf16x8 (&a)[2][KS], const unsigned short* ytile, int ldy,
                                       f32x4 (&acc)[2][4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bf16x8 b = *reinterpret_cast<const bf16x8*>(ytile + (c * 16 + (lane & 15)) * ldy + s * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][s], b, acc[i][c], 0, 0, 0);
    }
  }
}

template <int KS>
__global__ __launch_bounds__(256) void ib_fwd_kernel(const unsigned short* __restrict__ X,  // (nx, DP) queries
                                                     const unsigned short* __restrict__ Y,  // (ny, DP) docs
                                                     float* __restrict__ sumexp, int nx, int ny, int per_split,
                                                     float gamma, int clip) {
  constexpr int DP = KS * 32, LDY = DP + PADK;
  __shared__ __attribute__((aligned(16))) unsigned short yt[TD * LDY];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * TQ + wave * 32;
  const int c_begin = blockIdx.y * per_split, c_end = min(ny, c_begin + per_split);
  bf16x8 a[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int r = r0 + i * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      a[i][s] = r < nx ? *reinterpret_cast<const bf16x8*>(X + (size_t)r * DP + s * 32 + (lane >> 4) * 8)
                       : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  float rs[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int c0 = c_begin; c0 < c_end; c0 += TD) {
    __syncthreads();
    for (int q = threadIdx.x; q < TD * (DP / 8); q += 256) {
      int r = q / (DP / 8), cc = (q % (DP / 8)) * 8;
      u32x4 v = (c0 + r < c_end) ? *reinterpret_cast<const u32x4*>(Y + (size_t)(c0 + r) * DP + cc) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<u32x4*>(yt + r * LDY + cc) = v;
    }
    __syncthreads();
    f32x4 acc[2][4];
    s_tile<KS>(a, yt, LDY, acc);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool cv = c0 + c * 16 + (lane & 15) < c_end;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float r = acc[i][c][k];
          if (clip) r = fminf(fmaxf(r, 0.f), 1.f);
          rs[i][k] += cv ? __expf(gamma * (r - 1.f)) : 0.f;
        }
    }
  }
  // reduce over the 16 column lanes (xor 1,2,4,8), lanes with (lane&15)==0 write rows 4*(lane>>4)+k
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = rs[i][k];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      int r = r0 + i * 16 + 4 * (lane >> 4) + k;
      if ((lane & 15) == 0 && r < nx) atomicAdd(&sumexp[r], v);
    }
}

// ROW = true : rows = queries (X=Qn), cols = docs (Y=Dn), out = dQ, scale per row
// ROW = false: rows = docs (X=Dn),    cols = queries (Y=Qn), out = dD, scale per col
// scale[i] = gscale_i * gamma / sumexp_i (per query). G = scale * exp(g*(clip(R)-1)) * clip'(R)
template <int KS, bool ROW>
__global__ __launch_bounds__(256) void ib_bwd_kernel(const unsigned short* __restrict__ X,   // (nx, DP)
                                                     const unsigned short* __restrict__ Y,   // (ny, DP)
                                                     const unsigned short* __restrict__ YT,  // (DP, ny)
                                                     const float* __restrict__ scale, float* __restrict__ out,
                                                     int nx, int ny, int per_split, float gamma, int clip) {
  constexpr int DP = KS * 32, LDY = DP + PADK, LDT = TD + PADK, NC = DP / 16;
  __shared__ __attribute__((aligned(16))) unsigned short yt[TD * LDY];     // [col][feat]
  __shared__ __attribute__((aligned(16))) unsigned short ytt[DP * LDT];    // [feat][col]
  __shared__ __attribute__((aligned(16))) unsigned short gt[4][32 * LDT];  // per-wave G tile [row][col]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * TQ + wave * 32;
  const int c_begin = blockIdx.y * per_split, c_end = min(ny, c_begin + per_split);
  bf16x8 a[2][KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int r = r0 + i * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      a[i][s] = r < nx ? *reinterpret_cast<const bf16x8*>(X + (size_t)r * DP + s * 32 + (lane >> 4) * 8)
                       : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  float rsc[2][4];
  if (ROW) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int r = r0 + i * 16 + 4 * (lane >> 4) + k;
        rsc[i][k] = r < nx ? scale[r] : 0.f;
      }
  }
  f32x4 o[2][NC];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int n = 0; n < NC; ++n) o[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned short* gw = gt[wave];

  for (int c0 = c_begin; c0 < c_end; c0 += TD) {
    __syncthreads();
    for (int q = threadIdx.x; q < TD * (DP / 8); q += 256) {
      int r = q / (DP / 8), cc = (q % (DP / 8)) * 8;
      u32x4 v = (c0 + r < c_end) ? *reinterpret_cast<const u32x4*>(Y + (size_t)(c0 + r) * DP + cc) : u32x4{0, 0, 0, 0};
      *reinterpret_cast<u32x4*>(yt + r * LDY + cc) = v;
    }
    for (int q = threadIdx.x; q < DP * (TD / 8); q += 256) {
      int f = q / (TD / 8), cc = (q % (TD / 8)) * 8;
      u32x4 v = u32x4{0, 0, 0, 0};
      if (c0 + cc + 8 <= c_end && (ny & 7) == 0) v = *reinterpret_cast<const u32x4*>(YT + (size_t)f * ny + c0 + cc);
      else {
        unsigned short tmp[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) tmp[t] = (c0 + cc + t < c_end) ? YT[(size_t)f * ny + c0 + cc + t] : 0;
        v = *reinterpret_cast<u32x4*>(tmp);
      }
      *reinterpret_cast<u32x4*>(ytt + f * LDT + cc) = v;
    }
    __syncthreads();
    f32x4 acc[2][4];
    s_tile<KS>(a, yt, LDY, acc);
    // G tile -> LDS (bf16), row-major [32 rows][64 cols]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int col = c0 + c * 16 + (lane & 15);
      const bool cv = col < c_end;
      const float csc = (!ROW && cv) ? scale[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float r = acc[i][c][k];
          bool pass = !clip || (r >= 0.f && r <= 1.f);
          float rc = clip ? fminf(fmaxf(r, 0.f), 1.f) : r;
          float sc = ROW ? rsc[i][k] : csc;
          float g = (cv && pass) ? sc * __expf(gamma * (rc - 1.f)) : 0.f;
          gw[(i * 16 + 4 * (lane >> 4) + k) * LDT + c * 16 + (lane & 15)] = f32_to_bf16(g);
        }
    }
    // o[rows][feat] += G[rows][cols] . Y[cols][feat]  (A from gw, B from ytt)
#pragma unroll
    for (int s = 0; s < TD / 32; ++s) {
      bf16x8 ga[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        ga[i] = *reinterpret_cast<const bf16x8*>(gw + (i * 16 + (lane & 15)) * LDT + s * 32 + (lane >> 4) * 8);
#pragma unroll
      for (int n = 0; n < NC; ++n) {
        bf16x8 b = *reinterpret_cast<const bf16x8*>(ytt + (n * 16 + (lane & 15)) * LDT + s * 32 + (lane >> 4) * 8);
#pragma unroll
        for (int i = 0; i < 2; ++i) o[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ga[i], b, o[i][n], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int n = 0; n < NC; ++n)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int r = r0 + i * 16 + 4 * (lane >> 4) + k;
        int f = n * 16 + (lane & 15);
        float v = o[i][n][k];
        if (r < nx && v != 0.f) atomicAdd(&out[(size_t)r * DP + f], v);
      }
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

// Row-materialised variant for wide vectors (D > 192, e.g. BERT's 768) or small M: the
// (B x M) cosine matrix S comes from a hipBLASLt GEMM; one wave per row computes the
// log-sum-exp, the loss and the full logit gradient dS = gscale*g*(P - onehot)*clip'
// in place (the two products dQ = dS.D, dD = dS^T.Q are again library GEMMs).
__global__ __launch_bounds__(256) void ib_rows_kernel(float* __restrict__ S, const int* __restrict__ pos,
                                                      const float* __restrict__ gscale, float* __restrict__ loss,
                                                      int B, int M, float gamma, int clip) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float* s = S + (size_t)row * M;
  float sum = 0.f;
  for (int c = lane; c < M; c += 64) {
    float r = s[c];
    if (clip) r = fminf(fmaxf(r, 0.f), 1.f);
    sum += __expf(gamma * (r - 1.f));
  }
  sum = wave_sum(sum);
  const int p = pos[row];
  float rp = s[p];
  if (clip) rp = fminf(fmaxf(rp, 0.f), 1.f);
  if (lane == 0 && loss) loss[row] = gamma + __logf(sum) - gamma * rp;
  if (!gscale) return;
  const float g = gscale[row] * gamma;
  for (int c = lane; c < M; c += 64) {
    const float raw = s[c];
    const bool pass = !clip || (raw >= 0.f && raw <= 1.f);
    const float r = clip ? fminf(fmaxf(raw, 0.f), 1.f) : raw;
    const float P = __expf(gamma * (r - 1.f)) / sum;
    s[c] = pass ? g * (P - (c == p ? 1.f : 0.f)) : 0.f;
  }
}

// bf16 transpose (n, DP) -> (DP, n)
__global__ void transpose_bf16_kernel(const unsigned short* __restrict__ in, unsigned short* __restrict__ out, int n,
                                      int DP) {
  __shared__ unsigned short t[32][33];
  int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    int r = bx + k, c = by + tx;
    t[k][tx] = (r < n && c < DP) ? in[(size_t)r * DP + c] : 0;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    int c = by + k, r = bx + tx;
    if (c < DP && r < n) out[(size_t)c * n + r] = t[tx][k];
  }
}

}  // namespace loss
}  // namespace pv

using namespace pv;

PV_API int pv_dssm_explicit(const float* q, const float* d, float* loss, float* prob, float* dq, float* dd, int B,
                            int J1, int D, float gamma, float gscale, int clip, void* stream) {
  if (J1 > 16 || D > 512) return -1;
  hipLaunchKernelGGL(pv::loss::dssm_explicit_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, q, d, loss,
                     prob, dq, dd, B, J1, D, gamma, gscale, clip);
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

PV_API int pv_ib_fwd(const void* X, const void* Y, float* sumexp, int nx, int ny, int DP, float gamma, int clip,
                     void* stream) {
  using namespace pv::loss;
  if (DP % 32) return -2;
  int ns = ib_splits(nx, ny, 256);
  int per = ((ny + ns - 1) / ns + TD - 1) / TD * TD;
  ns = (ny + per - 1) / per;
  dim3 grid((nx + TQ - 1) / TQ, ns);
  IB_DISPATCH(DP / 32, hipLaunchKernelGGL(ib_fwd_kernel<KS>, grid, dim3(256), 0, (hipStream_t)stream,
                                          (const unsigned short*)X, (const unsigned short*)Y, sumexp, nx, ny, per,
                                          gamma, clip));
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_ib_bwd(const void* X, const void* Y, const void* YT, const float* scale, float* out, int nx, int ny,
                     int DP, float gamma, int clip, int row_scale, void* stream) {
  using namespace pv::loss;
  if (DP % 32 || DP > 192) return -2;
  int ns = ib_splits(nx, ny, 256);
  int per = ((ny + ns - 1) / ns + TD - 1) / TD * TD;
  ns = (ny + per - 1) / per;
  dim3 grid((nx + TQ - 1) / TQ, ns);
  hipStream_t s = (hipStream_t)stream;
  if (row_scale) {
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib_bwd_kernel<KS, true>), grid, dim3(256), 0, s, (const unsigned short*)X,
                                            (const unsigned short*)Y, (const unsigned short*)YT, scale, out, nx, ny,
                                            per, gamma, clip));
  } else {
    IB_DISPATCH(DP / 32, hipLaunchKernelGGL((ib_bwd_kernel<KS, false>), grid, dim3(256), 0, s,
                                            (const unsigned short*)X, (const unsigned short*)Y,
                                            (const unsigned short*)YT, scale, out, nx, ny, per, gamma, clip));
  }
  PV_LAUNCH_CHECK();
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

PV_API int pv_ib_rows(float* S, const int* pos, const float* gscale, float* loss, int B, int M, float gamma, int clip,
                      void* stream) {
  hipLaunchKernelGGL(pv::loss::ib_rows_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, S, pos, gscale,
                     loss, B, M, gamma, clip);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_transpose_bf16(const void* in, void* out, int n, int DP, void* stream) {
  dim3 grid((n + 31) / 32, (DP + 31) / 32);
  hipLaunchKernelGGL(pv::loss::transpose_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)in, (unsigned short*)out, n, DP);
  PV_LAUNCH_CHECK();
  return 0;
}
