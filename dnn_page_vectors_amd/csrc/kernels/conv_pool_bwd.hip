// K3b + K1b: sparse backward of gather -> dropout -> conv -> global-max-pool -> ReLU.
//
// Because of the global max-pool (cnn_dssm_th.py:94, pool_length = L-k+1) the
// gradient of filter f of sample n reaches exactly ONE window: a = argmax[n,f].
// With g[n,f] = dL/dpooled[n,f] * [pooled[n,f] > 0] (ReLU) and s = 1/(1-p):
//
//   db[f]          = sum_n g[n,f]
//   dW[f,j,e]      = s * sum_n g[n,f] * Xm[n, a+j, e]          (Xm = masked bf16 rows)
//   dTable[v,e]   += s * g[n,f] * W[f,j,e] * m[n,a+j,e]        for v = ids[n, a+j]
//
// Cost is O(N * F * k * E), independent of L (the dense Keras/Theano backward is
// O(N * L * F * k * E)).  The dropout mask m is regenerated from the counter hash
// (same function as the forward staging), never stored.
//
// dTable without 17M x 400-byte float atomics:
//   emit   : one thread per (n, f) writes up to k small entries
//            {key = token id, row = n*L + a + j, fj = f<<2|j, g} (sentinel key = V);
//   sort   : stable radix sort of (key, entry index) (sort.hip);
//   reduce : each wave walks a fixed chunk of sorted entries, recomputes the
//            contribution s*g*W[f,j,:]*m on the fly (W is L2-resident) and sums it
//            in registers per token; one row-atomic per (chunk, token) boundary.
#include "common.h"

namespace pv {
namespace convbwd {
PV_DEBUG_FLAG

constexpr int EP = 104;
constexpr int FW = 150;

__device__ __forceinline__ unsigned mask_byte(unsigned hr, int e, int token_mode) {
  return token_mode ? (hr & 0xFF) : ((dropout_group_hash(hr, (unsigned)(e >> 2)) >> (8 * (e & 3))) & 0xFF);
}

// ---- dW, db -----------------------------------------------------------------------
// grid (2*FW, nsplit), block 256 (4 waves).  Each wave takes its samples 64 at a time:
// lane l loads sample (base+l)'s g / ReLU flag / argmax and the k token ids of its
// argmax window (independent loads, issued together), then the wave walks the live
// samples with v_readlane broadcasts.  Lane l owns the 4-element groups q = l, l+64 of
// the (k x EP) window (EP % 4 == 0, so a group never crosses rows and ONE group hash
// yields its 4 dropout bytes); table loads for 4 samples are issued before use.
template <int K>
__device__ __forceinline__ void dw_filter(const float* __restrict__ gpool, const float* __restrict__ pooled,
                                          const int* __restrict__ argmax, const int* __restrict__ ids,
                                          const unsigned short* __restrict__ table, float* __restrict__ dw,
                                          float* __restrict__ db, float* red, int L, int E, int V, int fg, int fl,
                                          int n0, int n1, unsigned seed, unsigned row_offset, int thr, int token_mode,
                                          float scale) {
  constexpr int NG = K * EP / 4;  // groups per window
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float gsum = 0.f;
  int jj[2], ee[2];
  bool gv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = lane + 64 * i;
    jj[i] = (q * 4) / EP;
    ee[i] = (q * 4) % EP;
    gv[i] = q < NG && ee[i] < E;
  }
  for (int base = n0 + wave * 64; base < n1; base += 256) {
    const int n = base + lane;
    float g = 0.f;
    int a = 0;
    bool live = false;
    int tok[4] = {-1, -1, -1, -1};
    if (n < n1) {
      const size_t o = (size_t)n * (2 * FW) + fg;
      g = gpool[o];
      live = pooled[o] > 0.f && g != 0.f;
      a = argmax[o];
      if (live) {
#pragma unroll
        for (int j = 0; j < K; ++j) tok[j] = (a + j < L) ? ids[(size_t)n * L + a + j] : -1;
      }
    }
    gsum += live ? g : 0.f;
    unsigned long long m = __ballot(live);
    while (m) {
      int sl[4];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sl[u] = m ? (int)__builtin_ctzll(m) : -1;
        if (m) { m &= m - 1; ++cnt; }
      }
      uint2 raw[4][2];
      unsigned hh[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) break;
        const int s_ = sl[u];
        const int a_ = __builtin_amdgcn_readlane(a, s_);
        const int nn = base + s_;
        int tj[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) tj[j] = __builtin_amdgcn_readlane(tok[j], s_);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int t = jj[i] == 0 ? tj[0] : jj[i] == 1 ? tj[1] : jj[i] == 2 ? tj[2] : tj[3];
          const bool ok = gv[i] && t >= 0 && t < V;
          raw[u][i] = ok ? *reinterpret_cast<const uint2*>(table + (size_t)t * EP + ee[i]) : uint2{0u, 0u};
          unsigned h = 0xFFFFFFFFu;
          if (thr > 0) {
            const unsigned hr = dropout_row_hash(seed, row_offset + (unsigned)(nn * L + a_ + jj[i]));
            h = token_mode ? (hr & 0xFF) * 0x01010101u : dropout_group_hash(hr, (unsigned)(ee[i] >> 2));
          }
          hh[u][i] = h;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) break;
        const float gj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), sl[u]));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const unsigned h = hh[u][i];
          const uint2 r = raw[u][i];
          float x0 = __uint_as_float(r.x << 16), x1 = __uint_as_float(r.x & 0xFFFF0000u);
          float x2 = __uint_as_float(r.y << 16), x3 = __uint_as_float(r.y & 0xFFFF0000u);
          if (thr > 0) {
            x0 = ((int)(h & 0xFF) >= thr) ? x0 : 0.f;
            x1 = ((int)((h >> 8) & 0xFF) >= thr) ? x1 : 0.f;
            x2 = ((int)((h >> 16) & 0xFF) >= thr) ? x2 : 0.f;
            x3 = ((int)(h >> 24) >= thr) ? x3 : 0.f;
          }
          acc[i][0] += gj * x0;
          acc[i][1] += gj * x1;
          acc[i][2] += gj * x2;
          acc[i][3] += gj * x3;
        }
      }
    }
  }
  // cross-wave reduction through LDS: red[wave][K*EP]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = lane + 64 * i;
    if (q < NG) {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[wave * (K * EP) + q * 4 + c] = acc[i][c];
    }
  }
  const float gs = wave_sum(gsum);
  __syncthreads();
  for (int x = threadIdx.x; x < K * EP; x += 256) {
    float v = red[x] + red[K * EP + x] + red[2 * K * EP + x] + red[3 * K * EP + x];
    int j = x / EP, e = x % EP;
    if (e < E && v != 0.f) atomicAdd(&dw[((size_t)fl * K + j) * E + e], v * scale);
  }
  __shared__ float gsw[4];
  if (lane == 0) gsw[wave] = gs;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = gsw[0] + gsw[1] + gsw[2] + gsw[3];
    if (t != 0.f) atomicAdd(&db[fg], t);
  }
}

__global__ __launch_bounds__(256) void conv_bwd_dw_kernel(const float* gpool, const float* pooled, const int* argmax,
                                                          const int* ids, const unsigned short* table, float* dw3,
                                                          float* dw4, float* db, int N, int L, int E, int V, int nsplit,
                                                          unsigned seed, unsigned row_offset, int thr,
                                                          int token_mode, float scale) {
  __shared__ float red[4 * 4 * EP];
  const int f = blockIdx.x;
  const int per = ((N + nsplit - 1) / nsplit + 255) / 256 * 256;
  const int n0 = blockIdx.y * per, n1 = min(N, n0 + per);
  if (f < FW)
    dw_filter<3>(gpool, pooled, argmax, ids, table, dw3, db, red, L, E, V, f, f, n0, n1, seed, row_offset, thr,
                 token_mode, scale);
  else
    dw_filter<4>(gpool, pooled, argmax, ids, table, dw4, db, red, L, E, V, f, f - FW, n0, n1, seed, row_offset, thr,
                 token_mode, scale);
}

// ---- dTable: emit ------------------------------------------------------------------
// 4 slots per (n,f) pair; slot j >= k or dead (ReLU / g == 0 / t >= L) gets key = V.
__global__ __launch_bounds__(256) void conv_bwd_emit_kernel(const float* gpool, const float* pooled,
                                                            const int* argmax, const int* ids, unsigned* keys,
                                                            unsigned* vals, unsigned* erow, unsigned* efj, float* eg,
                                                            int N, int L, int V) {
  const long pair = (long)blockIdx.x * 256 + threadIdx.x;
  if (pair >= (long)N * 2 * FW) return;
  const int n = (int)(pair / (2 * FW)), f = (int)(pair % (2 * FW));
  const int K = f < FW ? 3 : 4;
  const float g = gpool[pair];
  const bool live = pooled[pair] > 0.f && g != 0.f;
  const int a = argmax[pair];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long s = pair * 4 + j;
    const int t = a + j;
    const bool ok = live && j < K && t < L;
    const int v = ok ? ids[(size_t)n * L + t] : V;
    PV_CHECK(v >= 0 && v <= V, PV_ERR_ID);
    keys[s] = (unsigned)v < (unsigned)V ? (unsigned)v : (unsigned)V;  // invalid ids: zero rows, as in fwd
    vals[s] = (unsigned)s;
    erow[s] = (unsigned)(n * L + t);
    efj[s] = (unsigned)((f << 2) | j);
    eg[s] = g;
  }
}

// ---- dTable: reduce over sorted entries ----------------------------------------------
// One wave per chunk of 64 sorted entries.  The entry metadata is loaded lane-parallel
// (lane i <- entry b+i: key, f/j, g, row hash) so the per-entry loop has no dependent
// global loads: entries are broadcast with v_readlane (uniform loop index) and lane l owns
// the contiguous columns e = l, l+64 (coalesced W loads and row atomics).
// Dropout bits: an entry needs ceil(E/4) group hashes; per PAIR of entries each lane of
// half h computes the group hash (lane&31) of entry j0+h (one mix32 for two entries),
// and the lanes fetch their groups' hashes with ds_bpermute — instead of every lane
// hashing both of its columns for every entry.  W values are fetched for 8 entries
// before they are used (W is L2-resident).
__global__ __launch_bounds__(256) void conv_bwd_reduce_kernel(const unsigned* __restrict__ skeys,
                                                              const unsigned* __restrict__ svals,
                                                              const unsigned* __restrict__ erow,
                                                              const unsigned* __restrict__ efj,
                                                              const float* __restrict__ eg, const float* __restrict__ w3,
                                                              const float* __restrict__ w4, float* __restrict__ dtable,
                                                              long M, int E, int V, unsigned seed, unsigned row_offset,
                                                              int thr, int token_mode, float scale) {
  const int lane = threadIdx.x & 63;
  const long chunk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long b = chunk * 64;
  if (b >= M) return;
  const long i = b + lane;
  unsigned key = (unsigned)V, fj = 0, hr = 0;
  float g = 0.f;
  if (i < M) {
    key = skeys[i];
    PV_CHECK(key <= (unsigned)V, PV_ERR_KEY);
    if (key < (unsigned)V) {
      const unsigned idx = svals[i];
      fj = efj[idx];
      g = eg[idx] * scale;
      if (thr > 0) hr = dropout_row_hash(seed, row_offset + erow[idx]);
    }
  }
  const unsigned long long live = __ballot(key < (unsigned)V);
  const int n = __popcll(live);  // sorted: live entries are a prefix of the chunk
  if (n == 0) return;
  const int c0 = lane, c1 = lane + 64;
  const bool h0 = c0 < E, h1 = c1 < E;
  // bpermute byte addresses of the lanes holding my two groups' hashes (per half)
  const int src0 = (c0 >> 2) * 4, src1 = ((c1 >> 2) & 31) * 4 + (c1 >= 128 ? 0 : 0);
  const int sh0 = 8 * (c0 & 3), sh1 = 8 * (c1 & 3);
  unsigned cur = __builtin_amdgcn_readfirstlane(key);
  float s0 = 0.f, s1 = 0.f;
  for (int j0 = 0; j0 < n; j0 += 8) {
    float wv0[8], wv1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int jj = min(j0 + u, n - 1);
      const unsigned f_j = (unsigned)__builtin_amdgcn_readlane((int)fj, jj);
      const int f = (int)(f_j >> 2), j = (int)(f_j & 3);
      const float* w = f < FW ? (w3 + ((size_t)f * 3 + j) * E) : (w4 + ((size_t)(f - FW) * 4 + j) * E);
      wv0[u] = h0 ? w[c0] : 0.f;
      wv1[u] = h1 ? w[c1] : 0.f;
    }
    unsigned hv[8];
    if (thr > 0 && !token_mode) {
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        const int ja = min(j0 + u, n - 1), jb = min(j0 + u + 1, n - 1);
        const unsigned ha = (unsigned)__builtin_amdgcn_readlane((int)hr, ja);
        const unsigned hb = (unsigned)__builtin_amdgcn_readlane((int)hr, jb);
        const unsigned gh = dropout_group_hash(lane < 32 ? ha : hb, (unsigned)(lane & 31));
        // entry A's groups live in lanes 0..31, entry B's in lanes 32..63
        const unsigned a0 = (unsigned)__builtin_amdgcn_ds_bpermute(src0, (int)gh);
        const unsigned a1 = (unsigned)__builtin_amdgcn_ds_bpermute(src1, (int)gh);
        const unsigned b0 = (unsigned)__builtin_amdgcn_ds_bpermute(src0 + 128, (int)gh);
        const unsigned b1 = (unsigned)__builtin_amdgcn_ds_bpermute(src1 + 128, (int)gh);
        hv[u] = (((a0 >> sh0) & 0xFF) << 8) | ((a1 >> sh1) & 0xFF);
        hv[u + 1] = (((b0 >> sh0) & 0xFF) << 8) | ((b1 >> sh1) & 0xFF);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int jj = j0 + u;
      if (jj >= n) break;
      const unsigned k = (unsigned)__builtin_amdgcn_readlane((int)key, jj);
      if (k != cur) {
        if (h0) atomicAdd(&dtable[(size_t)cur * E + c0], s0);
        if (h1) atomicAdd(&dtable[(size_t)cur * E + c1], s1);
        s0 = s1 = 0.f;
        cur = k;
      }
      const float gj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), jj));
      float v0 = gj * wv0[u], v1 = gj * wv1[u];
      if (thr > 0) {
        unsigned m0, m1;
        if (token_mode) {
          m0 = m1 = (unsigned)__builtin_amdgcn_readlane((int)hr, jj) & 0xFF;
        } else {
          m0 = hv[u] >> 8;
          m1 = hv[u] & 0xFF;
        }
        if ((int)m0 < thr) v0 = 0.f;
        if ((int)m1 < thr) v1 = 0.f;
      }
      s0 += v0;
      s1 += v1;
    }
  }
  if (h0) atomicAdd(&dtable[(size_t)cur * E + c0], s0);
  if (h1) atomicAdd(&dtable[(size_t)cur * E + c1], s1);
}

PV_DEBUG_EXPORT(convbwd)
}  // namespace convbwd
}  // namespace pv

using namespace pv;

PV_API int pv_conv_pool_bwd_dw(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                               const void* table, float* dw3, float* dw4, float* db, int N, int L, int E, int V,
                               unsigned seed, unsigned row_offset, int thr, int token_mode, float scale,
                               void* stream) {
  using namespace pv::convbwd;
  if (E > EP || L < 4) return -1;
  int nsplit = (N + 255) / 256;
  if (nsplit > 64) nsplit = 64;
  if (nsplit < 1) nsplit = 1;
  hipLaunchKernelGGL(conv_bwd_dw_kernel, dim3(2 * FW, nsplit), dim3(256), 0, (hipStream_t)stream, gpool, pooled,
                     argmax, ids, (const unsigned short*)table, dw3, dw4, db, N, L, E, V, nsplit, seed, row_offset, thr,
                     token_mode, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// Entries: M = N*2*FW*4 slots.
PV_API int pv_conv_pool_bwd_emit(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                 unsigned* keys, unsigned* vals, unsigned* erow, unsigned* efj, float* eg, int N,
                                 int L, int V, void* stream) {
  using namespace pv::convbwd;
  long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_bwd_emit_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     gpool, pooled, argmax, ids, keys, vals, erow, efj, eg, N, L, V);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_conv_pool_bwd_reduce(const unsigned* skeys, const unsigned* svals, const unsigned* erow,
                                   const unsigned* efj, const float* eg, const float* w3, const float* w4,
                                   float* dtable, long M, int E, int V, unsigned seed, unsigned row_offset, int thr,
                                   int token_mode, float scale, void* stream) {
  using namespace pv::convbwd;
  if (E > 128) return -1;
  long chunks = (M + 63) / 64;
  hipLaunchKernelGGL(conv_bwd_reduce_kernel, dim3((unsigned)((chunks + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, skeys, svals, erow, efj, eg, w3, w4, dtable, M, E, V, seed, row_offset,
                     thr, token_mode, scale);
  PV_LAUNCH_CHECK();
  return 0;
}
