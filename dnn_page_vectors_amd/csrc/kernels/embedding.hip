// K0 / K1: device featurizer (letter-trigram hashing) and embedding-bag kernels.
//
// * trigram_hash: ASCII-cleaned text bytes (N, Lmax) + lengths -> hashed trigram ids
//   (N, L), id = 1 + fnv1a(3 bytes) % (V-1), PAD = 0.  Same function as the C++
//   featurizer (csrc/runtime/featurize.cpp) restricted to single-byte code points, so
//   the host can ship raw bytes and let the GPU hash them (DSSM "word hashing").
// * embedding_bag: out[n,:] = scale_n * sum_{t: ids[n,t] != pad} W[ids[n,t], :] — the
//   multi-hot x W1 first layer of the DSSM MLP tower, for short bags (queries):
//   one wave per sample, 16-byte row chunks per lane, 4 rows in flight; it also emits the
//   16-bit sort keys of the sparse backward (bag_bwd_sorted: sort (token, slot) entries
//   by token, sum each token's run of dY rows, one atomic add per run and column).
// * bag_counts: for LONG bags (2k-token pages) the same product is computed as a dense
//   GEMM  C (N x V counts, bf16) x W  on the matrix cores (hipBLASLt), and the backward
//   dW = C^T x dY likewise — 126 GFLOP of MFMA instead of 8 GB of gathers / 4G float
//   atomics per step.  This kernel builds C (and the bag lengths) with one atomic
//   increment per token into a zeroed buffer (counts <= 256 are exact in bf16).
#include "common.h"
#include <stdlib.h>

namespace pv {
namespace embed {
PV_DEBUG_FLAG

__global__ void trigram_hash_kernel(const unsigned char* __restrict__ text, const int* __restrict__ lens,
                                    int* __restrict__ out, int N, int Lmax, int L, int V) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)N * L) return;
  const int n = (int)(i / L), t = (int)(i % L);
  const int len = lens[n];
  int id = 0;
  if (t + 3 <= len && t + 3 <= Lmax) {
    const unsigned char* p = text + (size_t)n * Lmax + t;
    unsigned h = 0x811C9DC5u;
    h = (h ^ p[0]) * 0x01000193u;
    h = (h ^ p[1]) * 0x01000193u;
    h = (h ^ p[2]) * 0x01000193u;
    id = 1 + (int)(h % (unsigned)(V - 1));
  }
  out[i] = id;
}

// W is bf16 (V, E) with E % 8 == 0 (E <= 1024). One wave per sample.
__global__ __launch_bounds__(256) void embedding_bag_kernel(const int* __restrict__ ids,
                                                            const unsigned short* __restrict__ W,
                                                            float* __restrict__ out, float* __restrict__ lens_out,
                                                            unsigned short* __restrict__ keys_out,
                                                            const float* __restrict__ bias, int act,
                                                            int N, int L, int E, int V, int pad, int mean) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (n >= N) return;
  const int nchunk = E / 8;  // 16-byte chunks per row
  float acc[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
  int cnt = 0;
  const int* row = ids + (size_t)n * L;
  for (int t0 = 0; t0 < L; t0 += 64) {
    const int tl = t0 + lane;
    const int myid = tl < L ? row[tl] : pad;
    PV_CHECK(myid == pad || (myid >= 0 && myid < V), PV_ERR_ID);
    const bool live = myid != pad && myid >= 0 && myid < V;
    unsigned long long m = __ballot(live);
    cnt += __popcll(m);
    // the sparse backward's sort keys: token id, or the sentinel V (sorts last) for pads
    if (keys_out && tl < L) keys_out[(size_t)n * L + tl] = (unsigned short)(live ? myid : V);
    while (m) {
      int src[4];
      int k = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        src[u] = m ? (int)__builtin_ctzll(m) : -1;
        if (m) { m &= m - 1; ++k; }
      }
      u32x4 v[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < k) {
          const int tok = __builtin_amdgcn_readlane(myid, src[u]);
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int ch = lane + 64 * c;
            v[u][c] = ch < nchunk ? *reinterpret_cast<const u32x4*>(W + (size_t)tok * E + ch * 8) : u32x4{0, 0, 0, 0};
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < k) {
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const u32x4 x = v[u][c];
            acc[c][0] += __uint_as_float(x.x << 16);
            acc[c][1] += __uint_as_float(x.x & 0xFFFF0000u);
            acc[c][2] += __uint_as_float(x.y << 16);
            acc[c][3] += __uint_as_float(x.y & 0xFFFF0000u);
            acc[c][4] += __uint_as_float(x.z << 16);
            acc[c][5] += __uint_as_float(x.z & 0xFFFF0000u);
            acc[c][6] += __uint_as_float(x.w << 16);
            acc[c][7] += __uint_as_float(x.w & 0xFFFF0000u);
          }
        }
      }
    }
  }
  const float s = (mean && cnt > 0) ? 1.f / (float)cnt : 1.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nchunk) {
      // epilogue: act(mean + bias) (the MLP tower's first layer, fused)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float y = acc[c][k] * s;
        if (bias) y += bias[ch * 8 + k];
        acc[c][k] = act == 1 ? fmaxf(y, 0.f) : act == 3 ? tanhf(y) : y;
      }
      f32x4 lo = {acc[c][0], acc[c][1], acc[c][2], acc[c][3]};
      f32x4 hi = {acc[c][4], acc[c][5], acc[c][6], acc[c][7]};
      *reinterpret_cast<f32x4*>(out + (size_t)n * E + ch * 8) = lo;
      *reinterpret_cast<f32x4*>(out + (size_t)n * E + ch * 8 + 4) = hi;
    }
  }
  if (lens_out && lane == 0) lens_out[n] = (float)cnt;
}

// Sparse bag backward (short bags): dW[tok] += scale_n * g[n] over the N*L (token, slot)
// entries sorted by token (keys from embedding_bag_kernel, values = slot = n*L + t).  Wave w
// walks sorted entries [w*EPW, (w+1)*EPW) run by run (sentinel keys V sort last and end the
// walk), 8 rows in flight, and adds each run's sum into dW: runs wholly inside the range
// with a plain vector read-modify-write (no other writer), the two boundary runs with float
// atomics (a hot token's run spreads over many waves and stays exact).
// Lane l owns columns {4l + 256 j}, j < NJ (E <= 256 NJ, E % 4 == 0).  dW may be the flat
// gradient buffer itself (accumulate semantics, ops/grad_sink.py).
template <int NJ>
__global__ __launch_bounds__(256) void bag_bwd_sorted_kernel(const unsigned short* __restrict__ skeys,
                                                             const unsigned* __restrict__ svals,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ lens, float* __restrict__ dW,
                                                             long M, int EPW, int L, int E, int V, int mean,
                                                             long long* fx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long wbeg = ((long)blockIdx.x * 4 + wave) * EPW;
  if (wbeg >= M) return;
  const long wend = min(M, wbeg + (long)EPW);
  const unsigned UV = (unsigned)V;
  // runs shared with the neighbouring waves: the one entering at wbeg, the one leaving at wend
  const unsigned k_in = wbeg > 0 ? (unsigned)skeys[wbeg - 1] : UV;
  const unsigned k_out = wend < M ? (unsigned)skeys[wend] : UV;
  unsigned cur = UV;
  bool first = true;
  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto flush = [&](bool last) {
    if (cur < UV) {
      float* drow = dW + (size_t)cur * E;
      // a run wholly inside this wave's range has no other writer: vector read-modify-write;
      // a boundary run may be split over waves: float atomics
      if ((first && cur == k_in) || (last && cur == k_out)) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = 4 * lane + 256 * j;
          if (c < E && fx) {  // deterministic mode (common.h): order-free fixed-point sums
#pragma unroll
            for (int k = 0; k < 4; ++k) fx_add(fx, (size_t)cur * E + c + k, acc[j][k]);
          } else if (c < E) {
            atomicAdd(&drow[c + 0], acc[j][0]);
            atomicAdd(&drow[c + 1], acc[j][1]);
            atomicAdd(&drow[c + 2], acc[j][2]);
            atomicAdd(&drow[c + 3], acc[j][3]);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = 4 * lane + 256 * j;
          if (c < E) {
            f32x4* p = reinterpret_cast<f32x4*>(drow + c);
            *p = *p + acc[j];
          }
        }
      }
      first = false;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  for (long i0 = wbeg; i0 < wend; i0 += 64) {
    const long il = i0 + lane;
    const unsigned kl = il < wend ? (unsigned)skeys[il] : UV;
    const unsigned rl = (il < wend && kl < UV) ? svals[il] : 0u;
    const int n = __popcll(__ballot(kl < UV));  // live entries are a prefix (sorted)
    for (int e0 = 0; e0 < n; e0 += 8) {
      f32x4 x[8][NJ];
      unsigned kk[8];
      float sc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u < n ? e0 + u : e0;
        kk[u] = (unsigned)__builtin_amdgcn_readlane((int)kl, e);
        const unsigned slot = (unsigned)__builtin_amdgcn_readlane((int)rl, e);
        PV_CHECK((long)slot < M, PV_ERR_SLOT);
        const unsigned smp = slot / (unsigned)L;
        sc[u] = mean ? 1.f / fmaxf(lens[smp], 1.f) : 1.f;
        const float* src = g + (size_t)smp * E;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int c = 4 * lane + 256 * j;
          x[u][j] = c < E ? *reinterpret_cast<const f32x4*>(src + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (e0 + u >= n) break;
        if (kk[u] != cur) {
          flush(false);
          cur = kk[u];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] += sc[u] * x[u][j];
      }
    }
    if (n < 64) break;
  }
  flush(true);
}

// counts: (N, ldc) bf16, zeroed; lens: (N) float (non-pad tokens per bag)
__global__ void bag_counts_kernel(const int* __restrict__ ids, unsigned short* __restrict__ counts,
                                  float* __restrict__ lens, int N, int L, int V, int ldc, int pad) {
  const int n = blockIdx.x;
  const int* row = ids + (size_t)n * L;
  unsigned short* crow = counts + (size_t)n * ldc;
  int local = 0;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const int v = row[t];
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    if (v != pad && v >= 0 && v < V) {
      ++local;
      // bf16 +1.0 on a 16-bit cell: CAS on the containing 32-bit word
      unsigned* word = reinterpret_cast<unsigned*>(crow + (v & ~1));
      const int sh = (v & 1) * 16;
      unsigned old = *word, assumed;
      do {
        assumed = old;
        const unsigned short cur = (unsigned short)(assumed >> sh);
        const unsigned short nxt = f32_to_bf16(bf16_to_f32(cur) + 1.f);
        const unsigned nw = (assumed & ~(0xFFFFu << sh)) | ((unsigned)nxt << sh);
        old = atomicCAS(word, assumed, nw);
      } while (old != assumed);
    }
  }
  local = (int)wave_sum((float)local);
  __shared__ float part[16];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = (float)local;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    lens[n] = s;
  }
}

// LDS-histogram variant (V <= HIST_MAX): one workgroup per bag counts its tokens with
// LDS atomics (no CAS loops on global bf16 cells, no contention between bags), then
// writes the WHOLE bf16 row (zeros included) with 8-byte stores — the caller does not
// have to clear the (N, ldc) matrix.
// Vocabularies wider than HIST_MAX (word level): blockIdx.y walks windows of HIST_MAX ids, each
// block re-reading its page's ids (round 6: the previous wide-vocabulary kernel added bf16 +1.0
// by compare-and-swap on the count matrix, so a count stuck at 256 — 256 + 1 rounds to 256 in
// bf16 — for any id repeated more than 256 times in a page).
constexpr int HIST_MAX = 38912;  // 152 KB of u32 counters
__global__ __launch_bounds__(1024) void bag_counts_lds_kernel(const int* __restrict__ ids,
                                                              unsigned short* __restrict__ counts,
                                                              float* __restrict__ lens, int N, int L, int V, int ldc,
                                                              int pad) {
  extern __shared__ unsigned hist[];
  __shared__ int part[16];
  const int n = blockIdx.x;
  const int v0 = blockIdx.y * HIST_MAX, w = min(HIST_MAX, ldc - v0);  // this window's ids
  for (int c = threadIdx.x; c < w; c += blockDim.x) hist[c] = 0u;
  __syncthreads();
  const int* row = ids + (size_t)n * L;
  int local = 0;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const int v = row[t];
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    if (v != pad && v >= 0 && v < V) {
      ++local;
      if (v >= v0 && v < v0 + w) atomicAdd(&hist[v - v0], 1u);
    }
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = local;
  __syncthreads();
  uint2* crow = reinterpret_cast<uint2*>(counts + (size_t)n * ldc + v0);
  for (int c4 = threadIdx.x; c4 < w / 4; c4 += blockDim.x) {
    const unsigned* h = hist + 4 * c4;
    crow[c4] = uint2{pack_bf16x2((float)h[0], (float)h[1]), pack_bf16x2((float)h[2], (float)h[3])};
  }
  if (threadIdx.x == 0 && blockIdx.y == 0) {
    int s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    lens[n] = (float)s;
  }
}

// Same, with two 16-bit counters per LDS word (bag length < 65536, so a counter never
// carries into its neighbour): half the LDS (60 KB at V = 30 k), two blocks per CU, so one
// block's histogram phase overlaps the other's row write.  Word w holds ids (2w, 2w+1) in
// (low, high) halves: exactly the bf16 pair order of the output row.
__global__ __launch_bounds__(1024) void bag_counts_lds16_kernel(const int* __restrict__ ids,
                                                                unsigned short* __restrict__ counts,
                                                                float* __restrict__ lens, int N, int L, int V,
                                                                int ldc, int pad) {
  extern __shared__ unsigned hist2[];
  __shared__ int part[16];
  const int n = blockIdx.x;
  const int words = ldc / 2;
  for (int c = threadIdx.x; c < words; c += blockDim.x) hist2[c] = 0u;
  __syncthreads();
  const int* row = ids + (size_t)n * L;
  int local = 0;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const int v = row[t];
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    if (v != pad && v >= 0 && v < V) {
      ++local;
      atomicAdd(&hist2[v >> 1], 1u << ((v & 1) * 16));
    }
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = local;
  __syncthreads();
  uint2* crow = reinterpret_cast<uint2*>(counts + (size_t)n * ldc);
  for (int c4 = threadIdx.x; c4 < ldc / 4; c4 += blockDim.x) {
    const unsigned a = hist2[2 * c4], b = hist2[2 * c4 + 1];
    crow[c4] = uint2{pack_bf16x2((float)(a & 0xFFFFu), (float)(a >> 16)),
                     pack_bf16x2((float)(b & 0xFFFFu), (float)(b >> 16))};
  }
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    lens[n] = (float)s;
  }
}

// counts for the MX fp8 bag GEMM: the same 16-bit LDS histogram, the row written as e4m3
// bytes (c8, ldc8 % 4 == 0: counts <= 16 exact, larger ones rounded to the nearest e4m3
// value, saturated at 448) and, when the weight gradient is needed, ALSO as bf16 (c16,
// exact, the operand of the backward's C^T G); columns V..ldc are zeros in both.
__global__ __launch_bounds__(1024) void bag_counts8_kernel(const int* __restrict__ ids,
                                                           unsigned short* __restrict__ c16, int ldc16,
                                                           unsigned char* __restrict__ c8, int ldc8,
                                                           float* __restrict__ lens, int N, int L, int V, int pad) {
  extern __shared__ unsigned hist2[];
  __shared__ int part[16];
  const int n = blockIdx.x;
  const int ldh = ldc8 > ldc16 ? ldc8 : ldc16;
  for (int c = threadIdx.x; c < ldh / 2; c += blockDim.x) hist2[c] = 0u;
  __syncthreads();
  const int* row = ids + (size_t)n * L;
  int local = 0;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const int v = row[t];
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    if (v != pad && v >= 0 && v < V) {
      ++local;
      atomicAdd(&hist2[v >> 1], 1u << ((v & 1) * 16));
    }
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = local;
  __syncthreads();
  unsigned* r8 = reinterpret_cast<unsigned*>(c8 + (size_t)n * ldc8);
  for (int c4 = threadIdx.x; c4 < ldc8 / 4; c4 += blockDim.x) {
    const unsigned a = hist2[2 * c4], b = hist2[2 * c4 + 1];
    unsigned w = 0;
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf((float)(a & 0xFFFFu), 448.f), fminf((float)(a >> 16), 448.f), w, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf((float)(b & 0xFFFFu), 448.f), fminf((float)(b >> 16), 448.f), w, true);
    r8[c4] = w;
  }
  if (c16) {
    uint2* r16 = reinterpret_cast<uint2*>(c16 + (size_t)n * ldc16);
    for (int c4 = threadIdx.x; c4 < ldc16 / 4; c4 += blockDim.x) {
      const unsigned a = hist2[2 * c4], b = hist2[2 * c4 + 1];
      r16[c4] = uint2{pack_bf16x2((float)(a & 0xFFFFu), (float)(a >> 16)),
                      pack_bf16x2((float)(b & 0xFFFFu), (float)(b >> 16))};
    }
  }
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    lens[n] = (float)s;
  }
}

PV_DEBUG_EXPORT(embed)
}  // namespace embed
}  // namespace pv

using namespace pv;

PV_API int pv_trigram_hash(const void* text, const int* lens, int* out, int N, int Lmax, int L, int V, void* stream) {
  if (V < 2) return -1;
  long total = (long)N * L;
  hipLaunchKernelGGL(pv::embed::trigram_hash_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const unsigned char*)text, lens, out, N, Lmax, L, V);
  PV_LAUNCH_CHECK();
  return 0;
}

// act: 0 none, 1 relu, 3 tanh (applied after the optional bias)
PV_API int pv_embedding_bag(const int* ids, const void* W, float* out, float* lens, void* keys, const float* bias,
                            int act, int N, int L, int E, int V, int pad, int mean, void* stream) {
  if (E % 8 || E > 1024 || (act != 0 && act != 1 && act != 3)) return -1;
  if (keys && V >= 65535) return -2;  // 16-bit sort keys (sentinel V)
  hipLaunchKernelGGL(pv::embed::embedding_bag_kernel, dim3((N + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids,
                     (const unsigned short*)W, out, lens, (unsigned short*)keys, bias, act, N, L, E, V, pad, mean);
  PV_LAUNCH_CHECK();
  return 0;
}

// Sparse bag backward over sorted (token, slot) entries: dW (V, E) fp32 += ... (atomics).
PV_API int pv_bag_bwd_sorted(const void* skeys, const unsigned* svals, const float* g, const float* lens, float* dW,
                             long M, int epw, int L, int E, int V, int mean, void* stream) {
  if (E % 4 || E > 1024 || epw < 8 || V >= 65535) return -1;
  const long waves = (M + epw - 1) / epw;
  const dim3 grid((unsigned)((waves + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const unsigned short* k = (const unsigned short*)skeys;
  long long* fx = pv::det_on() ? pv::det_scratch((size_t)V * E, st) : nullptr;
  if (pv::det_on() && !fx) return -4;
  if (E <= 256)
    hipLaunchKernelGGL(pv::embed::bag_bwd_sorted_kernel<1>, grid, dim3(256), 0, st, k, svals, g, lens, dW, M, epw, L,
                       E, V, mean, fx);
  else if (E <= 512)
    hipLaunchKernelGGL(pv::embed::bag_bwd_sorted_kernel<2>, grid, dim3(256), 0, st, k, svals, g, lens, dW, M, epw, L,
                       E, V, mean, fx);
  else
    hipLaunchKernelGGL(pv::embed::bag_bwd_sorted_kernel<4>, grid, dim3(256), 0, st, k, svals, g, lens, dW, M, epw, L,
                       E, V, mean, fx);
  PV_LAUNCH_CHECK();
  return fx ? pv::det_flush(fx, dW, (size_t)V * E, st) : 0;
}

// counts (N, ldc) bf16.  ldc <= HIST_MAX and ldc % 4 == 0: the LDS path writes every
// element (no zeroing needed); otherwise the caller's zeroed matrix is accumulated into
// (zeroed must be 1).
PV_API int pv_bag_counts(const int* ids, void* counts, float* lens, int N, int L, int V, int ldc, int pad,
                         int zeroed, void* stream) {
  if (ldc < V || (ldc & 1)) return -1;
  static const bool packed16 = [] {  // PAGEVEC_BAG_COUNTS16=0: one u32 counter per id (A/B switch)
    const char* e = getenv("PAGEVEC_BAG_COUNTS16");
    return !(e && e[0] == '0');
  }();
  if (packed16 && L < 65536 && ldc <= 40960 && (ldc & 3) == 0) {
    static bool attr16 = false;
    if (!attr16) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&pv::embed::bag_counts_lds16_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 40960 * 2) != hipSuccess)
        return -3;
      attr16 = true;
    }
    hipLaunchKernelGGL(pv::embed::bag_counts_lds16_kernel, dim3(N), dim3(1024), (ldc / 2) * sizeof(unsigned),
                       (hipStream_t)stream, ids, (unsigned short*)counts, lens, N, L, V, ldc, pad);
    PV_LAUNCH_CHECK();
    return 0;
  }
  if (ldc <= pv::embed::HIST_MAX && (ldc & 3) == 0) {
    static bool attr = false;
    if (!attr) {  // > 64 KB of dynamic LDS (gfx950: 160 KB per CU)
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&pv::embed::bag_counts_lds_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              pv::embed::HIST_MAX * (int)sizeof(unsigned)) != hipSuccess)
        return -3;
      attr = true;
    }
    hipLaunchKernelGGL(pv::embed::bag_counts_lds_kernel, dim3(N), dim3(1024), ldc * sizeof(unsigned),
                       (hipStream_t)stream, ids, (unsigned short*)counts, lens, N, L, V, ldc, pad);
    PV_LAUNCH_CHECK();
    return 0;
  }
  if ((ldc & 3) == 0) {  // wide vocabularies: windows of HIST_MAX ids (every element written)
    static bool attrw = false;
    if (!attrw) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&pv::embed::bag_counts_lds_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              pv::embed::HIST_MAX * (int)sizeof(unsigned)) != hipSuccess)
        return -3;
      attrw = true;
    }
    const int nwin = (ldc + pv::embed::HIST_MAX - 1) / pv::embed::HIST_MAX;
    hipLaunchKernelGGL(pv::embed::bag_counts_lds_kernel, dim3(N, nwin), dim3(1024),
                       pv::embed::HIST_MAX * sizeof(unsigned), (hipStream_t)stream, ids, (unsigned short*)counts,
                       lens, N, L, V, ldc, pad);
    PV_LAUNCH_CHECK();
    return 0;
  }
  if (!zeroed) return -2;
  hipLaunchKernelGGL(pv::embed::bag_counts_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, ids,
                     (unsigned short*)counts, lens, N, L, V, ldc, pad);
  PV_LAUNCH_CHECK();
  return 0;
}

// counts8 (N, ldc8) e4m3 (+ counts16 (N, ldc16) bf16 when non-null), every element written.
PV_API int pv_bag_counts8(const int* ids, void* counts16, int ldc16, void* counts8, int ldc8, float* lens, int N,
                          int L, int V, int pad, void* stream) {
  if (ldc8 < V || ldc8 % 4 || (counts16 && (ldc16 < V || ldc16 % 4)) || L >= 65536) return -1;
  const int ldh = counts16 && ldc16 > ldc8 ? ldc16 : ldc8;
  if (ldh > 40960) return -2;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&pv::embed::bag_counts8_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 40960 * 2) != hipSuccess)
      return -3;
    attr = true;
  }
  hipLaunchKernelGGL(pv::embed::bag_counts8_kernel, dim3(N), dim3(1024), (ldh / 2) * sizeof(unsigned),
                     (hipStream_t)stream, ids, (unsigned short*)counts16, counts16 ? ldc16 : 0,
                     (unsigned char*)counts8, ldc8, lens, N, L, V, pad);
  PV_LAUNCH_CHECK();
  return 0;
}
