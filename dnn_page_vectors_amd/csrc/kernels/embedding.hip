// K0 / K1: device featurizer (letter-trigram hashing) and embedding-bag kernels.
//
// * trigram_hash: ASCII-cleaned text bytes (N, Lmax) + lengths -> hashed trigram ids
//   (N, L), id = 1 + fnv1a(3 bytes) % (V-1), PAD = 0.  Same function as the C++
//   featurizer (csrc/runtime/featurize.cpp) restricted to single-byte code points, so
//   the host can ship raw bytes and let the GPU hash them (DSSM "word hashing").
// * embedding_bag: out[n,:] = scale_n * sum_{t: ids[n,t] != pad} W[ids[n,t], :] — the
//   multi-hot x W1 first layer of the DSSM MLP tower, for short bags (queries):
//   one wave per sample, 16-byte row chunks per lane, 4 rows in flight.
// * bag_counts: for LONG bags (2k-token pages) the same product is computed as a dense
//   GEMM  C (N x V counts, bf16) x W  on the matrix cores (hipBLASLt), and the backward
//   dW = C^T x dY likewise — 126 GFLOP of MFMA instead of 8 GB of gathers / 4G float
//   atomics per step.  This kernel builds C (and the bag lengths) with one atomic
//   increment per token into a zeroed buffer (counts <= 256 are exact in bf16).
#include "common.h"

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
    unsigned long long m = __ballot(myid != pad && myid >= 0 && myid < V);
    cnt += __popcll(m);
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
      f32x4 lo = {acc[c][0] * s, acc[c][1] * s, acc[c][2] * s, acc[c][3] * s};
      f32x4 hi = {acc[c][4] * s, acc[c][5] * s, acc[c][6] * s, acc[c][7] * s};
      *reinterpret_cast<f32x4*>(out + (size_t)n * E + ch * 8) = lo;
      *reinterpret_cast<f32x4*>(out + (size_t)n * E + ch * 8 + 4) = hi;
    }
  }
  if (lens_out && lane == 0) lens_out[n] = (float)cnt;
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
constexpr int HIST_MAX = 38912;  // 152 KB of u32 counters
__global__ __launch_bounds__(1024) void bag_counts_lds_kernel(const int* __restrict__ ids,
                                                              unsigned short* __restrict__ counts,
                                                              float* __restrict__ lens, int N, int L, int V, int ldc,
                                                              int pad) {
  extern __shared__ unsigned hist[];
  __shared__ int part[16];
  const int n = blockIdx.x;
  for (int c = threadIdx.x; c < ldc; c += blockDim.x) hist[c] = 0u;
  __syncthreads();
  const int* row = ids + (size_t)n * L;
  int local = 0;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const int v = row[t];
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    if (v != pad && v >= 0 && v < V) {
      ++local;
      atomicAdd(&hist[v], 1u);
    }
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = local;
  __syncthreads();
  uint2* crow = reinterpret_cast<uint2*>(counts + (size_t)n * ldc);
  for (int c4 = threadIdx.x; c4 < ldc / 4; c4 += blockDim.x) {
    const unsigned* h = hist + 4 * c4;
    crow[c4] = uint2{pack_bf16x2((float)h[0], (float)h[1]), pack_bf16x2((float)h[2], (float)h[3])};
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

PV_API int pv_embedding_bag(const int* ids, const void* W, float* out, float* lens, int N, int L, int E, int V, int pad,
                            int mean, void* stream) {
  if (E % 8 || E > 1024) return -1;
  hipLaunchKernelGGL(pv::embed::embedding_bag_kernel, dim3((N + 3) / 4), dim3(256), 0, (hipStream_t)stream, ids,
                     (const unsigned short*)W, out, lens, N, L, E, V, pad, mean);
  PV_LAUNCH_CHECK();
  return 0;
}

// counts (N, ldc) bf16.  ldc <= HIST_MAX and ldc % 4 == 0: the LDS path writes every
// element (no zeroing needed); otherwise the caller's zeroed matrix is accumulated into
// (zeroed must be 1).
PV_API int pv_bag_counts(const int* ids, void* counts, float* lens, int N, int L, int V, int ldc, int pad,
                         int zeroed, void* stream) {
  if (ldc < V || (ldc & 1)) return -1;
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
  if (!zeroed) return -2;
  hipLaunchKernelGGL(pv::embed::bag_counts_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, ids,
                     (unsigned short*)counts, lens, N, L, V, ldc, pad);
  PV_LAUNCH_CHECK();
  return 0;
}
