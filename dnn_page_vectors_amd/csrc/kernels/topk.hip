// K9: brute-force cosine top-k retrieval (Recall@k evaluation, page-vector search).
//
// S^T = Pn . Qn^T with v_mfma_f32_16x16x32_bf16 in the SWAPPED orientation (pages on
// the accumulator rows, queries on the lanes): every lane then owns ONE query column
// (lane & 15) and sees 4 pages of each 16-page subtile, so it keeps a private sorted
// top-K list (K <= 16) in registers with no cross-lane traffic in the hot loop; a
// new score costs one compare against the list tail and the K-step insertion runs only
// when some lane beats its tail.  Page tiles (64 x DP bf16) are staged once per
// workgroup in LDS and shared by its 4 waves (64 queries).  The page range is split
// over workgroups (grid.y) and a merge kernel selects the final top-k of the
// 4 * nsplit partial lists per query.
#include "common.h"

namespace pv {
namespace topk {

constexpr int K = 16;
constexpr int TP = 64;  // pages per split granule (and per LDS tile up to DP = 256)
constexpr int PADK = 8;

// Wide vectors (BERT's 768-d CLS, DP > 256) stage 32-page tiles: 32 x 776 bf16 = 49.7 KB LDS.
template <int KS>
__device__ constexpr int tile_pages() { return KS <= 8 ? TP : 32; }

template <int KS>
__global__ __launch_bounds__(256) void topk_partial_kernel(const unsigned short* __restrict__ Q,
                                                           const unsigned short* __restrict__ Pg,
                                                           float* __restrict__ pv, int* __restrict__ pi, int B,
                                                           int N, int per_split, int nsplit) {
  constexpr int DP = KS * 32, LDP = DP + PADK, T = tile_pages<KS>();
  __shared__ __attribute__((aligned(16))) unsigned short pt[T * LDP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x * 64 + wave * 16 + (lane & 15);
  const int p_begin = blockIdx.y * per_split, p_end = min(N, p_begin + per_split);
  // B operand: Q[q][feat 32s + 8(lane>>4) + j]
  bf16x8 b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    b[s] = q < B ? *reinterpret_cast<const bf16x8*>(Q + (size_t)q * DP + s * 32 + (lane >> 4) * 8)
                 : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  float vals[K];
  int idx[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    vals[i] = -INFINITY;
    idx[i] = -1;
  }
  for (int p0 = p_begin; p0 < p_end; p0 += T) {
    __syncthreads();
    for (int x = threadIdx.x; x < T * (DP / 8); x += 256) {
      int r = x / (DP / 8), cc = (x % (DP / 8)) * 8;
      u32x4 v = (p0 + r < p_end) ? *reinterpret_cast<const u32x4*>(Pg + (size_t)(p0 + r) * DP + cc)
                                 : u32x4{0, 0, 0, 0};
      *reinterpret_cast<u32x4*>(pt + r * LDP + cc) = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < T / 16; ++c) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(pt + (c * 16 + (lane & 15)) * LDP + s * 32 + (lane >> 4) * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[s], acc, 0, 0, 0);
      }
      // acc[r] = score(page = p0 + 16c + 4(lane>>4) + r, query = lane & 15)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int page = p0 + c * 16 + 4 * (lane >> 4) + r;
        float x = page < p_end ? acc[r] : -INFINITY;
        int xi = page;
        if (__any(x > vals[K - 1])) {
#pragma unroll
          for (int i = 0; i < K; ++i) {
            const bool sw = x > vals[i];
            const float tv = vals[i];
            const int ti = idx[i];
            vals[i] = sw ? x : tv;
            idx[i] = sw ? xi : ti;
            x = sw ? tv : x;
            xi = sw ? ti : xi;
          }
        }
      }
    }
  }
  if (q < B) {
    // partial lists: [q][split][lane>>4][K]
    const size_t o = (((size_t)q * nsplit + blockIdx.y) * 4 + (lane >> 4)) * K;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      pv[o + i] = vals[i];
      pi[o + i] = idx[i];
    }
  }
}

// One wave per query: select the top-k of its 4*nsplit*K candidates.  Every partial list
// is sorted, so only its first k entries can matter.  One pass: each lane keeps a sorted
// register list of the best k of its strided candidates (insertion only when a candidate
// beats the list tail); then k rounds of a wave arg-max over the 64 list heads, the
// winning lane popping its head.  (The previous form re-scanned all candidates k times:
// 1.2 ms for one query over 1 M pages, 512 splits.)  Order: descending score, ascending
// page index on ties.
__device__ __forceinline__ bool topk_better(float a, int ia, float b, int ib) {
  return a > b || (a == b && ia < ib);
}

__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                                         float* __restrict__ vals, int* __restrict__ idx, int B,
                                                         int nc, int k) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= B) return;
  const float* cv = pv + (size_t)q * nc;
  const int* ci = pi + (size_t)q * nc;
  float lv[K];
  int li[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    lv[i] = -INFINITY;
    li[i] = 0x7FFFFFFF;
  }
  // candidate c of list l sits at l*K + c; lane walks (list, c < k) pairs with stride 64
  const int nl = nc / K;
  for (int j = lane; j < nl * k; j += 64) {
    const int l = j / k, c = j - l * k;
    float v = cv[l * K + c];
    int ix = ci[l * K + c];
    if (ix < 0 || !topk_better(v, ix, lv[K - 1], li[K - 1])) continue;
#pragma unroll
    for (int i = 0; i < K; ++i) {  // insertion: carry the displaced entry down
      const bool sw = topk_better(v, ix, lv[i], li[i]);
      const float tv = lv[i];
      const int ti = li[i];
      lv[i] = sw ? v : tv;
      li[i] = sw ? ix : ti;
      v = sw ? tv : v;
      ix = sw ? ti : ix;
    }
  }
  for (int r = 0; r < k; ++r) {
    float best = lv[0];
    int bi = li[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (topk_better(ov, oi, best, bi)) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      vals[(size_t)q * k + r] = best;
      idx[(size_t)q * k + r] = bi == 0x7FFFFFFF ? -1 : bi;
    }
    if (li[0] == bi && bi != 0x7FFFFFFF) {  // page indices are unique: exactly one lane pops
#pragma unroll
      for (int i = 0; i + 1 < K; ++i) {
        lv[i] = lv[i + 1];
        li[i] = li[i + 1];
      }
      lv[K - 1] = -INFINITY;
      li[K - 1] = 0x7FFFFFFF;
    }
  }
}

}  // namespace topk
}  // namespace pv

using namespace pv;

// Split of the page range over workgroups (grid.y); the caller allocates the partial
// lists (B x nsplit x 4 x 16 floats + ints) so the launcher never allocates.
PV_API int pv_topk_splits(int B, int N) {
  using namespace pv::topk;
  // ~512 workgroups: more splits stream the pages from more CUs but grow the one-wave-per-
  // query merge (2048: 1 query over 1 M pages 1.41 ms vs 0.56 ms at 512)
  const int qb = (B + 63) / 64;
  int nsplit = (512 + qb - 1) / qb;
  const int maxs = (N + TP - 1) / TP;
  if (nsplit > maxs) nsplit = maxs;
  if (nsplit < 1) nsplit = 1;
  const int per = ((N + nsplit - 1) / nsplit + TP - 1) / TP * TP;
  return (N + per - 1) / per;
}

PV_API int pv_topk_cos(const void* Q, const void* Pg, float* vals, int* idx, float* pv, int* pi, int B, int N, int DP,
                       int k, int nsplit, void* stream) {
  using namespace pv::topk;
  if (k > K || k < 1 || DP % 32 || DP > 768 || nsplit < 1) return -1;
  const int qb = (B + 63) / 64;
  const int per = ((N + nsplit - 1) / nsplit + TP - 1) / TP * TP;
  if ((N + per - 1) / per > nsplit) return -1;
  const size_t nc = (size_t)nsplit * 4 * K;
  dim3 grid(qb, nsplit);
  hipStream_t s = (hipStream_t)stream;
#define PV_TOPK(KSV) hipLaunchKernelGGL(topk_partial_kernel<KSV>, grid, dim3(256), 0, s, (const unsigned short*)Q, \
                                        (const unsigned short*)Pg, pv, pi, B, N, per, nsplit)
  switch (DP / 32) {
    case 1: PV_TOPK(1); break;
    case 2: PV_TOPK(2); break;
    case 3: PV_TOPK(3); break;
    case 4: PV_TOPK(4); break;
    case 5: PV_TOPK(5); break;
    case 6: PV_TOPK(6); break;
    case 8: PV_TOPK(8); break;
    case 12: PV_TOPK(12); break;
    case 16: PV_TOPK(16); break;
    case 24: PV_TOPK(24); break;
    default: return -1;
  }
#undef PV_TOPK
  // splits whose page range is empty leave their lists untouched: they were -inf/-1 filled by the caller
  hipLaunchKernelGGL(topk_merge_kernel, dim3((B + 3) / 4), dim3(256), 0, s, pv, pi, vals, idx, B, (int)nc, k);
  PV_LAUNCH_CHECK();
  return 0;
}
