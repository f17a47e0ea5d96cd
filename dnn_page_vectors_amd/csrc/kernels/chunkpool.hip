// Masked mean over the chunk vectors of a long page (BASELINE config 5, models/chunked.py):
//   live[n, c] = any(ids[n, c*CL : (c+1)*CL] != 0)          (an all-padding chunk is empty)
//   out[n, :]  = sum_c live[n, c] * v[n, c, :] / max(1, sum_c live[n, c])
// and its backward dv[n, c, :] = live[n, c] / max(1, cnt[n]) * g[n, :].
// One workgroup per page: the 4 waves scan the page's chunks for a non-pad id (16-byte
// loads + a wave ballot), then every thread sums columns over the chunks.  Replaces the
// torch chain pad / compare / any / cast / mul / sum / sum / clamp / div (and the matching
// backward ops): ~a dozen launches per step of a 1.1 ms step.
#include "common.h"

namespace pv {
namespace chunkpool {

constexpr int MAXC = 64;  // chunks per page

__global__ __launch_bounds__(256) void chunk_mean_fwd_kernel(const float* __restrict__ v,
                                                             const int* __restrict__ ids, int C, int CL, int D,
                                                             float* __restrict__ out, float* __restrict__ scale_out) {
  __shared__ float live[MAXC];
  __shared__ float inv;
  const int n = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int* row = ids + (size_t)n * C * CL;
  for (int c = w; c < C; c += 4) {
    const int* p = row + (size_t)c * CL;
    bool nz = false;
    if ((CL & 3) == 0) {
      for (int i = lane * 4; i < CL; i += 256) {
        const int4 q = *reinterpret_cast<const int4*>(p + i);
        nz |= (q.x | q.y | q.z | q.w) != 0;
      }
    } else {
      for (int i = lane; i < CL; i += 64) nz |= p[i] != 0;
    }
    const unsigned long long any = __ballot(nz);  // every lane takes part
    if (lane == 0) live[c] = any ? 1.f : 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float cnt = 0.f;
    for (int c = 0; c < C; ++c) cnt += live[c];
    inv = 1.f / fmaxf(cnt, 1.f);
  }
  __syncthreads();
  // per-chunk backward scale live / max(1, cnt), saved for the backward
  for (int c = threadIdx.x; c < C; c += blockDim.x) scale_out[(size_t)n * C + c] = live[c] * inv;
  const float* vn = v + (size_t)n * C * D;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += live[c] * vn[(size_t)c * D + d];
    out[(size_t)n * D + d] = s * inv;
  }
}

__global__ __launch_bounds__(256) void chunk_mean_bwd_kernel(const float* __restrict__ g,
                                                             const float* __restrict__ scale, int C, int D,
                                                             float* __restrict__ dv) {
  const int n = blockIdx.x;
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    const int c = i / D, d = i - c * D;
    dv[(size_t)n * C * D + i] = scale[(size_t)n * C + c] * g[(size_t)n * D + d];
  }
}

}  // namespace chunkpool
}  // namespace pv

using namespace pv;

// v: (N, C, D) fp32, ids: (N, C*CL) int32 -> out (N, D) fp32, scale (N, C) = live / max(1, cnt)
PV_API int pv_chunk_mean_fwd(const float* v, const int* ids, int N, int C, int CL, int D, float* out, float* scale,
                             void* stream) {
  using namespace pv::chunkpool;
  if (N < 1 || C < 1 || C > MAXC || CL < 1 || D < 1) return -1;
  if ((CL & 3) == 0 && (reinterpret_cast<uintptr_t>(ids) & 15)) return -2;  // int4 loads
  hipLaunchKernelGGL(chunk_mean_fwd_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, v, ids, C, CL, D, out, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_chunk_mean_bwd(const float* g, const float* scale, int N, int C, int D, float* dv, void* stream) {
  if (N < 1 || C < 1 || D < 1) return -1;
  hipLaunchKernelGGL(pv::chunkpool::chunk_mean_bwd_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, g, scale, C, D,
                     dv);
  PV_LAUNCH_CHECK();
  return 0;
}
