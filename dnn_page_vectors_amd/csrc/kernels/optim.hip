// K8: fused flat-buffer Adam + helper elementwise kernels.
//
// Reference optimizer: model.compile(optimizer="adam") (cnn_dssm_th.py:182) = Keras-1
// Adam(lr=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-8):
//   lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t);  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p   -= lr_t * m / (sqrt(v) + eps)
// All parameters of a model live in ONE fp32 flat buffer (params / grads / m / v are
// parallel flat buffers), so the whole update is a single vectorised streaming launch
// (7 x 4 B per parameter) and the DP all-reduce works on the same flat gradient buffer.
// The same launch can emit a bf16 shadow copy of selected ranges (e.g. the embedding
// tables the fused conv kernel gathers from), with a row-padded layout.
#include "common.h"

namespace pv {
namespace optim {

__device__ __forceinline__ void store_bf16x4(unsigned short* dst, const f32x4& v) {
  const unsigned lo = (unsigned)f32_to_bf16(v[0]) | ((unsigned)f32_to_bf16(v[1]) << 16);
  const unsigned hi = (unsigned)f32_to_bf16(v[2]) | ((unsigned)f32_to_bf16(v[3]) << 16);
  *reinterpret_cast<uint2*>(dst) = uint2{lo, hi};
}

// tdev = {step, warmup steps}: the learning rate ramps linearly over the first warmup steps
// (0 = none), read on the device so a captured step replays the schedule
__device__ __forceinline__ float warmup_scale(const float* tdev) {
  const float w = tdev[1];
  return w > 0.f ? fminf(1.f, tdev[0] / w) : 1.f;
}

// (non-temporal loads / stores were measured as an A/B arm in round 5 — 16 M parameters 86.5
// vs 67.7 us — and removed: docs/PERF.md "Dense Adam streams")
__device__ __forceinline__ f32x4 ld4(const float* b, long i) { return reinterpret_cast<const f32x4*>(b)[i]; }
__device__ __forceinline__ void st4(float* b, long i, const f32x4& x) { reinterpret_cast<f32x4*>(b)[i] = x; }

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n, float lr_t,
                                                   float b1, float b2, float eps, float wd, int torch_style,
                                                   float bc2_sqrt_inv, const float* __restrict__ skip,
                                                   const float* __restrict__ tdev,
                                                   unsigned short* __restrict__ p16) {
  if (skip && *skip != 0.f) return;  // non-finite guard: skip the whole step
  if (tdev) {  // step count on the device (hipGraph replays): bias corrections computed here
    const float t = tdev[0], lr = lr_t * warmup_scale(tdev);
    const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
    if (torch_style) {
      lr_t = lr / bc1;
      bc2_sqrt_inv = rsqrtf(bc2);
    } else {
      lr_t = lr * sqrtf(bc2) / bc1;
    }
  }
  long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x);
  const long stride = (long)gridDim.x * blockDim.x;
  const long n4 = n / 4;
  auto upd = [&](f32x4& pp, const f32x4& gg, f32x4& mm, f32x4& vv) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gg[k] + wd * pp[k];
      mm[k] = b1 * mm[k] + (1.f - b1) * gk;
      vv[k] = b2 * vv[k] + (1.f - b2) * gk * gk;
      float den = torch_style ? (sqrtf(vv[k]) * bc2_sqrt_inv + eps) : (sqrtf(vv[k]) + eps);
      pp[k] -= lr_t * mm[k] / den;
    }
  };
  // two 16-byte groups per thread per trip: 8 independent 16-byte loads in flight per lane
  // (the update is a pure 28 B/parameter stream; one group per trip left HBM at ~3 TB/s)
  long i = i4;
  for (; i + stride < n4; i += 2 * stride) {
    const long j = i + stride;
    f32x4 p0 = ld4(p, i), p1 = ld4(p, j);
    f32x4 g0 = ld4(g, i), g1 = ld4(g, j);
    f32x4 m0 = ld4(m, i), m1 = ld4(m, j);
    f32x4 v0 = ld4(v, i), v1 = ld4(v, j);
    upd(p0, g0, m0, v0);
    upd(p1, g1, m1, v1);
    if (p16) {  // bf16 compute copy of the updated weights (consumers skip their cast kernel)
      store_bf16x4(p16 + 4 * i, p0);
      store_bf16x4(p16 + 4 * j, p1);
    }
    st4(p, i, p0);
    st4(m, i, m0);
    st4(v, i, v0);
    st4(p, j, p1);
    st4(m, j, m1);
    st4(v, j, v1);
  }
  for (; i < n4; i += stride) {
    f32x4 pp = ld4(p, i);
    f32x4 gg = ld4(g, i);
    f32x4 mm = ld4(m, i);
    f32x4 vv = ld4(v, i);
    upd(pp, gg, mm, vv);
    if (p16) store_bf16x4(p16 + 4 * i, pp);
    st4(p, i, pp);
    st4(m, i, mm);
    st4(v, i, vv);
  }
  for (long i = n4 * 4 + i4; i < n; i += stride) {
    float gk = g[i] + wd * p[i];
    m[i] = b1 * m[i] + (1.f - b1) * gk;
    v[i] = b2 * v[i] + (1.f - b2) * gk * gk;
    float den = torch_style ? (sqrtf(v[i]) * bc2_sqrt_inv + eps) : (sqrtf(v[i]) + eps);
    p[i] -= lr_t * m[i] / den;
    if (p16) p16[i] = f32_to_bf16(p[i]);
  }
}

__global__ void step_inc_kernel(float* t) { *t += 1.f; }

// Lazy (sparse-row) Adam over an embedding table (rows, cols) of the flat buffer: a row
// whose gradient is all zero this step (its tokens were not in the batch) keeps p, m and v
// untouched, so the step reads 4 B and writes nothing for it instead of the dense 28 B per
// parameter (TF LazyAdam semantics; the bias corrections use the global step *tdev).
// LPR lanes per row (cols <= 4 LPR, or LPR = 64 with up to 4 column groups per lane), so a
// 100-wide table puts two rows in each wave; two row groups per trip keep loads in flight.
template <int LPR>
__global__ __launch_bounds__(256) void adam_lazy_rows_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                             float* __restrict__ m, float* __restrict__ v, long rows,
                                                             int cols, float lr, float b1, float b2, float eps,
                                                             float wd, int torch_style,
                                                             const float* __restrict__ skip,
                                                             const float* __restrict__ tdev,
                                                             unsigned short* __restrict__ p16,
                                                             const int* __restrict__ rowlist) {
  // rowlist (optional): `rows` entries naming the candidate rows (< 0: none), e.g. the rows a
  // sparse-gradient table touched this step (parallel/sparse_rows.py); the all-zero test
  // still applies to each listed row
  constexpr int NJ = LPR == 64 ? 4 : 1;  // column groups per lane
  constexpr int RPW = 64 / LPR;          // rows per wave and trip
  if (skip && *skip != 0.f) return;
  const float t = tdev[0];
  lr *= warmup_scale(tdev);
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float lr_t = torch_style ? lr / bc1 : lr * sqrtf(bc2) / bc1;
  const float bc2_sqrt_inv = torch_style ? rsqrtf(bc2) : 1.f;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, ln = lane % LPR;
  const unsigned long long gmask = LPR == 64 ? ~0ull : (((1ull << LPR) - 1ull) << (sub * LPR));
  const long wave0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r0 = wave0 * 2 * RPW; r0 < rows; r0 += nwaves * 2 * RPW) {
    f32x4 gg[2][NJ];
    bool live[2];
    long rr[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long i = r0 + h * RPW + sub;
      const long r = i >= rows ? -1 : rowlist ? (long)rowlist[i] : i;
      rr[h] = r;
      bool nz = false;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = 4 * ln + 4 * LPR * j;
        gg[h][j] = (r >= 0 && c < cols) ? *reinterpret_cast<const f32x4*>(g + (size_t)r * cols + c)
                                        : f32x4{0.f, 0.f, 0.f, 0.f};
        nz |= gg[h][j][0] != 0.f || gg[h][j][1] != 0.f || gg[h][j][2] != 0.f || gg[h][j][3] != 0.f;
      }
      live[h] = (__ballot(nz) & gmask) != 0ull;  // any column of MY row
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long r = rr[h];
      if (!live[h] || r < 0) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = 4 * ln + 4 * LPR * j;
        if (c >= cols) continue;
        const size_t o = (size_t)r * cols + c;
        f32x4 pp = *reinterpret_cast<f32x4*>(p + o);
        f32x4 mm = *reinterpret_cast<f32x4*>(m + o);
        f32x4 vv = *reinterpret_cast<f32x4*>(v + o);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float gk = gg[h][j][k] + wd * pp[k];
          mm[k] = b1 * mm[k] + (1.f - b1) * gk;
          vv[k] = b2 * vv[k] + (1.f - b2) * gk * gk;
          const float den = torch_style ? (sqrtf(vv[k]) * bc2_sqrt_inv + eps) : (sqrtf(vv[k]) + eps);
          pp[k] -= lr_t * mm[k] / den;
        }
        *reinterpret_cast<f32x4*>(p + o) = pp;
        *reinterpret_cast<f32x4*>(m + o) = mm;
        *reinterpret_cast<f32x4*>(v + o) = vv;
        if (p16) store_bf16x4(p16 + o, pp);
      }
    }
  }
}

// fp32 (rows, cols) -> bf16 (rows, ldo) with zero padding of columns cols..ldo-1
__global__ void cast_pad_bf16_kernel(const float* __restrict__ in, unsigned short* __restrict__ out, long rows, int cols,
                                     int ldo) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  long total = rows * ldo;
  for (; i < total; i += stride) {
    long r = i / ldo;
    int c = (int)(i - r * ldo);
    out[i] = c < cols ? f32_to_bf16(in[r * cols + c]) : (unsigned short)0;
  }
}

// sum of squares + non-finite flag over a flat buffer.  One workgroup per CU-pair at most
// (<= 512 same-address atomics per call: 4096 of them serialised at one L2 channel cost
// ~40 us), 16-byte loads with four in flight per lane.
__device__ __forceinline__ void sq_acc(const f32x4& v, float& s, float& bad) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (!isfinite(v[k])) bad = 1.f;
    else s += v[k] * v[k];
  }
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ out2,
                                                    long long* fx) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const long n4 = ((uintptr_t)x & 15) ? 0 : n / 4;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  float s = 0.f, bad = 0.f;
  long i = t;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const f32x4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
    sq_acc(a, s, bad);
    sq_acc(b, s, bad);
    sq_acc(c, s, bad);
    sq_acc(d, s, bad);
  }
  for (; i < n4; i += stride) sq_acc(x4[i], s, bad);
  for (long j = n4 * 4 + t; j < n; j += stride) {
    const float v = x[j];
    if (!isfinite(v)) bad = 1.f;
    else s += v * v;
  }
  s = wave_sum(s);
  bad = wave_max(bad);
  __shared__ float ws[4], wb[4];
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { ws[w] = s; wb[w] = bad; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = ws[0] + ws[1] + ws[2] + ws[3];
    float b = fmaxf(fmaxf(wb[0], wb[1]), fmaxf(wb[2], wb[3]));
    if (fx) fx_add(fx, 0, tot);  // deterministic mode (common.h)
    else atomicAdd(&out2[0], tot);
    if (b != 0.f) atomicExch(&out2[1], 1.f);
  }
}

__global__ void scale_kernel(float* __restrict__ x, long n, float s) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) x[i] *= s;
}

}  // namespace optim
}  // namespace pv

using namespace pv;

static int g_adam_grid = 16384;  // 16384: -2..4 % vs 4096 (tools/adam_stream_micro.py)
static void launch_adam(dim3 grid, hipStream_t st, float* p, const float* g, float* m, float* v, long n, float lr,
                        float b1, float b2, float eps, float wd, int torch_style, float bc2i, const float* skip,
                        const float* tdev, unsigned short* p16) {
  hipLaunchKernelGGL(pv::optim::adam_kernel, grid, dim3(256), 0, st, p, g, m, v, n, lr, b1, b2, eps, wd, torch_style,
                     bc2i, skip, tdev, p16);
}

static unsigned grid_for(long n, int per_thread) {
  long b = (n / per_thread + 255) / 256;
  if (b > g_adam_grid) b = g_adam_grid;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// Device-counter variant: *tdev += 1, then the update with the bias corrections of step
// *tdev computed in the kernel — the whole optimizer step is replayable from a hipGraph.
PV_API int pv_adam_dev(float* p, const float* g, float* m, float* v, long n, float* tdev, float lr, float b1,
                       float b2, float eps, float wd, int torch_style, const float* skip, void* stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  hipLaunchKernelGGL(pv::optim::step_inc_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, tdev);
  PV_LAUNCH_CHECK();
  launch_adam(dim3(grid_for(n, 4)), (hipStream_t)stream, p, g, m, v, n, lr, b1, b2, eps, wd, torch_style, 1.f, skip,
              (const float*)tdev, (unsigned short*)nullptr);
  PV_LAUNCH_CHECK();
  return 0;
}

// Segmented step (lazy embedding rows): pv_step_inc once, then one pv_adam_seg per range of
// the flat buffer — row_len 0: dense update of n elements; row_len > 0: lazy rows of an
// (n / row_len, row_len) table.
// A/B: the dense launch's workgroup cap
PV_API int pv_adam_set_grid(int grid_cap) {
  if (grid_cap >= 256 && grid_cap <= 65536) g_adam_grid = grid_cap;
  return 0;
}

PV_API int pv_step_inc(float* tdev, void* stream) {
  hipLaunchKernelGGL(pv::optim::step_inc_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, tdev);
  PV_LAUNCH_CHECK();
  return 0;
}

// p16: optional bf16 copy of the segment written with the update (8-byte aligned).
PV_API int pv_adam_seg(float* p, const float* g, float* m, float* v, long n, int row_len, const float* tdev, float lr,
                       float b1, float b2, float eps, float wd, int torch_style, const float* skip, void* p16,
                       void* stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15 || ((uintptr_t)p16 & 7)) return -1;
  if (n <= 0) return 0;
  unsigned short* h = (unsigned short*)p16;
  if (row_len == 0) {
    launch_adam(dim3(grid_for(n, 4)), (hipStream_t)stream, p, g, m, v, n, lr, b1, b2, eps, wd, torch_style, 1.f, skip,
                tdev, h);
  } else {
    if (row_len % 4 || row_len > 1024 || n % row_len) return -2;
    const long rows = n / row_len;
    const int lpr = row_len <= 32 ? 8 : row_len <= 64 ? 16 : row_len <= 128 ? 32 : 64;
    long blocks = (rows + 8L * (64 / lpr) - 1) / (8L * (64 / lpr));  // 4 waves x 2 row groups
    if (blocks > 16384) blocks = 16384;
    const dim3 grid((unsigned)blocks);
    hipStream_t st = (hipStream_t)stream;
#define PV_LAZY(LPR)                                                                                          \
  hipLaunchKernelGGL(pv::optim::adam_lazy_rows_kernel<LPR>, grid, dim3(256), 0, st, p, g, m, v, rows, row_len, lr, \
                     b1, b2, eps, wd, torch_style, skip, tdev, h, (const int*)nullptr)
    if (lpr == 8) PV_LAZY(8);
    else if (lpr == 16) PV_LAZY(16);
    else if (lpr == 32) PV_LAZY(32);
    else PV_LAZY(64);
#undef PV_LAZY
  }
  PV_LAUNCH_CHECK();
  return 0;
}

// Lazy Adam over a LIST of rows of a (rows_total, row_len) table: rowlist[0..nlist) (entries
// < 0 skipped); p16 (optional) the table's bf16 mirror.  The sparse-gradient tables' update
// (parallel/sparse_rows.py): it streams only the candidate rows instead of the whole table.
PV_API int pv_adam_rows(float* p, const float* g, float* m, float* v, int row_len, const int* rowlist, long nlist,
                        const float* tdev, float lr, float b1, float b2, float eps, float wd, int torch_style,
                        const float* skip, void* p16, void* stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15 || ((uintptr_t)p16 & 7)) return -1;
  if (row_len % 4 || row_len > 1024 || row_len <= 0) return -2;
  if (nlist <= 0) return 0;
  const int lpr = row_len <= 32 ? 8 : row_len <= 64 ? 16 : row_len <= 128 ? 32 : 64;
  long blocks = (nlist + 8L * (64 / lpr) - 1) / (8L * (64 / lpr));
  if (blocks > 16384) blocks = 16384;
  const dim3 grid((unsigned)blocks);
  hipStream_t st = (hipStream_t)stream;
  unsigned short* h = (unsigned short*)p16;
#define PV_LAZYL(LPR)                                                                                          \
  hipLaunchKernelGGL(pv::optim::adam_lazy_rows_kernel<LPR>, grid, dim3(256), 0, st, p, g, m, v, nlist, row_len, \
                     lr, b1, b2, eps, wd, torch_style, skip, tdev, h, rowlist)
  if (lpr == 8) PV_LAZYL(8);
  else if (lpr == 16) PV_LAZYL(16);
  else if (lpr == 32) PV_LAZYL(32);
  else PV_LAZYL(64);
#undef PV_LAZYL
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_adam(float* p, const float* g, float* m, float* v, long n, int step, float lr, float b1, float b2,
                   float eps, float wd, int torch_style, const float* skip, void* stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  float lr_t, bc2i = 1.f;
  if (torch_style) {
    lr_t = (float)(lr / bc1);
    bc2i = (float)(1.0 / sqrt(bc2));
  } else {
    lr_t = (float)(lr * sqrt(bc2) / bc1);
  }
  launch_adam(dim3(grid_for(n, 4)), (hipStream_t)stream, p, g, m, v, n, lr_t, b1, b2, eps, wd, torch_style, bc2i, skip,
              (const float*)nullptr, (unsigned short*)nullptr);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_cast_pad_bf16(const float* in, void* out, long rows, int cols, int ldo, void* stream) {
  hipLaunchKernelGGL(pv::optim::cast_pad_bf16_kernel, dim3(grid_for(rows * ldo, 4)), dim3(256), 0,
                     (hipStream_t)stream, in, (unsigned short*)out, rows, cols, ldo);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_sumsq(const float* x, long n, float* out2, void* stream) {
  unsigned blocks = grid_for(n, 16);
  if (blocks > 512) blocks = 512;
  hipStream_t st = (hipStream_t)stream;
  long long* fx = pv::det_on() ? pv::det_scratch(1, st) : nullptr;
  if (pv::det_on() && !fx) return -4;
  hipLaunchKernelGGL(pv::optim::sumsq_kernel, dim3(blocks), dim3(256), 0, st, x, n, out2, fx);
  PV_LAUNCH_CHECK();
  return fx ? pv::det_flush(fx, out2, 1, st) : 0;
}

PV_API int pv_scale(float* x, long n, float s, void* stream) {
  hipLaunchKernelGGL(pv::optim::scale_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, x, n, s);
  PV_LAUNCH_CHECK();
  return 0;
}
