// Deterministic reduction mode: the fixed-point accumulator buffer and its flush
// (see common.h, "deterministic reduction mode").  pv_set_deterministic(1) switches the
// conv backward (dW, db, dTable), the column-sum kernel and the gradient-norm kernel from
// float atomics to fixed-point ones; ops/determinism.py also keeps a training step on one
// HIP stream while it is on.
#include "common.h"

namespace pv {
namespace {
int g_det = 0;
constexpr int kMaxDev = 64;
long long* g_fx[kMaxDev] = {};  // one buffer per device (the current device at the call)
size_t g_cap[kMaxDev] = {};

__global__ __launch_bounds__(256) void fx_flush_kernel(const long long* __restrict__ fx, float* __restrict__ dst,
                                                       long n, const unsigned* __restrict__ flag) {
  const long stride = (long)gridDim.x * blockDim.x;
  const bool poisoned = flag != nullptr && *flag != 0u;  // an addend was clamped (common.h fx_add)
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long v = fx[i];
    // |total| >= 2^62: the sum may have wrapped -> NaN, which the non-finite gradient guard
    // turns into a skipped step
    const bool overflow = poisoned || v >= (1LL << 62) || v <= -(1LL << 62);
    if (overflow) dst[i] = __builtin_nanf("");
    else if (v != 0) dst[i] += (float)((double)v * (1.0 / 1099511627776.0));
  }
}
}  // namespace

bool det_on() { return g_det != 0; }

long long* det_scratch_flag(size_t n, hipStream_t st, unsigned* flag) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  if (n > g_cap[dev]) {
    if (g_fx[dev]) {
      if (hipDeviceSynchronize() != hipSuccess) return nullptr;
      (void)hipFree(g_fx[dev]);
      g_fx[dev] = nullptr;
      g_cap[dev] = 0;
    }
    const size_t cap = n < ((size_t)1 << 20) ? ((size_t)1 << 20) : n;
    if (hipMalloc(&g_fx[dev], cap * sizeof(long long)) != hipSuccess) {
      g_fx[dev] = nullptr;
      return nullptr;
    }
    g_cap[dev] = cap;
  }
  if (hipMemsetAsync(g_fx[dev], 0, n * sizeof(long long), st) != hipSuccess) return nullptr;
  if (flag != nullptr && hipMemsetAsync(flag, 0, sizeof(unsigned), st) != hipSuccess) return nullptr;
  return g_fx[dev];
}

int det_flush_flag(const long long* fx, float* dst, size_t n, hipStream_t st, const unsigned* flag) {
  if (n == 0) return 0;
  long blocks = ((long)n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fx_flush_kernel, dim3((unsigned)blocks), dim3(256), 0, st, fx, dst, (long)n, flag);
  PV_LAUNCH_CHECK();
  return 0;
}
}  // namespace pv

PV_API void pv_set_deterministic(int on) { pv::g_det = on ? 1 : 0; }
PV_API int pv_get_deterministic() { return pv::g_det; }
