// MFMA issue-rate micro (gfx950): cycles per instruction and chip FLOP/s for the bf16 shapes the
// conv forward can use — v_mfma_f32_16x16x32_bf16 (production), v_mfma_f32_16x16x16_bf16 (a
// half-depth step for the K tails: k3 K = 300 = 9 x 32 + 12) and v_mfma_f32_32x32x16_bf16.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_micro.hip -o /tmp/mfma_micro && /tmp/mfma_micro
//
// Every wave runs ITERS x 8 independent MFMAs on random bf16 register operands (4 or 8
// accumulators), s_memtime brackets the loop (cycles per MFMA, per wave); the grid fills every
// SIMD with W waves and hipEvents give the chip's FLOP/s at the clock it holds under load.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int ITERS = 4096;

template <int SHAPE>
__global__ void mfma_loop(const unsigned* seed, float* out, long long* cyc) {
  const int lane = threadIdx.x & 63;
  unsigned s = seed[0] + blockIdx.x * 977u + threadIdx.x * 131u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return (short)(0x3C00 | ((s >> 9) & 0x807F));  // bf16 in +-[2^-7, 2^-6)
  };
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = rnd(); b[i] = rnd(); }
  bf16x4 a4, b4;
  for (int i = 0; i < 4; ++i) { a4[i] = rnd(); b4[i] = rnd(); }
  f32x4 c[8];
  f32x16 d[4];
  for (int i = 0; i < 8; ++i) c[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 4; ++i) d[i] = f32x16{};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (SHAPE == 0) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[j], 0, 0, 0);
      if constexpr (SHAPE == 1) c[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c[j], 0, 0, 0);
      if constexpr (SHAPE == 2) d[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, d[j & 3], 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int i = 0; i < 8; ++i) acc += c[i][0] + c[i][3];
  for (int i = 0; i < 4; ++i) acc += d[i][0] + d[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int SHAPE>
void run(const char* name, double flop_per_mfma, int waves_per_simd) {
  const int threads = 256 * waves_per_simd;  // one workgroup per CU: 4 SIMDs x W waves
  const int blocks = 256;
  unsigned* seed;
  float* out;
  long long* cyc;
  hipMalloc(&seed, 4);
  hipMemset(seed, 0x5A, 4);
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(threads), 0, 0, seed, out, cyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 20;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mfma_loop<SHAPE>, dim3(blocks), dim3(threads), 0, 0, seed, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int nw = blocks * threads / 64;
  long long* h = (long long*)malloc(sizeof(long long) * nw);
  hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < nw; ++i) mean += (double)h[i];
  mean /= nw;
  const double n_mfma = (double)ITERS * 8;
  const double flops = flop_per_mfma * n_mfma * nw * reps;
  printf("%-22s waves/SIMD %d: %6.2f cycles per MFMA per wave (%.2f per SIMD), %7.1f TFLOP/s chip\n", name,
         waves_per_simd, mean / n_mfma, mean / n_mfma / waves_per_simd, flops / (ms * 1e-3) / 1e12);
  free(h);
  hipFree(seed);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 4; ++w) {
    run<0>("16x16x32_bf16", 2.0 * 16 * 16 * 32, w);
    run<1>("16x16x16_bf16", 2.0 * 16 * 16 * 16, w);
    run<2>("32x32x16_bf16", 2.0 * 32 * 32 * 16, w);
  }
  return 0;
}
