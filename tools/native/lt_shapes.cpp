// Standalone hipBLASLt timing of the BERT GEMM shapes against the SYSTEM ROCm (this image's
// /opt/rocm hipBLASLt), outside any torch process — to compare with the library build torch
// bundles (tools/ffn_micro.py, profiles/r5_prof_bert_kernel_stats.md).  bf16 in, fp32
// accumulate, bf16 (or fp32 for the weight gradients) out; best of the heuristic's top 8.
//   hipcc --offload-arch=gfx950 -O2 tools/native/lt_shapes.cpp -lhipblaslt -o /tmp/lt_shapes
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

// random bf16 in [-1, 1) (constant operands draw less power and clock higher: not comparable)
static int fill_random(void* dst, size_t n, unsigned seed) {
  std::vector<uint16_t> h(n);
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  for (size_t i = 0; i < n; ++i) {
    const float f = u(g);
    uint32_t b;
    std::memcpy(&b, &f, 4);
    h[i] = (uint16_t)(b >> 16);
  }
  return (int)hipMemcpy(dst, h.data(), n * 2, hipMemcpyHostToDevice);
}

#define CK(x)                                                             \
  do {                                                                    \
    auto e_ = (x);                                                        \
    if ((int)e_ != 0) {                                                   \
      std::printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__);    \
      return 1;                                                           \
    }                                                                     \
  } while (0)

struct Shape {
  const char* name;
  int m, n, k, ta, tb, d32;
};

int main() {
  // column-major problems equivalent to the row-major BERT layers (T = 73728 tokens)
  const int T = 73728;
  std::vector<Shape> shapes = {
      {"qkv_fwd  T x 2304 x 768", 2304, T, 768, 1, 0, 0},
      {"ffn1_fwd T x 3072 x 768", 3072, T, 768, 1, 0, 0},
      {"ffn2_fwd T x 768 x 3072", 768, T, 3072, 1, 0, 0},
      {"ffn2_dx  T x 3072 x 768", 3072, T, 768, 0, 0, 0},
      {"ffn1_dw  3072 x 768 x T (fp32)", 768, 3072, T, 0, 1, 1},
      {"square 8192", 8192, 8192, 8192, 1, 0, 0},
  };
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  size_t wsb = 64 << 20;
  void* ws;
  CK(hipMalloc(&ws, wsb));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (auto& s : shapes) {
    const int rowsA = s.ta ? s.k : s.m, colsA = s.ta ? s.m : s.k;
    const int rowsB = s.tb ? s.n : s.k, colsB = s.tb ? s.k : s.n;
    void *A, *B, *D;
    CK(hipMalloc(&A, (size_t)rowsA * colsA * 2));
    CK(hipMalloc(&B, (size_t)rowsB * colsB * 2));
    CK(hipMalloc(&D, (size_t)s.m * s.n * (s.d32 ? 4 : 2)));
    CK(fill_random(A, (size_t)rowsA * colsA, 1));
    CK(fill_random(B, (size_t)rowsB * colsB, 2));
    hipblasLtMatmulDesc_t op;
    CK(hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t oa = s.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = s.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa)));
    CK(hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob)));
    hipblasLtMatrixLayout_t la, lb, ld;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, rowsA, colsA, rowsA));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, rowsB, colsB, rowsB));
    CK(hipblasLtMatrixLayoutCreate(&ld, s.d32 ? HIP_R_32F : HIP_R_16BF, s.m, s.n, s.m));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
    hipblasLtMatmulHeuristicResult_t res[8];
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, op, la, lb, ld, ld, pref, 8, res, &got));
    float alpha = 1.f, beta = 0.f, best = 1e30f, first = 0.f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int c = 0; c < got; ++c) {
      bool ok = true;
      for (int i = 0; i < 3 && ok; ++i)
        ok = hipblasLtMatmul(h, op, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[c].algo, ws,
                             res[c].workspaceSize, st) == HIPBLAS_STATUS_SUCCESS;
      if (!ok) continue;
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < 10; ++i)
        hipblasLtMatmul(h, op, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[c].algo, ws, res[c].workspaceSize, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 10.f;
      if (c == 0) first = ms;
      if (ms < best) best = ms;
    }
    const double fl = 2.0 * s.m * (double)s.n * s.k;
    std::printf("%-32s candidates %d  heuristic#1 %.3f ms (%.0f TF/s)  best %.3f ms (%.0f TF/s)\n", s.name, got,
                first, fl / first / 1e9, best, fl / best / 1e9);
    hipFree(A);
    hipFree(B);
    hipFree(D);
  }
  int v = 0;
  hipblasLtGetVersion(h, &v);
  std::printf("hipBLASLt version %d\n", v);
  return 0;
}
