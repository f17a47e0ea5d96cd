// hipBLASLt GEMMs with fused epilogues for the transformer FFN (ops/transformer.py::_FfnFn).
//
// The BERT FFN is  f = gelu(x W1^T + b1),  y = f W2^T.  With plain library GEMMs the bias +
// GELU forward and the GELU backward are separate streaming kernels over the (T x 3072)
// activation — per layer at T = 73728: one read + one write of h forward (~0.9 GB) and
// three passes backward (dF, h, dH: ~1.4 GB), 6 % + 3.4 % of the step in the round-4 profile
// (profiles/r4_profiles/bert_kernel_stats_r4.md).  hipBLASLt applies them in the GEMM's own
// epilogue while the tile is in registers:
//
//   forward   GELU_AUX_BIAS : D = gelu(A B + bias), AUX = A B + bias (kept for the backward)
//   backward  DGELU_BGRAD   : D = (A B) * gelu'(AUX), bias = column sums of D (db1)
//
// Plain library GEMMs stay plain (no hand-written schedule: round-4 measured the in-tree GEMM
// engine at 60-90 % of hipBLASLt, PERF.md).  The library is torch's own hipBLASLt (same
// soname, already loaded when this one is), so the tuned solution tables are shared.
//
// Layout: column-major as hipBLASLt sees it; ops/transformer.py maps PyTorch's row-major
// operands (D^T = B^T A^T).  Descriptors + the heuristic's algorithm are cached per problem.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"

namespace {

enum Epi : int {
  EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU_AUX_BIAS = 2, EPI_DGELU = 3, EPI_DGELU_BGRAD = 4,
  EPI_GELU = 5, EPI_GELU_BIAS = 6, EPI_GELU_AUX = 7
};
constexpr int EPI_NO_AUX_TYPE = 100;  // + epi: leave the aux data type attribute unset (probe)

hipblasLtEpilogue_t lt_epilogue(int e) {
  switch (e % EPI_NO_AUX_TYPE) {
    case EPI_BIAS: return HIPBLASLT_EPILOGUE_BIAS;
    case EPI_GELU_AUX_BIAS: return HIPBLASLT_EPILOGUE_GELU_AUX_BIAS;
    case EPI_DGELU: return HIPBLASLT_EPILOGUE_DGELU;
    case EPI_DGELU_BGRAD: return HIPBLASLT_EPILOGUE_DGELU_BGRAD;
    case EPI_GELU: return HIPBLASLT_EPILOGUE_GELU;
    case EPI_GELU_BIAS: return HIPBLASLT_EPILOGUE_GELU_BIAS;
    case EPI_GELU_AUX: return HIPBLASLT_EPILOGUE_GELU_AUX;
    default: return HIPBLASLT_EPILOGUE_DEFAULT;
  }
}

constexpr int MAX_CAND = 16;

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulHeuristicResult_t cand[MAX_CAND];
  int ncand = 0;
  int pick = 0;        // candidate in use
  bool tuned = false;  // timed once (autotune on)
  bool ok = false;
};

using Key = std::tuple<int, int, int, int, int, int, int, int, int, int, int, int, long, int>;

int g_tune = 0;  // pv_lt_set_tune: time the heuristic's candidates once per problem

struct State {
  std::mutex mu;
  std::map<int, hipblasLtHandle_t> handles;  // per device
  std::map<Key, Plan> plans;
};

State& state() {
  static State* s = new State();  // never destroyed: no teardown order against the HIP runtime
  return *s;
}

#define LT_TRY(x)                                   \
  do {                                              \
    hipblasStatus_t st_ = (x);                      \
    if (st_ != HIPBLAS_STATUS_SUCCESS) return -100 - (int)st_; \
  } while (0)

int make_plan(hipblasLtHandle_t h, Plan& p, int ta, int tb, int m, int n, int k, int lda, int ldb, int ldd,
              int epi, int bias_f32, long ws_bytes, int d_f32) {
  LT_TRY(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  hipblasLtEpilogue_t e = lt_epilogue(epi);
  LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  const bool aux_type = epi < EPI_NO_AUX_TYPE;
  epi %= EPI_NO_AUX_TYPE;
  if (epi == EPI_BIAS || epi == EPI_GELU_AUX_BIAS || epi == EPI_DGELU_BGRAD || epi == EPI_GELU_BIAS) {
    hipDataType bt = bias_f32 ? HIP_R_32F : HIP_R_16BF;
    LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (epi == EPI_GELU_AUX_BIAS || epi == EPI_DGELU || epi == EPI_DGELU_BGRAD || epi == EPI_GELU_AUX) {
    int64_t ld = ldd;
    LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    if (aux_type) {
      hipDataType at = HIP_R_16BF;
      LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
    }
  }
  // stored (rows, cols) of each operand, column-major
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ta ? k : m, ta ? m : k, lda));
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb));
  LT_TRY(hipblasLtMatrixLayoutCreate(&p.d, d_f32 ? HIP_R_32F : HIP_R_16BF, m, n, ldd));
  hipblasLtMatmulPreference_t pref;
  LT_TRY(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wsb = (uint64_t)ws_bytes;
  LT_TRY(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  int got = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.a, p.b, p.d, p.d, pref, MAX_CAND, p.cand, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || got < 1) return -3;  // no solution for this epilogue / shape
  p.ncand = got;
  p.ok = true;
  return 0;
}

// Time every candidate (1 warm-up + 3 runs each, events on the caller's stream) and keep the
// fastest; outside stream capture only, a host sync once per problem.  beta = 0 problems time
// in place (each run rewrites D / AUX / the bias gradient with the same values); beta != 0
// ones (D += A B, the residual dX) time with beta = 0 into a scratch D, so D keeps its input.
void autotune(hipblasLtHandle_t h, Plan& p, const void* A, const void* B, void* D, bool acc, size_t dbytes, void* ws,
              hipStream_t st) {
  p.tuned = true;
  if (p.ncand < 2) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  void* dst = D;
  if (acc && hipMalloc(&dst, dbytes) != hipSuccess) return;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return;
  if (hipEventCreate(&e1) != hipSuccess) { hipEventDestroy(e0); return; }
  const float alpha = 1.f, beta = 0.f;
  float best = 1e30f;
  int besti = p.pick;
  for (int c = 0; c < p.ncand; ++c) {
    auto run = [&]() {
      return hipblasLtMatmul(h, p.op, &alpha, A, p.a, B, p.b, &beta, dst, p.d, dst, p.d, &p.cand[c].algo, ws,
                             p.cand[c].workspaceSize, st);
    };
    if (run() != HIPBLAS_STATUS_SUCCESS) continue;
    hipEventRecord(e0, st);
    bool ok = true;
    for (int i = 0; i < 3 && ok; ++i) ok = run() == HIPBLAS_STATUS_SUCCESS;
    hipEventRecord(e1, st);
    if (!ok || hipEventSynchronize(e1) != hipSuccess) continue;
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) { best = ms; besti = c; }
  }
  p.pick = besti;
  if (acc) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(dst);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

}  // namespace

PV_API void pv_lt_set_tune(int on) { g_tune = on; }

// D (m x n, ldd) = op(A) op(B) [+ beta D] with epilogue `epi` (see Epi); bf16 A / B / AUX, D
// bf16 (fp32 when d_f32), fp32 accumulation and scalars.  bias: length m (bf16, or fp32 when bias_f32); for
// DGELU_BGRAD it is the OUTPUT bias gradient.  aux: m x n with leading dimension ldd.
// Returns 0, -3 when hipBLASLt has no solution (the caller falls back to plain GEMM + kernels),
// or -100 - hipblasStatus_t.
PV_API int pv_lt_gemm(int ta, int tb, int m, int n, int k, const void* A, int lda, const void* B, int ldb, void* D,
                      int ldd, int d_f32, float beta, const void* bias, int bias_f32, void* aux, int epi,
                      void* ws, long ws_bytes, void* stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  State& S = state();
  std::lock_guard<std::mutex> lock(S.mu);
  auto hit = S.handles.find(dev);
  if (hit == S.handles.end()) {
    hipblasLtHandle_t h;
    LT_TRY(hipblasLtCreate(&h));
    hit = S.handles.emplace(dev, h).first;
  }
  Key key{dev, ta, tb, m, n, k, lda, ldb, ldd, epi, bias_f32, beta != 0.f, ws_bytes, d_f32};
  auto it = S.plans.find(key);
  if (it == S.plans.end()) {
    Plan p;
    int r = make_plan(hit->second, p, ta, tb, m, n, k, lda, ldb, ldd, epi, bias_f32, ws_bytes, d_f32);
    it = S.plans.emplace(key, p).first;  // a failed plan is cached too: no retry per call
    if (r != 0) return r;
  }
  Plan& p = it->second;
  if (!p.ok) return -3;
  if (bias) LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
  if (aux) LT_TRY(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
  if (g_tune && !p.tuned)
    autotune(hit->second, p, A, B, D, beta != 0.f, (size_t)ldd * n * (d_f32 ? 4 : 2), ws, (hipStream_t)stream);
  const float alpha = 1.f;
  const hipblasLtMatmulHeuristicResult_t& c = p.cand[p.pick];
  LT_TRY(hipblasLtMatmul(hit->second, p.op, &alpha, A, p.a, B, p.b, &beta, D, p.d, D, p.d, &c.algo, ws,
                         c.workspaceSize, (hipStream_t)stream));
  return 0;
}
