// Word2Vec training (CBOW or skip-gram, negative sampling) — the reference trains its word
// vectors with gensim (dssm_cnn_v2/w2v.py:8-53, dssm_cnn/w2v.py: identical):
// Word2Vec(sentences, size=num_features, min_count, window=context, sample=1e-3) with
// gensim's defaults sg=0 (CBOW, cbow_mean=1), negative=5, alpha 0.025 -> 0.0001.
//
// MI355X design: one wave per center position (lanes over the vector dimensions, DPL
// values per lane), asynchronous SGD like gensim's / word2vec.c's worker threads: the
// centers of a launch read the shared tables concurrently and ADD their updates with
// no-return float atomics (one wave adds one contiguous row: full-rate 256-B atomics).
// Plain read-modify-write (Hogwild proper) loses most updates of hot rows at GPU
// concurrency — a 72-word corpus collapsed to one direction — while summed updates behave
// like the mini-batch SGD of the torch oracle.  The host side (models/word2vec.py)
// subsamples and compacts the corpus on the device each epoch and launches chunks of
// centers (sized to the vocabulary, so small vocabularies see small effective batches)
// with the linearly decayed learning rate.
//
// Random draws are counter hashes of (seed, center, k) — w2v_rng below, restated in
// ops/word2vec.py for the fp32 torch oracle — so a run is reproducible given the launch
// order:  k = 0 the reduced window b (window - b = effective half-width, gensim's
// `reduced_windows`), k >= 1 the negatives (skip-gram: k = 1 + slot * negative + j).
#include "common.h"

namespace pv {
namespace w2v {

__device__ __forceinline__ unsigned w2v_rng(unsigned seed, unsigned i, unsigned k) {
  return mix32(mix32(seed ^ i) + k * 0x9E3779B9u);
}

struct Args {
  const int* words;  // (T) compacted corpus of this epoch (vocabulary ids)
  const int* sbeg;   // (T) index of the first token of the token's sentence
  const int* send;   // (T) one past the last token of the token's sentence
  const int* table;  // (table_size) unigram^0.75 sampling table
  float* win;        // (V, D) input vectors (gensim syn0)
  float* wout;       // (V, D) output vectors (gensim syn1neg)
  long begin, end;   // centers of this launch
  int table_size, D, window, negative;
  unsigned seed;
  float alpha;
};

template <int DPL>
__device__ __forceinline__ void load_row(const float* __restrict__ row, int D, int lane, float (&v)[DPL]) {
#pragma unroll
  for (int d = 0; d < DPL; ++d) {
    const int c = lane + 64 * d;
    v[d] = c < D ? row[c] : 0.f;
  }
}

// One (h -> target) logistic step for the positive and the negatives: accumulates the
// input-side error e += g * wout[t] and applies wout[t] += g * h (gensim
// fast_sentence_{cbow,sg}_neg).  Returns nothing; rows are updated in place.
template <int DPL>
__device__ __forceinline__ void train_targets(const Args& a, unsigned ctr, unsigned kbase, int center,
                                              const float (&h)[DPL], float (&e)[DPL], int lane) {
  for (int k = 0; k <= a.negative; ++k) {
    int t = center;
    float label = 1.f;
    if (k > 0) {
      t = a.table[w2v_rng(a.seed, ctr, kbase + (unsigned)k) % (unsigned)a.table_size];
      if (t == center) continue;
      label = 0.f;
    }
    float* orow = a.wout + (size_t)t * a.D;
    float o[DPL];
    load_row<DPL>(orow, a.D, lane, o);
    float f = 0.f;
#pragma unroll
    for (int d = 0; d < DPL; ++d) f += h[d] * o[d];
    f = wave_sum(f);
    const float g = (label - 1.f / (1.f + __expf(-f))) * a.alpha;
#pragma unroll
    for (int d = 0; d < DPL; ++d) {
      const int c = lane + 64 * d;
      e[d] += g * o[d];
      if (c < a.D) atomicAdd(&orow[c], g * h[d]);
    }
  }
}

template <int DPL>
__device__ __forceinline__ void add_row(float* __restrict__ row, int D, int lane, const float (&e)[DPL]) {
#pragma unroll
  for (int d = 0; d < DPL; ++d) {
    const int c = lane + 64 * d;
    if (c < D) atomicAdd(&row[c], e[d]);
  }
}

template <int DPL, bool SG>
__global__ __launch_bounds__(256) void w2v_kernel(Args a) {
  const long i = a.begin + (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= a.end) return;
  const int lane = threadIdx.x & 63;
  const unsigned ctr = (unsigned)i;
  const int w = a.window - (int)(w2v_rng(a.seed, ctr, 0u) % (unsigned)a.window);  // 1..window
  const int lo = max(a.sbeg[i], (int)(i - w)), hi = min(a.send[i], (int)(i + w + 1));
  const int center = a.words[i];
  if constexpr (!SG) {
    // CBOW, cbow_mean=1: h = mean of the context input vectors; every context row gets the
    // full error e (gensim divides e only when cbow_mean=0)
    float h[DPL], e[DPL];
#pragma unroll
    for (int d = 0; d < DPL; ++d) h[d] = e[d] = 0.f;
    int cnt = 0;
    for (int c = lo; c < hi; ++c) {
      if (c == i) continue;
      float v[DPL];
      load_row<DPL>(a.win + (size_t)a.words[c] * a.D, a.D, lane, v);
#pragma unroll
      for (int d = 0; d < DPL; ++d) h[d] += v[d];
      ++cnt;
    }
    if (cnt == 0) return;
    const float inv = 1.f / (float)cnt;
#pragma unroll
    for (int d = 0; d < DPL; ++d) h[d] *= inv;
    train_targets<DPL>(a, ctr, 0u, center, h, e, lane);
    for (int c = lo; c < hi; ++c)
      if (c != i) add_row<DPL>(a.win + (size_t)a.words[c] * a.D, a.D, lane, e);
  } else {
    // skip-gram: every context word's input vector predicts the center word
    for (int c = lo; c < hi; ++c) {
      if (c == i) continue;
      float* irow = a.win + (size_t)a.words[c] * a.D;
      float h[DPL], e[DPL];
      load_row<DPL>(irow, a.D, lane, h);
#pragma unroll
      for (int d = 0; d < DPL; ++d) e[d] = 0.f;
      train_targets<DPL>(a, ctr, (unsigned)(c - lo) * (unsigned)a.negative, center, h, e, lane);
      add_row<DPL>(irow, a.D, lane, e);
    }
  }
}

}  // namespace w2v
}  // namespace pv

using namespace pv;

// Train the centers [begin, end) of the compacted corpus with learning rate alpha.
// D <= 512 (8 values per lane), window >= 1.
PV_API int pv_w2v_train(const int* words, const int* sbeg, const int* send, const int* table, float* win,
                        float* wout, long begin, long end, int table_size, int D, int window, int negative,
                        unsigned seed, float alpha, int sg, void* stream) {
  using namespace pv::w2v;
  if (D <= 0 || D > 512 || window < 1 || negative < 0 || table_size <= 0) return -1;
  if (end <= begin) return 0;
  Args a{words, sbeg, send, table, win, wout, begin, end, table_size, D, window, negative, seed, alpha};
  const long n = end - begin;
  dim3 grid((unsigned)((n + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const int dpl = (D + 63) / 64;
#define PV_W2V(DV)                                                                                      \
  case DV:                                                                                              \
    if (sg) hipLaunchKernelGGL((w2v_kernel<DV, true>), grid, dim3(256), 0, st, a);                      \
    else hipLaunchKernelGGL((w2v_kernel<DV, false>), grid, dim3(256), 0, st, a);                        \
    break;
  switch (dpl) {
    PV_W2V(1) PV_W2V(2) PV_W2V(3) PV_W2V(4) PV_W2V(5) PV_W2V(6) PV_W2V(7) PV_W2V(8)
    default: return -1;
  }
#undef PV_W2V
  PV_LAUNCH_CHECK();
  return 0;
}
