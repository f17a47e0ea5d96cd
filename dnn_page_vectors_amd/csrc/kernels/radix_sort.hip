// Stable LSD radix sort of (key, uint32 value) pairs — the bucketing step of the conv
// backward's embedding-table gradient (conv_pool_bwd.hip: emit -> sort -> reduce).
//
// Written for hipGraph capture and for wave64:
//  * no host-side memsets, no device atomics, no decoupled look-back, no ordered block ids:
//    every counter a launch reads was written by an earlier launch of the same sequence
//    (rocPRIM's onesweep resets its look-back / block-id state with hipMemsetAsync nodes
//    and faulted after ~100 graph replays interleaved with eager work; see docs/PERF.md);
//  * 8-bit digits, 3 launches per pass: count (per-tile digit histogram), scan (per digit,
//    over the tiles), scatter (stable in-tile ranking, LDS-staged coalesced writes);
//  * in-tile ranking without atomics: a wave takes its 64 x IPT items in rounds of 64
//    consecutive items; the lanes holding the same digit find each other with one ballot
//    per digit bit, the lowest of them (the leader) advances the wave's counter for that
//    digit.  Rank order = (digit, wave, round, lane) = input order within a digit: stable.
//
// Layout of the temp buffer: key ping-pong copy (n keys), value copy (n u32), hist
// (256 x tiles u32, digit-major), totals (256 u32).
#include "common.h"
#include <stdlib.h>

namespace pv {
namespace rsort {
PV_DEBUG_FLAG

constexpr int BT = 256;             // threads per block (4 waves)
constexpr int NW = BT / WAVE;
constexpr int IPT = 16;             // items per thread
constexpr int TILE = BT * IPT;      // 4096 items per tile
constexpr int RADIX = 256;
constexpr int WTILE = WAVE * IPT;   // items per wave

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return (1ull << lane) - 1ull;
}

// Lanes of this wave whose (valid) digit equals mine, from one ballot per digit bit.
__device__ __forceinline__ unsigned long long peers_of(unsigned d, bool valid, int nbits) {
  unsigned long long m = __ballot(valid);
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long bb = __ballot(valid && bit);
    m &= bit ? bb : ~bb;
  }
  return valid ? m : 0ull;
}

// Exclusive scan of one value per thread over the 256 threads of the block; returns the
// block total in *total.  ws: NW words of LDS scratch.
__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned* ws, unsigned* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  unsigned base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const unsigned s = ws[i];
    base += i < w ? s : 0u;
    tot += s;
  }
  __syncthreads();  // ws reusable after return
  *total = tot;
  return base + x - v;
}

// ---- pass kernel 1: per-tile digit histogram -> hist[d * nb + tile] ----------------------
template <typename KT, int IPT_>
__global__ __launch_bounds__(BT) void rs_count_kernel(const KT* __restrict__ keys, long n, int shift, int nbits,
                                                      unsigned* __restrict__ hist, int nb) {
  __shared__ unsigned cnt[NW][RADIX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < NW * RADIX; i += BT) (&cnt[0][0])[i] = 0u;
  __syncthreads();
  const unsigned mask = (1u << nbits) - 1u;
  const long base = (long)blockIdx.x * (BT * IPT_) + (long)w * (WAVE * IPT_);
  unsigned d[IPT_];
#pragma unroll
  for (int j = 0; j < IPT_; ++j) {
    const long i = base + j * WAVE + lane;
    d[j] = i < n ? ((unsigned)keys[i] >> shift) & mask : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int j = 0; j < IPT_; ++j) {
    const bool valid = d[j] != 0xFFFFFFFFu;
    const unsigned long long pm = peers_of(d[j], valid, nbits);
    const bool leader = valid && (pm & lanemask_lt()) == 0ull;
    if (leader) cnt[w][d[j]] += (unsigned)__popcll(pm);
  }
  __syncthreads();
  const int t = threadIdx.x;  // BT == RADIX: thread t owns digit t
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += cnt[i][t];
  hist[(long)t * nb + blockIdx.x] = s;
}

// ---- pass kernel 2: exclusive scan of each digit's row over the tiles (in place) ---------
__global__ __launch_bounds__(BT) void rs_scan_kernel(unsigned* __restrict__ hist, int nb,
                                                     unsigned* __restrict__ totals) {
  __shared__ unsigned ws[NW];
  unsigned* row = hist + (long)blockIdx.x * nb;
  unsigned carry = 0;
  for (int c = 0; c < nb; c += BT) {
    const int i = c + threadIdx.x;
    const unsigned v = i < nb ? row[i] : 0u;
    unsigned tot;
    const unsigned ex = block_excl_scan(v, ws, &tot);
    if (i < nb) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// ---- pass kernel 3: stable scatter ---------------------------------------------------------
// vals_in == nullptr: values are the input positions (iota), i.e. the first pass of a sort
// whose payload is "where did this key come from".
template <typename KT, int IPT_>
__global__ __launch_bounds__(BT) void rs_scatter_kernel(const KT* __restrict__ keys_in,
                                                        const unsigned* __restrict__ vals_in,
                                                        KT* __restrict__ keys_out, unsigned* __restrict__ vals_out,
                                                        long n, int shift, int nbits,
                                                        const unsigned* __restrict__ hist,
                                                        const unsigned* __restrict__ totals, int nb) {
  __shared__ unsigned cnt[NW][RADIX];   // per-wave digit counters, then per-wave digit offsets
  __shared__ unsigned dstart[RADIX];    // first in-tile position of each digit
  __shared__ unsigned gbase[RADIX];     // global position of (digit, this tile)'s first item
  __shared__ unsigned ws[NW];
  __shared__ KT kst[(BT * IPT_)];
  __shared__ unsigned vst[(BT * IPT_)];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
  for (int i = t; i < NW * RADIX; i += BT) (&cnt[0][0])[i] = 0u;
  {  // global base of each digit: exclusive scan of the digit totals + this tile's offset
    unsigned tot;
    const unsigned ex = block_excl_scan(totals[t], ws, &tot);
    gbase[t] = ex + hist[(long)t * nb + blockIdx.x];
  }
  __syncthreads();
  const unsigned mask = (1u << nbits) - 1u;
  const long tbase = (long)blockIdx.x * (BT * IPT_);
  const long base = tbase + (long)w * (WAVE * IPT_);
  KT k[IPT_];
  unsigned v[IPT_];
#pragma unroll
  for (int j = 0; j < IPT_; ++j) {
    const long i = base + j * WAVE + lane;
    const bool ok = i < n;
    k[j] = ok ? keys_in[i] : (KT)0;
    v[j] = ok ? (vals_in ? vals_in[i] : (unsigned)i) : 0u;
  }
  unsigned rank[IPT_];
#pragma unroll
  for (int j = 0; j < IPT_; ++j) {
    const long i = base + j * WAVE + lane;
    const bool valid = i < n;
    const unsigned d = ((unsigned)k[j] >> shift) & mask;
    const unsigned long long pm = peers_of(d, valid, nbits);
    const unsigned old = valid ? cnt[w][d] : 0u;
    const bool leader = valid && (pm & lanemask_lt()) == 0ull;
    rank[j] = old + (unsigned)__popcll(pm & lanemask_lt());
    if (leader) cnt[w][d] = old + (unsigned)__popcll(pm);
  }
  __syncthreads();
  {  // digit t: per-wave exclusive offsets, in-tile start of the digit
    unsigned s = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const unsigned c = cnt[i][t];
      cnt[i][t] = s;
      s += c;
    }
    unsigned tot;
    dstart[t] = block_excl_scan(s, ws, &tot);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT_; ++j) {
    const long i = base + j * WAVE + lane;
    if (i < n) {
      const unsigned d = ((unsigned)k[j] >> shift) & mask;
      const unsigned pos = dstart[d] + cnt[w][d] + rank[j];
      PV_CHECK(pos < (unsigned)(BT * IPT_), PV_ERR_LDS);
      kst[pos] = k[j];
      vst[pos] = v[j];
    }
  }
  __syncthreads();
  const int tn = (int)min((long)(BT * IPT_), n - tbase);
  for (int i = t; i < tn; i += BT) {
    const KT kk = kst[i];
    const unsigned d = ((unsigned)kk >> shift) & mask;
    const unsigned g = gbase[d] + ((unsigned)i - dstart[d]);
    PV_CHECK((long)g < n, PV_ERR_POS);
    keys_out[g] = kk;
    vals_out[g] = vst[i];
  }
}

PV_DEBUG_EXPORT(rsort)

struct Layout {
  size_t ktmp, vtmp, hist, totals, bytes;
  int nb, passes;
};

__host__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Items per thread: 16 (4096-item tiles) for large sorts; small ones (the sparse bag
// backward's ~200k keys) use 1024-item tiles so the grid still covers the CUs.
// PAGEVEC_RSORT_IPT / pv_rsort_set_ipt: 4, 16 or 32 for every size (A/B; 0 = this rule).
inline int g_ipt_override = [] {
  const char* e = getenv("PAGEVEC_RSORT_IPT");
  return e ? atoi(e) : 0;
}();
__host__ inline int pick_ipt(long n) {
  if (g_ipt_override == 4 || g_ipt_override == 16 || g_ipt_override == 32) return g_ipt_override;
  return n <= (1L << 20) ? 4 : IPT;
}

__host__ inline Layout layout(long n, int end_bit, int key_bytes) {
  Layout L{};
  const long tile = (long)BT * pick_ipt(n);
  L.nb = (int)((n + tile - 1) / tile);
  L.passes = (end_bit + 7) / 8;
  size_t o = 0;
  L.ktmp = o;
  o = align256(o + (size_t)n * key_bytes);
  L.vtmp = o;
  o = align256(o + (size_t)n * 4);
  L.hist = o;
  o = align256(o + (size_t)RADIX * L.nb * 4);
  L.totals = o;
  o = align256(o + (size_t)RADIX * 4);
  L.bytes = o;
  return L;
}

template <typename KT>
int sort_impl(void* temp, long temp_bytes, const KT* keys_in, KT* keys_out, const unsigned* vals_in,
              unsigned* vals_out, long n, int end_bit, hipStream_t st) {
  if (n <= 0) return 0;
  if (end_bit < 1 || end_bit > (int)(8 * sizeof(KT)) || n >= (1L << 32) - TILE) return -1;
  const Layout L = layout(n, end_bit, (int)sizeof(KT));
  if (temp == nullptr || (size_t)temp_bytes < L.bytes) return -2;
  char* tb = (char*)temp;
  KT* ktmp = (KT*)(tb + L.ktmp);
  unsigned* vtmp = (unsigned*)(tb + L.vtmp);
  unsigned* hist = (unsigned*)(tb + L.hist);
  unsigned* totals = (unsigned*)(tb + L.totals);
  // ping-pong so that the last pass lands in the output buffers
  const KT* kin = keys_in;
  const unsigned* vin = vals_in;
  for (int p = 0; p < L.passes; ++p) {
    const int shift = 8 * p;
    const int nbits = min(8, end_bit - shift);
    const bool to_out = ((L.passes - 1 - p) & 1) == 0;
    KT* kout = to_out ? keys_out : ktmp;
    unsigned* vout = to_out ? vals_out : vtmp;
    if (pick_ipt(n) == 4)
      hipLaunchKernelGGL((rs_count_kernel<KT, 4>), dim3(L.nb), dim3(BT), 0, st, kin, n, shift, nbits, hist, L.nb);
    else if (pick_ipt(n) == 32)
      hipLaunchKernelGGL((rs_count_kernel<KT, 32>), dim3(L.nb), dim3(BT), 0, st, kin, n, shift, nbits, hist, L.nb);
    else
      hipLaunchKernelGGL((rs_count_kernel<KT, IPT>), dim3(L.nb), dim3(BT), 0, st, kin, n, shift, nbits, hist, L.nb);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(RADIX), dim3(BT), 0, st, hist, L.nb, totals);
    if (pick_ipt(n) == 4)
      hipLaunchKernelGGL((rs_scatter_kernel<KT, 4>), dim3(L.nb), dim3(BT), 0, st, kin, vin, kout, vout, n, shift,
                         nbits, (const unsigned*)hist, (const unsigned*)totals, L.nb);
    else if (pick_ipt(n) == 32)
      hipLaunchKernelGGL((rs_scatter_kernel<KT, 32>), dim3(L.nb), dim3(BT), 0, st, kin, vin, kout, vout, n, shift,
                         nbits, (const unsigned*)hist, (const unsigned*)totals, L.nb);
    else
      hipLaunchKernelGGL((rs_scatter_kernel<KT, IPT>), dim3(L.nb), dim3(BT), 0, st, kin, vin, kout, vout, n, shift,
                         nbits, (const unsigned*)hist, (const unsigned*)totals, L.nb);
    PV_LAUNCH_CHECK();
    kin = kout;
    vin = vout;
  }
  return 0;
}

}  // namespace rsort
}  // namespace pv

using namespace pv;

PV_API void pv_rsort_set_ipt(int ipt) { pv::rsort::g_ipt_override = ipt; }

PV_API long pv_rsort_temp_bytes(long n, int end_bit, int key_bytes) {
  return (long)pv::rsort::layout(n, end_bit, key_bytes).bytes;
}

// key_bytes 2 (uint16 keys) or 4 (uint32 keys); vals_in may be null (values = positions).
// Sorts by bits [0, end_bit) of the key; stable; deterministic.
PV_API int pv_rsort_pairs(void* temp, long temp_bytes, const void* keys_in, void* keys_out, const unsigned* vals_in,
                          unsigned* vals_out, long n, int end_bit, int key_bytes, void* stream) {
  using namespace pv::rsort;
  hipStream_t st = (hipStream_t)stream;
  if (key_bytes == 2)
    return sort_impl<unsigned short>(temp, temp_bytes, (const unsigned short*)keys_in, (unsigned short*)keys_out,
                                     vals_in, vals_out, n, end_bit, st);
  if (key_bytes == 4)
    return sort_impl<unsigned>(temp, temp_bytes, (const unsigned*)keys_in, (unsigned*)keys_out, vals_in, vals_out, n,
                               end_bit, st);
  return -3;
}
