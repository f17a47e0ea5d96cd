// One-pass counting sort of small integer keys (< 2^15) with their input positions — the
// bucketing step of the conv backward's embedding-table gradient (conv_pool_bwd.hip:
// emit -> sort -> reduce), replacing the two 8-bit LSD passes of radix_sort.hip there.
//
// The keys are token ids of a <= 32k-row hashed vocabulary, so ONE pass over a per-key
// histogram does it: gfx950's 160 KB LDS holds a block's whole 2^15-bin histogram (128 KB).
//   count   : each block histograms its contiguous slice of the keys in LDS (ds_add),
//             writes the histogram row  hist[block][key];
//   scan    : one thread per key walks the block rows: hist[b][k] <- sum_{b' < b} hist[b'][k],
//             tot[k] = key total (loads coalesced across keys);
//   base    : one block scans the key totals: base[k] = sum_{k' < k} tot[k'];
//   scatter : each block loads base[k] + hist[b][k] into LDS and, for every key of its
//             slice, takes its slot with a returning LDS atomic (ds_add_rtn) and writes the
//             sorted key and the position there.
// 4 launches and one read of the keys per launch that needs them, against 6 launches and
// two full key + value round trips for the 2-pass LSD sort.  Graph-safe like radix_sort.hip:
// every global word a launch reads was written by an earlier launch of the sequence (no
// memsets, no global atomics).  NOT stable: within one key the order follows LDS atomic
// arrival (the sum the reduce forms per key is then order-dependent in its last bits);
// the deterministic reduction mode keeps the stable LSD sort (ops/conv_pool.py).
#include "common.h"

namespace pv {
namespace csort {
PV_DEBUG_FLAG

constexpr int BT = 1024;   // threads per block (16 waves: atomics latency hiding at 1 block / CU)
constexpr int VEC = 8;     // 2-byte keys per 16-byte load
constexpr int MAXBINS = 1 << 15;  // 128 KB of LDS counters (static: one block per CU)

template <typename KT>
__device__ __forceinline__ void load8(const KT* __restrict__ keys, long i, unsigned (&k)[VEC]) {
  if constexpr (sizeof(KT) == 2) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(keys + i);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      k[2 * w] = v[w] & 0xFFFFu;
      k[2 * w + 1] = v[w] >> 16;
    }
  } else {
    const u32x4 a = *reinterpret_cast<const u32x4*>(keys + i);
    const u32x4 b = *reinterpret_cast<const u32x4*>(keys + i + 4);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      k[w] = a[w];
      k[4 + w] = b[w];
    }
  }
}

template <typename KT>
__global__ __launch_bounds__(BT) void cs_count_kernel(const KT* __restrict__ keys, long n, long per, int nbins,
                                                      unsigned* __restrict__ hist) {
  __shared__ unsigned h[MAXBINS];
  for (int i = threadIdx.x; i < nbins; i += BT) h[i] = 0u;
  __syncthreads();
  const long b0 = (long)blockIdx.x * per, b1 = min(n, b0 + per);
  const unsigned kmax = (unsigned)nbins - 1u;
  long i = b0 + (long)threadIdx.x * VEC;
  for (; i + VEC <= b1; i += (long)BT * VEC) {
    unsigned k[VEC];
    load8(keys, i, k);
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      PV_CHECK(k[u] <= kmax, PV_ERR_ID);
      atomicAdd(&h[min(k[u], kmax)], 1u);
    }
  }
  for (long t = max(i, b0); t < b1 && t < i + VEC; ++t) atomicAdd(&h[min((unsigned)keys[t], kmax)], 1u);
  __syncthreads();
  unsigned* row = hist + (size_t)blockIdx.x * nbins;
  for (int k = threadIdx.x; k < nbins; k += BT) row[k] = h[k];
}

// one thread per key: exclusive prefix over the block rows (in place), key total
__global__ __launch_bounds__(256) void cs_scan_kernel(unsigned* __restrict__ hist, int nblk, int nbins,
                                                      unsigned* __restrict__ tot) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= nbins) return;
  unsigned s = 0u;
  int b = 0;
  for (; b + 4 <= nblk; b += 4) {  // 4 independent loads in flight
    unsigned c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = hist[(size_t)(b + u) * nbins + k];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      hist[(size_t)(b + u) * nbins + k] = s;
      s += c[u];
    }
  }
  for (; b < nblk; ++b) {
    const unsigned c = hist[(size_t)b * nbins + k];
    hist[(size_t)b * nbins + k] = s;
    s += c;
  }
  tot[k] = s;
}

// one block: base[k] = exclusive prefix of tot over the keys
__global__ __launch_bounds__(BT) void cs_base_kernel(const unsigned* __restrict__ tot, int nbins,
                                                     unsigned* __restrict__ base) {
  __shared__ unsigned ws[BT / WAVE];
  const int per = (nbins + BT - 1) / BT;
  const int k0 = threadIdx.x * per;
  unsigned s = 0u;
  for (int j = 0; j < per; ++j)
    if (k0 + j < nbins) s += tot[k0 + j];
  // block exclusive scan of s
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  unsigned pre = 0u;
  for (int i = 0; i < w; ++i) pre += ws[i];
  unsigned run = pre + x - s;
  for (int j = 0; j < per; ++j)
    if (k0 + j < nbins) {
      base[k0 + j] = run;
      run += tot[k0 + j];
    }
}

template <typename KT>
__global__ __launch_bounds__(BT) void cs_scatter_kernel(const KT* __restrict__ keys, long n, long per, int nbins,
                                                        const unsigned* __restrict__ hist,
                                                        const unsigned* __restrict__ base, KT* __restrict__ skeys,
                                                        unsigned* __restrict__ svals) {
  __shared__ unsigned off[MAXBINS];
  const unsigned* row = hist + (size_t)blockIdx.x * nbins;
  for (int k = threadIdx.x; k < nbins; k += BT) off[k] = base[k] + row[k];
  __syncthreads();
  const long b0 = (long)blockIdx.x * per, b1 = min(n, b0 + per);
  const unsigned kmax = (unsigned)nbins - 1u;
  long i = b0 + (long)threadIdx.x * VEC;
  for (; i + VEC <= b1; i += (long)BT * VEC) {
    unsigned k[VEC], p[VEC];
    load8(keys, i, k);
#pragma unroll
    for (int u = 0; u < VEC; ++u) p[u] = atomicAdd(&off[min(k[u], kmax)], 1u);
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      skeys[p[u]] = (KT)k[u];
      svals[p[u]] = (unsigned)(i + u);
    }
  }
  for (long t = max(i, b0); t < b1 && t < i + VEC; ++t) {
    const unsigned k = min((unsigned)keys[t], kmax);
    const unsigned p = atomicAdd(&off[k], 1u);
    skeys[p] = (KT)k;
    svals[p] = (unsigned)t;
  }
}

struct Plan {
  int nblk, nbins;
  long per;
};

inline Plan plan(long n, int end_bit) {
  Plan pl;
  pl.nbins = 1 << end_bit;
  // >= 16k keys per block (the 128 KB histogram row is written and read once per block),
  // at most one block per CU-slot worth of parallelism beyond that
  long nb = (n + 16383) / 16384;
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  long per = (n + nb - 1) / nb;
  per = (per + VEC - 1) / VEC * VEC;  // 16-byte aligned block slices
  pl.per = per;
  pl.nblk = (int)((n + per - 1) / per);
  if (pl.nblk < 1) pl.nblk = 1;
  return pl;
}

PV_DEBUG_EXPORT(csort)
}  // namespace csort
}  // namespace pv

using namespace pv;

PV_API long pv_csort_temp_bytes(long n, int end_bit) {
  if (end_bit < 1 || end_bit > 15 || n < 0) return -1;
  const csort::Plan pl = csort::plan(n, end_bit);
  return ((long)pl.nblk * pl.nbins + 2L * pl.nbins) * 4;
}

// keys (n, 2- or 4-byte, values < 2^end_bit, end_bit <= 15) -> skeys (sorted), svals (input
// positions).  Not stable (see above).
PV_API int pv_csort_pairs(void* temp, long temp_bytes, const void* keys, void* skeys, unsigned* svals, long n,
                          int end_bit, int key_bytes, void* stream) {
  using namespace pv::csort;
  if (n <= 0) return 0;
  if (end_bit < 1 || end_bit > 15 || (key_bytes != 2 && key_bytes != 4)) return -1;
  if (n > 0xFFFFFFFFL) return -2;
  if (((size_t)keys & 15) != 0) return -4;  // 16-byte vector loads of the key slices
  const Plan pl = plan(n, end_bit);
  if (temp_bytes < pv_csort_temp_bytes(n, end_bit)) return -3;
  unsigned* hist = (unsigned*)temp;
  unsigned* tot = hist + (size_t)pl.nblk * pl.nbins;
  unsigned* base = tot + pl.nbins;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = 0;  // static 128 KB histograms
  if (key_bytes == 2) {
    hipLaunchKernelGGL((cs_count_kernel<unsigned short>), dim3(pl.nblk), dim3(BT), lds, st,
                       (const unsigned short*)keys, n, pl.per, pl.nbins, hist);
  } else {
    hipLaunchKernelGGL((cs_count_kernel<unsigned>), dim3(pl.nblk), dim3(BT), lds, st, (const unsigned*)keys, n,
                       pl.per, pl.nbins, hist);
  }
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(cs_scan_kernel, dim3((pl.nbins + 255) / 256), dim3(256), 0, st, hist, pl.nblk, pl.nbins, tot);
  PV_LAUNCH_CHECK();
  hipLaunchKernelGGL(cs_base_kernel, dim3(1), dim3(BT), 0, st, tot, pl.nbins, base);
  PV_LAUNCH_CHECK();
  if (key_bytes == 2) {
    hipLaunchKernelGGL((cs_scatter_kernel<unsigned short>), dim3(pl.nblk), dim3(BT), lds, st,
                       (const unsigned short*)keys, n, pl.per, pl.nbins, hist, base, (unsigned short*)skeys, svals);
  } else {
    hipLaunchKernelGGL((cs_scatter_kernel<unsigned>), dim3(pl.nblk), dim3(BT), lds, st, (const unsigned*)keys, n,
                       pl.per, pl.nbins, hist, base, (unsigned*)skeys, svals);
  }
  PV_LAUNCH_CHECK();
  return 0;
}
