// K1 long bags: the bag-of-trigrams product of the MLP / chunked towers on in-tree MFMA kernels
// whose count operand never exists in HBM.
//
// Reference layer: the first Dense of the DSSM tower over the multi-hot trigram bag
// (dssm_cnn_v2/cnn_dssm_th.py:136-138; SURVEY K1 "EmbeddingBag sum for the trigram bag").
//
//   forward   out[n][e]  = sum_v C[n][v] W[v][e]        (C = per-page token counts, N x V)
//   backward  dW[v][e]   = sum_n C[n][v] Gs[n][e]      (Gs = bf16 dZ / len)
//
// A 2000-token page touches ~700 of the 30k vocabulary ids: C is >97% zeros and, as a dense
// bf16 matrix, 246 MB per 4096 pages — the old plan wrote it with a histogram kernel and read it
// back through two hipBLASLt GEMMs (profiles/r4_profiles/mlp_kernel_stats_r4.md).  Here:
//
//  1. bag_rle_kernel (one workgroup per page): an LDS histogram of the page's ids (two 16-bit
//     counters per word), then the page's non-zero (id, count) pairs in id order, cut into
//     64-id SEGMENTS, with the start of every segment (u16 offsets) — ~3 KB per page instead of
//     a 60 KB dense row.  Entry = bf16(count) << 16 | segment << 6 | (id & 63) (V <= 65536).
//  2. bag_mm_kernel<FWD>: 256 x 128 output tiles, K in steps of 64, role-split workgroup
//     (12 waves): 8 MFMA waves (64 x 64 each, v_mfma_f32_16x16x32_bf16) read LDS only; 4 loader
//     waves build the NEXT step's count tile in LDS from the segment lists (zero the rows,
//     scatter the few entries: ~190 per 256 x 64 tile) and stage the dense operand's 64 x 128
//     tile (W rows for the forward, Gs rows for the weight gradient); one barrier per step.
//     The dense operand is k-major in memory (row = id or page), so its LDS image is read with
//     ds_read_b64_tr_b16 (hardware transpose) as the MFMA B operand; chunk j of k-row r sits at
//     chunk j ^ 4h(r) (h = r & 3 | (r >> 3 & 1) << 2): conflict-free for the transposed reads of
//     both 32-lane halves.  The count tile's 16-byte chunk c of row m sits at c ^ (m & 7):
//     conflict-free ds_read_b128 A reads (brute-forced against the 4 lane groups of b128).
//     Forward: rows = pages, K = vocabulary split over `splits` workgroup slices -> fp32
//     partial slabs (the colsum kernel sums them with the bag mean / bias / activation).
//     Weight gradient: rows = vocabulary ids (4 segments per tile), K = pages -> dW rows
//     straight into the flat gradient (store or accumulate), no split, no atomics.
#include "common.h"

namespace pv {
namespace bagmm {
PV_DEBUG_FLAG

constexpr int SEG = 64;       // ids per segment = K-step of the forward
constexpr int BM = 256;       // output rows per workgroup
constexpr int BN = 128;       // output columns per workgroup
constexpr int BK = 64;        // K per step (one barrier)
constexpr int NTH = 768;      // 8 MFMA waves + 4 loader waves
constexpr int NLD = 256;      // loader threads
constexpr int A_ROWB = BK * 2;                 // 128 B per count-tile row
constexpr int A_BYTES = BM * A_ROWB;           // 32 KB
constexpr int B_ROWB = BN * 2;                 // 256 B per dense-tile k row
constexpr int B_BYTES = BK * B_ROWB;           // 16 KB
constexpr int BUF = A_BYTES + B_BYTES;         // 48 KB per stage, 2 stages
constexpr int EPL = 8;                         // entries per loader lane kept in registers per step

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int b_hsw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
// byte offset of 8-byte chunk j (4 columns) of dense-tile k row r
__device__ __forceinline__ int b_off(int r, int j) { return r * B_ROWB + ((j ^ (4 * b_hsw(r))) << 3); }
// byte offset of column c (k index) of count-tile row m
__device__ __forceinline__ int a_off(int m, int c) { return m * A_ROWB + ((((c >> 3) ^ (m & 7))) << 4) + ((c & 7) << 1); }

// ---------------------------------------------------------------- 1. atom-major count lists
// An ATOM is the (64-page group q, 64-id segment s) block of the count matrix: ~1 non-zero per
// page on the bench distribution.  Its entries (bf16(count) << 16 | page-in-group << 6 | id & 63)
// are contiguous, atoms ordered segment-major: ao[s * Q + q] .. ao[s * Q + q + 1].  A forward
// K-step of a 256-page tile is 4 consecutive atoms (one per loader wave); a weight-gradient step
// of a 256-id tile is the 4 atoms (4v .. 4v+3, q) — one per loader wave as well.
// Built without any V-sized histogram or global atomics, in four launches:
//  a. bag_sort_kernel (one workgroup per page): the page's non-pad ids sorted in LDS (bitonic,
//     P = next power of two >= L keys), runs -> distinct (id, count) pairs in id order
//     (page-major scratch), distinct ids per segment c[n][s] (u8), non-pad length;
//  b. bag_group_scan_kernel: per page group and segment, the pages' offsets inside the atom
//     (u16 within[n][s]) and the atom totals tot[s][q] (a sequential scan over 64 pages);
//  c. bag_atom_scan_kernel: exclusive scan of tot in (s, q) order -> ao;
//  d. bag_place_kernel (one wave per page): every distinct pair to its atom-major slot.
constexpr int SORT_MAX = 8192;  // keys per page sorted in LDS (32 KB); longer bags: library plan

__global__ __launch_bounds__(1024) void bag_sort_kernel(const int* __restrict__ ids, unsigned* __restrict__ dist,
                                                        unsigned char* __restrict__ cseg, float* __restrict__ lens,
                                                        int N, int L, int V, int pad, int P) {
  extern __shared__ unsigned key[];  // P keys, then P + 1 run starts
  __shared__ int wsum[16];
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int S = (V + SEG - 1) / SEG;
  const int* row = ids + (size_t)n * L;
  for (int i = t; i < P; i += 1024) {
    const int v = i < L ? row[i] : pad;
    PV_CHECK(v == pad || (v >= 0 && v < V), PV_ERR_ID);
    key[i] = (v != pad && v >= 0 && v < V) ? (unsigned)v : 0xFFFFFFFFu;
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < P / 2; i += 1024) {
        const int lo = 2 * i - (i & (j - 1)), hi = lo + j;
        const bool up = (lo & k) == 0;
        const unsigned a = key[lo], b = key[hi];
        if ((a > b) == up) {
          key[lo] = b;
          key[hi] = a;
        }
      }
      __syncthreads();
    }
  // run starts -> compact start positions (block scan of the start flags in index order)
  unsigned* st = key + P;
  const int per = P / 1024 > 0 ? P / 1024 : 1;
  const int i0 = t * per;
  int c = 0;
  for (int i = i0; i < i0 + per && i < P; ++i)
    c += (key[i] != 0xFFFFFFFFu && (i == 0 || key[i] != key[i - 1])) ? 1 : 0;
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0, nd = 0;
  for (int i = 0; i < 16; ++i) {
    base += i < w ? wsum[i] : 0;
    nd += wsum[i];
  }
  int d = base + inc - c;
  for (int i = i0; i < i0 + per && i < P; ++i)
    if (key[i] != 0xFFFFFFFFu && (i == 0 || key[i] != key[i - 1])) st[d++] = (unsigned)i;
  // valid keys = index of the first INF (binary search over the sorted keys)
  __syncthreads();
  if (t == 0) {
    int lo = 0, hi = P;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (key[m] == 0xFFFFFFFFu) hi = m; else lo = m + 1;
    }
    st[nd] = (unsigned)lo;
    lens[n] = (float)lo;
  }
  __syncthreads();
  unsigned* drow = dist + (size_t)n * L;
  for (int q = t; q < nd; q += 1024) {
    const unsigned i = st[q], cnt = st[q + 1] - i, id = key[i];
    drow[q] = ((unsigned)f32_to_bf16((float)cnt) << 16) | id;  // id < 65536
  }
  // distinct ids per segment: lower_bound of the segment's first id among the distinct ids
  auto first_of = [&](int sg) {
    int lo = 0, hi = nd;
    const unsigned idv = (unsigned)sg * SEG;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (key[st[m]] < idv) lo = m + 1; else hi = m;
    }
    return lo;
  };
  unsigned char* crow = cseg + (size_t)n * S;
  for (int sg = t; sg < S; sg += 1024) crow[sg] = (unsigned char)(first_of(sg + 1) - first_of(sg));
}

// per (page group q, segment s): offsets of the group's pages inside atom (s, q) and its total
__global__ __launch_bounds__(256) void bag_group_scan_kernel(const unsigned char* __restrict__ cseg,
                                                             unsigned short* __restrict__ within, int* __restrict__ tot,
                                                             int N, int S, int Q) {
  const int q = blockIdx.y;
  const int sg = blockIdx.x * 256 + threadIdx.x;
  if (sg >= S) return;
  int run = 0;
  const int n0 = q * 64, n1 = min(N, n0 + 64);
  for (int n = n0; n < n1; ++n) {
    within[(size_t)n * S + sg] = (unsigned short)run;
    run += cseg[(size_t)n * S + sg];
  }
  tot[sg * Q + q] = run;
}

// exclusive scan of tot (T = S * Q ints) -> ao (T + 1), one 1024-thread workgroup
__global__ __launch_bounds__(1024) void bag_atom_scan_kernel(const int* __restrict__ tot, int* __restrict__ ao, int T) {
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int per = (T + 1023) / 1024;
  const int a0 = min(T, t * per), a1 = min(T, a0 + per);
  int c = 0;
  for (int i = a0; i < a1; ++i) c += tot[i];
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
  for (int i = 0; i < 16; ++i) {
    base += i < w ? wsum[i] : 0;
    all += wsum[i];
  }
  int pos = base + inc - c;
  for (int i = a0; i < a1; ++i) {
    ao[i] = pos;
    pos += tot[i];
  }
  if (t == 0) ao[T] = all;
}

// one wave per page: distinct pair q of the page (id order) -> ao[s Q + group] + within + rank
__global__ __launch_bounds__(256) void bag_place_kernel(const unsigned* __restrict__ dist,
                                                        const unsigned char* __restrict__ cseg,
                                                        const unsigned short* __restrict__ within,
                                                        const int* __restrict__ ao, unsigned* __restrict__ ent, int N,
                                                        int L, int S, int Q) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const unsigned* drow = dist + (size_t)n * L;
  const unsigned char* crow = cseg + (size_t)n * S;
  const unsigned pg = (unsigned)(n & 63) << 6;
  const int q = n / 64;
  // walk the segments in chunks of 64 (one per lane), prefix-summing their distinct counts
  int d0 = 0;
  for (int s0 = 0; s0 < S; s0 += 64) {
    const int sg = s0 + lane;
    const int c = sg < S ? crow[sg] : 0;
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    const int first = d0 + inc - c;  // this segment's first distinct index
    if (c) {
      const int dst = ao[sg * Q + q] + within[(size_t)n * S + sg];
      for (int r = 0; r < c; ++r) {
        const unsigned x = drow[first + r];
        ent[dst + r] = (x & 0xFFFF0000u) | pg | (x & 63u);
      }
    }
    d0 += __shfl(inc, 63, 64);
  }
}

// ---------------------------------------------------------------- 2. the MFMA product
struct MmParams {
  const unsigned* ent;          // atom-major entries
  const int* ao;                // (S * Q + 1) atom starts
  const unsigned short* dense;  // FWD: W (V, E) bf16; WGRAD: Gs (N, E) bf16
  float* out;                   // FWD: (splits, N, E) partials; WGRAD: dW rows (V, ldo)
  int N, V, E, S, Q;            // S = segments, Q = 64-page groups
  int splits, steps_per_split;  // FWD
  int ldo, accumulate;          // WGRAD
};

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void wait_vm12() { asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS: two count tiles (built by the loader waves, 32 KB each) + a ring of NBD dense tiles
// (16 KB each, landed by LDS-DMA DAHEAD steps ahead of their use)
constexpr int NBD = 4, DAHEAD = 3;
constexpr int LDS_MAIN = 2 * A_BYTES + NBD * B_BYTES;  // 128 KB
constexpr int AOCH = 256;                              // atom bounds staged per loader wave
constexpr int LDS_AO = 4 * 2 * AOCH * 4;               // 8 KB
constexpr int LDS_TOTAL = LDS_MAIN + LDS_AO + 4 * NBD * 2 * 64 * 4;  // + 8 KB entry ring

// DBG (timing ablations, wrong results): 1 no dense DMA in the loop, 2 no count-tile builds in
// the loop, 4 no MFMAs, 8 no LDS fragment reads (tools/bag_gemm_micro.py --dbg)
template <bool FWD, int DBG = 0>
__global__ __launch_bounds__(NTH, 1) void bag_mm_kernel(MmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const abuf = smem;                 // [2][A_BYTES]
  char* const dring = smem + 2 * A_BYTES;  // [NBD][B_BYTES]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  // tile of this workgroup
  int row0, col0, k_begin, k_end;
  {
    const int ncol = (p.E + BN - 1) / BN;
    if (FWD) {
      const int nrow = (p.N + BM - 1) / BM;
      // blocks b and b + 8 share an XCD: one (split, column) W slab per XCD's L2
      const int b = xcd_remap(blockIdx.x, gridDim.x);
      const int rt = b % nrow, rest = b / nrow;
      const int ct = rest % ncol, sp = rest / ncol;
      row0 = rt * BM;
      col0 = ct * BN;
      k_begin = sp * p.steps_per_split;
      k_end = min(p.S, k_begin + p.steps_per_split);
    } else {
      const int b = blockIdx.x;
      const int ct = b % ncol, vt = b / ncol;
      row0 = vt * BM;  // vocabulary ids
      col0 = ct * BN;
      k_begin = 0;
      k_end = (p.N + BK - 1) / BK;
    }
  }
  const int nsteps = max(0, k_end - k_begin);
  if (wave >= 8) {
    // ------------------------------------------------------------ loader waves
    const int lw = wave - 8, lt = threadIdx.x - 8 * 64;
    const int drows = FWD ? p.V : p.N;
    // dense tile of step k -> ring slot: wave lw's 4 DMA instructions cover rows 16 lw .. +15;
    // LDS piece pc' of row r holds global piece pc' ^ 2h(r) (the b_off swizzle), clamped rows /
    // columns re-read real data (they meet zero counts or discarded output columns)
    auto dma_dense = [&](int k) {
      char* slot = dring + (k % NBD) * B_BYTES;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (lw * 4 + i) * 4 + (lane >> 4);
        const int pc = (lane & 15) ^ (2 * b_hsw(r));
        const int gr = min(k * BK + r, drows - 1), gc = min(col0 + pc * 8, p.E - 8);
        glds16(p.dense + (size_t)gr * p.E + gc, slot + (lw * 4 + i) * 1024);
      }
    };
    // this wave's atom of step k: FWD (segment k, page group row0 / 64 + lw), WGRAD (segment
    // row0 / 64 + lw, page group k); entry -> count-tile (row, column)
    auto atom_of = [&](int k) {
      const int sg = FWD ? k : row0 / SEG + lw, q = FWD ? row0 / 64 + lw : k;
      return (k < k_end && sg < p.S && q < p.Q) ? sg * p.Q + q : -1;
    };
    auto put = [&](char* A, unsigned x, unsigned short c) {
      const int id = (int)(x & 63u), pg = (int)((x >> 6) & 63u);
      const int m = FWD ? 64 * lw + pg : 64 * lw + id;
      const int col = FWD ? id : pg;
      *reinterpret_cast<unsigned short*>(A + a_off(m, col)) = c;
    };
    // zero both count tiles once; afterwards each build clears exactly what it wrote last time
    {
      u32x4* z0 = reinterpret_cast<u32x4*>(abuf + lt * A_ROWB);
      u32x4* z1 = reinterpret_cast<u32x4*>(abuf + A_BYTES + lt * A_ROWB);
#pragma unroll
      for (int i = 0; i < A_ROWB / 16; ++i) z0[i] = z1[i] = u32x4{0u, 0u, 0u, 0u};
    }
    constexpr int RR = 2;  // rounds of 64 entries DMA'd per step (an atom holds ~64-150)
    unsigned old[2][RR];   // entries last written into each count tile
    int nold[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < RR; ++r) old[0][r] = old[1][r] = 0u;
    // The loop issues no vector loads whose VALUES it waits for (hipcc would then wait on the
    // whole vmcnt queue, DMA groups included, every step): the atom bounds of this wave's steps
    // are staged in LDS in chunks of AOCH steps, and each step's entries arrive by LDS-DMA into
    // a ring beside the dense tile (ENT slot = RR x 64 dwords per wave).
    int* aol = reinterpret_cast<int*>(smem + LDS_MAIN) + lw * (2 * AOCH);
    unsigned* ering = reinterpret_cast<unsigned*>(smem + LDS_MAIN + LDS_AO) + lw * (NBD * RR * 64);
    int* sinfo = aol + 2 * AOCH - 2 * NBD;  // (lo, n) of the step in each ring slot (last 2 NBD ints)
    int chunk = -1;
    auto stage_bounds = [&](int c) {
      for (int i = lane; i < AOCH - NBD; i += 64) {
        const int at = atom_of(k_begin + c * (AOCH - NBD) + i);
        const int a0 = p.ao[max(at, 0)], a1 = p.ao[max(at, 0) + 1];
        aol[2 * i] = at >= 0 ? a0 : 0;
        aol[2 * i + 1] = at >= 0 ? a1 - a0 : 0;
      }
      chunk = c;
    };
    auto bounds = [&](int kk, int& lo, int& n) {  // kk: step index inside this workgroup
      constexpr int CH = AOCH - NBD;
      if (kk / CH != chunk) stage_bounds(kk / CH);  // wave-uniform, once per CH steps
      lo = aol[2 * (kk % CH)];
      n = aol[2 * (kk % CH) + 1];
    };
    // step kk's DMA group: this wave's entries (RR dword DMAs, clamped in-bounds indices) and
    // its 4 pieces of the dense tile — exactly RR + 4 vector-memory operations
    auto dma_step = [&](int kk) {
      int lo, n;
      bounds(kk, lo, n);
      const int sl = kk % NBD;
      if (lane == 0) {
        sinfo[2 * sl] = lo;
        sinfo[2 * sl + 1] = n;
      }
#pragma unroll
      for (int r = 0; r < RR; ++r)
        __builtin_amdgcn_global_load_lds(p.ent + lo + min(r * 64 + lane, max(n - 1, 0)),
                                         (__attribute__((address_space(3))) void*)(ering + (sl * RR + r) * 64), 4, 0,
                                         0);
      dma_dense(k_begin + kk);
    };
    auto build = [&](int kk) {
      const int b = kk & 1, sl = kk % NBD;
      char* A = abuf + b * A_BYTES;
      if (nold[b] > RR * 64) {  // a big atom last time: clear this wave's 64 rows whole
        for (int rr = 0; rr < 64; ++rr) {
          u32x4* zr = reinterpret_cast<u32x4*>(A + (64 * lw + rr) * A_ROWB);
          if (lane < A_ROWB / 16) zr[lane] = u32x4{0u, 0u, 0u, 0u};
        }
      } else {
#pragma unroll
        for (int r = 0; r < RR; ++r)
          if (r * 64 + lane < nold[b]) put(A, old[b][r], 0);
      }
      const int n = sinfo[2 * sl + 1], lo = sinfo[2 * sl];
      unsigned e[RR];
#pragma unroll
      for (int r = 0; r < RR; ++r) e[r] = ering[(sl * RR + r) * 64 + lane];
#pragma unroll
      for (int r = 0; r < RR; ++r)
        if (r * 64 + lane < n) put(A, e[r], (unsigned short)(e[r] >> 16));
      for (int i = RR * 64 + lane; i < n; i += 64) {  // rare: atoms of > RR x 64 entries
        const unsigned x = p.ent[lo + i];
        put(A, x, (unsigned short)(x >> 16));
      }
#pragma unroll
      for (int r = 0; r < RR; ++r) old[b][r] = e[r];
      nold[b] = n;
    };
    // ---- prologue: steps 0 .. DAHEAD-1 in flight, step 0 built
    for (int d = 0; d < DAHEAD; ++d)
      if (d < nsteps) dma_step(d);
    wait_vm0();
    if (nsteps > 0) build(0);
    for (int it = 0; it < nsteps; ++it) {
      __syncthreads();  // B_it: count tile it&1 and dense slot it%NBD complete
      // step it+DAHEAD in flight; then step it+1's group must have landed: younger than it are
      // the groups of steps it+2 and it+3 (RR + 4 each), so vmcnt(2 (RR + 4)) suffices; near the
      // end (fewer groups in flight) wait for everything
      if (it + DAHEAD < nsteps) {
        if (!(DBG & 1)) dma_step(it + DAHEAD);
        wait_vm12();
      } else {
        wait_vm0();
      }
      if (it + 1 < nsteps && !(DBG & 2)) build(it + 1);
    }
    __syncthreads();  // B_end: pairs with the MFMA waves' last barrier
    return;
  }
  // -------------------------------------------------------------- MFMA waves
  const int wm = wave & 3, wn = wave >> 2;  // 64-row block, 64-column block
  const int m16 = lane & 15, g = lane >> 4;
  const int q = (lane & 15) >> 2, pp = lane & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int aoff[2][4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wm * 64 + 16 * i + m16;
      aoff[ks][i] = m * A_ROWB + ((((ks * 4 + g) ^ (m16 & 7))) << 4);
    }
  int boff[2][4][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * ks + 8 * g + 4 * h + q;
        const int jc = (wn * 64 + 16 * j) / 4 + pp;
        boff[ks][j][h] = b_off(r, jc);
      }
  for (int it = 0; it < nsteps; ++it) {
    __syncthreads();
    const char* A = abuf + (it & 1) * A_BYTES;
    const char* B = dring + ((k_begin + it) % NBD) * B_BYTES;
    // both sub-steps' fragments first (24 LDS reads in flight, separate registers), then the 32
    // MFMAs: hipcc otherwise re-reads A fragments just in time into the same 8 VGPRs and each
    // pair's LDS latency sits in front of its MFMAs
    bf16x8 a[2][4], b[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr ((DBG & 8) != 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[ks][i] = b[ks][i] = bf16x8{(short)it, 1, 2, 3, 4, 5, 6, (short)lane};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[ks][i] = *reinterpret_cast<const bf16x8*>(A + aoff[ks][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          typedef __attribute__((address_space(3))) v4s lds_v4s;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(B + boff[ks][j][0]));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(B + boff[ks][j][1]));
          b[ks][j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr ((DBG & 4) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks][i], b[ks][j], acc[i][j], 0, 0, 0);
      } else {
        acc[0][0][0] += (float)a[ks][0][0] + (float)b[ks][3][1];
      }
    }
  }
  __syncthreads();  // B_end
  // epilogue: lane holds rows 4g + r, column m16 of each 16 x 16 tile
  const int col_l = col0 + wn * 64 + m16;
  float* dst;
  int ld, nrows;
  if (FWD) {
    const int sp = k_begin / max(1, p.steps_per_split);
    dst = p.out + (size_t)sp * p.N * p.E;
    ld = p.E;
    nrows = p.N;
  } else {
    dst = p.out;
    ld = p.ldo;
    nrows = p.V;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + wm * 64 + 16 * i + 4 * g + r;
      if (row < nrows) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = col_l + 16 * j;
          if (c < p.E) {
            float* o = dst + (size_t)row * ld + c;
            *o = (!FWD && p.accumulate) ? *o + acc[i][j][r] : acc[i][j][r];
          }
        }
      }
    }
}

// ---------------------------------------------------------------- 3. dense-count products
// (round 6) The counts plan on in-tree MFMA kernels: the dense bf16 count matrix C (N x ldc, one
// LDS-histogram kernel, embedding.hip) read by LDS-DMA instead of two hipBLASLt GEMMs.
//   forward   part[z] (N x E) = C[:, K slice z] . W16[K slice z]        A = C rows (pages, k = ids),
//                                                                        B = W16 rows (k = ids)
//   wgrad     dW (V x E) = (Gt . C)^T, Gt = (bf16 dZ / len)^T (E x Np)   A = Gt rows (e, k = pages),
//                                                                        B = C rows (k = pages, n = ids)
// Tiles and MFMA waves as bag_mm_kernel (256 x 128, K-steps of 64, 8 MFMA waves of 64 x 64 + 4
// loader waves), but the loader waves only issue DMA: both operands land in a 3-slot ring two
// steps ahead — A (m-major, k-contiguous rows) with 16-byte chunk c of row m at c ^ (m & 7) (the
// conflict-free ds_read_b128 layout of the count tile), B (k-major) as in bag_mm_kernel.  The
// weight gradient stores its transposed tile straight into the dW rows (16-byte stores).
struct DmParams {
  const unsigned short* A;  // rows: tile M dimension, k contiguous; lda elements per row
  const unsigned short* B;  // rows: k, n contiguous; ldb elements per row
  float* out;
  long lda, ldb, ldo;
  int M, N;          // output rows (A rows) / columns (B columns) that exist
  int arows, brows;  // A rows / B rows (k) that may be read (clamp)
  int bcols;         // B columns that may be read (clamp; multiple of 8)
  int ksteps;        // K-steps of 64 over the whole reduction (A columns are zero-padded to it)
  int splits, steps_per_split;
  int accumulate;    // WGRAD: add into dW
};

constexpr int DNB = 3, DDA = 2;                       // ring slots, DMA steps ahead
constexpr int DSLOT = A_BYTES + B_BYTES;              // 48 KB
constexpr int DLDS = DNB * DSLOT;                     // 144 KB

template <bool WGRAD>
__global__ __launch_bounds__(NTH, 1) void bagd_mm_kernel(DmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int row0, col0, k_begin, k_end;
  {
    const int ncol = (p.N + BN - 1) / BN, nrow = (p.M + BM - 1) / BM;
    // neighbouring logical blocks run on one XCD at the same time (xcd_remap): the tiles that
    // share the big operand — the count matrix — are neighbours, so it streams through that
    // XCD's L2 once instead of once per tile.  Forward: the E / 128 column tiles of a (row tile,
    // split) share C's rows; weight gradient: the E / 256 row tiles of a column tile share C's
    // columns.
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    int rt, ct, sp;
    if (WGRAD) {
      rt = b % nrow;
      ct = (b / nrow) % ncol;
      sp = b / (nrow * ncol);
    } else {
      ct = b % ncol;
      rt = (b / ncol) % nrow;
      sp = b / (nrow * ncol);
    }
    row0 = rt * BM;
    col0 = ct * BN;
    k_begin = sp * p.steps_per_split;
    k_end = min(p.ksteps, k_begin + p.steps_per_split);
  }
  const int nsteps = max(0, k_end - k_begin);
  if (wave >= 8) {
    // ------------------------------------------------------------ loader waves: DMA only
    const int lw = wave - 8;
    auto dma_step = [&](int kk) {  // step kk (inside this workgroup's K slice) -> ring slot kk % DNB
      char* slot = smem + (kk % DNB) * DSLOT;
      const int k = k_begin + kk;
      // A: 8 instructions x 8 rows of 128 B; lane l -> row 8 i' + (l >> 3), LDS chunk l & 7
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int blk = lw * 8 + i;
        const int r = blk * 8 + (lane >> 3);
        const int c = (lane & 7) ^ (r & 7);
        const int gr = min(row0 + r, p.arows - 1);
        glds16(p.A + (size_t)gr * p.lda + (size_t)k * BK + c * 8, slot + blk * 1024);
      }
      // B: 4 instructions x 4 k-rows of 256 B, the b_off swizzle (as bag_mm_kernel's dense tile)
      char* bs = slot + A_BYTES;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (lw * 4 + i) * 4 + (lane >> 4);
        const int pc = (lane & 15) ^ (2 * b_hsw(r));
        const int gr = min(k * BK + r, p.brows - 1), gc = min(col0 + pc * 8, p.bcols - 8);
        glds16(p.B + (size_t)gr * p.ldb + gc, bs + (lw * 4 + i) * 1024);
      }
    };
    for (int d = 0; d < DDA; ++d)
      if (d < nsteps) dma_step(d);
    if (nsteps > 1) wait_vm12();  // step 0 landed (step 1's 12 DMAs may stay in flight)
    else wait_vm0();
    for (int it = 0; it < nsteps; ++it) {
      __syncthreads();  // B_it: slot it % DNB complete for everyone; slot (it + 2) % DNB free
      if (it + DDA < nsteps) {
        dma_step(it + DDA);
        wait_vm12();  // step it + 1 landed; step it + 2 may stay in flight
      } else {
        wait_vm0();
      }
    }
    __syncthreads();  // B_end
    return;
  }
  // -------------------------------------------------------------- MFMA waves (bag_mm_kernel's)
  const int wm = wave & 3, wn = wave >> 2;
  const int m16 = lane & 15, g = lane >> 4;
  const int q = (lane & 15) >> 2, pp = lane & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int aoff[2][4];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wm * 64 + 16 * i + m16;
      aoff[ks][i] = m * A_ROWB + ((((ks * 4 + g) ^ (m16 & 7))) << 4);
    }
  int boff[2][4][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * ks + 8 * g + 4 * h + q;
        const int jc = (wn * 64 + 16 * j) / 4 + pp;
        boff[ks][j][h] = A_BYTES + b_off(r, jc);
      }
  for (int it = 0; it < nsteps; ++it) {
    __syncthreads();
    const char* S = smem + (it % DNB) * DSLOT;
    bf16x8 a[2][4], b[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[ks][i] = *reinterpret_cast<const bf16x8*>(S + aoff[ks][i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        typedef __attribute__((address_space(3))) v4s lds_v4s;
        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(S + boff[ks][j][0]));
        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(S + boff[ks][j][1]));
        b[ks][j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks][i], b[ks][j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // B_end
  // epilogue: lane holds rows 4g + r, column m16 of each 16 x 16 tile
  if (WGRAD) {  // rows = e, columns = vocabulary ids: dW[id][e .. e + 3] as one 16-byte store
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = row0 + wm * 64 + 16 * i + 4 * g;
      if (e >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int id = col0 + wn * 64 + 16 * j + m16;
        if (id >= p.N) continue;
        f32x4* o = reinterpret_cast<f32x4*>(p.out + (size_t)id * p.ldo + e);
        *o = p.accumulate ? *o + acc[i][j] : acc[i][j];
      }
    }
  } else {
    const int sp = k_begin / max(1, p.steps_per_split);
    float* dst = p.out + (size_t)sp * p.M * p.ldo;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * 64 + 16 * i + 4 * g + r;
        if (row >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = col0 + wn * 64 + 16 * j + m16;
          if (c < p.N) dst[(size_t)row * p.ldo + c] = acc[i][j][r];
        }
      }
  }
}

// gs (N, E) bf16 -> gt (E, Np) bf16, columns N .. Np-1 zero (64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void bag_transpose16_kernel(const unsigned short* __restrict__ gs,
                                                               unsigned short* __restrict__ gt, int N, int E,
                                                               int Np) {
  __shared__ unsigned short t[64][65];
  const int n0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;  // r: n, c: e
    const int n = n0 + r, e = e0 + c;
    t[r][c] = (n < N && e < E) ? gs[(size_t)n * E + e] : (unsigned short)0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;  // r: e, c: n
    const int e = e0 + r, n = n0 + c;
    if (e < E && n < Np) gt[(size_t)e * Np + n] = t[c][r];
  }
}

PV_DEBUG_EXPORT(bagmm)
}  // namespace bagmm
}  // namespace pv

using namespace pv::bagmm;

PV_API int pv_bag_segments(int V) { return (V + SEG - 1) / SEG; }

static int g_bag_dbg = 0;
PV_API void pv_bag_set_dbg(int d) { g_bag_dbg = d; }

template <bool FWD, int DBG>
static int launch_mm(const MmParams& p, int grid, hipStream_t st) {
  static bool done = false;
  if (!done) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bag_mm_kernel<FWD, DBG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL) != hipSuccess)
      return -3;
    done = true;
  }
  hipLaunchKernelGGL((bag_mm_kernel<FWD, DBG>), dim3(grid), dim3(NTH), LDS_TOTAL, st, p);
  PV_LAUNCH_CHECK();
  return 0;
}

template <bool FWD>
static int launch_mm_dbg(const MmParams& p, int grid, hipStream_t st) {
  switch (g_bag_dbg) {
    case 0: return launch_mm<FWD, 0>(p, grid, st);
    case 1: return launch_mm<FWD, 1>(p, grid, st);
    case 2: return launch_mm<FWD, 2>(p, grid, st);
    case 3: return launch_mm<FWD, 3>(p, grid, st);
    case 4: return launch_mm<FWD, 4>(p, grid, st);
    case 8: return launch_mm<FWD, 8>(p, grid, st);
    case 12: return launch_mm<FWD, 12>(p, grid, st);
    case 15: return launch_mm<FWD, 15>(p, grid, st);
    default: return -7;
  }
}

// ids (N, L) int32 -> ent (<= N * L u32, atom-major), ao (S * Q + 1 int32), lens (N f32);
// workspaces: dist (N * L u32), cseg (N * S u8), within (N * S u16), tot (S * Q int32)
PV_API int pv_bag_rle(const int* ids, void* ent, int* ao, void* dist, void* cseg, void* within, int* tot, float* lens,
                      int N, int L, int V, int pad, void* stream) {
  if (N <= 0 || L <= 0 || L > SORT_MAX || V <= 0 || V > 65536) return -1;
  const int S = (V + SEG - 1) / SEG, Q = (N + 63) / 64;
  int P = 64;
  while (P < L) P <<= 1;
  const size_t lds = (size_t)(2 * P + 1) * sizeof(unsigned);
  static size_t attr = 0;
  if (lds > attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bag_sort_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -3;
    attr = lds;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bag_sort_kernel, dim3(N), dim3(1024), lds, st, ids, (unsigned*)dist, (unsigned char*)cseg, lens,
                     N, L, V, pad, P);
  hipLaunchKernelGGL(bag_group_scan_kernel, dim3((S + 255) / 256, Q), dim3(256), 0, st, (const unsigned char*)cseg,
                     (unsigned short*)within, tot, N, S, Q);
  hipLaunchKernelGGL(bag_atom_scan_kernel, dim3(1), dim3(1024), 0, st, (const int*)tot, ao, S * Q);
  hipLaunchKernelGGL(bag_place_kernel, dim3((N + 3) / 4), dim3(256), 0, st, (const unsigned*)dist,
                     (const unsigned char*)cseg, (const unsigned short*)within, (const int*)ao, (unsigned*)ent, N, L,
                     S, Q);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_bag_groups(int N) { return (N + 63) / 64; }

// forward partials: part (splits, N, E) f32 = C[:, split range] @ W16[split range]
PV_API int pv_bag_mm_fwd(const void* ent, const int* ao, const void* W16, float* part, int N, int V, int E,
                         int splits, void* stream) {
  if (N <= 0 || E < 8 || E % 8 || splits <= 0) return -1;
  const int S = (V + SEG - 1) / SEG, Q = (N + 63) / 64;
  const int sps = (S + splits - 1) / splits;
  MmParams p{(const unsigned*)ent, ao, (const unsigned short*)W16, part, N, V, E, S, Q, splits, sps, E, 0};
  const int grid = ((N + BM - 1) / BM) * ((E + BN - 1) / BN) * splits;
  return launch_mm_dbg<true>(p, grid, (hipStream_t)stream);
}

// weight gradient: dW (V rows, leading dim ldo) (+)= C^T @ Gs, Gs (N, E) bf16
PV_API int pv_bag_mm_wgrad(const void* ent, const int* ao, const void* Gs, float* dW, int ldo, int accumulate, int N,
                           int V, int E, void* stream) {
  if (N <= 0 || E < 8 || E % 8 || ldo < E) return -1;
  const int S = (V + SEG - 1) / SEG, Q = (N + 63) / 64;
  MmParams p{(const unsigned*)ent, ao, (const unsigned short*)Gs, dW, N, V, E, S, Q, 1, 0, ldo, accumulate};
  const int grid = ((V + BM - 1) / BM) * ((E + BN - 1) / BN);
  return launch_mm_dbg<false>(p, grid, (hipStream_t)stream);
}

template <bool WG>
static int launch_dm(const DmParams& p, int grid, hipStream_t st) {
  static bool done = false;
  if (!done) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&bagd_mm_kernel<WG>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, DLDS) != hipSuccess)
      return -3;
    done = true;
  }
  hipLaunchKernelGGL((bagd_mm_kernel<WG>), dim3(grid), dim3(NTH), DLDS, st, p);
  PV_LAUNCH_CHECK();
  return 0;
}

// dense-count forward partials: part (splits, N, E) f32 = C[:, slice] @ W16[slice]; C (N, ldc)
// bf16 with zero columns V .. ldc-1 (ldc % 64 == 0), W16 (V, E) bf16
PV_API int pv_bagd_fwd(const void* C, int ldc, const void* W16, float* part, int N, int V, int E, int splits,
                       void* stream) {
  if (N <= 0 || V <= 0 || E < 8 || E % 8 || ldc < V || ldc % BK || splits <= 0) return -1;
  const int ks = ldc / BK, sps = (ks + splits - 1) / splits;
  splits = (ks + sps - 1) / sps;
  DmParams p{(const unsigned short*)C, (const unsigned short*)W16, part, ldc, E, E, N, E, N, V, E, ks, splits, sps, 0};
  const int grid = ((N + BM - 1) / BM) * ((E + BN - 1) / BN) * splits;
  return launch_dm<false>(p, grid, (hipStream_t)stream);
}

PV_API int pv_bagd_splits(int N, int V, int E, int ldc, int splits) {  // slabs pv_bagd_fwd writes
  const int ks = ldc / BK, sps = (ks + splits - 1) / splits;
  (void)N; (void)V; (void)E;
  return (ks + sps - 1) / sps;
}

// dense-count weight gradient: dW (V rows, leading dim ldo) (+)= C[:, :V]^T @ gs, via
// gt = gs^T (E, Np) bf16 (Np = ceil64(N), zero-padded; ws: E * Np bf16 scratch)
PV_API int pv_bagd_wgrad(const void* C, int ldc, const void* gs, void* ws, float* dW, int ldo, int accumulate, int N,
                         int V, int E, void* stream) {
  if (N <= 0 || V <= 0 || E < 8 || E % 8 || ldc < V || ldc % 8 || ldo < E || ldo % 4) return -1;
  const int Np = (N + BK - 1) / BK * BK;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bag_transpose16_kernel, dim3(Np / 64, (E + 63) / 64), dim3(256), 0, st,
                     (const unsigned short*)gs, (unsigned short*)ws, N, E, Np);
  PV_LAUNCH_CHECK();
  DmParams p{(const unsigned short*)ws, (const unsigned short*)C, dW, Np, ldc, ldo, E, V, E, N, ldc, Np / BK, 1,
             Np / BK, accumulate};
  const int grid = ((E + BM - 1) / BM) * ((V + BN - 1) / BN);
  return launch_dm<true>(p, grid, st);
}
