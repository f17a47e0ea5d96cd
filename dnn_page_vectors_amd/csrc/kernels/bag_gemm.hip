// K1 long bags: the bag-of-trigrams product of the MLP / chunked towers on in-tree MFMA kernels.
//
// Reference layer: the first Dense of the DSSM tower over the multi-hot trigram bag
// (dssm_cnn_v2/cnn_dssm_th.py:136-138; SURVEY K1 "EmbeddingBag sum for the trigram bag").
//
//   forward   out[n][e]  = sum_v C[n][v] W[v][e]        (C = per-page token counts, N x V)
//   backward  dW[v][e]   = sum_n C[n][v] Gs[n][e]      (Gs = bf16 dZ / len)
//
// C is the dense bf16 count matrix of embedding.hip's LDS-histogram kernel (N x ldc, ldc =
// ceil64(V), zero columns past V).  (Round 5 built count tiles in LDS from per-atom segment lists
// instead, so that C never reached HBM; its list build — 300 us against the histogram's 45 — and
// its two-round weight gradient lost to the library, and it was removed in round 6:
// profiles/r5_bag/README.md.)
#include "common.h"

namespace pv {
namespace bagmm {
PV_DEBUG_FLAG

constexpr int BM = 256;       // output rows per workgroup
constexpr int BN = 128;       // output columns per workgroup
constexpr int BK = 64;        // K per step (one barrier)
constexpr int NTH = 768;      // 8 MFMA waves + 4 loader waves
constexpr int A_ROWB = BK * 2;                 // 128 B per A-tile row
constexpr int A_BYTES = BM * A_ROWB;           // 32 KB
constexpr int B_ROWB = BN * 2;                 // 256 B per dense-tile k row
constexpr int B_BYTES = BK * B_ROWB;           // 16 KB

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int b_hsw(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
// byte offset of 8-byte chunk j (4 columns) of dense-tile k row r
__device__ __forceinline__ int b_off(int r, int j) { return r * B_ROWB + ((j ^ (4 * b_hsw(r))) << 3); }
// (A tiles: 16-byte chunk c of row m at c ^ (m & 7) — conflict-free ds_read_b128 fragment reads)

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void wait_vm12() { asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------- dense-count products
// (round 6) The counts plan on in-tree MFMA kernels: the dense bf16 count matrix C (N x ldc, one
// LDS-histogram kernel, embedding.hip) read by LDS-DMA instead of two hipBLASLt GEMMs.
//   forward   part[z] (N x E) = C[:, K slice z] . W16[K slice z]        A = C rows (pages, k = ids),
//                                                                        B = W16 rows (k = ids)
//   wgrad     dW (V x E) = (Gt . C)^T, Gt = (bf16 dZ / len)^T (E x Np)   A = Gt rows (e, k = pages),
//                                                                        B = C rows (k = pages, n = ids)
// 256 x 128 tiles, K-steps of 64, 8 MFMA waves of 64 x 64 (v_mfma_f32_16x16x32_bf16) + 4 loader
// waves that only issue DMA: both operands land in a 3-slot ring two steps ahead — A (m-major,
// k-contiguous rows) with 16-byte chunk c of row m at c ^ (m & 7) (conflict-free ds_read_b128
// fragment reads), B (k-major) with 8-byte chunk j of k-row r at j ^ 4 h(r) (b_off: conflict-free
// ds_read_b64_tr_b16 transposed reads for both 32-lane halves).  The weight gradient stores its
// transposed tile straight into the dW rows (16-byte stores).
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
      // B: 4 instructions x 4 k-rows of 256 B in the b_off swizzle
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
  // -------------------------------------------------------------- MFMA waves
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
