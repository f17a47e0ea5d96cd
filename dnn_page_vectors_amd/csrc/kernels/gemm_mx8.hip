// Block-scaled fp8 GEMM on v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, fp32 accumulate):
//   C[M][N] = epilogue( alpha * A8[M][K] . B8[N][K]^T ),   K contiguous in both operands.
//
// The hot GEMM of the long-page chunked encoder (BASELINE config 5): the page-chunk bag
// C (4096 chunks x 30k vocabulary, token counts) times the embedding table, 126 GFLOP per
// step.  The scaled fp8 MFMA issues twice the bf16 FLOPs per cycle (MI355X_MICROARCH: the
// 16x16x128 form takes twice the cycles of the bf16 16x16x32 at 4x the K); operands are
// per-tensor scaled (the e8m0 block scales are all 1.0, the dequantisation 2^e * amax / 448
// is one alpha in the epilogue), so the MFMA's scale operands are constants.
//
// Operand packing (tests/test_kernels_gpu.py::test_mx_fp8_mfma_layout, "halves16"): lane l
// supplies row (l & 15) of its operand, bytes 0-15 = k [16g, 16g + 16) and bytes 16-31 =
// k [64 + 16g, 64 + 16g + 16) of the 128-k step, g = l >> 4 — two 16-byte chunks (g and
// 4 + g) of the row's 128-byte K tile, i.e. two ds_read_b128 per fragment.
//
// Workgroup tile 256 x 128 x 128 bytes, 8 waves (4 x 2), each wave 64 x 64 = 4 x 4 MFMA
// tiles (64 accumulator VGPRs).  Staging: direct-to-LDS
// loads (global_load_lds_dwordx4), double-buffered (2 x 48 KB); 128-byte rows with the
// 16-byte chunk c of row r stored at c ^ (r & 7) (source-side swizzle, conflict-free reads).
// Split-K: each K slice writes alpha * partial into its fp32 slab (the caller's column-sum
// kernel applies the bag mean / bias / activation, ops/embedding.py).
#include "common.h"

namespace pv {
namespace gemm8 {
PV_DEBUG_FLAG

constexpr int BM = 256, BN = 128, BK = 128;  // BK in bytes (= e4m3 elements)
constexpr int NTH = 512;
constexpr int A_BYTES = BM * BK, B_BYTES = BN * BK, STAGE = A_BYTES + B_BYTES;  // 32 + 16 KB
constexpr int E8M0_ONE = 127;
typedef int v8i __attribute__((ext_vector_type(8)));

struct Params {
  const unsigned char* A;
  const unsigned char* B;
  long lda, ldb;          // bytes between rows
  void* C;
  long ldc;
  int M, N, K;            // K in bytes, K % 128 == 0
  int ksplit;
  long slab;              // elements between split-K partial slabs (ksplit > 1)
  const float* bias;
  float alpha;
  const float* alpha_ptr;  // optional device scalar multiplied into alpha (e.g. amax / 448)
  int act;                 // 0 none, 1 relu, 3 tanh
  int out_bf16;
  int tiles_m, tiles_n, n_fastest;
};

__device__ __forceinline__ void glds16(const unsigned char* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// per-lane source rows of the staging pieces (rows [r0, r0 + ROWS) of X, 16-byte chunk
// swizzled): ROWS / 64 pieces of 1 KB per wave; computed once, advanced by 128 bytes per K tile
template <int ROWS>
__device__ __forceinline__ void stage_ptrs(const unsigned char* __restrict__ X, long ld, int r0, int rmax, int wave,
                                           const unsigned char* (&src)[ROWS / 64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < ROWS / 64; ++u) {
    const int r = (wave * (ROWS / 64) + u) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    src[u] = X + (size_t)min(r0 + r, rmax) * ld + c * 16;  // clamped rows are never stored
  }
}

template <int ROWS>
__device__ __forceinline__ void stage(const unsigned char* const (&src)[ROWS / 64], int k0, char* dst, int wave) {
#pragma unroll
  for (int u = 0; u < ROWS / 64; ++u) glds16(src[u] + k0, dst + (wave * (ROWS / 64) + u) * 1024);
}

// fragment of rows [rb, rb + 16): chunks g and 4 + g of row rb + (lane & 15)
__device__ __forceinline__ v8i frag(const char* t, int rb) {
  const int lane = threadIdx.x & 63;
  const int r = rb + (lane & 15), g = lane >> 4;
  const char* row = t + r * BK;
  const u32x4 lo = *reinterpret_cast<const u32x4*>(row + ((g ^ (r & 7)) * 16));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(row + (((4 + g) ^ (r & 7)) * 16));
  return v8i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

__device__ __forceinline__ f32x4 mx(const v8i& a, const v8i& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, E8M0_ONE, 0, E8M0_ONE);
}

__device__ __forceinline__ float act_f(float x, int act) {
  if (act == 1) return x > 0.f ? x : 0.f;
  if (act == 3) return 1.f - 2.f / (__expf(2.f * x) + 1.f);
  return x;
}

// NS staging buffers: NS = 2 (round 3) stages tile kt + 2 after tile kt's barrier, i.e. one
// tile (~1000 MFMA cycles per SIMD, ~0.4 us) ahead — less than the HBM latency under load,
// and the round-5 PMC pass showed 55 % of wave-cycles waiting (35 % MFMA busy,
// profiles/r5_mx8/).  NS = 3 (144 KB of LDS) keeps two tiles in flight: tile kt + 3 is staged
// into tile kt's buffer, and the switch waits only for tile kt + 1 (vmcnt(6): the 6 DMA
// pieces a wave issues per tile for kt + 2 may still be in flight).
template <int NS>
__global__ __launch_bounds__(NTH, 1) void gemm_mx8_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [NS][A | B]
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = p.tiles_m * p.tiles_n;
  const int split = bid / ntile, t = bid - split * ntile;
  const int tm = p.n_fastest ? t / p.tiles_n : t % p.tiles_m;
  const int tn = p.n_fastest ? t % p.tiles_n : t / p.tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / BK;
  const int per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * per, kt1 = min(ktiles, kt0 + per);
  const int arb = wr * 64, brb = wc * 64;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    const unsigned char* sa[BM / 64];
    const unsigned char* sb[BN / 64];
    stage_ptrs<BM>(p.A, p.lda, m0, p.M - 1, wave, sa);
    stage_ptrs<BN>(p.B, p.ldb, n0, p.N - 1, wave, sb);
    stage<BM>(sa, kt0 * BK, smem, wave);
    stage<BN>(sb, kt0 * BK, smem + A_BYTES, wave);
    if constexpr (NS == 3) {  // tile kt0 + 1 in flight behind tile kt0 (clamped: never read past kt1)
      const int k1 = min(kt0 + 1, kt1 - 1) * BK;
      stage<BM>(sa, k1, smem + STAGE, wave);
      stage<BN>(sb, k1, smem + STAGE + A_BYTES, wave);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    {
      const int k2 = min(kt0 + NS - 1, kt1 - 1) * BK;  // NS = 2: kt0 + 1; NS = 3: kt0 + 2
      char* st = smem + (NS - 1) * STAGE;
      stage<BM>(sa, k2, st, wave);
      stage<BN>(sb, k2, st + A_BYTES, wave);
    }
    // B fragments of a whole K tile (4) double-buffered across tiles; A fragments streamed
    // one 16-row block at a time (read block i + 1 while block i's 4 MFMAs run): 64 acc +
    // 64 B + 16 A VGPRs.  The tile switch sits before the last A block: next tile landed ->
    // barrier -> its first fragments, behind the last 4 MFMAs of this tile.
    v8i b[2][4], a0, a1;
#pragma unroll
    for (int j = 0; j < 4; ++j) b[0][j] = frag(smem + A_BYTES, brb + 16 * j);
    a0 = frag(smem, arb);
    auto tile = [&](int kt, int buf, v8i (&bc)[4], v8i (&bn)[4]) {
      const char* ta = smem + buf * STAGE;
      // sched_barrier: keep each A read beside the MFMAs it hides behind (the scheduler
      // would otherwise hoist all reads and hold three fragment sets + renamed accumulators)
      a1 = frag(ta, arb + 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[0][j] = mx(a0, bc[j], acc[0][j]);
      __builtin_amdgcn_sched_barrier(0);
      a0 = frag(ta, arb + 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[1][j] = mx(a1, bc[j], acc[1][j]);
      __builtin_amdgcn_sched_barrier(0);
      a1 = frag(ta, arb + 48);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[2][j] = mx(a0, bc[j], acc[2][j]);
      __builtin_amdgcn_sched_barrier(0);
      // branch-free tile switch (one basic block, so the sched_barriers hold): the reads of
      // the next tile's first fragments and the staging of the tile NS - 1 ahead are issued
      // unconditionally — past the split's end they re-read / re-load a clamped tile into a
      // buffer nobody reads again
      if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
      const int nbuf = buf + 1 == NS ? 0 : buf + 1;
      {
        const char* nt = smem + nbuf * STAGE;
#pragma unroll
        for (int j = 0; j < 4; ++j) bn[j] = frag(nt + A_BYTES, brb + 16 * j);
        a0 = frag(nt, arb);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[3][j] = mx(a1, bc[j], acc[3][j]);
      __builtin_amdgcn_sched_barrier(0);
      {
        char* st = smem + buf * STAGE;
        const int k2 = min(kt + NS, kt1 - 1) * BK;
        stage<BM>(sa, k2, st, wave);
        stage<BN>(sb, k2, st + A_BYTES, wave);
      }
      return nbuf;
    };
    int buf = 0;
#pragma unroll 1
    for (int kt = kt0; kt < kt1; kt += 2) {
      buf = tile(kt, buf, b[0], b[1]);
      if (kt + 1 >= kt1) break;
      buf = tile(kt + 1, buf, b[1], b[0]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped extra loads land before exit
  }

  // acc[i][j][r] = C[m0 + arb + 16i + 4(lane >> 4) + r][n0 + brb + 16j + (lane & 15)]
  const float alpha = p.alpha * (p.alpha_ptr ? *p.alpha_ptr : 1.f);
  const int colb = n0 + brb + (lane & 15);
  const int rowb = m0 + arb + 4 * (lane >> 4);
  if (p.ksplit > 1) {
    float* Cs = reinterpret_cast<float*>(p.C) + (size_t)split * p.slab;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rowb + 16 * i + r;
        if (row >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = colb + 16 * j;
          if (col < p.N) Cs[(size_t)row * p.ldc + col] = acc[i][j][r] * alpha;
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = colb + 16 * j;
    if (col >= p.N) continue;
    const float bj = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rowb + 16 * i + r;
        if (row >= p.M) continue;
        const float v = act_f(acc[i][j][r] * alpha + bj, p.act);
        const size_t o = (size_t)row * p.ldc + col;
        if (p.out_bf16) reinterpret_cast<unsigned short*>(p.C)[o] = f32_to_bf16(v);
        else reinterpret_cast<float*>(p.C)[o] = v;
      }
  }
}

PV_DEBUG_EXPORT(gemm8)
}  // namespace gemm8
}  // namespace pv

using namespace pv;

namespace {
// pv_gemm_mx8_set_stages: staging buffers (2 = round 3, 3 = two tiles in flight); measured equal
// (bag forward 68-76 vs 74-78 us, weight gradient 90-94 vs 91-93, square 8192 1.69-1.71 PF/s
// both; profiles/r5_mx8/): the waits the PMC pass counts are not the DMA latency
int g_mx8_stages = 2;
}  // namespace

PV_API void pv_gemm_mx8_set_stages(int n) { g_mx8_stages = n; }

// C = epi(alpha * (*alpha_ptr) * A8 . B8^T); A8 (M x K) and B8 (N x K) e4m3 bytes, K % 128 == 0,
// 16-byte aligned rows.  ksplit > 1: C is a workspace of ksplit fp32 slabs (slab = elements
// per slab) the caller reduces; bias / act / bf16 then belong to the caller's reduction.
PV_API int pv_gemm_mx8(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                       int ksplit, long slab, const float* bias, float alpha, const float* alpha_ptr, int act,
                       int out_bf16, void* stream) {
  using namespace pv::gemm8;
  if (M <= 0 || N <= 0 || K <= 0 || K % BK) return -1;
  if (ksplit < 1) ksplit = 1;
  if (ksplit > 1 && (out_bf16 || bias || act)) return -2;
  if (((size_t)A & 15) || ((size_t)B & 15) || lda % 16 || ldb % 16) return -3;
  if (act != 0 && act != 1 && act != 3) return -4;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mx8_kernel<2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * STAGE) != hipSuccess ||
        hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_mx8_kernel<3>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 3 * STAGE) != hipSuccess)
      return -5;
    attr = true;
  }
  Params p{(const unsigned char*)A, (const unsigned char*)B, lda, ldb, C, ldc, M, N, K, ksplit, slab, bias, alpha,
           alpha_ptr, act, out_bf16, (M + BM - 1) / BM, (N + BN - 1) / BN, N <= M ? 1 : 0};
  const int grid = p.tiles_m * p.tiles_n * ksplit;
  if (g_mx8_stages == 3)
    hipLaunchKernelGGL(gemm_mx8_kernel<3>, dim3(grid), dim3(NTH), 3 * STAGE, (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(gemm_mx8_kernel<2>, dim3(grid), dim3(NTH), 2 * STAGE, (hipStream_t)stream, p);
  PV_LAUNCH_CHECK();
  return 0;
}
