// K3b + K1b: sparse backward of gather -> dropout -> conv -> global-max-pool -> ReLU.
//
// Because of the global max-pool (cnn_dssm_th.py:94, pool_length = L-k+1) the
// gradient of filter f of sample n reaches exactly ONE window: a = argmax[n,f].
// With g[n,f] = dL/dpooled[n,f] * [pooled[n,f] > 0] (ReLU) and s = 1/(1-p):
//
//   db[f]          = sum_n g[n,f]
//   dW[f,j,e]      = s * sum_n g[n,f] * Xm[n, a+j, e]          (Xm = masked bf16 rows)
//   dTable[v,e]   += s * g[n,f] * W[f,j,e] * m[n,a+j,e]        for v = ids[n, a+j]
//
// Cost is O(N * F * k * E), independent of L (the dense Keras/Theano backward is
// O(N * L * F * k * E)).  The dropout mask m is regenerated from the counter hash
// (same function as the forward staging), never stored.
//
// dTable without 17M x 400-byte float atomics:
//   keys   : the slot keys (token id, sentinel V when dead) of every (n, f) pair — written
//            by the conv forward's loader waves (conv_pool_fwd.hip, loader7_emit), or by
//            the emit kernel here — plus one {g*scale, argmax} record per pair;
//   sort   : stable radix sort of (key, slot id) (radix_sort.hip);
//   reduce : each wave walks EPW sorted entries, 4 at a time (one per 16-lane group),
//            recomputes the contribution s*g*W[f,j,:]*m on the fly (bf16 W rows are
//            L2-resident) and sums it in registers per token, carrying its open run
//            across sub-chunks; one row-atomic per (wave, token) boundary.
#include "common.h"

namespace pv {
namespace convbwd {
PV_DEBUG_FLAG

constexpr int EP = 104;
constexpr int FW = 150;

// ---- dW, db -----------------------------------------------------------------------
// grid (2*FW, nsplit), block 256 (4 waves).  Each wave takes its samples 64 at a time:
// lane l loads sample (base+l)'s g / ReLU flag / argmax and the k token ids of its
// argmax window (independent loads, issued together), then the wave walks the live
// samples with v_readlane broadcasts.  Lane l owns the 16-byte piece l of the (k x EP)
// window (row l / 13, columns 8*(l % 13) .. +7): one 16-byte table load, the dropout mask
// of the piece from keep_piece (one group hash in the nibble mode), 8 FMAs.  The k row
// hashes of a sample are computed once by lanes 0..k-1 and fetched with ds_bpermute.
// Table loads for 4 samples are issued before use.
constexpr int PIECES_ROW = EP / 8;  // 13
template <int K, int DM>
__device__ __forceinline__ void dw_filter(const float* __restrict__ gpool, const float* __restrict__ pooled,
                                          const int* __restrict__ argmax, const int* __restrict__ ids,
                                          const unsigned short* __restrict__ table, float* __restrict__ dw,
                                          float* __restrict__ db, float* red, int L, int E, int V, int fg, int fl,
                                          int n0, int n1, unsigned seed, unsigned row_offset, int thr, int token_mode,
                                          float scale, long long* fxw, long long* fxb) {
  constexpr int NP = K * PIECES_ROW;  // pieces per window (39 / 52)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float gsum = 0.f;
  const int jj = lane / PIECES_ROW, pc = lane - jj * PIECES_ROW;
  const bool pv_ = lane < NP && pc * 8 < E;
  const int jsel = jj < K ? jj : 0;
  for (int base = n0 + wave * 64; base < n1; base += 256) {
    const int n = base + lane;
    float g = 0.f;
    int a = 0;
    bool live = false;
    int tok[4] = {-1, -1, -1, -1};
    if (n < n1) {
      const size_t o = (size_t)n * (2 * FW) + fg;
      g = gpool[o];
      a = argmax[o];
      live = pooled[o] > 0.f && g != 0.f && PV_OK(a >= 0 && a < L, PV_ERR_ARGMAX);
      if (live) {
#pragma unroll
        for (int j = 0; j < K; ++j) tok[j] = (a + j < L) ? ids[(size_t)n * L + a + j] : -1;
      }
    }
    gsum += live ? g : 0.f;
    unsigned long long m = __ballot(live);
    while (m) {
      int sl[4];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sl[u] = m ? (int)__builtin_ctzll(m) : -1;
        if (m) { m &= m - 1; ++cnt; }
      }
      u32x4 raw[4];
      // dropout row hashes of the (up to) 4 samples of this round in ONE pass: lane 4u + j
      // hashes row (n_u, a_u + j), then every lane fetches its row's hash with a bpermute
      // ... and the same lanes fetch the window's token ids of those samples (4 bpermutes for
      // the round instead of 4 readlanes + 3 selects per sample)
      unsigned hq = 0u;
      int tq;
      {
        const int uu = (lane >> 2) & 3, jq = lane & 3;
        int su = sl[0];
        su = uu == 1 ? sl[1] : su;
        su = uu == 2 ? sl[2] : su;
        su = uu == 3 ? sl[3] : su;
        su = su < 0 ? sl[0] : su;
        int tv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) tv[j] = __builtin_amdgcn_ds_bpermute(su * 4, tok[j]);
        tq = jq == 0 ? tv[0] : jq == 1 ? tv[1] : jq == 2 ? tv[2] : tv[3];
        if (DM < 0 ? thr > 0 : DM != 0) {
          const int au = __builtin_amdgcn_ds_bpermute(su * 4, a);
          hq = (lane < 16 && jq < K) ? dropout_row_hash(seed, row_offset + (unsigned)((base + su) * L + au + jq)) : 0u;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) break;
        const int t = __builtin_amdgcn_ds_bpermute((4 * u + jsel) * 4, tq);
        const bool ok = pv_ && t >= 0 && t < V;
        // 32-bit element offset (V * EP < 2^31): no 64-bit multiply per piece
        raw[u] = ok ? *reinterpret_cast<const u32x4*>(table + (unsigned)(t * EP + pc * 8)) : u32x4{0u, 0u, 0u, 0u};
        if (DM < 0 ? thr > 0 : DM != 0) {  // dropout mask of this lane's piece (ops/reference.py dropout_keep_mask)
          const unsigned hr = (unsigned)__builtin_amdgcn_ds_bpermute((4 * u + jsel) * 4, (int)hq);
          if (DM == 3 || (DM < 0 && token_mode)) {
            const unsigned k = ((int)(hr & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
            raw[u] &= u32x4{k, k, k, k};
          } else {
            raw[u] &= keep_piece(hr, pc, dm_thr(DM, thr));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) break;
        const float gj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), sl[u]));
        const f32x2 g2 = {gj, gj};
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // packed fp32 FMA (v_pk_fma_f32): two columns per op
          const f32x2 x2 = {__uint_as_float(raw[u][w] << 16), __uint_as_float(raw[u][w] & 0xFFFF0000u)};
          f32x2 a2 = {acc[2 * w], acc[2 * w + 1]};
          a2 = __builtin_elementwise_fma(g2, x2, a2);
          acc[2 * w] = a2[0];
          acc[2 * w + 1] = a2[1];
        }
      }
    }
  }
  // cross-wave reduction through LDS: red[wave][K*EP], piece l -> elements 8l .. 8l+7
  if (lane < NP) {
#pragma unroll
    for (int c = 0; c < 8; ++c) red[wave * (K * EP) + lane * 8 + c] = acc[c];
  }
  const float gs = wave_sum(gsum);
  __syncthreads();
  for (int x = threadIdx.x; x < K * EP; x += 256) {
    float v = red[x] + red[K * EP + x] + red[2 * K * EP + x] + red[3 * K * EP + x];
    int j = x / EP, e = x % EP;
    if (e < E && v != 0.f) {
      const size_t o = ((size_t)fl * K + j) * E + e;
      if (fxw) fx_add(fxw, o, v * scale);  // deterministic mode (common.h)
      else atomicAdd(&dw[o], v * scale);
    }
  }
  __shared__ float gsw[4];
  if (lane == 0) gsw[wave] = gs;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = gsw[0] + gsw[1] + gsw[2] + gsw[3];
    if (t != 0.f) {
      if (fxb) fx_add(fxb, fg, t);
      else atomicAdd(&db[fl], t);  // db: this width's bias gradient (filter fl of the width)
    }
  }
}

// DM: compile-time dropout mode (0 off, 1 element p = 0.25, 2 element any p, 3 token; the runtime-mode
// instantiation, 0.537 vs 0.495 ms, is gone)
template <int DM>
__global__ __launch_bounds__(256) void conv_bwd_dw_kernel(const float* gpool, const float* pooled, const int* argmax,
                                                          const int* ids, const unsigned short* table, float* dw3,
                                                          float* dw4, float* db3, float* db4, int N, int L, int E, int V,
                                                          int nsplit,
                                                          unsigned seed, const unsigned* seed_ptr,
                                                          unsigned row_offset, int thr, int token_mode, float scale,
                                                          int xcd_map, long long* fx) {
  __shared__ float red[4 * 4 * EP];
  if (seed_ptr) seed += *seed_ptr;  // device seed offset (captured hipGraph steps)
  // XCD-aware work mapping: workgroups are dealt round-robin to the 8 XCDs (each with its
  // own L2).  The natural (f = blockIdx.x, split = blockIdx.y) order puts filters f, f+1 of
  // one sample range on different XCDs, so every L2 fetches the same gpool / argmax /
  // pooled / id lines (rows of 2*FW floats hold all filters of a sample).  Remapped, the
  // 2*FW filter blocks of a split run on ONE XCD and share those lines in its L2.
  int f = blockIdx.x, split = blockIdx.y;
  if (xcd_map && (nsplit & 7) == 0) {
    const int b = blockIdx.x + gridDim.x * blockIdx.y;
    const int logical = (b & 7) * (gridDim.x * (nsplit >> 3)) + (b >> 3);
    f = logical % (int)gridDim.x;
    split = logical / (int)gridDim.x;
  }
  const int per = ((N + nsplit - 1) / nsplit + 255) / 256 * 256;
  const int n0 = split * per, n1 = min(N, n0 + per);
  if (f < FW)
    dw_filter<3, DM>(gpool, pooled, argmax, ids, table, dw3, db3, red, L, E, V, f, f, n0, n1, seed, row_offset, thr,
                 token_mode, scale, fx, fx ? fx + (size_t)7 * FW * E : nullptr);
  else
    dw_filter<4, DM>(gpool, pooled, argmax, ids, table, dw4, db4, red, L, E, V, f, f - FW, n0, n1, seed, row_offset, thr,
                 token_mode, scale, fx ? fx + (size_t)3 * FW * E : nullptr, fx ? fx + (size_t)7 * FW * E : nullptr);
}

// ---- dTable emit (compact): keys + slot values + one 8-byte record per (n,f) pair -------
// Slots are numbered per sample without the dead 4th row of the k=3 filters:
//   sample n owns slots [n*SPS, (n+1)*SPS), SPS = 3*FW + 4*FW = 1050; k=3 filter f (< FW) row j
//   is slot n*SPS + 3f + j, k=4 filter f row j is n*SPS + 3*FW + 4(f - FW) + j
// (a 12.5% smaller sort than 4 slots per pair).  Everything the reduce needs per entry
// follows from the slot and rec[pair] = {g * scale, argmax}: ONE 8-byte gather per sorted
// entry instead of three 4-byte gathers from per-slot arrays (the sorted order scatters them).
constexpr int SPS = 7 * FW;

__device__ __forceinline__ void slot_decode(unsigned sl, unsigned& n, unsigned& f, unsigned& j) {
  n = sl / (unsigned)SPS;
  const unsigned r = sl - n * (unsigned)SPS;
  if (r < 3u * FW) {
    f = r / 3u;
    j = r - 3u * f;
  } else {
    const unsigned q = r - 3u * FW;
    f = FW + (q >> 2);
    j = q & 3u;
  }
}

// KT: unsigned (any V) or unsigned short (V < 65535: 2-byte sort keys, a quarter less sort /
// emit / reduce key traffic)
template <typename KT>
__global__ __launch_bounds__(256) void conv_bwd_emit3_kernel(const float* gpool, const float* pooled,
                                                             const int* argmax, const int* ids, KT* keys,
                                                             unsigned* vals, int2* rec, int N, int L, int V,
                                                             float scale) {
  const long pair = (long)blockIdx.x * 256 + threadIdx.x;
  if (pair >= (long)N * 2 * FW) return;
  const int n = (int)(pair / (2 * FW)), f = (int)(pair % (2 * FW));
  const int K = f < FW ? 3 : 4;
  const float g = gpool[pair];
  const int a = argmax[pair];
  const bool live = pooled[pair] > 0.f && g != 0.f && PV_OK(a >= 0 && a < L, PV_ERR_ARGMAX);
  rec[pair] = int2{__float_as_int(g * scale), a};
  const unsigned s0 = (unsigned)n * SPS + (f < FW ? 3u * f : 3u * FW + 4u * (f - FW));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < K) {
      const int t = a + j;
      const bool ok = live && t < L;
      const int v = ok ? ids[(size_t)n * L + t] : V;
      PV_CHECK(v >= 0 && v <= V, PV_ERR_ID);
      keys[s0 + j] = (KT)((unsigned)v < (unsigned)V ? (unsigned)v : (unsigned)V);
      if (vals) vals[s0 + j] = s0 + j;  // null: the sort generates the positions itself
    }
  }
}

// ---- dTable reduce: the round (4 entries per wave-instruction) --------------------------
// A 16-lane group owns one sorted entry per round (4 entries per round per wave); lane p
// of the group owns columns 8p..8p+7 of the 104-wide padded row: one 16-byte load of the
// bf16 weight row W[f][j] (layout [2*FW][4][EP], zero padded), the two dropout group
// hashes of those 8 columns, 8 FMAs into its accumulator.  Entries are sorted by key, so
// a round's keys are ascending across the groups: the common round (all 4 keys equal the
// current run's key) just accumulates; a round with a key change flushes the finished
// run — the 4 groups' partials meet in a wave-private LDS slab (write 104 floats per
// group, read back lane-linear) and lane l adds columns l, l+64 to dTable with two
// 256-byte-shaped atomic instructions.
constexpr int RPIECES = EP / 8;  // 13 pieces of 8 columns
__device__ __forceinline__ void reduce4_flush(float* slab, const float (&acc)[8], int g, int p, int lane, int E,
                                              unsigned key, float* __restrict__ dtable, long long* fx) {
  if (p < RPIECES) {
    *reinterpret_cast<f32x4*>(slab + g * EP + 8 * p) = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *reinterpret_cast<f32x4*>(slab + g * EP + 8 * p + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's slab writes are done
  const int c0 = lane, c1 = lane + 64;
  if (c0 < E) {
    const float v = slab[c0] + slab[EP + c0] + slab[2 * EP + c0] + slab[3 * EP + c0];
    if (fx) fx_add(fx, (unsigned)(key * (unsigned)E + c0), v);  // deterministic mode
    else atomicAdd(&dtable[(unsigned)(key * (unsigned)E + c0)], v);
  }
  if (c1 < E) {
    const float v = slab[c1] + slab[EP + c1] + slab[2 * EP + c1] + slab[3 * EP + c1];
    if (fx) fx_add(fx, (unsigned)(key * (unsigned)E + c1), v);
    else atomicAdd(&dtable[(unsigned)(key * (unsigned)E + c1)], v);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // slab reads done before the next flush overwrites it
}

// ---- dTable reduce, long runs: each wave owns EPW consecutive sorted entries --------------
// The rounds above, with a wave walking EPW entries (64 per sub-chunk) and
// carries its open run (key + register partials) across sub-chunks, so a token whose run
// spans many sub-chunks is flushed once per wave instead of once per 64 entries: under the
// Zipf token distribution of real (and synthetic) pages the most frequent rows otherwise
// take thousands of serialised row-atomics at one L2 channel.  Entry metadata is software-
// pipelined: keys/slots two sub-chunks ahead, the {g, argmax} record gather one ahead.
template <typename KT>
__device__ __forceinline__ void rd_meta(const KT* __restrict__ skeys, const unsigned* __restrict__ svals,
                                        long i, long wend, unsigned V, unsigned& key, unsigned& sl) {
  key = V;
  sl = 0u;
  if (i < wend) {
    key = skeys[i];
    PV_CHECK(key <= V, PV_ERR_KEY);
    if (key < V) sl = svals[i];
  }
}

// DM: dropout mode as a template parameter (0 off, 1 element p = 0.25, 2 element any p,
// 3 token); the common round's multiply + add are packed FMAs.  Earlier generations (a
// 64-entry-per-wave kernel, a runtime dropout mode, RB rounds of row gathers in flight) were
// measured slower and removed: docs/PERF.md "dTable reduce generations".
// OCC: minimum waves per SIMD the register allocation must allow (1 = compiler's choice,
// 74 VGPRs / 6 waves; 8 caps it at 64 VGPRs)
template <typename KT, int DM, int OCC = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void conv_bwd_reduce7_kernel(const KT* __restrict__ skeys,
                                                               const unsigned* __restrict__ svals,
                                                               const int2* __restrict__ rec,
                                                               const unsigned short* __restrict__ wrow,
                                                               float* __restrict__ dtable, long M, int EPW, int L,
                                                               int E, int V, unsigned seed, const unsigned* seed_ptr,
                                                               unsigned row_offset, int thr, int token_mode, long long* fx) {
  __shared__ __attribute__((aligned(16))) float slabs[4][4 * EP];
  if (seed_ptr) seed += *seed_ptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, p = lane & 15;
  float* slab = slabs[wave];
  const long wbeg = ((long)blockIdx.x * 4 + wave) * EPW;
  if (wbeg >= M) return;
  const long wend = min(M, wbeg + (long)EPW);
  const unsigned UV = (unsigned)V;
  // pipeline: (k0, s0, r0) = current sub-chunk, (k1, s1) = next, (k2, s2) = the one after
  unsigned k0, s0, k1, s1, k2, s2;
  rd_meta(skeys, svals, wbeg + lane, wend, UV, k0, s0);
  rd_meta(skeys, svals, wbeg + 64 + lane, wend, UV, k1, s1);
  auto ld_rec = [&](unsigned key, unsigned sl) -> int2 {
    if (!(key < UV && PV_OK((long)sl < M, PV_ERR_SLOT))) return int2{0, 0};
    unsigned nn, f, j;
    slot_decode(sl, nn, f, j);
    return rec[nn * (2 * FW) + f];
  };
  int2 r0 = ld_rec(k0, s0);
  unsigned cur = UV;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const bool act = p < RPIECES;
  for (long b = wbeg; b < wend; b += 64) {
    rd_meta(skeys, svals, b + 128 + lane, wend, UV, k2, s2);
    const int2 r1 = ld_rec(k1, s1);
    // this lane's entry of sub-chunk b
    const unsigned key = k0;
    unsigned fj = 0, hr = 0;
    float gg = 0.f;
    if (key < UV) {
      unsigned nn, f, j;
      slot_decode(s0, nn, f, j);
      fj = (f << 2) | j;
      gg = __int_as_float(r0.x);
      if (DM != 0) hr = dropout_row_hash(seed, row_offset + nn * (unsigned)L + (unsigned)r0.y + j);
    }
    const int n = __popcll(__ballot(key < UV));  // live entries are a prefix (sorted)
    if (n == 0) break;
    if (cur == UV) cur = __builtin_amdgcn_readfirstlane(key);
    const unsigned klast = (unsigned)__builtin_amdgcn_readlane((int)key, n - 1);
    for (int q0 = 0; q0 < n; q0 += 4) {
      const int e = q0 + g;
      const bool valid = e < n;
      const int src = (valid ? e : q0) * 4;
      unsigned kg = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)key);
      const unsigned f_j = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)fj);
      float ge = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(gg)));
      const unsigned he = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)hr);
      if (!valid) ge = 0.f;
      float x[8];
      {
        // every lane loads (lanes p >= 13 re-read piece 12; their sums are never flushed):
        // no exec-masked load
        u32x4 w = *reinterpret_cast<const u32x4*>(wrow + (unsigned)(f_j * EP + 8 * (act ? p : RPIECES - 1)));
        if constexpr (DM == 3) {
          const unsigned k = ((int)(he & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
          w &= u32x4{k, k, k, k};
        } else if constexpr (DM == 1 || DM == 4) {
          w &= keep_piece(he, p, dm_thr(DM, thr));  // compile-time p = 0.25 (the reference's rate) / 0.125
        } else if constexpr (DM == 2) {
          w &= keep_piece(he, p, thr);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = __uint_as_float((k & 1) ? (w[k >> 1] & 0xFFFF0000u) : (w[k >> 1] << 16));
      }
      if (!valid) kg = klast;
      const unsigned ka = (unsigned)__builtin_amdgcn_readlane((int)kg, 0);
      const unsigned kb = (unsigned)__builtin_amdgcn_readlane((int)kg, 48);
      if (ka == cur && kb == cur) {  // common round: packed FMAs straight into the run sums
        const f32x2 g2 = {ge, ge};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f32x2 a2 = {acc[2 * k], acc[2 * k + 1]};
          a2 = __builtin_elementwise_fma(g2, f32x2{x[2 * k], x[2 * k + 1]}, a2);
          acc[2 * k] = a2[0];
          acc[2 * k + 1] = a2[1];
        }
        continue;
      }
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ge * x[k];
      bool done = false;
      for (int it = 0; it < 5; ++it) {
        const bool mine = !done && kg == cur;
        if (mine) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += v[k];
          done = true;
        }
        const unsigned long long left = __ballot(!done);
        if (left == 0) break;
        reduce4_flush(slab, acc, g, p, lane, E, cur, dtable, fx);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
        cur = (unsigned)__builtin_amdgcn_readlane((int)kg, (int)__builtin_ctzll(left));
      }
    }
    if (n < 64) break;  // the dead (key == V) tail starts inside this sub-chunk
    k0 = k1; s0 = s1; r0 = r1;
    k1 = k2; s1 = s2;
  }
  if (cur != UV) reduce4_flush(slab, acc, g, p, lane, E, cur, dtable, fx);
}

// ---- dTable for short sequences (query towers: L <= DENSE_MAXL) ------------------------------
// A 45-token query has ~45 touched embedding rows but 1050 (f, j) gradient entries, so the
// entry-level emit -> sort -> reduce moves 23x more entries than there are rows.  Instead:
//  dx_dense : one workgroup per sample builds the sample's dense input gradient in LDS,
//               dX[t, :] = s * sum_{(f, j): argmax[n,f] + j == t, live} g[n,f] * W[f, j, :]
//             (LDS float atomics: the (f, j) of a sample collide on the same t), applies the
//             regenerated dropout mask and writes each touched row (fp32, stride EP) plus its
//             token key (sentinel V for untouched / fully dropped rows);
//  sort     : the row keys (radix_sort.hip), values = row index;
//  rows_reduce: each wave sums EPW consecutive sorted rows per token in registers, one
//             row-atomic per (wave, token) run.  Summing per token BEFORE the global atomics
//             matters: direct per-row atomics from dx_dense serialise on the Zipf-hot rows
//             (measured 2.4 ms vs 0.49 ms for the sort path at 4096 x 45).
constexpr int DENSE_MAXL = 256;  // LDS: L * EP fp32 (104 KB at L = 256)

// dx_dense, one workgroup per sample, no atomics:
//  1. per-filter {g*scale (0 = dead), argmax} -> LDS;
//  2. wave 0 ranks the (f, j) entries by their position t = argmax + j in entry order (one
//     ballot per bit of t finds the lanes of a round with the same t; per-t running counts in
//     LDS): bucket position = stable, so each row sums its entries in a fixed order;
//  3. exclusive scan of the per-t counts, scatter of the entry ids into their buckets;
//  4. wave w sums rows t = w, w+4, ...: lane c < 52 owns columns 2c, 2c+1 (one 4-byte load of
//     the bf16 weight row per entry, 4 entries in flight), applies the dropout mask of those
//     columns and writes the row (fp32, stride EP) + its token key.
constexpr int DX_ENT = 2 * FW * 4;  // entry ids f*4 + j (k=3 filters leave j = 3 unused)
constexpr int DX_BATCH = 8;          // entries per load batch in the row sums
constexpr int DX_THREADS = 512;      // 8 waves: rows t = wave, wave + 8, ...

template <typename KT, int DM>
__global__ __launch_bounds__(DX_THREADS) void conv_bwd_dx_dense_kernel(const float* __restrict__ gpool,
                                                                const float* __restrict__ pooled,
                                                                const int* __restrict__ argmax,
                                                                const int* __restrict__ ids,
                                                                const unsigned short* __restrict__ wrow,
                                                                float* __restrict__ rows, KT* __restrict__ keys,
                                                                int L, int V, unsigned seed,
                                                                const unsigned* seed_ptr, unsigned row_offset,
                                                                int thr, int token_mode, float scale) {
  __shared__ float gsl[2 * FW];
  __shared__ int al[2 * FW];
  __shared__ unsigned cnt[DENSE_MAXL];
  __shared__ unsigned start[DENSE_MAXL];
  __shared__ unsigned short rnk[DX_ENT];
  __shared__ unsigned short ent[DX_ENT];
  __shared__ unsigned ws[DX_THREADS / 64];
  if (seed_ptr) seed += *seed_ptr;
  const int n = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const size_t rb = (size_t)n * (2 * FW);
  for (int f = tid; f < 2 * FW; f += DX_THREADS) {
    const float g = gpool[rb + f];
    const int a = argmax[rb + f];
    const bool live = pooled[rb + f] > 0.f && g != 0.f && PV_OK(a >= 0 && a < L, PV_ERR_ARGMAX);
    gsl[f] = live ? g * scale : 0.f;
    al[f] = a;
  }
  for (int t = tid; t < DENSE_MAXL; t += DX_THREADS) cnt[t] = 0u;
  __syncthreads();
  // (2) stable ranks by t, wave 0
  int nb = 0;  // bits of t
  while ((1 << nb) < L) ++nb;
  if (wave == 0) {
    for (int e0 = 0; e0 < DX_ENT; e0 += 64) {
      const int e = e0 + lane;
      const int f = e >> 2, j = e & 3;
      int t = -1;
      if (e < DX_ENT && (j < 3 || f >= FW) && gsl[f] != 0.f) {
        t = al[f] + j;
        if (t >= L) t = -1;
      }
      const bool valid = t >= 0;
      unsigned long long m = __ballot(valid);
      for (int b = 0; b < nb; ++b) {
        const bool bit = valid && ((t >> b) & 1);
        const unsigned long long bb = __ballot(bit);
        m &= bit ? bb : ~bb;
      }
      m = valid ? m : 0ull;
      const unsigned long long lt = (1ull << lane) - 1ull;
      const unsigned old = valid ? cnt[t] : 0u;
      if (e < DX_ENT) rnk[e] = valid ? (unsigned short)(old + __popcll(m & lt)) : (unsigned short)0xFFFF;
      if (valid && (m & lt) == 0ull) cnt[t] = old + (unsigned)__popcll(m);
    }
  }
  __syncthreads();
  {  // (3) scan of the per-t counts (L <= 256 <= threads)
    const unsigned v = tid < L ? cnt[tid] : 0u;
    unsigned x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    unsigned base = 0;
    for (int i = 0; i < wave; ++i) base += ws[i];
    if (tid < L) start[tid] = base + x - v;
  }
  __syncthreads();
  for (int e = tid; e < DX_ENT; e += DX_THREADS) {
    const unsigned r = rnk[e];
    if (r != 0xFFFFu) {
      const int t = al[e >> 2] + (e & 3);
      ent[start[t] + r] = (unsigned short)e;
    }
  }
  __syncthreads();
  // (4) rows
  const int c = lane;          // column pair (2c, 2c+1)
  const bool act = c < EP / 2;  // 52 pairs
  for (int t = wave; t < L; t += DX_THREADS / 64) {
    const size_t r = (size_t)n * L + t;
    const int tok = ids[r];
    PV_CHECK(tok >= 0 && tok < V, PV_ERR_ID);
    const int b0 = (int)start[t], b1 = b0 + (int)cnt[t];
    float x0 = 0.f, x1 = 0.f;
    for (int i = b0; i < b1; i += DX_BATCH) {  // DX_BATCH weight-row loads in flight per lane
      unsigned w[DX_BATCH];
      float g[DX_BATCH];
#pragma unroll
      for (int u = 0; u < DX_BATCH; ++u) {
        const int e = ent[i + u < b1 ? i + u : b0];
        g[u] = i + u < b1 ? gsl[e >> 2] : 0.f;
        w[u] = act ? *reinterpret_cast<const unsigned*>(wrow + (size_t)e * EP + 2 * c) : 0u;
      }
#pragma unroll
      for (int u = 0; u < DX_BATCH; ++u) {
        x0 += g[u] * __uint_as_float(w[u] << 16);
        x1 += g[u] * __uint_as_float(w[u] & 0xFFFF0000u);
      }
    }
    bool keep_row = tok >= 0 && tok < V && b1 > b0;
    if (keep_row && (DM < 0 ? thr > 0 : DM != 0)) {
      const unsigned hr = dropout_row_hash(seed, row_offset + (unsigned)n * (unsigned)L + (unsigned)t);
      if (DM == 3 || (DM < 0 && token_mode)) {
        keep_row = (int)(hr & 0xFFu) >= thr;
      } else {
        const u32x4 k = keep_piece(hr, c >> 2, dm_thr(DM, thr));
        const unsigned kw = k[c & 3];
        x0 = (kw & 1u) ? x0 : 0.f;
        x1 = (kw & 0x10000u) ? x1 : 0.f;
      }
    }
    if (lane == 0) keys[r] = (KT)(keep_row ? (unsigned)tok : (unsigned)V);
    if (keep_row && act) *reinterpret_cast<f32x2*>(rows + r * EP + 2 * c) = f32x2{x0, x1};
  }
}

// Sorted rows -> dTable: wave w sums entries [w*EPW, (w+1)*EPW) run by run (sentinel keys V
// sort last and end the walk); rows are loaded 4 entries ahead.
template <typename KT>
__global__ __launch_bounds__(256) void conv_bwd_rows_reduce_kernel(const KT* __restrict__ skeys,
                                                                   const unsigned* __restrict__ svals,
                                                                   const float* __restrict__ rows,
                                                                   float* __restrict__ dtable, long M, int EPW,
                                                                   int E, int V, long long* fx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long wbeg = ((long)blockIdx.x * 4 + wave) * EPW;
  if (wbeg >= M) return;
  const long wend = min(M, wbeg + (long)EPW);
  const int c0 = lane, c1 = lane + 64;
  const unsigned UV = (unsigned)V;
  unsigned cur = UV;
  float a0 = 0.f, a1 = 0.f;
  auto flush = [&]() {
    if (cur < UV) {
      if (fx) {  // deterministic mode
        if (c0 < E) fx_add(fx, (size_t)cur * E + c0, a0);
        if (c1 < E) fx_add(fx, (size_t)cur * E + c1, a1);
      } else {
        float* drow = dtable + (size_t)cur * E;
        if (c0 < E) atomicAdd(&drow[c0], a0);
        if (c1 < E) atomicAdd(&drow[c1], a1);
      }
    }
    a0 = 0.f;
    a1 = 0.f;
  };
  for (long i0 = wbeg; i0 < wend; i0 += 64) {
    // this sub-chunk's keys / row ids: one per lane, broadcast by readlane
    const long il = i0 + lane;
    const unsigned kl = il < wend ? (unsigned)skeys[il] : UV;
    const unsigned rl = (il < wend && kl < UV) ? svals[il] : 0u;
    const int n = __popcll(__ballot(kl < UV));  // live entries are a prefix (sorted)
    for (int e0 = 0; e0 < n; e0 += 8) {
      float x0[8], x1[8];
      unsigned kk[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u < n ? e0 + u : e0;
        kk[u] = (unsigned)__builtin_amdgcn_readlane((int)kl, e);
        const unsigned row = (unsigned)__builtin_amdgcn_readlane((int)rl, e);
        PV_CHECK((long)row < M, PV_ERR_SLOT);
        const float* src = rows + (size_t)row * EP;
        x0[u] = src[c0];
        x1[u] = c1 < E ? src[c1] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (e0 + u >= n) break;
        if (kk[u] != cur) {
          flush();
          cur = kk[u];
        }
        a0 += x0[u];
        a1 += x1[u];
      }
    }
    if (n < 64) break;
  }
  flush();
}

PV_DEBUG_EXPORT(convbwd)
}  // namespace convbwd
}  // namespace pv

using namespace pv;

// deterministic mode (common.h): fixed-point accumulators for an n-float target, flushed
// into it after the kernel; a no-op otherwise
struct DetAcc {
  long long* fx = nullptr;
  int err = 0;
  DetAcc(size_t n, hipStream_t st) {
    if (pv::det_on()) {
      fx = pv::det_scratch(n, st);
      if (!fx) err = -4;
    }
  }
  int finish(float* dst, size_t n, hipStream_t st) const { return fx ? pv::det_flush(fx, dst, n, st) : 0; }
};


// db3 / db4: the two widths' bias gradients (150 floats each; separate so they can be the
// bias parameters' own slices of the flat gradient buffer — ops/grad_sink.py)
PV_API int pv_conv_pool_bwd_dw2(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                const void* table, float* dw3, float* dw4, float* db3, float* db4, int N, int L, int E,
                                int V, unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr,
                                int token_mode, float scale, void* stream) {
  using namespace pv::convbwd;
  if (E > EP || L < 4 || (long)V * EP >= (1L << 31)) return -1;  // 32-bit table offsets in the kernel
  int nsplit = (N + 255) / 256;
  if (nsplit > 64) nsplit = 64;
  if (nsplit < 1) nsplit = 1;
  static const int xcd_map = [] {  // PAGEVEC_DW_XCD=0: natural block order (A/B switch)
    const char* e = getenv("PAGEVEC_DW_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  hipStream_t st = (hipStream_t)stream;
  // deterministic mode: fixed-point accumulators [dW3 | dW4 | db], flushed in order below
  const size_t nfx = (size_t)7 * FW * E + 2 * FW;
  long long* fx = det_on() ? det_scratch(nfx, st) : nullptr;
  if (det_on() && !fx) return -4;
  const int dm = dm_of(thr, token_mode);
#define PV_DW(DMV)                                                                                               \
  hipLaunchKernelGGL((conv_bwd_dw_kernel<DMV>), dim3(2 * FW, nsplit), dim3(256), 0, st, gpool, pooled, argmax, ids, \
                     (const unsigned short*)table, dw3, dw4, db3, db4, N, L, E, V, nsplit, seed, seed_ptr,           \
                     row_offset, thr, token_mode, scale, xcd_map, fx)
  if (dm == 0) PV_DW(0);
  else if (dm == 1) PV_DW(1);
  else if (dm == 4) PV_DW(4);
  else if (dm == 3) PV_DW(3);
  else PV_DW(2);
#undef PV_DW
  PV_LAUNCH_CHECK();
  if (fx) {
    int rc = det_flush(fx, dw3, (size_t)3 * FW * E, st);
    if (!rc) rc = det_flush(fx + (size_t)3 * FW * E, dw4, (size_t)4 * FW * E, st);
    if (!rc) rc = det_flush(fx + (size_t)7 * FW * E, db3, FW, st);
    if (!rc) rc = det_flush(fx + (size_t)7 * FW * E + FW, db4, FW, st);
    return rc;
  }
  return 0;
}

// db: both widths' bias gradients as one (2 * FW) array
PV_API int pv_conv_pool_bwd_dw(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                               const void* table, float* dw3, float* dw4, float* db, int N, int L, int E, int V,
                               unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                               float scale, void* stream) {
  return pv_conv_pool_bwd_dw2(gpool, pooled, argmax, ids, table, dw3, dw4, db, db + pv::convbwd::FW, N, L, E, V, seed,
                              seed_ptr, row_offset, thr, token_mode, scale, stream);
}

// keys/vals: M = N * pv_conv_bwd_slots_per_sample() slots; rec: N*2*FW records {g*scale, argmax}.
PV_API int pv_conv_bwd_slots_per_sample() { return pv::convbwd::SPS; }

PV_API int pv_conv_pool_bwd_emit3(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                  unsigned* keys, unsigned* vals, void* rec, int N, int L, int V, float scale,
                                  void* stream) {
  using namespace pv::convbwd;
  const long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_bwd_emit3_kernel<unsigned>, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gpool, pooled, argmax, ids, keys, vals, (int2*)rec, N, L, V, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// Records only (the keys were written by the conv forward's epilogue, conv_pool_fwd.hip
// emit_keys): rec[pair] = {g * scale, argmax}, one coalesced pass.
__global__ __launch_bounds__(256) void conv_bwd_rec_kernel(const float* __restrict__ gpool,
                                                           const int* __restrict__ argmax, int2* __restrict__ rec,
                                                           long pairs, float scale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < pairs) rec[i] = int2{__float_as_int(gpool[i] * scale), argmax[i]};
}

PV_API int pv_conv_pool_bwd_rec(const float* gpool, const int* argmax, void* rec, int N, float scale, void* stream) {
  using namespace pv::convbwd;
  const long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_bwd_rec_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     gpool, argmax, (int2*)rec, pairs, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// 2-byte-key variants (V < 65535): emit -> pv_sort_iota_u16 -> reduce
PV_API int pv_conv_pool_bwd_emit3_u16(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                      void* keys, void* rec, int N, int L, int V, float scale, void* stream) {
  using namespace pv::convbwd;
  if (V >= 65535) return -1;
  const long pairs = (long)N * 2 * FW;
  hipLaunchKernelGGL(conv_bwd_emit3_kernel<unsigned short>, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gpool, pooled, argmax, ids, (unsigned short*)keys, (unsigned*)nullptr,
                     (int2*)rec, N, L, V, scale);
  PV_LAUNCH_CHECK();
  return 0;
}

// reduce7 occupancy (same process at the bench shape): capped at 64 VGPRs
// (8 waves / SIMD, 2 VGPRs spilled) 0.443 ms vs 0.473 ms at the compiler's 74 VGPRs (6 waves);
// PMC: 47% of wave-cycles parked at s_waitcnt, 26% L2 miss rate (the random {g, argmax}
// record gathers) — latency-bound, so more waves pay.  PAGEVEC_R7_OCC=1 restores 74 VGPRs.
static int g_r7_occ = getenv("PAGEVEC_R7_OCC") ? atoi(getenv("PAGEVEC_R7_OCC")) : 8;
PV_API void pv_conv_r7_set_occ(int occ) { g_r7_occ = occ; }

template <typename KT>
int launch_reduce7(const void* skeys, const unsigned* svals, const void* rec, const void* wrow, float* dtable, long M,
                   int epw, int L, int E, int V, unsigned seed, const unsigned* seed_ptr, unsigned row_offset,
                   int thr, int token_mode, hipStream_t st) {
  using namespace pv::convbwd;
  if (E > EP || epw < 64 || (epw & 63) || (sizeof(KT) == 2 && V >= 65535) || (long)V * E >= (1L << 32)) return -1;
  const long waves = (M + epw - 1) / epw;
  const dim3 grid((unsigned)((waves + 3) / 4));
  const DetAcc det((size_t)V * E, st);
  if (det.err) return det.err;
  const int dm = dm_of(thr, token_mode);
#define PV_R7(DMV)                                                                                               \
  if (g_r7_occ == 8)                                                                                             \
    hipLaunchKernelGGL((conv_bwd_reduce7_kernel<KT, DMV, 8>), grid, dim3(256), 0, st, (const KT*)skeys, svals,   \
                       (const int2*)rec, (const unsigned short*)wrow, dtable, M, epw, L, E, V, seed, seed_ptr,    \
                       row_offset, thr, token_mode, det.fx);                                                     \
  else                                                                                                           \
    hipLaunchKernelGGL((conv_bwd_reduce7_kernel<KT, DMV>), grid, dim3(256), 0, st, (const KT*)skeys, svals,      \
                       (const int2*)rec, (const unsigned short*)wrow, dtable, M, epw, L, E, V, seed, seed_ptr,    \
                       row_offset, thr, token_mode, det.fx)
  switch (dm) {
    case 0: PV_R7(0); break;
    case 1: PV_R7(1); break;
    case 4: PV_R7(4); break;
    case 3: PV_R7(3); break;
    default: PV_R7(2); break;
  }
#undef PV_R7
  PV_LAUNCH_CHECK();
  return det.finish(dtable, (size_t)V * E, st);
}

// skeys: sorted 2-byte (V < 65535) or 4-byte token keys (dead sentinel V), svals their slots;
// rec: {g * scale, argmax} per (n, f); wrow: bf16 [2*FW][4][EP] weight rows; epw: sorted entries
// per wave (multiple of 64)
PV_API int pv_conv_pool_bwd_reduce7_u16(const void* skeys, const unsigned* svals, const void* rec, const void* wrow,
                                        float* dtable, long M, int epw, int L, int E, int V, unsigned seed,
                                        const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                                        void* stream) {
  return launch_reduce7<unsigned short>(skeys, svals, rec, wrow, dtable, M, epw, L, E, V, seed, seed_ptr, row_offset,
                                        thr, token_mode, (hipStream_t)stream);
}

PV_API int pv_conv_pool_bwd_reduce7(const void* skeys, const unsigned* svals, const void* rec, const void* wrow,
                                    float* dtable, long M, int epw, int L, int E, int V, unsigned seed,
                                    const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode,
                                    void* stream) {
  return launch_reduce7<unsigned>(skeys, svals, rec, wrow, dtable, M, epw, L, E, V, seed, seed_ptr, row_offset, thr,
                                  token_mode, (hipStream_t)stream);
}

// Short-sequence dTable, step 1: rows (N*L, EP) fp32 (touched rows written), keys (N*L) u16
// (V < 65535) or u32 with sentinel V; wrow as for the reduce kernels; L <= pv_conv_dx_dense_maxl().
PV_API int pv_conv_dx_dense_maxl() { return pv::convbwd::DENSE_MAXL; }

PV_API int pv_conv_pool_bwd_dx_dense(const float* gpool, const float* pooled, const int* argmax, const int* ids,
                                     const void* wrow, float* rows, void* keys, int key_bytes, int N, int L, int V,
                                     unsigned seed, const unsigned* seed_ptr, unsigned row_offset, int thr,
                                     int token_mode, float scale, void* stream) {
  using namespace pv::convbwd;
  if (L > DENSE_MAXL || L < 4 || N <= 0 || (key_bytes == 2 && V >= 65535)) return -1;
  hipStream_t st = (hipStream_t)stream;
  const int dm = dm_of(thr, token_mode);
#define PV_DX_LAUNCH(KT, DMV)                                                                                   \
  hipLaunchKernelGGL((conv_bwd_dx_dense_kernel<KT, DMV>), dim3(N), dim3(DX_THREADS), 0, st, gpool, pooled, argmax, ids, \
                     (const unsigned short*)wrow, rows, (KT*)keys, L, V, seed, seed_ptr, row_offset, thr,        \
                     token_mode, scale)
  if (key_bytes == 2) {
    switch (dm) {
      case 0: PV_DX_LAUNCH(unsigned short, 0); break;
      case 1: PV_DX_LAUNCH(unsigned short, 1); break;
      case 3: PV_DX_LAUNCH(unsigned short, 3); break;
      default: PV_DX_LAUNCH(unsigned short, 2); break;
    }
  } else {
    switch (dm) {
      case 0: PV_DX_LAUNCH(unsigned, 0); break;
      case 1: PV_DX_LAUNCH(unsigned, 1); break;
      case 3: PV_DX_LAUNCH(unsigned, 3); break;
      default: PV_DX_LAUNCH(unsigned, 2); break;
    }
  }
#undef PV_DX_LAUNCH
  PV_LAUNCH_CHECK();
  return 0;
}

// Short-sequence dTable, step 3 (after sorting keys with values = row ids): dtable += rows.
PV_API int pv_conv_bwd_rows_reduce(const void* skeys, int key_bytes, const unsigned* svals, const float* rows,
                                   float* dtable, long M, int epw, int E, int V, void* stream) {
  using namespace pv::convbwd;
  if (E > EP || epw < 64 || (epw & 63)) return -1;
  const long waves = (M + epw - 1) / epw;
  hipStream_t st = (hipStream_t)stream;
  const DetAcc det((size_t)V * E, st);
  if (det.err) return det.err;
  if (key_bytes == 2)
    hipLaunchKernelGGL(conv_bwd_rows_reduce_kernel<unsigned short>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       st, (const unsigned short*)skeys, svals, rows, dtable, M, epw, E, V, det.fx);
  else
    hipLaunchKernelGGL(conv_bwd_rows_reduce_kernel<unsigned>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st,
                       (const unsigned*)skeys, svals, rows, dtable, M, epw, E, V, det.fx);
  PV_LAUNCH_CHECK();
  return det.finish(dtable, (size_t)V * E, st);
}
