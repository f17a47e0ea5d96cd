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
// lane l loads sample (base+l)'s g / ReLU flag / argmax and the k token ids of its argmax
// window, hashes the k dropout rows of that window itself (k full-wave lowbias32 rounds per 64
// samples) and parks {token, row hash} per window row in a wave-private LDS table; the wave then
// walks the live samples 4 per round: lane l owns the 16-byte piece l of the (k x EP) window
// (row l / 13, columns 8*(l % 13) .. +7) and reads its row's {token, hash} with ONE ds_read_b64
// per sample — one 16-byte table load, the dropout mask of the piece from keep_piece, 8 FMAs.
// (Round 5 hashed the rows inside each round — 16 active lanes, a bpermute -> lowbias32 ->
// bpermute chain in front of every mask — and moved the ids with 4 + 1 bpermutes per sample:
// dW 1.10 ms per step with dropout against 0.61 without, profiles/r6_first/.)
constexpr int PIECES_ROW = EP / 8;  // 13
template <int K, int DM>
__device__ __forceinline__ void dw_filter(const float* __restrict__ gpool, const float* __restrict__ pooled,
                                          const int* __restrict__ argmax, const int* __restrict__ ids,
                                          const unsigned short* __restrict__ table, float* __restrict__ dw,
                                          float* __restrict__ db, float* red, int2* trow, int L, int E, int V,
                                          int fg, int fl, int n0, int n1, unsigned seed, unsigned row_offset,
                                          int thr, int token_mode, float scale, long long* fxw, long long* fxb) {
  constexpr int NP = K * PIECES_ROW;  // pieces per window (39 / 52)
  constexpr bool DROP = DM != 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int2* tw = trow + wave * (64 * 4);  // this wave's {token, row hash} table: [sample lane][window row]
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float gsum = 0.f;
  const int jj = lane / PIECES_ROW, pc = lane - jj * PIECES_ROW;
  const bool pv_ = lane < NP && pc * 8 < E;
  const int jsel = jj < K ? jj : 0;
  const unsigned hseed = DROP ? mix32(seed) : 0u;  // dropout_row_hash(seed, r) = mix32(r ^ mix32(seed))
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
    const unsigned rbase = row_offset + (unsigned)n * (unsigned)L + (unsigned)a;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const unsigned hr = DROP ? mix32((rbase + (unsigned)j) ^ hseed) : 0u;
      tw[lane * 4 + j] = int2{tok[j], (int)hr};
    }
    unsigned long long m = __ballot(live);
    while (m) {
      int sl[4];
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        sl[u] = m ? (int)__builtin_ctzll(m) : -1;
        if (m) { m &= m - 1; ++cnt; }
      }
      int2 th[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) th[u] = tw[(u < cnt ? sl[u] : sl[0]) * 4 + jsel];
      u32x4 raw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= cnt) break;
        const int t = th[u].x;
        const bool ok = pv_ && t >= 0 && t < V;
        // 32-bit element offset (V * EP < 2^31): no 64-bit multiply per piece
        raw[u] = ok ? *reinterpret_cast<const u32x4*>(table + (unsigned)(t * EP + pc * 8)) : u32x4{0u, 0u, 0u, 0u};
        if constexpr (DROP) {  // dropout mask of this lane's piece (ops/reference.py dropout_keep_mask)
          const unsigned hr = (unsigned)th[u].y;
          if (DM == 3 || (DM < 0 && token_mode)) {
            const unsigned k = ((int)(hr & 0xFFu) >= thr) ? 0xFFFFFFFFu : 0u;
            raw[u] &= u32x4{k, k, k, k};
          } else if (DM > 0 || thr > 0) {
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
                                                          long long* fx) {
  __shared__ float red[4 * 4 * EP];
  __shared__ int2 trow[4 * 64 * 4];  // per wave: {token, dropout row hash} of 64 samples x 4 window rows
  if (seed_ptr) seed += *seed_ptr;  // device seed offset (captured hipGraph steps)
  // (an XCD-aware remap of (filter, split) blocks — a split's filter blocks on one XCD sharing
  // its L2 — measured neutral in round 4 and was removed in round 6)
  const int f = blockIdx.x, split = blockIdx.y;
  const int per = ((N + nsplit - 1) / nsplit + 255) / 256 * 256;
  const int n0 = split * per, n1 = min(N, n0 + per);
  if (f < FW)
    dw_filter<3, DM>(gpool, pooled, argmax, ids, table, dw3, db3, red, trow, L, E, V, f, f, n0, n1, seed, row_offset, thr,
                 token_mode, scale, fx, fx ? fx + (size_t)7 * FW * E : nullptr);
  else
    dw_filter<4, DM>(gpool, pooled, argmax, ids, table, dw4, db4, red, trow, L, E, V, f, f - FW, n0, n1, seed, row_offset, thr,
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
  hipStream_t st = (hipStream_t)stream;
  // deterministic mode: fixed-point accumulators [dW3 | dW4 | db], flushed in order below
  const size_t nfx = (size_t)7 * FW * E + 2 * FW;
  long long* fx = det_on() ? det_scratch(nfx, st) : nullptr;
  if (det_on() && !fx) return -4;
  const int dm = dm_of(thr, token_mode);
#define PV_DW(DMV)                                                                                               \
  hipLaunchKernelGGL((conv_bwd_dw_kernel<DMV>), dim3(2 * FW, nsplit), dim3(256), 0, st, gpool, pooled, argmax, ids, \
                     (const unsigned short*)table, dw3, dw4, db3, db4, N, L, E, V, nsplit, seed, seed_ptr,           \
                     row_offset, thr, token_mode, scale, fx)
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
