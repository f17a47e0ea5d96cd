// K1+K2+K3: fused embedding gather -> dropout -> Conv1D(k=3,4; 150 filters each, valid)
//           -> global max-pool over time (+argmax) -> bias -> ReLU.
//
// Reference op chain: dssm_cnn_v2/cnn_dssm_th.py:86-109 (Convolution1D + MaxPooling1D
// + Flatten + concat) preceded by Embedding + Dropout(0.25) (:111-134).
//
// MI355X design (gfx950, wave64, v_mfma_f32_16x16x32_bf16):
//  * Implicit GEMM with rows = window start t, cols = filters, K = k*EP where each
//    embedding row is stored with a padded stride EP=104 (cols 100..103 are zero in
//    the bf16 table copy AND in the packed weights), so window t is the *contiguous*
//    LDS span X[t*EP, (t+k)*EP): no im2col, and the A fragment of K-step s is one
//    16-byte-aligned ds_read_b128 at byte 208*t + 64*s + 16*(lane>>4).  Both widths
//    share the A fragments of steps 0..9; k=4 adds steps 10..12.
//  * All 2 x 150 filters live in REGISTERS for the whole persistent workgroup, as 9 k3
//    tiles + 9 k4 tiles of 16 columns + ONE mixed 13-step tile (k3 filters 144..149 with
//    a zero 4th tap beside k4 filters 144..149; v4): 220 MFMAs per 16-row block (the
//    plain 2 x 160 padding needs 230).  8 waves, two per SIMD (waves w and w+4 share a
//    SIMD under the dispatcher's cyclic wave->SIMD order): per-SIMD loads {56,56,56,52}
//    MFMAs per block, split over its two waves so each wave holds <= 120 weight VGPRs —
//    no AGPR spills/copies — and one wave's max/argmax VALU epilogue overlaps its
//    partner's MFMAs.  Weights are loaded once per workgroup, not per sample.
//  * Conv activations never leave registers: each lane keeps a running max and the
//    argmax row for its 4 accumulator rows; the cross-lane reduction happens once per
//    sample.  ReLU(max + bias) == max(ReLU(conv + bias)) because ReLU is monotone.
//  * Dropout: counter-based hash of (seed, row, column) applied while staging the
//    gathered rows into LDS (mask only, exact in bf16); the 1/(1-p) scale is applied
//    to the pooled maximum (max(s*y) = s*max(y), s > 0).  The backward regenerates
//    the same mask at the argmax windows only.
//  * Production (v7, below): the workgroup is role-split — 8 MFMA waves read LDS only, 4
//    loader waves gather / mask / stage the next chunk meanwhile (token ids two chunks
//    ahead), so neither the id->row dependent loads nor the dropout hashes sit in the
//    MFMA waves' instruction stream.  v4 (every wave stages between its MFMA phases) is
//    kept as the bit-identity reference of the v7 tests.
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace pv {
namespace convpool {
PV_DEBUG_FLAG

constexpr int EP = 104;            // padded embedding stride (elements)
constexpr int ROWB = EP * 2;       // bytes per LDS row (208 = 13 * 16)
constexpr int PIECES = ROWB / 16;  // 16-byte pieces per row
constexpr int S3 = 10;             // K-steps of 32 for k=3 (K = 312 -> 320)
constexpr int S4 = 13;             // K-steps of 32 for k=4 (K = 416)
constexpr int NT = 10;             // 16-column tiles per width (150 -> 160 filters)
constexpr int FW = 150;            // real filters per width
#ifndef PV_CONV_R
#define PV_CONV_R 112                // tools/conv_variant_build.py builds other chunk sizes for A/B runs
#endif
constexpr int R = PV_CONV_R;       // window rows per chunk (7 blocks; 3 staged pieces per thread)
static_assert(R % 16 == 0, "chunk = whole 16-window blocks");
constexpr int CROWS = R + 3;       // LDS rows per chunk
constexpr int NTHREADS = 512;
// staging work per thread for a workgroup of NTH threads (v5: 256 threads, one wave per SIMD)
template <int NTH> constexpr int ppt_of() { return (CROWS * PIECES + NTH - 1) / NTH; }  // 16-byte pieces
template <int NTH> constexpr int ids_of() { return (CROWS + NTH - 1) / NTH; }           // token ids
constexpr int PPT = ppt_of<NTHREADS>();     // pieces per thread (4)
constexpr int IDS_PT = ids_of<NTHREADS>();  // ids per thread (1)

struct Params {
  const int* ids;              // (N, L)
  const unsigned short* table; // (V, EP) bf16
  const bf16x8* wpack;         // [tile][step][lane] fragments
  const float* bias;           // (2*FW)
  float* pooled;               // (N, 2*FW)
  int* argmax;                 // (N, 2*FW)
  int N, L, V;
  unsigned seed, row_offset;
  int thr;                     // dropout byte threshold (0 = off)
  int token_mode;              // 1: one keep decision per row
  float scale;                 // 1/(1-p)
  const unsigned* seed_ptr;    // optional device seed offset (added to seed; captured hipGraph steps)
  const float* bias4;          // (FW) k=4 filters' bias; bias holds the k=3 filters' (FW)
  void* keys;                  // optional dTable sort keys (conv_pool_bwd.hip slot layout), or null
  int key_bytes;               // 2 (V < 65535) or 4
};

// The dTable emit fused into the conv forward (v7 loader waves, one sample behind the MFMA
// waves): filter f of sample n (its argmax window at a, post-ReLU output y) owns slots
// n*SPS + {3f | 3*FW + 4(f-FW)} + j, j < k; each slot's key is the token at window row j, or
// the dead sentinel V when y <= 0 (zero gradient).  Same layout as conv_pool_bwd.hip's emit
// kernel, which this replaces for the page / query towers.
constexpr int SPS = 7 * FW;  // slots per sample (3 per k=3 filter, 4 per k=4 filter)
__device__ __forceinline__ void emit_keys(const Params& p, int n, int f, int a, bool live) {
  const int K = f < FW ? 3 : 4;
  const size_t s0 = (size_t)n * SPS + (f < FW ? 3 * f : 3 * FW + 4 * (f - FW));
  const int* row = p.ids + (size_t)n * p.L + a;
  int tok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) tok[j] = (j < K && live) ? row[j] : p.V;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < K) {
      const unsigned v = (unsigned)tok[j] < (unsigned)p.V ? (unsigned)tok[j] : (unsigned)p.V;
      if (p.key_bytes == 2) static_cast<unsigned short*>(p.keys)[s0 + j] = (unsigned short)v;
      else static_cast<unsigned*>(p.keys)[s0 + j] = v;
    }
  }
}

// Diagnostic ablations are COMPILE-TIME (template DBG; production instantiation DBG = 0
// carries no branches): 1 no gather, 2 max-only epilogue, 4 no dropout hash,
// 8 no A-fragment LDS reads (tools/conv_micro.py times them interleaved in one process).

// Conflict-free A-fragment reads.  ds_read_b128 is serviced in 4 lane groups
// {0-3,12-15,20-27} {4-11,16-19,28-31} {32-35,44-47,52-59} {36-43,48-51,60-63}; with the
// fixed 208-byte row stride (13 quads) lane (row i, k-chunk c) hits quad 13*w(i) + c (mod
// 16).  Mapping the MFMA A rows 4..11 to the EVEN windows and rows 0..3, 12..15 to the ODD
// windows, and letting lane group kq read k-chunk {0,2,1,3}[kq] of each 32-wide step, puts
// the 16 lanes of every group on 16 distinct quads (the natural order is 2-way on most
// groups: measured SQ_LDS_BANK_CONFLICT ~3.6 cycles per read).  The packed weights use the
// same k-chunk order; the epilogue maps accumulator row i back to window w(i).
__device__ __forceinline__ int win_of_row(int i) {
  return (i >= 4 && i < 12) ? 2 * (i - 4) : (i < 4 ? 2 * i + 1 : 2 * (i - 12) + 9);
}
__device__ __forceinline__ int chunk_of_kq(int kq) { return kq == 1 ? 2 : (kq == 2 ? 1 : kq); }

// fragment base index of tile T in wpack (tiles 0..9 k3 with S3 steps, 10..19 k4 with S4)
__device__ __forceinline__ int tile_base(int T) {
  return T < NT ? T * S3 : NT * S3 + (T - NT) * S4;  // T = 2*NT: the mixed tile (v4), after all others
}
constexpr int MIXT = 2 * NT;  // mixed tile: k3 filters 144..149 (cols 0-5) + k4 filters 144..149 (cols 6-11)
constexpr int MIXC = 6;       // k3 columns of the mixed tile

struct Cursor {
  int n, c, nchunks;
};

__device__ __forceinline__ void advance(Cursor& cu) {
  if (++cu.c >= cu.nchunks) {
    cu.c = 0;
    cu.n += gridDim.x;
  }
}

// Load the token ids of chunk (n,c) row `r` for this thread.
template <int NTH = NTHREADS>
__device__ __forceinline__ void load_ids(const Params& p, const Cursor& cu, int (&tok)[ids_of<NTH>()]) {
#pragma unroll
  for (int i = 0; i < ids_of<NTH>(); ++i) {
    int r = threadIdx.x + i * NTH;
    int t = cu.c * R + r;
    tok[i] = (cu.n < p.N && r < CROWS && t < p.L) ? p.ids[(size_t)cu.n * p.L + t] : -1;
    PV_CHECK(tok[i] < p.V && (tok[i] >= 0 || !(cu.n < p.N && r < CROWS && t < p.L)), PV_ERR_ID);
  }
}

// Issue the 16-byte table loads for this thread's pieces of chunk (n,c).
// tok_of_row(r) reads another thread's id through LDS scratch (ids_lds).
template <int DBG, int NTH = NTHREADS>
__device__ __forceinline__ void load_rows(const Params& p, const int* ids_lds, u32x4 (&v)[ppt_of<NTH>()]) {
#pragma unroll
  for (int i = 0; i < ppt_of<NTH>(); ++i) {
    int q = threadIdx.x + i * NTH;
    int r = q / PIECES, pc = q - r * PIECES;
    int tok = (q < CROWS * PIECES) ? ids_lds[r] : -1;
    if constexpr ((DBG & 128) != 0) {  // ablation: synthetic non-zero rows, no table gather
      const unsigned h = mix32((unsigned)tok * 13u + (unsigned)pc);
      const unsigned w = (h & 0x807F807Fu) | 0x3C003C00u;  // two bf16 of magnitude [2^-7, 2^-6)
      v[i] = u32x4{w, w ^ 0x80008000u, w ^ 0x00400040u, w ^ 0x80408040u};
    } else if ((DBG & 1) == 0 && tok >= 0 && tok < p.V) {
      v[i] = *reinterpret_cast<const u32x4*>(p.table + (size_t)tok * EP + pc * 8);
    } else {
      v[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

// Apply dropout to the staged pieces and write them into the LDS chunk buffer.
// hrow[r] holds the per-row hash of this chunk (computed once per row when its token id
// was loaded), so each 16-byte piece costs only its two group hashes.
// DM (dropout mode, compile time): -1 runtime (p.thr / p.token_mode), 0 off, 1 element
// dropout at thr = 64 (p = 0.25, the reference's rate: one nibble-decision group hash per
// piece), 2 element dropout at any thr, 3 token dropout.  The compile-time forms drop the
// runtime mode branches (and their code) from the staging path.
template <int DM>
__device__ __forceinline__ bool dm_on(const Params& p) {
  return DM < 0 ? p.thr > 0 : DM != 0;
}

template <int DBG, int DM = -1, int NTH = NTHREADS>
__device__ __forceinline__ void store_rows(const Params& p, char* xl, const unsigned* hrow,
                                           u32x4 (&v)[ppt_of<NTH>()]) {
#pragma unroll
  for (int i = 0; i < ppt_of<NTH>(); ++i) {
    int q = threadIdx.x + i * NTH;
    if (q < CROWS * PIECES) {
      int r = q / PIECES, pc = q - r * PIECES;
      u32x4 x = v[i];
      if ((DBG & 4) == 0 && dm_on<DM>(p)) {
        const unsigned hr = hrow[r];
        if (DM == 3 || (DM < 0 && p.token_mode)) {
          unsigned m = ((int)(hr & 0xFF) >= p.thr) ? 0xFFFFFFFFu : 0u;
          x = x & u32x4{m, m, m, m};
        } else {
          x &= keep_piece(hr, pc, dm_thr(DM, p.thr));
        }
      }
      *reinterpret_cast<u32x4*>(xl + r * ROWB + pc * 16) = x;
    }
  }
}

// per-row dropout hash of chunk (n,c) row r (0 when dropout is off)
template <int DM = -1>
__device__ __forceinline__ unsigned row_hash(const Params& p, const Cursor& cu, int r) {
  if (!dm_on<DM>(p)) return 0u;
  return dropout_row_hash(p.seed, p.row_offset + (unsigned)(cu.n * p.L + cu.c * R + r));
}

// ---- v2 schedule: double-buffered chunk tiles + tag-encoded argmax -----------------
// * Two LDS chunk buffers: a wave stores chunk i+1's staged rows into the idle buffer
//   right after ITS OWN MFMA phase on chunk i (no wait for slower waves), then ONE
//   barrier per chunk (v1: store between two barriers).
// * Running max with the argmax in the low TAGB mantissa bits: value bits & ~mask |
//   block index (uniform SGPR) -> v_and_or + v_max per accumulator (v1: v_cmp + two
//   v_cndmask), and no argmax registers.  The pooled value loses the low TAGB mantissa
//   bits (relative change < 2^-(23-TAGB)); ties within that are broken by block order.
constexpr int TAGB = 10;                      // <= 1024 blocks of 16 windows (L <= 16386)
constexpr unsigned TAGM = (1u << TAGB) - 1u;

__device__ __forceinline__ float tagged(float x, unsigned blk) {
  return __uint_as_float((__float_as_uint(x) & ~TAGM) | blk);
}

// m = max(m, tag(x)): the tag is plain C++ (v_and/v_or, whose MFMA-result read hazards the
// compiler resolves); only the max is inline asm — fmaxf in IEEE mode would canonicalise
// BOTH operands (two extra v_max x,x per accumulator), and both operands here come from
// ordinary VALU ops, so the asm needs no MFMA hazard handling.
__device__ __forceinline__ float max_tagged(float m, float x, unsigned keep, unsigned btag) {
  const float t = __uint_as_float((__float_as_uint(x) & keep) | btag);
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(m), "v"(t));
  return r;
}

template <int N3, int N4, int PF, int DBG, int OPT = 0, int DM = -1, bool MIX = false, int NTH = NTHREADS>
__device__ __forceinline__ void run_wave2(const Params& p, int t3base, int t4base, char* xl0, int* ids_lds) {
  constexpr int IDS_PT = ids_of<NTH>(), PPT = ppt_of<NTH>();
  const int lane = threadIdx.x & 63;
  constexpr int A3 = N3 > 0 ? N3 : 1, A4 = N4 > 0 ? N4 : 1;
  bf16x8 w3[A3][S3];
  bf16x8 w4[A4][S4];
#pragma unroll
  for (int i = 0; i < N3; ++i)
#pragma unroll
    for (int s = 0; s < S3; ++s) w3[i][s] = p.wpack[(tile_base(t3base + i) + s) * 64 + lane];
#pragma unroll
  for (int i = 0; i < N4; ++i)
#pragma unroll
    for (int s = 0; s < S4; ++s)
      w4[i][s] = p.wpack[(tile_base((MIX && i == N4 - 1) ? MIXT : NT + t4base + i) + s) * 64 + lane];

  const int nchunks = (p.L - 3 + 1 + R - 1) / R;
  // chunk cursors: cur (MFMA), c1 (staged in regs / stored this iteration), c2 (ids in LDS), c3 (ids in regs)
  Cursor cur{(int)blockIdx.x, 0, nchunks};
  Cursor c1 = cur;
  advance(c1);
  Cursor c2 = c1;
  advance(c2);
  Cursor c3 = c2;
  advance(c3);
  unsigned* hs = reinterpret_cast<unsigned*>(ids_lds + 2 * CROWS);  // 2 x CROWS row hashes
  int tok[IDS_PT];
  unsigned hrw[IDS_PT];
  u32x4 stage[PPT];
  // prologue: chunk 0 -> xl[0]; chunk 1 rows -> regs; chunk 2 ids + hashes -> LDS slot 0; chunk 3 ids -> regs
  load_ids<NTH>(p, cur, tok);
#pragma unroll
  for (int i = 0; i < IDS_PT; ++i) {
    const int r = threadIdx.x + i * NTH;
    if (r < CROWS) {
      ids_lds[r] = tok[i];
      hs[r] = row_hash<DM>(p, cur, r);
    }
  }
  __syncthreads();
  load_rows<DBG, NTH>(p, ids_lds, stage);
  store_rows<DBG, DM, NTH>(p, xl0, hs, stage);
  load_ids<NTH>(p, c1, tok);
#pragma unroll
  for (int i = 0; i < IDS_PT; ++i) {
    const int r = threadIdx.x + i * NTH;
    if (r < CROWS) {
      ids_lds[CROWS + r] = tok[i];
      hs[CROWS + r] = row_hash<DM>(p, c1, r);
    }
  }
  load_ids<NTH>(p, c2, tok);
#pragma unroll
  for (int i = 0; i < IDS_PT; ++i) hrw[i] = row_hash<DM>(p, c2, threadIdx.x + i * NTH);
  __syncthreads();
  load_rows<DBG, NTH>(p, ids_lds + CROWS, stage);  // rows of c1
  // slot bookkeeping: ids/hashes of chunk c live in slot (c parity); the stage regs hold c1
  int par = 0;  // parity of `cur` (xl buffer and id/hash slot of cur)
  const int nw3 = p.L - 2, nw4 = p.L - 3;
  f32x4 m3[A3], m4[A4];
  auto reset_state = [&]() {
#pragma unroll
    for (int i = 0; i < N3; ++i) m3[i] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < N4; ++i) m4[i] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  };
  reset_state();
  const int rsub = lane & 15, kq = lane >> 4;
  // valid-window limit of k4 tile i in a partial block (the mixed tile's k3 columns reach one more window)
  auto lim4 = [&](int i) { return (MIX && i == N4 - 1 && rsub < MIXC) ? nw3 : nw4; };
  unsigned keep = ~TAGM;
  if constexpr ((OPT & 4) != 0) {
    // the tag mask in a VGPR: (x & keep) | btag can then be ONE v_and_or_b32 (VGPR, VGPR, SGPR)
    // — a literal mask forces v_and + v_or (gfx9 VOP3 has no literal operand)
    asm("v_mov_b32 %0, 0xfffffc00" : "=v"(keep));
  }
  while (cur.n < p.N) {
    const char* xl = xl0 + par * (CROWS * ROWB);
    const int tc = cur.c * R;
    // A fragments are prefetched PF K-steps ahead ACROSS blocks: the last steps of block b
    // already fetch block b+1's first fragments (the block loop is not unrolled, so the
    // compiler cannot pipeline it by itself)
    const char* abase0 = xl + win_of_row(rsub) * ROWB + chunk_of_kq(kq) * 16;
    bf16x8 ab[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) ab[u] = *reinterpret_cast<const bf16x8*>(abase0 + u * 64);
    // one 16-window block: MFMAs over all K-steps, then the running max/argmax.  FULL blocks
    // (every window valid for both widths) take the unmasked epilogue.
    auto block = [&](const int blk, auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
      const int t0 = tc + blk * 16;
      const unsigned btag = (unsigned)(t0 >> 4);
      f32x4 c3[A3], c4[A4];
#pragma unroll
      for (int i = 0; i < N3; ++i) c3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < N4; ++i) c4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* abase = abase0 + blk * 16 * ROWB;
      const char* anext = blk + 1 < R / 16 ? abase + 16 * ROWB : abase;
      constexpr int NS = N4 > 0 ? S4 : S3;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        bf16x8 a = ab[0];
#pragma unroll
        for (int u = 0; u + 1 < PF; ++u) ab[u] = ab[u + 1];
        if constexpr ((DBG & 8) == 0) {
          if (s + PF < NS) ab[PF - 1] = *reinterpret_cast<const bf16x8*>(abase + (s + PF) * 64);
          else ab[PF - 1] = *reinterpret_cast<const bf16x8*>(anext + (s + PF - NS) * 64);
        }
        if (s < S3) {
#pragma unroll
          for (int i = 0; i < N3; ++i) c3[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w3[i][s], c3[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < N4; ++i) c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w4[i][s], c4[i], 0, 0, 0);
      }
      if constexpr ((DBG & 2) != 0) {
#pragma unroll
        for (int i = 0; i < N3; ++i) m3[i] += c3[i];
#pragma unroll
        for (int i = 0; i < N4; ++i) m4[i] += c4[i];
      } else if constexpr (FULL) {
#pragma unroll
        for (int i = 0; i < N3; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) m3[i][r] = max_tagged(m3[i][r], c3[i][r], keep, btag);
#pragma unroll
        for (int i = 0; i < N4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) m4[i][r] = max_tagged(m4[i][r], c4[i][r], keep, btag);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = t0 + win_of_row(4 * kq + r);
#pragma unroll
          for (int i = 0; i < N3; ++i)
            if (row < nw3) m3[i][r] = max_tagged(m3[i][r], c3[i][r], keep, btag);
#pragma unroll
          for (int i = 0; i < N4; ++i)
            if (row < lim4(i)) m4[i][r] = max_tagged(m4[i][r], c4[i][r], keep, btag);
        }
      }
    };
    // the full blocks of the chunk in one loop, the (at most 2) partial tail blocks of the
    // sample in a second one — the hot loop carries no masked-epilogue path
    const int nvalid = min(R / 16, (nw3 - tc + 15) / 16);
    const int nfull = nw4 - tc >= 16 ? min(nvalid, (nw4 - tc - 16) / 16 + 1) : 0;
    int blk = 0;
#pragma unroll 1
    for (; blk < nfull; ++blk) block(blk, std::true_type{});
#pragma unroll 1
    for (; blk < nvalid; ++blk) block(blk, std::false_type{});
    // sample epilogue: decode (value, window) per register, reduce over regs and lane groups
    if (cur.c == cur.nchunks - 1) {
      auto finish = [&](f32x4& m, int colbase, bool mixed = false) {
        float bv = -INFINITY;
        int bi = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned u = __float_as_uint(m[r]);
          const float v = m[r] == -INFINITY ? -INFINITY : __uint_as_float(u & ~TAGM);
          const int row = (int)(u & TAGM) * 16 + win_of_row(4 * kq + r);
          const bool take = v > bv || (v == bv && row < bi) || r == 0;
          bv = take ? v : bv;
          bi = take ? row : bi;
        }
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
          const float ov = __shfl_xor(bv, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          const bool take = ov > bv || (ov == bv && oi < bi);
          bv = take ? ov : bv;
          bi = take ? oi : bi;
        }
        // the mixed tile's lanes map to k3 filter 144+rsub (rsub < 6) or k4 filter 144+rsub-6 (rsub < 12)
        const int col = mixed ? (rsub < MIXC ? 144 + rsub : rsub < 2 * MIXC ? 160 + 144 + rsub - MIXC : 159)
                              : colbase + rsub;
        if (kq == 0 && (col % 160) < FW) {
          const int f = (col / 160) * FW + (col % 160);
          PV_CHECK(bi >= 0 && bi < (col < 160 ? nw3 : nw4), PV_ERR_ARGMAX);
          const float y = bv * p.scale + (f < FW ? p.bias[f] : p.bias4[f - FW]);
          p.pooled[(size_t)cur.n * (2 * FW) + f] = y > 0.f ? y : 0.f;
          p.argmax[(size_t)cur.n * (2 * FW) + f] = bi;
        }
      };
#pragma unroll
      for (int i = 0; i < N3; ++i) finish(m3[i], (t3base + i) * 16);
#pragma unroll
      for (int i = 0; i < N4; ++i) finish(m4[i], 160 + (t4base + i) * 16, MIX && i == N4 - 1);
      reset_state();
    }
    // stage chunk c1 into the idle buffer (its hashes are in slot par^1), publish c2's ids/hashes
    store_rows<DBG, DM, NTH>(p, xl0 + (par ^ 1) * (CROWS * ROWB), hs + (par ^ 1) * CROWS, stage);
#pragma unroll
    for (int i = 0; i < IDS_PT; ++i) {
      const int r = threadIdx.x + i * NTH;
      if (r < CROWS) {
        ids_lds[par * CROWS + r] = tok[i];  // c2 has the parity of cur
        hs[par * CROWS + r] = hrw[i];
      }
    }
    if constexpr ((DBG & 64) == 0) __syncthreads();
    load_rows<DBG, NTH>(p, ids_lds + par * CROWS, stage);  // rows of c2
    load_ids<NTH>(p, c3, tok);
#pragma unroll
    for (int i = 0; i < IDS_PT; ++i) hrw[i] = row_hash<DM>(p, c3, threadIdx.x + i * NTH);
    cur = c1;
    c1 = c2;
    c2 = c3;
    advance(c3);
    par ^= 1;
  }
}

// v4 = v3 with the padding columns packed: 9 k3 tiles (filters 0..143), 9 k4 tiles and ONE
// mixed 13-step tile holding k3 filters 144..149 (zero 4th tap) beside k4 filters 144..149.
// 220 MFMAs per 16-window block instead of 230, and the per-SIMD load {56,56,56,52}
// instead of {56,56,59,59}: the chunk barrier waits for the slowest SIMD.
template <int PF, int DBG, int OPT, int DM>
__global__ __launch_bounds__(NTHREADS, 2) void conv_pool_fwd4_kernel(Params p) {
  if (p.seed_ptr) p.seed += *p.seed_ptr;
  __shared__ __attribute__((aligned(16))) char smem[2 * CROWS * ROWB + 4 * CROWS * 4 + 16];
  char* xl = smem;
  int* ids_lds = reinterpret_cast<int*>(smem + 2 * CROWS * ROWB);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr ((OPT & 1) != 0) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  // SIMD s hosts waves s and s+4: {k3 0-2 | k4 0-1}, {k3 3-5 | k4 2-3}, {k3 6-8 | k4 4-5}, {k4 6-7 | k4 8 + mixed}
  if (wave < 3) {
    run_wave2<3, 0, PF, DBG, OPT, DM>(p, 3 * wave, 0, xl, ids_lds);
  } else if (wave == 7) {
    run_wave2<0, 2, PF, DBG, OPT, DM, true>(p, 0, 8, xl, ids_lds);
  } else {
    run_wave2<0, 2, PF, DBG, OPT, DM>(p, 0, wave == 3 ? 6 : 2 * (wave - 4), xl, ids_lds);
  }
}

// ---- v7: role-split workgroup --------------------------------------------------------
// 768 threads = 12 waves, three per SIMD (SIMD s hosts waves s, s+4, s+8):
//  * waves 0-7 are MFMA waves with exactly v4's register-resident tile sets and K-loop; they
//    never touch global memory inside the chunk loop (no staging registers, no vmcnt in
//    their MFMA stream);
//  * waves 8-11 (one per SIMD) are LOADER waves: while the MFMA waves compute chunk k from
//    LDS buffer k%2, they gather chunk k+1's table rows (global_load_dwordx4), apply the
//    same counter-hash dropout mask as v4, write buffer (k+1)%2, and publish chunk k+2's
//    token ids + row hashes.  Their VALU (the mask hashes) issues in the MFMA waves' shadow
//    instead of as a staging burst that every wave of v4 runs between two chunks.
// One workgroup barrier per chunk.  Outputs are bit-identical to v4 (same data, same mask,
// same per-wave MFMA order).  The MFMA waves fit the 168-VGPR budget of three waves per SIMD
// because they hold no staging state.
constexpr int NTH7 = 768;
constexpr int NLD7 = 256;                                   // loader threads (waves 8-11)
// chunk of RR windows: CR = RR + 3 LDS rows, LPPT 16-byte pieces per loader lane (6 at RR = 112)
template <int RR> constexpr int cr_of() { return RR + 3; }
template <int RR> constexpr int lppt_of() { return (cr_of<RR>() * PIECES + NLD7 - 1) / NLD7; }

template <int DM, int RR>
__device__ __forceinline__ unsigned row_hash7(const Params& p, const Cursor& cu, int r) {
  if (!dm_on<DM>(p)) return 0u;
  return dropout_row_hash(p.seed, p.row_offset + (unsigned)(cu.n * p.L + cu.c * RR + r));
}

template <int RR>
__device__ __forceinline__ int chunk_tok(const Params& p, const Cursor& cu, int r) {
  constexpr int CROWS = cr_of<RR>();
  const int t = cu.c * RR + r;
  const bool ok = cu.n < p.N && r < CROWS && t < p.L;
  const int tok = ok ? p.ids[(size_t)cu.n * p.L + t] : -1;
  PV_CHECK(!ok || (tok >= 0 && tok < p.V), PV_ERR_ID);
  return tok;
}

// loader lane lt: rows of the chunk whose ids / hashes sit in (ids_s, hs_s) -> LDS buffer xl
template <int DM, int RR>
__device__ __forceinline__ void loader7_stage(const Params& p, int lt, const int* ids_s, const unsigned* hs_s,
                                              char* xl, u32x4 (&v)[lppt_of<RR>()]) {
  constexpr int CROWS = cr_of<RR>(), LPPT = lppt_of<RR>();
#pragma unroll
  for (int i = 0; i < LPPT; ++i) {
    const int q = lt + i * NLD7;
    const int r = q / PIECES, pc = q - r * PIECES;
    const int tok = q < CROWS * PIECES ? ids_s[r] : -1;
    v[i] = (tok >= 0 && tok < p.V) ? *reinterpret_cast<const u32x4*>(p.table + (size_t)tok * EP + pc * 8)
                                   : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < LPPT; ++i) {
    const int q = lt + i * NLD7;
    if (q < CROWS * PIECES) {
      const int r = q / PIECES, pc = q - r * PIECES;
      u32x4 x = v[i];
      if (dm_on<DM>(p)) {
        const unsigned hr = hs_s[r];
        if (DM == 3 || (DM < 0 && p.token_mode)) {
          const unsigned m = ((int)(hr & 0xFF) >= p.thr) ? 0xFFFFFFFFu : 0u;
          x = x & u32x4{m, m, m, m};
        } else {
          x &= keep_piece(hr, pc, dm_thr(DM, p.thr));
        }
      }
      *reinterpret_cast<u32x4*>(xl + r * ROWB + pc * 16) = x;
    }
  }
}

// loader lane lt emits the dTable keys of filters lt and lt + 256 of sample n (whose pooled /
// argmax rows another wave of this workgroup stored before the barrier the loader passed)
__device__ __forceinline__ void loader7_emit(const Params& p, int lt, int n) {
#pragma unroll
  for (int f = lt; f < 2 * FW; f += NLD7) {
    const size_t o = (size_t)n * (2 * FW) + f;
    emit_keys(p, n, f, p.argmax[o], p.pooled[o] > 0.f);
  }
}

template <int DM, int RR, int OPT = 0>
__device__ __forceinline__ void loader7(const Params& p, char* xl0, int* ids_lds) {
  constexpr int CROWS = cr_of<RR>(), LPPT = lppt_of<RR>(), R = RR;
  static_assert(CROWS <= NLD7, "one loader lane per chunk row for the id / hash publish");
  const int lt = threadIdx.x - (NTH7 - NLD7);
  unsigned* hs = reinterpret_cast<unsigned*>(ids_lds + 2 * CROWS);  // 2 x CROWS row hashes
  const int nchunks = (p.L - 3 + 1 + R - 1) / R;
  Cursor cur{(int)blockIdx.x, 0, nchunks};
  Cursor c1 = cur;
  advance(c1);
  Cursor c2 = c1;
  advance(c2);
  // prologue: ids + row hashes of chunk 0 -> slot 0 and of chunk 1 -> slot 1 (S1), rows of
  // chunk 0 -> buffer 0 (B_0)
  if (lt < CROWS) {
    ids_lds[lt] = chunk_tok<RR>(p, cur, lt);
    hs[lt] = row_hash7<DM, RR>(p, cur, lt);
    ids_lds[CROWS + lt] = chunk_tok<RR>(p, c1, lt);
    hs[CROWS + lt] = row_hash7<DM, RR>(p, c1, lt);
  }
  __syncthreads();  // S1
  u32x4 v[LPPT];
  loader7_stage<DM, RR>(p, lt, ids_lds, hs, xl0, v);
  int par = 0;  // parity of cur: its LDS buffer and its id / hash slot
  int done_n = -1;  // a sample whose pooled / argmax the MFMA waves wrote before the last barrier
  while (cur.n < p.N) {
    if constexpr ((OPT & 512) == 0) __syncthreads();  // B_k: buffer par holds chunk k, slot par^1 chunk k+1's ids
    if (c1.n < p.N) {
      // chunk k+2's ids issued first: their latency hides behind the row gathers
      const int tk = lt < CROWS ? chunk_tok<RR>(p, c2, lt) : -1;
      loader7_stage<DM, RR>(p, lt, ids_lds + (par ^ 1) * CROWS, hs + (par ^ 1) * CROWS,
                        xl0 + (par ^ 1) * (CROWS * ROWB), v);
      if (lt < CROWS) {  // slot par: chunk k's ids were consumed in iteration k-1
        ids_lds[par * CROWS + lt] = tk;
        hs[par * CROWS + lt] = row_hash7<DM, RR>(p, c2, lt);
      }
    }
    if (p.keys && done_n >= 0) loader7_emit(p, lt, done_n);
    done_n = cur.c == cur.nchunks - 1 ? cur.n : -1;  // finished by the MFMA waves in iteration k
    cur = c1;
    c1 = c2;
    advance(c2);
    par ^= 1;
  }
  __syncthreads();  // B_end: the last sample's outputs are written
  if (p.keys && done_n >= 0) loader7_emit(p, lt, done_n);
}

// MFMA role: v4's K-loop, running max / argmax and sample epilogue, reading chunk k from
// buffer k%2 after barrier B_k (OPT: 1 = s_setprio 1 for waves 4-7; 4 = tag mask in a VGPR)
template <int N3, int N4, int PF, int OPT, bool MIX, int RR>
__device__ __forceinline__ void mfma7(const Params& p, int t3base, int t4base, const char* xl0) {
  constexpr int CROWS = cr_of<RR>(), R = RR;
  const int lane = threadIdx.x & 63;
  constexpr int A3 = N3 > 0 ? N3 : 1, A4 = N4 > 0 ? N4 : 1;
  bf16x8 w3[A3][S3];
  bf16x8 w4[A4][S4];
#pragma unroll
  for (int i = 0; i < N3; ++i)
#pragma unroll
    for (int s = 0; s < S3; ++s) w3[i][s] = p.wpack[(tile_base(t3base + i) + s) * 64 + lane];
#pragma unroll
  for (int i = 0; i < N4; ++i)
#pragma unroll
    for (int s = 0; s < S4; ++s)
      w4[i][s] = p.wpack[(tile_base((MIX && i == N4 - 1) ? MIXT : NT + t4base + i) + s) * 64 + lane];
  const int nchunks = (p.L - 3 + 1 + R - 1) / R;
  Cursor cur{(int)blockIdx.x, 0, nchunks};
  const int nw3 = p.L - 2, nw4 = p.L - 3;
  f32x4 m3[A3], m4[A4];
  auto reset_state = [&]() {
#pragma unroll
    for (int i = 0; i < N3; ++i) m3[i] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < N4; ++i) m4[i] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  };
  reset_state();
  const int rsub = lane & 15, kq = lane >> 4;
  auto lim4 = [&](int i) { return (MIX && i == N4 - 1 && rsub < MIXC) ? nw3 : nw4; };
  unsigned keep = ~TAGM;
  if constexpr ((OPT & 4) != 0) asm("v_mov_b32 %0, 0xfffffc00" : "=v"(keep));
  __syncthreads();  // S1 (the loaders publish chunk 0's and 1's ids)
  int par = 0;
  while (cur.n < p.N) {
    if constexpr ((OPT & 512) == 0) __syncthreads();  // B_k (OPT 512: timing ablation only)
    const char* xl = xl0 + par * (CROWS * ROWB);
    const int tc = cur.c * R;
    const char* abase0 = xl + win_of_row(rsub) * ROWB + chunk_of_kq(kq) * 16;
    bf16x8 ab[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) ab[u] = *reinterpret_cast<const bf16x8*>(abase0 + u * 64);
    auto block = [&](const int blk, auto full_c) {
      constexpr bool FULL = decltype(full_c)::value;
      const int t0 = tc + blk * 16;
      const unsigned btag = (unsigned)(t0 >> 4);
      f32x4 c3[A3], c4[A4];
#pragma unroll
      for (int i = 0; i < N3; ++i) c3[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < N4; ++i) c4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* abase = abase0 + blk * 16 * ROWB;
      const char* anext = blk + 1 < R / 16 ? abase + 16 * ROWB : abase;
      constexpr int NS = N4 > 0 ? S4 : S3;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        bf16x8 a = ab[0];
#pragma unroll
        for (int u = 0; u + 1 < PF; ++u) ab[u] = ab[u + 1];
        if constexpr ((OPT & 256) == 0) {  // OPT 256: no A-fragment reads (timing ablation only)
          if (s + PF < NS) ab[PF - 1] = *reinterpret_cast<const bf16x8*>(abase + (s + PF) * 64);
          else ab[PF - 1] = *reinterpret_cast<const bf16x8*>(anext + (s + PF - NS) * 64);
        }
        if (s < S3) {
#pragma unroll
          for (int i = 0; i < N3; ++i) c3[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w3[i][s], c3[i], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < N4; ++i) c4[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w4[i][s], c4[i], 0, 0, 0);
        // OPT 1024: pin the step order (prefetch read, then this step's MFMAs) — left alone,
        // hipcc pairs two steps' reads and waits for the first right away (PF 1 becomes PF 0
        // on every other step)
        if constexpr ((OPT & 1024) != 0) __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr ((OPT & 128) != 0) {  // OPT 128: sum instead of max/argmax (timing ablation only)
#pragma unroll
        for (int i = 0; i < N3; ++i) m3[i] += c3[i];
#pragma unroll
        for (int i = 0; i < N4; ++i) m4[i] += c4[i];
      } else if constexpr (FULL) {
#pragma unroll
        for (int i = 0; i < N3; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) m3[i][r] = max_tagged(m3[i][r], c3[i][r], keep, btag);
#pragma unroll
        for (int i = 0; i < N4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) m4[i][r] = max_tagged(m4[i][r], c4[i][r], keep, btag);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = t0 + win_of_row(4 * kq + r);
#pragma unroll
          for (int i = 0; i < N3; ++i)
            if (row < nw3) m3[i][r] = max_tagged(m3[i][r], c3[i][r], keep, btag);
#pragma unroll
          for (int i = 0; i < N4; ++i)
            if (row < lim4(i)) m4[i][r] = max_tagged(m4[i][r], c4[i][r], keep, btag);
        }
      }
    };
    const int nvalid = min(R / 16, (nw3 - tc + 15) / 16);
    const int nfull = nw4 - tc >= 16 ? min(nvalid, (nw4 - tc - 16) / 16 + 1) : 0;
    int blk = 0;
#pragma unroll 1
    for (; blk < nfull; ++blk) block(blk, std::true_type{});
#pragma unroll 1
    for (; blk < nvalid; ++blk) block(blk, std::false_type{});
    if (cur.c == cur.nchunks - 1) {
      auto finish = [&](f32x4& m, int colbase, bool mixed = false) {
        float bv = -INFINITY;
        int bi = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned u = __float_as_uint(m[r]);
          const float v = m[r] == -INFINITY ? -INFINITY : __uint_as_float(u & ~TAGM);
          const int row = (int)(u & TAGM) * 16 + win_of_row(4 * kq + r);
          const bool take = v > bv || (v == bv && row < bi) || r == 0;
          bv = take ? v : bv;
          bi = take ? row : bi;
        }
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
          const float ov = __shfl_xor(bv, o, 64);
          const int oi = __shfl_xor(bi, o, 64);
          const bool take = ov > bv || (ov == bv && oi < bi);
          bv = take ? ov : bv;
          bi = take ? oi : bi;
        }
        const int col = mixed ? (rsub < MIXC ? 144 + rsub : rsub < 2 * MIXC ? 160 + 144 + rsub - MIXC : 159)
                              : colbase + rsub;
        if (kq == 0 && (col % 160) < FW) {
          const int f = (col / 160) * FW + (col % 160);
          PV_CHECK(bi >= 0 && bi < (col < 160 ? nw3 : nw4), PV_ERR_ARGMAX);
          const float y = bv * p.scale + (f < FW ? p.bias[f] : p.bias4[f - FW]);
          p.pooled[(size_t)cur.n * (2 * FW) + f] = y > 0.f ? y : 0.f;
          p.argmax[(size_t)cur.n * (2 * FW) + f] = bi;
        }
      };
#pragma unroll
      for (int i = 0; i < N3; ++i) finish(m3[i], (t3base + i) * 16);
#pragma unroll
      for (int i = 0; i < N4; ++i) finish(m4[i], 160 + (t4base + i) * 16, MIX && i == N4 - 1);
      reset_state();
    }
    advance(cur);
    par ^= 1;
  }
  __syncthreads();  // B_end (the loaders emit the last sample's keys after it)
}

// OPT: 1 = s_setprio 1 for MFMA waves 4-7, 4 = tag mask in a VGPR
template <int PF, int OPT, int RR, int DM>
__global__ __launch_bounds__(NTH7, 1) void conv_pool_fwd7_kernel(Params p) {
  constexpr int CROWS = cr_of<RR>();
  if (p.seed_ptr) p.seed += *p.seed_ptr;
  __shared__ __attribute__((aligned(16))) char smem[2 * CROWS * ROWB + 4 * CROWS * 4 + 16];
  char* xl = smem;
  int* ids_lds = reinterpret_cast<int*>(smem + 2 * CROWS * ROWB);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave >= 8) {
    loader7<DM, RR, OPT>(p, xl, ids_lds);
    return;
  }
  if constexpr ((OPT & 1) != 0) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  // SIMD s hosts waves s and s+4 (and loader s+8): v4's tile sets
  if (wave < 3) {
    mfma7<3, 0, PF, OPT, false, RR>(p, 3 * wave, 0, xl);
  } else if (wave == 7) {
    mfma7<0, 2, PF, OPT, true, RR>(p, 0, 8, xl);
  } else {
    mfma7<0, 2, PF, OPT, false, RR>(p, 0, wave == 3 ? 6 : 2 * (wave - 4), xl);
  }
}

// (v5, measured and removed: v4's tile sets with ONE wave per SIMD in a 256-thread
// workgroup — A fragments read once per SIMD instead of twice — ran 7.23-7.31 ms against
// v4's 5.53 ms at the bench shape, bit-identical outputs: without a partner wave nothing
// covers the LDS / staging latencies between the MFMA bursts; docs/PERF.md round 3.)

PV_DEBUG_EXPORT(convfwd)
}  // namespace convpool
}  // namespace pv

using namespace pv;

// Pack conv weights (fp32, [F][k][E] per width) into MFMA B fragments (bf16).
// w3: (150,3,E) ; w4: (150,4,E). out: 20 tiles' fragments (NT*S3 + NT*S4) * 64 lanes * 8.
__device__ __forceinline__ bf16x8 pack_fragment(const float* w3, const float* w4, int E, int frag, int lane) {
  using namespace pv::convpool;
  int T, s;
  if (frag < NT * S3) { T = frag / S3; s = frag % S3; }
  else { T = NT + (frag - NT * S3) / S4; s = (frag - NT * S3) % S4; }
  int k = (T < NT) ? 3 : 4;
  const float* w = (T < NT) ? w3 : w4;
  int col = (T % NT) * 16 + (lane & 15);
  if (T == MIXT) {  // mixed tile (v4): k3 filters 144..149, then k4 filters 144..149, then zeros
    const int c = lane & 15;
    k = c < MIXC ? 3 : 4;
    w = c < MIXC ? w3 : w4;
    col = c < MIXC ? 144 + c : c < 2 * MIXC ? 144 + c - MIXC : FW;
  }
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int kk = s * 32 + chunk_of_kq(lane >> 4) * 8 + j;  // window element (k-chunk order of the A reads)
    int jj = kk / EP, e = kk % EP;
    float x = 0.f;
    if (col < FW && jj < k && e < E) x = w[((size_t)col * k + jj) * E + e];
    v[j] = (short)f32_to_bf16(x);
  }
  return v;
}

__global__ void pack_conv_weights_kernel(const float* w3, const float* w4, int E, bf16x8* out) {
  out[(size_t)blockIdx.x * 64 + threadIdx.x] = pack_fragment(w3, w4, E, blockIdx.x, threadIdx.x);
}

PV_API int pv_conv_pack_weights(const float* w3, const float* w4, int E, void* out, void* stream) {
  using namespace pv::convpool;
  if (E > EP) return -1;
  int nfrag = NT * S3 + NT * S4 + S4;  // + the mixed tile of v4
  hipLaunchKernelGGL(pack_conv_weights_kernel, dim3(nfrag), dim3(64), 0, (hipStream_t)stream, w3, w4, E,
                     (bf16x8*)out);
  PV_LAUNCH_CHECK();
  return 0;
}

// The per-step bf16 operands of up to 4 conv towers in ONE launch (round 6): each tower's table
// cast to the padded (V, EP) bf16 layout and its filters packed into MFMA fragments — what
// pv_cast_pad_bf16 + pv_conv_pack_weights did in two launches per tower at the start of every
// forward.  Blocks [0, cast_blocks) of a tower cast its table (grid-stride), the next
// pack_blocks blocks pack 4 fragments each (64 lanes per fragment).
struct PrepTower {
  const float* table;      // (V, E) fp32
  unsigned short* tbl16;   // (V, EP) bf16
  const float* w3;         // (FW, 3, E)
  const float* w4;         // (FW, 4, E)
  bf16x8* pack;            // pv_conv_packed_size() bf16
  int V;
};
struct PrepArgs {
  PrepTower t[4];
  int n, E, cast_blocks;
};

__global__ __launch_bounds__(256) void conv_prep_multi_kernel(PrepArgs a) {
  using namespace pv::convpool;
  constexpr int NFRAG = NT * S3 + NT * S4 + S4;
  constexpr int PACK_BLOCKS = (NFRAG + 3) / 4;
  const int per = a.cast_blocks + PACK_BLOCKS;
  const int ti = blockIdx.x / per, b = blockIdx.x - ti * per;
  if (ti >= a.n) return;
  const PrepTower& t = a.t[ti];
  if (b < a.cast_blocks) {
    const long total = (long)t.V * EP;
    for (long i = (long)b * 256 + threadIdx.x; i < total; i += (long)a.cast_blocks * 256) {
      const long r = i / EP;
      const int c = (int)(i - r * EP);
      t.tbl16[i] = c < a.E ? f32_to_bf16(t.table[r * a.E + c]) : (unsigned short)0;
    }
    return;
  }
  const int frag = (b - a.cast_blocks) * 4 + (threadIdx.x >> 6);
  if (frag < NFRAG) t.pack[(size_t)frag * 64 + (threadIdx.x & 63)] = pack_fragment(t.w3, t.w4, a.E, frag, threadIdx.x & 63);
}

// tables / tbl16 / w3 / w4 / packs: arrays of n (<= 4) device pointers; Vs: n vocabulary sizes
PV_API int pv_conv_prep_multi(int n, const void* const* tables, void* const* tbl16, const void* const* w3s,
                              const void* const* w4s, void* const* packs, const int* Vs, int E, void* stream) {
  using namespace pv::convpool;
  if (n < 1 || n > 4 || E > EP) return -1;
  PrepArgs a{};
  a.n = n;
  a.E = E;
  long vmax = 0;
  for (int i = 0; i < n; ++i) {
    a.t[i] = PrepTower{(const float*)tables[i], (unsigned short*)tbl16[i], (const float*)w3s[i], (const float*)w4s[i],
                       (bf16x8*)packs[i], Vs[i]};
    vmax = Vs[i] > vmax ? Vs[i] : vmax;
  }
  long cb = (vmax * EP / 4 + 255) / 256;  // ~4 elements per thread
  a.cast_blocks = (int)(cb < 1 ? 1 : cb > 4096 ? 4096 : cb);
  constexpr int NFRAG = NT * S3 + NT * S4 + S4;
  const int per = a.cast_blocks + (NFRAG + 3) / 4;
  hipLaunchKernelGGL(conv_prep_multi_kernel, dim3(n * per), dim3(256), 0, (hipStream_t)stream, a);
  PV_LAUNCH_CHECK();
  return 0;
}

// Backward weight rows: bf16 [2*FW][4][EP] (k=3 filters' 4th row and columns >= E zero), the
// operand of the sparse dTable kernels (conv_pool_bwd.hip) -- one launch instead of a
// zero fill + two strided copies.
__global__ void conv_weight_rows_kernel(const float* __restrict__ w3, const float* __restrict__ w4, int E,
                                        unsigned short* __restrict__ out) {
  using namespace pv::convpool;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // element of [2*FW][4][EP]
  if (i >= 2 * FW * 4 * EP) return;
  const int e = i % EP, j = (i / EP) % 4, f = i / (4 * EP);
  float x = 0.f;
  if (e < E) {
    if (f < FW) x = j < 3 ? w3[((size_t)f * 3 + j) * E + e] : 0.f;
    else x = w4[((size_t)(f - FW) * 4 + j) * E + e];
  }
  out[i] = f32_to_bf16(x);
}

PV_API int pv_conv_weight_rows(const float* w3, const float* w4, int E, void* out, void* stream) {
  using namespace pv::convpool;
  if (E > EP) return -1;
  const int n = 2 * FW * 4 * EP;
  hipLaunchKernelGGL(conv_weight_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w3, w4, E,
                     (unsigned short*)out);
  PV_LAUNCH_CHECK();
  return 0;
}

PV_API int pv_conv_packed_size() {
  using namespace pv::convpool;
  return (NT * S3 + NT * S4 + S4) * 64 * 8;  // bf16 elements
}

// Diagnostic ablation switch (tools/conv_micro.py): 0 in production.
static int g_conv_dbg = getenv("PAGEVEC_CONV_DBG") ? atoi(getenv("PAGEVEC_CONV_DBG")) : 0;
PV_API void pv_conv_set_dbg(int d) { g_conv_dbg = d; }
PV_API int pv_conv_get_dbg() { return g_conv_dbg; }
// Short sequences (the query tower, L = 45): one chunk of 48 window rows (3 blocks of 16)
// instead of 112 — a 45-token query filled 43 of 112 rows (62 % of the MFMA blocks padding).
// Same per-window arithmetic and block order: bit-identical (test_conv_short_chunk_bit_identical).
static int g_conv_short = getenv("PAGEVEC_CONV_SHORT") ? atoi(getenv("PAGEVEC_CONV_SHORT")) : 1;
PV_API void pv_conv_set_short(int on) { g_conv_short = on; }
constexpr int SHORT_RR = 48;

// bias3 / bias4: the two widths' biases (FW floats each, e.g. the parameters themselves)
PV_API int pv_conv_pool_fwd2(const int* ids, const void* table, const void* wpack, const float* bias3,
                             const float* bias4, float* pooled, int* argmax, int N, int L, int V, unsigned seed,
                             const unsigned* seed_ptr, unsigned row_offset, int thr, int token_mode, float scale,
                             int grid, void* stream, void* keys, int key_bytes) {
  using namespace pv::convpool;
  if (L < 4 || N <= 0) return -1;
  const int dbg = g_conv_dbg;
  if (keys && key_bytes != 2 && key_bytes != 4) return -4;
  if (keys && dbg != 0 && dbg < 16384) return -6;  // the key emit lives in the v7 loader waves
  if (keys && key_bytes == 2 && V >= 65535) return -5;
  if ((L - 2 + 15) / 16 > 1024) return -2;  // tagged argmax: block index must fit TAGB bits
  Params p{ids, (const unsigned short*)table, (const bf16x8*)wpack, bias3, pooled, argmax, N, L, V,
           seed, row_offset, thr, token_mode, scale, seed_ptr, bias4, keys, key_bytes};
  if (grid <= 0) grid = 256;
  if (grid > N) grid = N;
  hipStream_t st = (hipStream_t)stream;
  const int dm = dm_of(thr, token_mode);
#define PV_CONV_DM(KERNEL, NT_, ...)                                                             \
  switch (dm) {                                                                                  \
    case 0: hipLaunchKernelGGL((KERNEL<__VA_ARGS__, 0>), dim3(grid), dim3(NT_), 0, st, p); break; \
    case 1: hipLaunchKernelGGL((KERNEL<__VA_ARGS__, 1>), dim3(grid), dim3(NT_), 0, st, p); break; \
    case 2: hipLaunchKernelGGL((KERNEL<__VA_ARGS__, 2>), dim3(grid), dim3(NT_), 0, st, p); break; \
    case 4: hipLaunchKernelGGL((KERNEL<__VA_ARGS__, 4>), dim3(grid), dim3(NT_), 0, st, p); break; \
    default: hipLaunchKernelGGL((KERNEL<__VA_ARGS__, 3>), dim3(grid), dim3(NT_), 0, st, p); break; \
  }
  switch (dbg) {
    case 4096: {  // v4 (padding columns packed into one mixed tile, 220 MFMAs per block; same-process A/B
                  // vs v3 at the bench shape: 5.528 vs 5.691 ms, bit-identical)
      PV_CONV_DM(conv_pool_fwd4_kernel, NTHREADS, 2, 0, 13)
      break;
    }
    // v4 diagnostic ablations (DBG bits: 2 max-only epilogue, 4 no dropout hash) and schedule A/B arms
    case 4096 + 512 + 4: hipLaunchKernelGGL((conv_pool_fwd4_kernel<2, 4, 13, 1>), dim3(grid), dim3(NTHREADS), 0, st, p); break;
    case 4096 + 512 + 2: hipLaunchKernelGGL((conv_pool_fwd4_kernel<2, 2, 13, 1>), dim3(grid), dim3(NTHREADS), 0, st, p); break;
    case 4096 + 512 + 8: hipLaunchKernelGGL((conv_pool_fwd4_kernel<2, 8, 13, 1>), dim3(grid), dim3(NTHREADS), 0, st, p); break;
    case 4096 + 512 + 128: hipLaunchKernelGGL((conv_pool_fwd4_kernel<2, 128, 13, 1>), dim3(grid), dim3(NTHREADS), 0, st, p); break;
    // v7: role-split workgroup (8 MFMA waves + 4 loader waves), 16384 + 64 * PF + OPT
    case 0:  // production: v7, A prefetch depth 1, pinned K-step order (same process at the bench shape:
             // 4.858 vs 5.025 ms unpinned; v4 5.349 vs unpinned v7 4.838 on another box)
      if (g_conv_short && L - 2 <= SHORT_RR) {  // every window of both widths in one 48-row chunk
        PV_CONV_DM(conv_pool_fwd7_kernel, NTH7, 1, 5 + 1024, SHORT_RR)
        break;
      }
      [[fallthrough]];
    case 16384 + 64 + 5 + 1024: PV_CONV_DM(conv_pool_fwd7_kernel, NTH7, 1, 5 + 1024, 112) break;
    case 16384 + 64 + 5: hipLaunchKernelGGL((conv_pool_fwd7_kernel<1, 5, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    case 16384 + 128 + 5: hipLaunchKernelGGL((conv_pool_fwd7_kernel<2, 5, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    // pinned step order (OPT 1024) at A prefetch depth 2 / 3
    case 16384 + 128 + 5 + 1024: hipLaunchKernelGGL((conv_pool_fwd7_kernel<2, 5 + 1024, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    case 16384 + 192 + 5 + 1024: hipLaunchKernelGGL((conv_pool_fwd7_kernel<3, 5 + 1024, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    // timing ablations of v7 (wrong outputs): +128 max-only epilogue, +256 no A reads, +512 no chunk barriers
    case 16384 + 64 + 5 + 128: hipLaunchKernelGGL((conv_pool_fwd7_kernel<1, 5 + 128, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    case 16384 + 64 + 5 + 256: hipLaunchKernelGGL((conv_pool_fwd7_kernel<1, 5 + 256, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    case 16384 + 64 + 5 + 512: hipLaunchKernelGGL((conv_pool_fwd7_kernel<1, 5 + 512, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    case 16384 + 64 + 5 + 896: hipLaunchKernelGGL((conv_pool_fwd7_kernel<1, 5 + 896, 112, 1>), dim3(grid), dim3(NTH7), 0, st, p); break;
    default: return -3;
  }
#undef PV_CONV_DM
  PV_LAUNCH_CHECK();
  return 0;
}

// bias: both widths' biases as one (2 * FW) array
PV_API int pv_conv_pool_fwd(const int* ids, const void* table, const void* wpack, const float* bias,
                            float* pooled, int* argmax, int N, int L, int V, unsigned seed, const unsigned* seed_ptr,
                            unsigned row_offset, int thr, int token_mode, float scale, int grid, void* stream) {
  return pv_conv_pool_fwd2(ids, table, wpack, bias, bias + pv::convpool::FW, pooled, argmax, N, L, V, seed, seed_ptr,
                           row_offset, thr, token_mode, scale, grid, stream, nullptr, 0);
}
