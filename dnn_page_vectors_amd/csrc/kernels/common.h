// Shared device helpers for the gfx950 kernels (wave64, CDNA4 MFMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PV_API extern "C" __attribute__((visibility("default")))

namespace pv {

constexpr int WAVE = 64;

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16;  // 32x32 accumulator
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

__device__ __forceinline__ float bf16_to_f32(unsigned short h) {
  return __uint_as_float(((unsigned)h) << 16);
}

// Round-to-nearest-even f32 -> bf16: gfx950's v_cvt_pk_bf16_f32 (one instruction per pair).
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;

__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){lo, hi}, bf16x2v));
}

// lowbias32 finaliser — the counter-based RNG shared with ops/reference.py.
__host__ __device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// One lowbias32 round per row: mix32(seed) is loop-invariant in every caller (hoisted), so
// a row costs one finaliser (two 32-bit multiplies).
__device__ __forceinline__ unsigned dropout_row_hash(unsigned seed, unsigned row) {
  return mix32(row ^ mix32(seed));
}

// 24-bit multiply (v_mul_u32_u24 / v_mad_u32_u24: full rate; v_mul_lo_u32 is quarter rate):
// low 32 bits of (a mod 2^24) * (b mod 2^24).
// (the masks make both operands provably 24-bit, so the backend selects the u24 forms)
__host__ __device__ __forceinline__ unsigned umul24(unsigned a, unsigned b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }

// Group hash of a dropout row (round 6): the row hash is already a full lowbias32 round, so the
// 8- or 4-column groups of the row only need to be decorrelated from each other — two
// xorshift / 24-bit-multiply rounds, six full-rate VALU ops, instead of mix32's two quarter-rate
// 32-bit multiplies (the sparse backward kernels regenerate this hash for every gathered
// 16-byte piece and were VALU-bound on it: dW 1.10 -> 0.61 ms per step with dropout off,
// profiles/r6_first/).  Quality: keep rate, all pairwise correlations of a row's 104 decisions,
// and the per-piece / per-row / adjacent-piece count distributions at the statistical floor
// (tests/test_dropout_mask.py).  ops/reference.py::dropout_keep_mask is the specification.
constexpr unsigned DROP_GROUP_STEP = 0x9E3779u;  // 24-bit golden-ratio step between groups
__host__ __device__ __forceinline__ unsigned mix24(unsigned x) {
  x ^= x >> 16;
  x = umul24(x, 0xED5AD5u);
  x ^= x >> 15;
  return umul24(x, 0x9E3779u);
}
// (the round-5 stream, mix32(hrow + g * 0x9E3779B9) with nibble j = bits 4j..4j+3, was the A arm
// of the quality A/B, profiles/r6/hash_quality_ab.txt; its build switch was removed after it)
__host__ __device__ __forceinline__ unsigned dropout_group_hash(unsigned hrow, unsigned g) {
  return mix24(hrow + umul24(g, DROP_GROUP_STEP));
}

// Nibble mode (thr % 16 == 0, p = k/16 — the reference's 0.25 is k = 4): element j (column
// 8g + j) of a group reads the 4-bit value  h[P] h[P-8] h[P-4] h[P-12]  (MSB first) with
// P = 15 - (j >> 1) + 16 (j & 1), and is kept iff that value >= thr / 16.  The bit positions are
// chosen so the fast path below needs no per-element extraction: "value >= t" for t = 2, 4, 8,
// 12 is a bitwise function of h, h << 8, h << 4 landing on bit P, and v_perm_b32's sign-
// replicating selectors (8 -> bit 15, 9 -> bit 31, 10 -> bit 47, 11 -> bit 63 of {S0, S1})
// turn bits 15 / 31 of a word into the two 16-bit halves of a bf16-pair AND mask.
__host__ __device__ __forceinline__ int dropout_nib_pos(int j) { return 15 - (j >> 1) + 16 * (j & 1); }
__host__ __device__ __forceinline__ unsigned dropout_nibble(unsigned h, int j) {
  const int P = dropout_nib_pos(j);
  return (((h >> P) & 1u) << 3) | (((h >> (P - 8)) & 1u) << 2) | (((h >> (P - 4)) & 1u) << 1) | ((h >> (P - 12)) & 1u);
}
// rotate left by r (v_alignbit_b32); at the bit positions P the result equals h << r for
// r <= 12, and a rotate keeps the backend from folding the shift into the preceding 24-bit
// multiply (h * K << 8 became one quarter-rate v_mul_lo_u32 by K << 8)
__device__ __forceinline__ unsigned rotl32(unsigned h, int r) { return __builtin_amdgcn_alignbit(h, h, 32 - r); }
// word whose bit P_j is the keep decision of element j (other bits: don't care)
__device__ __forceinline__ unsigned dropout_keep_word(unsigned h, int t) {
  if (t == 4) return h | rotl32(h, 8);                   // value >= 4: either of the two top bits
  if (t == 2) return h | rotl32(h, 8) | rotl32(h, 4);    // value >= 2: any of the three top bits
  if (t == 8) return h;                                  // value >= 8: the top bit
  if (t == 12) return h & rotl32(h, 8);                  // value >= 12: both top bits
  unsigned w = 0u;
  for (int j = 0; j < 8; ++j) w |= (dropout_nibble(h, j) >= (unsigned)t ? 1u : 0u) << dropout_nib_pos(j);
  return w;
}
// keep decisions of the group's 8 columns as bits 0..7 (bit j = column 8g + j kept)
__device__ __forceinline__ unsigned dropout_keep_bits8(unsigned h, int t) {
  const unsigned w = dropout_keep_word(h, t);
  unsigned b = 0u;
  for (int j = 0; j < 8; ++j) b |= ((w >> dropout_nib_pos(j)) & 1u) << j;
  return b;
}

// Byte mode (any other thr): byte b of the group hash decides column 4g + b (kept iff >= thr).
__device__ __forceinline__ unsigned bytes_to_mask(unsigned x) { return (x << 8) - x; }
__device__ __forceinline__ unsigned keep_bytes(unsigned h, int thr) {
  unsigned b = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) b |= ((int)((h >> (8 * k)) & 0xFFu) >= thr ? 1u : 0u) << (8 * k);
  return bytes_to_mask(b);
}

// AND-mask for the bf16 pair (elements 2j, 2j+1) of a packed dword, from keep_bytes (v_perm_b32).
__device__ __forceinline__ unsigned keep_pair(unsigned kb, int j) {
  return __builtin_amdgcn_perm(0u, kb, j ? 0x03030202u : 0x01010000u);
}

// Element-dropout AND-masks for the 8 bf16 columns 8q..8q+7 (one 16-byte piece) of a row
// with row hash hrow (ops/reference.py dropout_keep_mask is the specification):
//  * thr % 16 == 0: ONE group hash per piece; the keep word's bits 15 / 31 (shifted by the
//    pair index) become the two halves of each pair mask through v_perm_b32 — at p = 0.25
//    one v_lshl_or + three shifts + four perms after the hash;
//  * otherwise two byte-wise group hashes (groups 2q, 2q+1, byte k decides column 4g+k).
__device__ __forceinline__ u32x4 keep_piece(unsigned hrow, int q, int thr) {
  if ((thr & 15) == 0) {
    const unsigned w0 = dropout_keep_word(dropout_group_hash(hrow, (unsigned)q), thr >> 4);
    const unsigned w1 = w0 << 1, w2 = w0 << 2, w3 = w0 << 3;
    return u32x4{__builtin_amdgcn_perm(w1, w0, 0x09090808u), __builtin_amdgcn_perm(w1, w0, 0x0B0B0A0Au),
                 __builtin_amdgcn_perm(w3, w2, 0x09090808u), __builtin_amdgcn_perm(w3, w2, 0x0B0B0A0Au)};
  }
  const unsigned k0 = keep_bytes(dropout_group_hash(hrow, (unsigned)(2 * q)), thr);
  const unsigned k1 = keep_bytes(dropout_group_hash(hrow, (unsigned)(2 * q + 1)), thr);
  return u32x4{keep_pair(k0, 0), keep_pair(k0, 1), keep_pair(k1, 0), keep_pair(k1, 1)};
}

// Dropout modes of the conv kernels (template DM): 0 off, 1 element p = 64/256 (the reference's
// 0.25), 2 element any p (runtime threshold), 3 token, 4 element p = 32/256 (the chunked-CDSSM
// preset's 0.125): 1 and 4 fold the threshold into keep_piece at compile time.
__host__ __device__ constexpr int dm_thr(int dm, int thr) { return dm == 1 ? 64 : dm == 4 ? 32 : thr; }
inline int dm_of(int thr, int token_mode) {
  return thr <= 0 ? 0 : token_mode ? 3 : thr == 64 ? 1 : thr == 32 ? 4 : 2;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 T1).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int x = bid % nx, i = bid / nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace pv

// ---- debug build (python -m dnn_page_vectors_amd._build --debug -> libpagevec_hip_debug.so)
// PV_CHECK(cond, bit) records a violated precondition (out-of-range id, LDS index
// outside its tile, ...) in a per-file device flag instead of faulting; the host reads
// and clears it with pv_debug_<file>(reset) (dnn_page_vectors_amd._native.debug_status).
// The release library compiles every check away.
// PV_OK(cond, bit) is the guarding form for data-dependent addresses: in the debug build it
// records a violation AND evaluates to cond so the caller skips the access; in the release
// build it is the constant true.
enum { PV_ERR_ID = 0, PV_ERR_LDS = 1, PV_ERR_SHAPE = 2, PV_ERR_KEY = 3, PV_ERR_ARGMAX = 4, PV_ERR_SLOT = 5,
       PV_ERR_POS = 6 };
#ifdef PAGEVEC_DEBUG
#define PV_DEBUG_FLAG static __device__ unsigned pv_dbg_flag_ = 0;
#define PV_CHECK(cond, bit)                                      \
  do {                                                           \
    if (!(cond)) atomicOr(&pv_dbg_flag_, 1u << (bit));           \
  } while (0)
#define PV_OK(cond, bit) ((cond) ? true : (atomicOr(&pv_dbg_flag_, 1u << (bit)), false))
#define PV_DEBUG_EXPORT(tu)                                                   \
  PV_API unsigned pv_debug_##tu(int reset) {                                 \
    unsigned v = 0;                                                           \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(pv_dbg_flag_), 4) != hipSuccess) \
      return 0xFFFFFFFFu;                                                     \
    if (reset) {                                                              \
      unsigned z = 0;                                                         \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(pv_dbg_flag_), &z, 4);               \
    }                                                                         \
    return v;                                                                 \
  }
#else
#define PV_DEBUG_FLAG
#define PV_CHECK(cond, bit) \
  do {                      \
  } while (0)
#define PV_OK(cond, bit) true
#define PV_DEBUG_EXPORT(tu)
#endif

// ---- deterministic reduction mode (ops/determinism.py, det.hip) ---------------
// Float atomics make a cross-workgroup sum depend on arrival order.  In deterministic mode
// the kernels that combine partial sums across workgroups add int64 fixed-point values
// (resolution 2^-40, range +-2^23) instead: integer addition is associative, so the total
// is the same for every arrival order, and det_flush adds it into the float target in one
// ordered pass.  Partial sums inside a workgroup are already formed in a fixed order.
namespace pv {
constexpr float PV_FX_SCALE = 1099511627776.0f;  // 2^40
constexpr float PV_FX_BIG = 2.3058430e18f;       // 2^61 (2^21 in value units): the addend clamp
namespace {
// Per translation unit: set by fx_add when an addend is not finite or had to be clamped to
// +-2^21 in value units; det_flush then writes NaN into the whole target, so the trainer's
// non-finite guard skips the step.  The flush also NaNs any element whose int64 total reached
// +-2^62.  What stays undetected: a TOTAL that wrapped past +-2^23 in value units although
// every addend was below 2^21 — far outside any gradient this mode sums.
__device__ unsigned g_fx_flag = 0;
__host__ inline unsigned* fx_flag_ptr() {
  void* q = nullptr;
  return hipGetSymbolAddress(&q, HIP_SYMBOL(g_fx_flag)) == hipSuccess ? (unsigned*)q : nullptr;
}
}  // namespace
__device__ __forceinline__ void fx_add(long long* fx, size_t i, float v) {
  const float s = v * PV_FX_SCALE;
  if (!(fabsf(s) < PV_FX_BIG)) atomicOr(&g_fx_flag, 1u);
  const float x = fminf(fmaxf(s, -PV_FX_BIG), PV_FX_BIG);
  atomicAdd(reinterpret_cast<unsigned long long*>(fx) + i, (unsigned long long)__float2ll_rn(x));
}
bool det_on();
// n zeroed int64 accumulators (and this TU's fx_add flag cleared), stream-ordered (one
// process-wide buffer: deterministic mode runs every kernel of a step on one stream); nullptr
// on allocation failure
long long* det_scratch_flag(size_t n, hipStream_t st, unsigned* flag);
int det_flush_flag(const long long* fx, float* dst, size_t n, hipStream_t st, const unsigned* flag);
namespace {
__host__ inline long long* det_scratch(size_t n, hipStream_t st) { return det_scratch_flag(n, st, fx_flag_ptr()); }
// dst += fx * 2^-40 (NaN where the total overflowed, everywhere when this TU's flag is set)
__host__ inline int det_flush(const long long* fx, float* dst, size_t n, hipStream_t st) {
  return det_flush_flag(fx, dst, n, st, fx_flag_ptr());
}
}  // namespace
}  // namespace pv

#define PV_LAUNCH_CHECK() \
  do {                    \
    hipError_t e__ = hipGetLastError(); \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)
