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
// a row costs one finaliser (two 32-bit multiplies) — the sparse backward kernels recompute
// it for every gradient entry and are VALU-bound.
__device__ __forceinline__ unsigned dropout_row_hash(unsigned seed, unsigned row) {
  return mix32(row ^ mix32(seed));
}

// Keep-bits for columns 4g..4g+3 of a row (byte b of the group hash >= thr).
__device__ __forceinline__ unsigned dropout_group_hash(unsigned hrow, unsigned g) {
  return mix32(hrow + g * 0x9E3779B9u);
}

// Bytes in {0, 1} -> bytes in {0, 0xFF}: x * 255 as (x << 8) - x (two full-rate ops instead
// of a quarter-rate v_mul_lo_u32; the sparse-backward kernels are VALU-bound).
__device__ __forceinline__ unsigned bytes_to_mask(unsigned x) { return (x << 8) - x; }

// Byte k of the result is 0xFF iff byte k of the group hash is >= thr (element 4g+k kept).
// thr = 64 / 128 / 192 (p = 0.25 — the reference's rate — / 0.5 / 0.75) is a function of the
// top two bits of each byte: 4 bit ops instead of 4 compares + selects.
__device__ __forceinline__ unsigned keep_bytes(unsigned h, int thr) {
  unsigned b;
  if (thr == 64) {
    b = ((h | (h << 1)) >> 7) & 0x01010101u;
  } else if (thr == 128) {
    b = (h >> 7) & 0x01010101u;
  } else if (thr == 192) {
    b = ((h & (h << 1)) >> 7) & 0x01010101u;
  } else {
    b = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) b |= ((int)((h >> (8 * k)) & 0xFFu) >= thr ? 1u : 0u) << (8 * k);
  }
  return bytes_to_mask(b);
}

// AND-mask for the bf16 pair (elements 2j, 2j+1) of a packed dword, from keep_bytes (v_perm_b32).
__device__ __forceinline__ unsigned keep_pair(unsigned kb, int j) {
  return __builtin_amdgcn_perm(0u, kb, j ? 0x03030202u : 0x01010000u);
}

// Element-dropout AND-masks for the 8 bf16 columns 8q..8q+7 (one 16-byte piece) of a row
// with row hash hrow (ops/reference.py dropout_keep_mask is the specification):
//  * thr % 16 == 0 (p = k/16, incl. the reference's 0.25): ONE group hash per piece, nibble
//    k decides column 8q+k (kept iff nibble >= thr/16);
//  * otherwise two byte-wise group hashes (groups 2q, 2q+1, byte k decides column 4g+k).
__device__ __forceinline__ u32x4 keep_piece(unsigned hrow, int q, int thr) {
  if ((thr & 15) == 0) {
    const unsigned h = dropout_group_hash(hrow, (unsigned)q);
    const int t = thr >> 4;
    unsigned b;  // bit 0 of nibble k = keep column k
    if (t == 2) {  // nibble >= 2: any of bits 1..3
      b = ((h >> 1) | (h >> 2) | (h >> 3)) & 0x11111111u;
    } else if (t == 4) {
      b = ((h | (h >> 1)) >> 2) & 0x11111111u;
    } else if (t == 8) {
      b = (h >> 3) & 0x11111111u;
    } else if (t == 12) {
      b = ((h & (h >> 1)) >> 2) & 0x11111111u;
    } else {
      b = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) b |= (((h >> (4 * k)) & 0xFu) >= (unsigned)t ? 1u : 0u) << (4 * k);
    }
    const unsigned lo = bytes_to_mask(b & 0x01010101u);         // byte j: column 2j (even nibbles)
    const unsigned hi = bytes_to_mask((b >> 4) & 0x01010101u);  // byte j: column 2j+1
    return u32x4{__builtin_amdgcn_perm(hi, lo, 0x04040000u), __builtin_amdgcn_perm(hi, lo, 0x05050101u),
                 __builtin_amdgcn_perm(hi, lo, 0x06060202u), __builtin_amdgcn_perm(hi, lo, 0x07070303u)};
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
