// Shared device/host helpers for libirc_hip.so (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "irc.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// GELU(x) = x Phi(x) for epilogues whose output is rounded to bf16 (or MX-fp8):
// x * sigmoid(p(x)) with p(x) = x (c1 + c3 x^2 + c5 x^4), a weighted minimax fit to
// the exact erf GELU of HF BertIntermediate ("gelu"), tools/gelu_fit.py: |error| <=
// 6.3e-5 absolute and <= 0.15 bf16 ulp wherever |GELU(x)| >= 1e-2 (<= 2 ulp down to
// 1e-4), so the bf16 outputs are those of the exact function up to a rare 1-ulp
// rounding flip.  3 packed FMAs + 1 packed multiply + clamp + v_exp_f32 + v_rcp_f32
// per pair, against ~11 packed ops + 4 transcendental + 4 scalar for the A&S erf
// form: the FFN1 epilogue runs with the matrix pipe idle and is VALU-bound.  The
// coefficients carry -log2(e), so the sigmoid is 1 / (1 + exp2(p)).  x is clamped to
// [-9, 9] inside p only (sigmoid saturates in fp32 there; q > 0 on the whole range).
// Not used where outputs stay fp32 (parity mode, GELU-save training forward).
__device__ __forceinline__ f32x2_t gelu_lite2(f32x2_t x) {
  constexpr float C1 = -2.300117254257202f, C3 = -0.1075558140873909f,
                  C5 = 0.001120027038268745f;
  const f32x2_t xc = {__builtin_amdgcn_fmed3f(x.x, -9.0f, 9.0f),
                      __builtin_amdgcn_fmed3f(x.y, -9.0f, 9.0f)};
  const f32x2_t u = xc * xc;
  f32x2_t q = u * C5 + C3;
  q = q * u + C1;
  const f32x2_t p = q * xc;
  const f32x2_t d = {1.0f + __builtin_amdgcn_exp2f(p.x), 1.0f + __builtin_amdgcn_exp2f(p.y)};
  return x * f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ float gelu_lite(float x) {
  return gelu_lite2(f32x2_t{x, x}).x;
}

#define IRC_LDS_BYTES (160 * 1024)

namespace irc {

// ---- host-side error plumbing (irc_runtime.hip) ----
void set_error(const char* fmt, ...);
int check_launch(const char* what);

#define IRC_REQUIRE(cond, ...)          \
  do {                                  \
    if (!(cond)) {                      \
      ::irc::set_error(__VA_ARGS__);    \
      return IRC_E_INVALID;             \
    }                                   \
  } while (0)

bool prof_on();
void prof_begin(hipStream_t st);
void prof_end(const char* name, hipStream_t st, double work = 0.0);
void prof_work(const char* name, double work);

static inline hipStream_t as_stream(irc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- device helpers ----

// s_waitcnt that waits only on vmcnt <= N (gfx9 encoding: vmcnt lo [3:0], hi [15:14];
// expcnt [6:4] and lgkmcnt [11:8] left at their maxima so they do not wait).
// Counts above the 6-bit maximum clamp to 63 (waiting for MORE ops is always safe).
template <int N0>
__device__ __forceinline__ void wait_vmcnt() {
  constexpr int N = N0 > 63 ? 63 : N0;
  static_assert(N >= 0, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// vmcnt(n) for a wave-uniform run-time n (clamped to 63: waiting for more is safe).
__device__ __forceinline__ void wait_vmcnt_n(int n) {
#define IRC_VMN(E) \
  case E:          \
    wait_vmcnt<E>(); \
    return;
  switch (n < 63 ? n : 63) {
    IRC_VMN(0) IRC_VMN(1) IRC_VMN(2) IRC_VMN(3) IRC_VMN(4) IRC_VMN(5) IRC_VMN(6) IRC_VMN(7)
    IRC_VMN(8) IRC_VMN(9) IRC_VMN(10) IRC_VMN(11) IRC_VMN(12) IRC_VMN(13) IRC_VMN(14)
    IRC_VMN(15) IRC_VMN(16) IRC_VMN(17) IRC_VMN(18) IRC_VMN(19) IRC_VMN(20) IRC_VMN(21)
    IRC_VMN(22) IRC_VMN(23) IRC_VMN(24) IRC_VMN(25) IRC_VMN(26) IRC_VMN(27) IRC_VMN(28)
    IRC_VMN(29) IRC_VMN(30) IRC_VMN(31) IRC_VMN(32) IRC_VMN(33) IRC_VMN(34) IRC_VMN(35)
    IRC_VMN(36) IRC_VMN(37) IRC_VMN(38) IRC_VMN(39) IRC_VMN(40) IRC_VMN(41) IRC_VMN(42)
    IRC_VMN(43) IRC_VMN(44) IRC_VMN(45) IRC_VMN(46) IRC_VMN(47) IRC_VMN(48) IRC_VMN(49)
    IRC_VMN(50) IRC_VMN(51) IRC_VMN(52) IRC_VMN(53) IRC_VMN(54) IRC_VMN(55) IRC_VMN(56)
    IRC_VMN(57) IRC_VMN(58) IRC_VMN(59) IRC_VMN(60) IRC_VMN(61) IRC_VMN(62)
    default:
      wait_vmcnt<63>();
      return;
  }
#undef IRC_VMN
}

// vmcnt(ahead*PW + extra) with ahead in {0,1,2} and a run-time extra in [0, 32]:
// s_waitcnt takes an immediate, so dispatch over the small range (counts above
// 63 clamp, which only waits for more).
template <int PW>
__device__ __forceinline__ void wait_vmcnt_dyn(int ahead, int extra) {
  if (ahead == 0) {
    wait_vmcnt<0>();
    return;
  }
#define IRC_VM_CASE(E)                     \
  case E:                                  \
    if (ahead == 2)                        \
      wait_vmcnt<2 * PW + E>();            \
    else                                   \
      wait_vmcnt<PW + E>();                \
    return;
  switch (extra) {
    IRC_VM_CASE(0) IRC_VM_CASE(1) IRC_VM_CASE(2) IRC_VM_CASE(3) IRC_VM_CASE(4)
    IRC_VM_CASE(5) IRC_VM_CASE(6) IRC_VM_CASE(7) IRC_VM_CASE(8) IRC_VM_CASE(9)
    IRC_VM_CASE(10) IRC_VM_CASE(11) IRC_VM_CASE(12) IRC_VM_CASE(13) IRC_VM_CASE(14)
    IRC_VM_CASE(15) IRC_VM_CASE(16) IRC_VM_CASE(17) IRC_VM_CASE(18) IRC_VM_CASE(19)
    IRC_VM_CASE(20) IRC_VM_CASE(21) IRC_VM_CASE(22) IRC_VM_CASE(23) IRC_VM_CASE(24)
    IRC_VM_CASE(25) IRC_VM_CASE(26) IRC_VM_CASE(27) IRC_VM_CASE(28) IRC_VM_CASE(29)
    IRC_VM_CASE(30) IRC_VM_CASE(31) IRC_VM_CASE(32)
    default:
      if (ahead == 2) wait_vmcnt<2 * PW>(); else wait_vmcnt<PW>();  // conservative
      return;
  }
#undef IRC_VM_CASE
}

// Grouped output-tile order of the large GEMMs: runs of gm row tiles walk their
// rows fastest, so the tiles one XCD has in flight share a few column tiles of B
// (the weights, read by every row tile) that stay in its L2, instead of each row
// block cycling through all of N.  gm <= 1: row-major (tm = t / tiles_n).  All
// operands are wave-uniform (scalar arithmetic).
__device__ __forceinline__ void grouped_tile(int t, int tiles_m, int tiles_n, int gm, int& tm,
                                             int& tn) {
  if (gm <= 1) {
    tm = t / tiles_n;
    tn = t % tiles_n;
    return;
  }
  const int per = gm * tiles_n;
  const int grp = t / per;
  const int first = grp * gm;
  const int rows = tiles_m - first < gm ? tiles_m - first : gm;
  const int r = t - grp * per;
  tm = first + r % rows;
  tn = r / rows;
}

// Raw workgroup barrier that does NOT drain vmcnt (so LDS-DMA prefetches stay in
// flight across it); the empty asm statements stop the compiler moving memory
// operations across the barrier.
// RULE: s_barrier does not wait for this wave's own LDS accesses either.  A barrier
// that publishes LDS writes to other waves (or frees LDS that other waves will
// overwrite after reading it) must be lds_barrier() below, which waits lgkmcnt(0)
// first; wg_barrier() alone is only for barriers that order DMA (vmcnt, waited
// explicitly before it) or whose LDS traffic was already waited for.  A raw barrier
// at an LDS exchange returned stale partial sums on MI355X (the scan's k-slice
// butterfly, round 3).
__device__ __forceinline__ void wg_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Barrier at an LDS exchange: this wave's LDS writes have landed and its LDS reads
// have returned before any wave passes (vmcnt is left alone, so LDS-DMA stays in flight).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  The LDS destination of
// lane l is (wave-uniform lds_base) + 16*l; the global source is per lane.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Same with an explicit cache-policy immediate (aux: 0 default, 2 nt, ...).
template <int AUX>
__device__ __forceinline__ void glds16_pol(const void* gsrc, void* lds_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)gsrc,
      (__attribute__((address_space(3))) void*)lds_base, 16, 0, AUX);
}

// Order-preserving map fp32 -> uint32 (larger float -> larger uint).  -0.0 is
// folded to +0.0 and NaN to 0 (lowest), matching oracle.canon_scores.
__device__ __forceinline__ uint32_t orderable_f32(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) == 0) u = 0;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return 0u;  // NaN
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float unorderable_f32(uint32_t h) {
  uint32_t u = (h & 0x80000000u) ? (h & 0x7fffffffu) : ~h;
  return __uint_as_float(u);
}

// Distinct 64-bit ranking key: score in the high word, bitwise-NOT of the global
// doc index in the low word, so a larger key = higher score, then LOWER index.
__device__ __forceinline__ uint64_t make_key(float score, uint32_t gidx) {
  return ((uint64_t)orderable_f32(score) << 32) | (uint64_t)(uint32_t)(~gidx);
}

__device__ __forceinline__ float bf16_to_f32(unsigned short b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(unsigned short, h);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Key blocks of 32 that the attention rows of one sequence must visit: through the block
// holding its last visible key.  Every key past it is masked (-1e30) or past L (-3e30), so
// its probability is exactly 0 and its block adds exactly nothing to the row maximum, the
// sum or P.V: skipping those blocks leaves the context bit-identical.  With no visible key
// at all the row averages every key, so all nj blocks stay.  mask_row: the sequence's L
// mask words (nonzero = visible), or null (all visible).  Called by all 64 lanes of a wave;
// the result is wave-uniform.
__device__ __forceinline__ int visible_key_blocks(const int64_t* mask_row, int L, int nj,
                                                  int lane) {
#ifdef IRC_ATTN_NO_SKIP  // A/B build: every key block
  return nj;
#endif
  if (mask_row == nullptr) return nj;
  int last = -1;
  for (int j = lane; j < L; j += 64)
    if (mask_row[j] != 0) last = j;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int t = __shfl_xor(last, o, 64);
    last = t > last ? t : last;
  }
  last = __builtin_amdgcn_readfirstlane(last);
  return last < 0 ? nj : last / 32 + 1;
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace irc
