// MX-fp8 (OCP e4m3 codes + one E8M0 power-of-two scale per 32 consecutive values
// of a row) helpers shared by the MX GEMM epilogue, the quantiser and the fused
// producers (LayerNorm, attention).  The scale layout in HBM is
// [K / 128][rows padded to 256][4] bytes, ordered within each 256-row block as
// mx_scale_index says (see gemm_pp.hip, MX_SC_OFF).
#pragma once
#include "irc_common.h"

namespace irc {
namespace gpp {

// Power-of-two scale exponent p of an MX block with max magnitude amax: the
// smallest p with amax / 2^p <= 448 (the e4m3 maximum), so nothing saturates;
// p = 0 for an all-zero block.  Matches oracle.quantize_mx_e4m3 bit for bit.
__device__ __forceinline__ int mx_exponent(float amax) {
  if (!(amax > 0.f)) return 0;
  // amax = m 2^E, m in [1, 2) (E = -127 for subnormals, which clamp anyway):
  // amax <= 448 2^p = 1.75 2^(p + 8)  <=>  p >= E - 8 + (m > 1.75), from the bits
  // (no division: this runs per lane in every MX epilogue)
  const uint32_t b = __float_as_uint(amax);
  const int e = (int)(b >> 23) - 135 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// max over the 4 lanes of a quad (lane ^ 1, lane ^ 2) by DPP quad permutes: no LDS
// traffic (the epilogues around this are LDS-bound already)
__device__ __forceinline__ float quad_max(float x) {
  const int xi = __float_as_int(x);
  float y = fmaxf(x, __int_as_float(__builtin_amdgcn_mov_dpp(xi, 0xB1, 0xF, 0xF, false)));  // [1,0,3,2]
  const int yi = __float_as_int(y);
  return fmaxf(y, __int_as_float(__builtin_amdgcn_mov_dpp(yi, 0x4E, 0xF, 0xF, false)));  // [2,3,0,1]
}

// Quantise 8 fp32 values of one 32-value MX block (the other 24 held by the lanes
// lane ^ 1, lane ^ 2, lane ^ 3) to e4m3 bytes; returns the block's E8M0 byte.
__device__ __forceinline__ unsigned mx_quant8(const float (&v)[8], uint2& out) {
  float am = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) am = fmaxf(am, fabsf(v[t]));
  am = quad_max(am);
  const int p = mx_exponent(am);
  const float inv = ldexpf(1.f, -p);
  uint32_t w0 = 0, w1 = 0;
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, w0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, w1, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
  out = make_uint2(w0, w1);
  return (unsigned)(p + 127);
}

// E8M0 scale byte of (row, column) in the MX layout: per 128-column K-tile kt and
// 256-row block rb one 1 KB record, [half g = row bit 7][k-block q = col bits 5-6]
// [r = row bits 0-3][i = row bits 4-6] -- so the lane of the GEMM that feeds rows
// 16 i + r (i = 0..7) of half g with k-block q reads its 8 scales as ONE 8-byte LDS
// word (byte i), and one half's 512 B arrive with one DMA wave-instruction.
__host__ __device__ __forceinline__ int64_t mx_scale_index(int64_t row, int64_t col,
                                                           int64_t mpad) {
  return (col >> 7) * mpad * 4 + (row >> 8) * 1024 + ((row >> 7) & 1) * 512 +
         ((col >> 5) & 3) * 128 + (row & 15) * 8 + ((row >> 4) & 7);
}

}  // namespace gpp
}  // namespace irc
