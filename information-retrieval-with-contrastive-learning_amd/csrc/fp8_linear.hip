// fp8 (OCP e4m3) linear layers for the frozen encoder (BASELINE config C5,
// "fp8 (CDNA4 MFMA) encoder weights"; reference call site: the BERT forward of
// src/contrastor/contrastive_module.py:36-41 -> HF modeling_bert nn.Linear).
//
//   y[m][n] = sa[m] * sb[n] * sum_k qa[m][k] * qb[n][k]  (+ bias / GELU / residual)
//
// qb = e4m3(W[n][:] / sb[n]) with sb[n] = amax|W[n][:]| / 448 (per output channel,
// once per weight); qa = e4m3(x[m][:] / sa[m]) with sa[m] = amax|x[m][:]| / 448
// (per token, every call: irc_quantize_rows_fp8).  The product runs on the
// ping-pong GEMM's F8 path (v_mfma_scale_f32_16x16x128_f8f6f4 with unit block
// scales: twice the bf16 MFMA rate), the scales are applied to the fp32
// accumulators in its epilogue, ahead of the bias / GELU / residual.
#include "gemm_pp.h"
#include "mx.h"

namespace irc {
namespace f8 {

// One wave per row: amax over the row, then e4m3(RNE(x * 448 / amax)), saturated;
// scale[m] = amax / 448 (1 for an all-zero row).  8 elements per lane per step.
template <typename T>
__global__ __launch_bounds__(256) void quantize_rows_kernel(const T* __restrict__ x, int64_t ldx,
                                                            int64_t M, int64_t K,
                                                            unsigned char* __restrict__ out,
                                                            int64_t ldo, float* __restrict__ scale) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  const T* xr = x + row * ldx;
  auto ld = [&](int64_t k) -> float {
    if constexpr (sizeof(T) == 2)
      return bf16_to_f32(reinterpret_cast<const unsigned short*>(xr)[k]);
    else
      return reinterpret_cast<const float*>(xr)[k];
  };
  float amax = 0.f;
  for (int64_t k = lane * 8; k < K; k += 512)
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(ld(k + j)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const float inv = amax > 0.f ? 448.f / amax : 1.f;
  if (lane == 0) scale[row] = amax > 0.f ? amax / 448.f : 1.f;
  unsigned char* orow = out + row * ldo;
  for (int64_t k = lane * 8; k < K; k += 512) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(ld(k + j) * inv, -448.f), 448.f);
    uint32_t w0 = 0, w1 = 0;
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], w1, true);
    *reinterpret_cast<uint2*>(orow + k) = make_uint2(w0, w1);
  }
}

// MX-fp8 quantiser (the encoder's weights, and any activation not produced by an
// MX epilogue): per 32 consecutive values of a row one power-of-two scale 2^p with
// p the smallest exponent for which amax / 2^p <= 448 (no saturation), values
// e4m3(RNE(x / 2^p)).  Codes [M][ldo] bytes; scales in the MX layout
// [K / 128][mpad][4] (E8M0 = p + 127).  One wave per row, 4 lanes per block.
template <typename T>
__global__ __launch_bounds__(256) void quantize_mx_kernel(const T* __restrict__ x, int64_t ldx,
                                                          int64_t M, int64_t K,
                                                          unsigned char* __restrict__ out,
                                                          int64_t ldo, unsigned char* __restrict__ sc,
                                                          int64_t mpad) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;  // wave-uniform
  const T* xr = x + row * ldx;
  for (int64_t k0 = 0; k0 < K; k0 += 512) {  // 64 lanes x 8 values
    const int64_t k = k0 + lane * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (sizeof(T) == 2)
        v[j] = k < K ? bf16_to_f32(reinterpret_cast<const unsigned short*>(xr)[k + j]) : 0.f;
      else
        v[j] = k < K ? reinterpret_cast<const float*>(xr)[k + j] : 0.f;
    }
    uint2 q;
    const unsigned e8 = gpp::mx_quant8(v, q);  // block = lanes 4b..4b+3 (K % 32 == 0)
    if (k < K) {
      *reinterpret_cast<uint2*>(out + row * ldo + k) = q;
      if ((lane & 3) == 0) sc[gpp::mx_scale_index(row, k, mpad)] = (unsigned char)e8;
    }
  }
}

}  // namespace f8
}  // namespace irc

using namespace irc;

extern "C" int irc_quantize_mx_fp8(int in_dtype, const void* x, int64_t ldx, int64_t M, int64_t K,
                                   void* out, int64_t ldo, void* scales, int64_t mpad,
                                   irc_stream_t stream) {
  IRC_REQUIRE(in_dtype == 0 || in_dtype == 1, "quantize_mx_fp8: in_dtype 0 (bf16) or 1 (fp32)");
  IRC_REQUIRE(M >= 0 && K % 128 == 0 && ldx % 8 == 0 && ldo % 16 == 0 && mpad >= M,
              "quantize_mx_fp8: K %% 128, ldx %% 8, ldo %% 16, mpad >= M (K=%lld)", (long long)K);
  IRC_REQUIRE(((uintptr_t)out & 15) == 0, "quantize_mx_fp8: output must be 16-byte aligned");
  if (M == 0) return IRC_OK;
  const dim3 grid((unsigned)((M + 3) / 4));
  hipStream_t st = as_stream(stream);
  if (in_dtype == 0)
    hipLaunchKernelGGL((f8::quantize_mx_kernel<unsigned short>), grid, dim3(256), 0, st,
                       static_cast<const unsigned short*>(x), ldx, M, K,
                       static_cast<unsigned char*>(out), ldo, static_cast<unsigned char*>(scales),
                       mpad);
  else
    hipLaunchKernelGGL((f8::quantize_mx_kernel<float>), grid, dim3(256), 0, st,
                       static_cast<const float*>(x), ldx, M, K, static_cast<unsigned char*>(out),
                       ldo, static_cast<unsigned char*>(scales), mpad);
  return check_launch("quantize_mx_fp8");
}

// MX-fp8 linear layer: C = A8 . B8^T with both operands' E8M0 block scales applied
// inside the MFMA (+ bias / GELU / residual).  out_mx: C is an MX-fp8 output (bytes,
// ldc in bytes, block scales cx in the MX layout with mpad rows), else bf16.
extern "C" int irc_gemm_mx(const void* A8, int64_t lda, const void* sa, int64_t mpad,
                           const void* B8, int64_t ldb, const void* sb, int64_t npad, int64_t M,
                           int64_t N, int64_t K, const float* bias, const void* R, int64_t ldr,
                           void* C, int64_t ldc, void* cx, int epi, irc_stream_t stream) {
  IRC_REQUIRE(epi >= 0 && epi <= 3, "gemm_mx: epilogue %d", epi);
  IRC_REQUIRE(M >= 0 && N >= 32 && K > 0 && K % 128 == 0 && N % 32 == 0,
              "gemm_mx: K %% 128 and N %% 32 required (M=%lld N=%lld K=%lld)", (long long)M,
              (long long)N, (long long)K);
  IRC_REQUIRE(mpad >= (M + 255) / 256 * 256 && npad >= (N + 255) / 256 * 256,
              "gemm_mx: scale rows must be padded to 256 (mpad=%lld npad=%lld)", (long long)mpad,
              (long long)npad);
  IRC_REQUIRE(lda % 16 == 0 && ldb % 16 == 0 && ldc % 16 == 0,
              "gemm_mx: lda / ldb / ldc must be multiples of 16");
  IRC_REQUIRE(((uintptr_t)A8 | (uintptr_t)B8 | (uintptr_t)C | (uintptr_t)sa | (uintptr_t)sb) % 16 == 0,
              "gemm_mx: operands and scales must be 16-byte aligned");
  IRC_REQUIRE(epi != 3 || (R != nullptr && ldr % 8 == 0 && (uintptr_t)R % 16 == 0 && cx == nullptr),
              "gemm_mx: residual epilogue needs an aligned R and a bf16 output");
  IRC_REQUIRE(epi == 0 || bias != nullptr, "gemm_mx: epilogue %d needs a bias", epi);
  IRC_REQUIRE(cx == nullptr || (N % 128 == 0 && (epi == 1 || epi == 2)),
              "gemm_mx: an MX output needs N %% 128 and a bias / bias+GELU epilogue");
  if (M == 0) return IRC_OK;
  gpp::PArgs a{};
  a.A = static_cast<const unsigned short*>(A8);
  a.B = static_cast<const unsigned short*>(B8);
  a.C = C;
  a.bias = bias;
  a.R = R;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)(K / 2);
  a.kchunk = (int)(K / 2);
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  a.ldr = ldr;
  a.alpha = 1.f;
  a.vec_c = 1;
  a.sax = static_cast<const unsigned char*>(sa);
  a.sbx = static_cast<const unsigned char*>(sb);
  a.mpad = (int)mpad;
  a.npad = (int)npad;
  a.cx = static_cast<unsigned char*>(cx);
  const bool on = prof_on();
  hipStream_t st = as_stream(stream);
  if (on) prof_begin(st);
  gpp::run_mx(epi, a, st);
  if (on) {
    prof_end("gemm_fp8", st, 2.0 * M * N * K);
    // algorithmic bytes: both operands' codes and E8M0 scales once, C once (bf16, or
    // MX codes + scales), the residual once
    const double mn = (double)M * N;
    prof_work("gemm_fp8_bytes", (double)(M + N) * K * (1.0 + 1.0 / 32) +
                                    (cx ? mn * (1.0 + 1.0 / 32) : 2.0 * mn) +
                                    (epi == 3 ? 2.0 * mn : 0.0));
  }
  return check_launch("gemm_mx");
}

extern "C" int irc_quantize_rows_fp8(int in_dtype, const void* x, int64_t ldx, int64_t M,
                                     int64_t K, void* out, int64_t ldo, float* scale,
                                     irc_stream_t stream) {
  IRC_REQUIRE(in_dtype == 0 || in_dtype == 1, "quantize_rows_fp8: in_dtype 0 (bf16) or 1 (fp32)");
  IRC_REQUIRE(M >= 0 && K % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0,
              "quantize_rows_fp8: K, ldx, ldo must be multiples of 8 (K=%lld)", (long long)K);
  IRC_REQUIRE(((uintptr_t)out & 7) == 0, "quantize_rows_fp8: output must be 8-byte aligned");
  if (M == 0) return IRC_OK;
  const dim3 grid((unsigned)((M + 3) / 4));
  hipStream_t st = as_stream(stream);
  if (in_dtype == 0)
    hipLaunchKernelGGL((f8::quantize_rows_kernel<unsigned short>), grid, dim3(256), 0, st,
                       static_cast<const unsigned short*>(x), ldx, M, K,
                       static_cast<unsigned char*>(out), ldo, scale);
  else
    hipLaunchKernelGGL((f8::quantize_rows_kernel<float>), grid, dim3(256), 0, st,
                       static_cast<const float*>(x), ldx, M, K, static_cast<unsigned char*>(out),
                       ldo, scale);
  return check_launch("quantize_rows_fp8");
}

// epi: 0 none, 1 bias, 2 bias + GELU, 3 bias + residual (bf16 R [M][ldr]); C bf16.
extern "C" int irc_gemm_fp8(const void* A8, int64_t lda, const float* sa, const void* B8,
                            int64_t ldb, const float* sb, int64_t M, int64_t N, int64_t K,
                            const float* bias, const void* R, int64_t ldr, void* C, int64_t ldc,
                            int epi, irc_stream_t stream) {
  IRC_REQUIRE(epi >= 0 && epi <= 3, "gemm_fp8: epilogue %d", epi);
  IRC_REQUIRE(M >= 0 && N >= 8 && K > 0 && K % 128 == 0,
              "gemm_fp8: K must be a positive multiple of 128 (M=%lld N=%lld K=%lld)",
              (long long)M, (long long)N, (long long)K);
  IRC_REQUIRE(lda % 16 == 0 && ldb % 16 == 0 && ldc % 8 == 0 && N % 8 == 0,
              "gemm_fp8: lda/ldb must be multiples of 16, ldc and N of 8");
  IRC_REQUIRE(((uintptr_t)A8 | (uintptr_t)B8 | (uintptr_t)C) % 16 == 0,
              "gemm_fp8: operands must be 16-byte aligned");
  IRC_REQUIRE(epi != 3 || (R != nullptr && ldr % 8 == 0 && (uintptr_t)R % 16 == 0),
              "gemm_fp8: residual epilogue needs an aligned R");
  IRC_REQUIRE(epi == 0 || bias != nullptr, "gemm_fp8: epilogue %d needs a bias", epi);
  IRC_REQUIRE(sa != nullptr && sb != nullptr, "gemm_fp8: scales required");
  if (M == 0) return IRC_OK;
  gpp::PArgs a{};
  a.A = static_cast<const unsigned short*>(A8);
  a.B = static_cast<const unsigned short*>(B8);
  a.C = C;
  a.bias = bias;
  a.R = R;
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)(K / 2);
  a.kchunk = (int)(K / 2);
  a.lda = lda / 2;
  a.ldb = ldb / 2;
  a.ldc = ldc;
  a.ldr = ldr;
  a.alpha = 1.f;
  a.vec_c = 1;
  a.sa = sa;
  a.sb = sb;
  const bool on = prof_on();
  hipStream_t st = as_stream(stream);
  if (on) prof_begin(st);
  gpp::run_fp8(epi, a, st);
  if (on) prof_end("gemm_fp8", st, 2.0 * M * N * K);
  return check_launch("gemm_fp8");
}
