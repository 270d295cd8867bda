// BERT-style encoder pieces other than the GEMMs (gfx950):
//  * embed_ln: LN(word[ids] + token_type[0] + position[l]) fused (HF BertEmbeddings,
//    reached from src/contrastor/contrastive_module.py:39, eps 1e-12).
//  * layernorm: y = LN(x) * gamma + beta, one wave per row (BertSelfOutput /
//    BertOutput LayerNorm; the residual add is fused into the producing GEMM).
//  * attention: per (sequence, head) softmax(Q K^T / sqrt(dh) + key mask) V with an
//    online softmax; PAD query rows are computed and kept, as HF does.
// Element type T is bf16 (uint16 bits) or fp32; statistics are always fp32.
#include "irc_common.h"

namespace irc {
namespace enc {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2)
    return bf16_to_f32(reinterpret_cast<const unsigned short*>(p)[i]);
  else
    return reinterpret_cast<const float*>(p)[i];
}
template <typename T>
__device__ __forceinline__ void st(T* p, int64_t i, float v) {
  if constexpr (sizeof(T) == 2)
    reinterpret_cast<unsigned short*>(p)[i] = f32_to_bf16(v);
  else
    reinterpret_cast<float*>(p)[i] = v;
}

constexpr int MAXH_PER_LANE = 32;  // H <= 2048

// One wave per row; the row is held in registers (H/64 values per lane).
template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       int64_t rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[MAXH_PER_LANE];
  const int per = (H + 63) / 64;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    v[i] = c < H ? ld(x, row * H + c) : 0.f;
    s += v[i];
  }
  const float mean = warp_sum(s) / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    const float d = c < H ? v[i] - mean : 0.f;
    s2 += d * d;
  }
  const float rstd = rsqrtf(warp_sum(s2) / H + eps);
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    if (c < H) st(y, row * H + c, (v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int64_t* __restrict__ ids, const T* __restrict__ word, const T* __restrict__ pos,
    const T* __restrict__ type0, const float* __restrict__ gamma, const float* __restrict__ beta,
    T* __restrict__ y, int64_t rows, int L, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t id = ids[row];
  const int l = (int)(row % L);
  float v[MAXH_PER_LANE];
  const int per = (H + 63) / 64;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    // HF order: (word + token_type) + position
    v[i] = c < H ? (ld(word, id * H + c) + ld(type0, c)) + ld(pos, (int64_t)l * H + c) : 0.f;
    s += v[i];
  }
  const float mean = warp_sum(s) / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    const float d = c < H ? v[i] - mean : 0.f;
    s2 += d * d;
  }
  const float rstd = rsqrtf(warp_sum(s2) / H + eps);
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) {
    if (i >= per) break;
    const int c = i * 64 + lane;
    if (c < H) st(y, row * H + c, (v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
}

// Attention: one workgroup per (sequence b, head a).  qkv is the fused
// projection output [B*L, 3H] (cols [0,H)=Q, [H,2H)=K, [2H,3H)=V, head a at
// a*dh); ctx [B*L, H].  K and V of the (b, a) pair are staged in LDS as fp32;
// each thread owns one query row (q in registers) and runs an online softmax
// over the unmasked keys.  dh <= 128, L <= 512.
template <typename T, int DH>
__global__ __launch_bounds__(256) void attention_kernel(const T* __restrict__ qkv,
                                                       const int64_t* __restrict__ mask,
                                                       T* __restrict__ ctx, int L, int H,
                                                       int heads, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);          // [L][DH]
  float* Vs = Ks + (size_t)L * DH;                     // [L][DH]
  int* valid = reinterpret_cast<int*>(Vs + (size_t)L * DH);  // [L] compacted key list
  __shared__ int nvalid;
  const int b = blockIdx.x / heads, a = blockIdx.x % heads;
  const int64_t base = (int64_t)b * L;
  const int64_t ld3 = 3LL * H;
  for (int e = threadIdx.x; e < L * DH; e += blockDim.x) {
    const int j = e / DH, d = e % DH;
    Ks[e] = ld(qkv, (base + j) * ld3 + H + a * DH + d);
    Vs[e] = ld(qkv, (base + j) * ld3 + 2 * H + a * DH + d);
  }
  if (threadIdx.x == 0) {
    int n = 0;
    for (int j = 0; j < L; ++j)
      if (mask == nullptr || mask[base + j] != 0) valid[n++] = j;
    nvalid = n;
  }
  __syncthreads();
  const int nv = nvalid;
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    float qv[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) qv[d] = ld(qkv, (base + i) * ld3 + a * DH + d) * scale;
    float m = -INFINITY, l = 0.f;
    float o[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) o[d] = 0.f;
    for (int t = 0; t < nv; ++t) {
      const int j = valid[t];
      const float* kr = Ks + j * DH;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s += qv[d] * kr[d];
      const float mn = fmaxf(m, s);
      const float corr = __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * corr + p;
      const float* vr = Vs + j * DH;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = o[d] * corr + p * vr[d];
      m = mn;
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int d = 0; d < DH; ++d) st(ctx, (base + i) * H + a * DH + d, o[d] * inv);
  }
}

}  // namespace enc
}  // namespace irc

using namespace irc;

extern "C" int irc_layernorm(int dtype, const void* x, void* y, const float* gamma,
                             const float* beta, int64_t rows, int64_t H, float eps,
                             irc_stream_t stream) {
  IRC_REQUIRE(H >= 1 && H <= 64 * enc::MAXH_PER_LANE, "layernorm: H=%lld unsupported",
              (long long)H);
  if (rows == 0) return IRC_OK;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == 0)
    hipLaunchKernelGGL((enc::layernorm_kernel<unsigned short>), grid, dim3(256), 0,
                       as_stream(stream), (const unsigned short*)x, (unsigned short*)y, gamma,
                       beta, rows, (int)H, eps);
  else
    hipLaunchKernelGGL((enc::layernorm_kernel<float>), grid, dim3(256), 0, as_stream(stream),
                       (const float*)x, (float*)y, gamma, beta, rows, (int)H, eps);
  return check_launch("layernorm_kernel");
}

extern "C" int irc_embed_ln(int dtype, const int64_t* ids, const void* word, const void* pos,
                            const void* type0, const float* gamma, const float* beta, void* y,
                            int64_t rows, int64_t L, int64_t H, float eps, irc_stream_t stream) {
  IRC_REQUIRE(H >= 1 && H <= 64 * enc::MAXH_PER_LANE, "embed_ln: H=%lld unsupported",
              (long long)H);
  if (rows == 0) return IRC_OK;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == 0)
    hipLaunchKernelGGL((enc::embed_ln_kernel<unsigned short>), grid, dim3(256), 0,
                       as_stream(stream), ids, (const unsigned short*)word,
                       (const unsigned short*)pos, (const unsigned short*)type0, gamma, beta,
                       (unsigned short*)y, rows, (int)L, (int)H, eps);
  else
    hipLaunchKernelGGL((enc::embed_ln_kernel<float>), grid, dim3(256), 0, as_stream(stream), ids,
                       (const float*)word, (const float*)pos, (const float*)type0, gamma, beta,
                       (float*)y, rows, (int)L, (int)H, eps);
  return check_launch("embed_ln_kernel");
}

template <typename T, int DH>
static int attn_launch(const void* qkv, const int64_t* mask, void* ctx, int64_t B, int64_t L,
                       int64_t H, int64_t heads, hipStream_t st) {
  const size_t lds = (size_t)2 * L * DH * 4 + (size_t)L * 4;
  hipLaunchKernelGGL((enc::attention_kernel<T, DH>), dim3((unsigned)(B * heads)), dim3(256), lds,
                     st, (const T*)qkv, mask, (T*)ctx, (int)L, (int)H, (int)heads,
                     1.0f / sqrtf((float)DH));
  return check_launch("attention_kernel");
}

extern "C" int irc_attention(int dtype, const void* qkv, const int64_t* mask, void* ctx,
                             int64_t B, int64_t L, int64_t H, int64_t heads,
                             irc_stream_t stream) {
  IRC_REQUIRE(heads >= 1 && H % heads == 0, "attention: H %% heads != 0");
  const int64_t dh = H / heads;
  IRC_REQUIRE(dh == 16 || dh == 32 || dh == 64 || dh == 128, "attention: head dim %lld",
              (long long)dh);
  IRC_REQUIRE(L >= 1 && (size_t)2 * L * dh * 4 + L * 4 <= (size_t)IRC_LDS_BYTES,
              "attention: L=%lld too long for LDS staging", (long long)L);
  if (B == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
#define IRC_ATT(DH)                                                                  \
  if (dh == DH)                                                                      \
    return dtype == 0 ? attn_launch<unsigned short, DH>(qkv, mask, ctx, B, L, H, heads, st) \
                      : attn_launch<float, DH>(qkv, mask, ctx, B, L, H, heads, st);
  IRC_ATT(16)
  IRC_ATT(32)
  IRC_ATT(64)
  IRC_ATT(128)
#undef IRC_ATT
  return IRC_E_INVALID;
}
