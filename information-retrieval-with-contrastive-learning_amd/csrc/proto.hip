// ProtoNCE / HProtoNCE on the GPU.
//
//  * irc_proto_ce -- the prototype cross entropy of NCELoss._compute_proto_loss
//    (src/contrastor/contrastive_loss.py:95-135): z = logits / temp (column
//    temperatures = cluster densities), CE with target column i for row i,
//    reduction sum; per-row losses, or dL/dlogits = (softmax(z) - onehot) / temp
//    times an optional device scalar (the upstream gradient).
//  * irc_argmax_bias / irc_centroid_accumulate / irc_centroid_finalize -- Lloyd
//    k-means for run_kmeans (src/contrastor/utils.py:50-110, faiss Clustering +
//    GpuIndexFlatL2 in the reference): nearest centroid = argmax_j (x.c_j -
//    |c_j|^2 / 2) over an fp32 score tile from irc_gemm, atomically accumulated
//    sums and counts, then means (an empty cluster keeps its centroid).
#include "irc_common.h"

namespace irc {
namespace proto {

constexpr int NT = 256;

__device__ __forceinline__ float block_reduce_max(float v, float* sh) {
  v = warp_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = sh[0];
  for (int w = 1; w < NT / 64; ++w) r = fmaxf(r, sh[w]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_reduce_sum(float v, float* sh) {
  v = warp_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < NT / 64; ++w) r += sh[w];  // fixed order
  __syncthreads();
  return r;
}

// one workgroup per row
__global__ __launch_bounds__(NT) void proto_ce_kernel(const float* __restrict__ logits,
                                                      const float* __restrict__ temp, int64_t C,
                                                      float* __restrict__ row_loss,
                                                      float* __restrict__ dlogits,
                                                      const float* __restrict__ gscale) {
  __shared__ float sh[NT / 64];
  const int64_t i = blockIdx.x;
  const float* l = logits + i * C;
  float mx = -__builtin_huge_valf();
  for (int64_t j = threadIdx.x; j < C; j += NT) mx = fmaxf(mx, l[j] / temp[j]);
  mx = block_reduce_max(mx, sh);
  float se = 0.f;
  for (int64_t j = threadIdx.x; j < C; j += NT) se += expf(l[j] / temp[j] - mx);
  se = block_reduce_sum(se, sh);
  const float lse = mx + logf(se);
  if (row_loss != nullptr && threadIdx.x == 0) row_loss[i] = lse - l[i] / temp[i];
  if (dlogits != nullptr) {
    const float gs = gscale != nullptr ? gscale[0] : 1.f;
    for (int64_t j = threadIdx.x; j < C; j += NT) {
      const float p = expf(l[j] / temp[j] - lse) - (j == i ? 1.f : 0.f);
      dlogits[i * C + j] = gs * p / temp[j];
    }
  }
}

// one wave per row: max_j S[r][j] + bias[j] (lowest j on ties)
__global__ __launch_bounds__(NT) void argmax_bias_kernel(const float* __restrict__ S,
                                                         const float* __restrict__ bias,
                                                         int64_t rows, int64_t k,
                                                         int64_t* __restrict__ idx,
                                                         float* __restrict__ val) {
  const int64_t r = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* s = S + r * k;
  float best = -__builtin_huge_valf();
  int64_t bj = k;
  for (int64_t j = lane; j < k; j += 64) {
    const float v = s[j] + bias[j];
    if (v > best) {
      best = v;
      bj = j;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int64_t oj = __shfl_xor(bj, o, 64);
    if (ov > best || (ov == best && oj < bj)) {
      best = ov;
      bj = oj;
    }
  }
  if (lane == 0) {
    idx[r] = bj;
    val[r] = best;
  }
}

__global__ __launch_bounds__(NT) void centroid_accumulate_kernel(const float* __restrict__ x,
                                                                 const int64_t* __restrict__ assign,
                                                                 int64_t n, int64_t D,
                                                                 float* __restrict__ sums,
                                                                 float* __restrict__ counts) {
  const int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (t >= n * D) return;
  const int64_t r = t / D, d = t - r * D;
  const int64_t c = assign[r];
  atomicAdd(&sums[c * D + d], x[t]);
  if (d == 0) atomicAdd(&counts[c], 1.f);
}

// one workgroup per centroid: mean of its members (kept when empty) and the
// assignment bias -|c|^2 / 2
__global__ __launch_bounds__(NT) void centroid_finalize_kernel(const float* __restrict__ sums,
                                                               const float* __restrict__ counts,
                                                               int64_t D,
                                                               float* __restrict__ centroids,
                                                               float* __restrict__ bias) {
  __shared__ float sh[NT / 64];
  const int64_t c = blockIdx.x;
  const float n = counts[c];
  float ss = 0.f;
  for (int64_t d = threadIdx.x; d < D; d += NT) {
    float v = centroids[c * D + d];
    if (n > 0.f) {
      v = sums[c * D + d] / n;
      centroids[c * D + d] = v;
    }
    ss += v * v;
  }
  ss = block_reduce_sum(ss, sh);
  if (threadIdx.x == 0) bias[c] = -0.5f * ss;
}

}  // namespace proto
}  // namespace irc

using namespace irc;
using namespace irc::proto;

extern "C" int irc_proto_ce(const float* logits, const float* temp, int64_t B, int64_t C,
                            float* row_loss, float* dlogits, const float* gscale,
                            irc_stream_t stream) {
  IRC_REQUIRE(B >= 0 && C >= 1 && B <= C, "proto_ce: need 0 <= B <= C (target column = row)");
  if (B == 0) return IRC_OK;
  hipLaunchKernelGGL(proto_ce_kernel, dim3((unsigned)B), dim3(NT), 0, as_stream(stream), logits,
                     temp, C, row_loss, dlogits, gscale);
  return check_launch("proto_ce_kernel");
}

extern "C" int irc_argmax_bias(const float* S, const float* bias, int64_t rows, int64_t k,
                               int64_t* idx, float* val, irc_stream_t stream) {
  IRC_REQUIRE(rows >= 0 && k >= 1, "argmax_bias: bad sizes");
  if (rows == 0) return IRC_OK;
  hipLaunchKernelGGL(argmax_bias_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(NT), 0,
                     as_stream(stream), S, bias, rows, k, idx, val);
  return check_launch("argmax_bias_kernel");
}

extern "C" int irc_centroid_accumulate(const float* x, const int64_t* assign, int64_t n, int64_t D,
                                       float* sums, float* counts, irc_stream_t stream) {
  IRC_REQUIRE(n >= 0 && D >= 1, "centroid_accumulate: bad sizes");
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(centroid_accumulate_kernel, dim3((unsigned)((n * D + NT - 1) / NT)),
                     dim3(NT), 0, as_stream(stream), x, assign, n, D, sums, counts);
  return check_launch("centroid_accumulate_kernel");
}

extern "C" int irc_centroid_finalize(const float* sums, const float* counts, int64_t k, int64_t D,
                                     float* centroids, float* bias, irc_stream_t stream) {
  IRC_REQUIRE(k >= 1 && D >= 1, "centroid_finalize: bad sizes");
  hipLaunchKernelGGL(centroid_finalize_kernel, dim3((unsigned)k), dim3(NT), 0, as_stream(stream),
                     sums, counts, D, centroids, bias);
  return check_launch("centroid_finalize_kernel");
}
