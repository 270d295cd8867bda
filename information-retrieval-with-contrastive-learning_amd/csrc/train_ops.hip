// Training-step kernels other than GEMM / encoder / LSTM (gfx950):
//  * seq2vec tail (src/contrastor/contrastive_module.py:102-112): mean over ALL L
//    positions (PAD included) and F.normalize (L2, eps 1e-12), forward + backward.
//  * InfoNCE row pass (src/contrastor/contrastive_loss.py:56-93): per row of the
//    [2N, 2N] in-batch logits (+ the q.queue logits, REUSED for rows N..2N-1 as
//    the reference's .repeat(2, 1) does) the log-sum-exp and NLL of the positive
//    column (i+N) mod 2N, then the softmax gradients G = 1/2 (P - onehot) / T.
//    The two logit GEMMs and the dq GEMMs run on gemm.hip in fp32-MFMA mode.
//  * deterministic reductions (fixed assignment + fixed-order final sum).
//  * clip_grad_norm_(1.0) + torch.optim.Adam step fused over the flat fp32
//    parameter buffer (src/train.py:155-165, src/model.py:52-57), momentum update
//    theta_k = m theta_k + (1-m) theta_q (contrastive_module.py:43-53) and the
//    queue enqueue with its device-side pointer (contrastive_module.py:55-68).
#include "irc_common.h"

namespace irc {
namespace tops {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2)
    return bf16_to_f32(reinterpret_cast<const unsigned short*>(p)[i]);
  else
    return reinterpret_cast<const float*>(p)[i];
}

// out[b, c] = mean_l x[b, l, c]  (fp32 accumulate in l order)
template <typename T>
__global__ void mean_rows_kernel(const T* __restrict__ x, float* __restrict__ out, int B, int L,
                                 int C, int64_t ldx) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * C) return;
  const int b = (int)(e / C), c = (int)(e % C);
  float s = 0.f;
  for (int l = 0; l < L; ++l) s += ldf(x, ((int64_t)b * L + l) * ldx + c);
  out[e] = s / (float)L;
}

// y[b, l, c] = g[b, c] * scale  (broadcast of d(mean) over positions)
__global__ void bcast_rows_kernel(const float* __restrict__ g, float* __restrict__ y, int B, int L,
                                  int C, float scale) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * L * C) return;
  const int c = (int)(e % C);
  const int b = (int)(e / ((int64_t)L * C));
  y[e] = g[(int64_t)b * C + c] * scale;
}

// one wave per row: y = x / max(||x||, eps); nrm[b] = ||x||
__global__ void l2norm_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                  float* __restrict__ nrm, int B, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float v = x[(int64_t)b * D + c];
    s += v * v;
  }
  const float n = sqrtf(warp_sum(s));
  const float inv = 1.f / fmaxf(n, eps);
  for (int c = lane; c < D; c += 64) y[(int64_t)b * D + c] = x[(int64_t)b * D + c] * inv;
  if (lane == 0 && nrm) nrm[b] = n;
}

// dx = (dy - e (dy . e)) / n  for n > eps (e = y), else dy / eps
__global__ void l2norm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                  const float* __restrict__ nrm, float* __restrict__ dx, int B,
                                  int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float n = nrm[b];
  if (n <= eps) {
    for (int c = lane; c < D; c += 64) dx[(int64_t)b * D + c] = dy[(int64_t)b * D + c] / eps;
    return;
  }
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += dy[(int64_t)b * D + c] * y[(int64_t)b * D + c];
  const float dot = warp_sum(s);
  for (int c = lane; c < D; c += 64)
    dx[(int64_t)b * D + c] = (dy[(int64_t)b * D + c] - y[(int64_t)b * D + c] * dot) / n;
}

// ---- InfoNCE ----
// S [2N, 2N] (ld 2N), LQ [N, K] (ld K) or K == 0.  One workgroup per row i.
__global__ __launch_bounds__(256) void nce_lse_kernel(const float* __restrict__ S,
                                                      const float* __restrict__ LQ, int N, int K,
                                                      float invT, float* __restrict__ lse,
                                                      float* __restrict__ loss_row) {
  __shared__ float red[4];
  const int i = blockIdx.x;
  const int n2 = 2 * N;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* srow = S + (int64_t)i * n2;
  const float* qrow = K > 0 ? LQ + (int64_t)(i % N) * K : nullptr;
  float m = -INFINITY;
  for (int j = tid; j < n2; j += 256)
    if (j != i) m = fmaxf(m, srow[j] * invT);
  for (int j = tid; j < K; j += 256) m = fmaxf(m, qrow[j] * invT);
  m = warp_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int j = tid; j < n2; j += 256)
    if (j != i) s += __expf(srow[j] * invT - m);
  for (int j = tid; j < K; j += 256) s += __expf(qrow[j] * invT - m);
  s = warp_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  if (tid == 0) {
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    const float l = m + logf(tot);
    lse[i] = l;
    const int p = (i + N) % n2;
    loss_row[i] = l - srow[p] * invT;
  }
}

// GS[i][j] = 0.5/T (exp(S_ij/T - lse_i) - [j == p_i]), GS[i][i] = 0, times the
// upstream gradient *gscale (read on device: no host sync for loss / acml).
__global__ void nce_grad_s_kernel(const float* __restrict__ S, const float* __restrict__ lse,
                                  float* __restrict__ GS, int N, float invT, float scale0,
                                  const float* __restrict__ gscale) {
  const int n2 = 2 * N;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n2 * n2) return;
  const float scale = gscale ? scale0 * gscale[0] : scale0;
  const int i = (int)(e / n2), j = (int)(e % n2);
  float g = 0.f;
  if (j != i) {
    g = __expf(S[e] * invT - lse[i]);
    if (j == (i + N) % n2) g -= 1.f;
  }
  GS[e] = g * scale;
}

// GQ[n][m] = 0.5/T (exp(LQ/T - lse_n) + exp(LQ/T - lse_{n+N}))
__global__ void nce_grad_q_kernel(const float* __restrict__ LQ, const float* __restrict__ lse,
                                  float* __restrict__ GQ, int N, int K, float invT, float scale0,
                                  const float* __restrict__ gscale) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)N * K) return;
  const float scale = gscale ? scale0 * gscale[0] : scale0;
  const int n = (int)(e / K);
  const float z = LQ[e] * invT;
  GQ[e] = (__expf(z - lse[n]) + __expf(z - lse[n + N])) * scale;
}

// ---- deterministic reductions ----
constexpr int RED_NT = 256;
// partial[blk] = sum over a fixed contiguous range of (scale * x)^p, p in {1, 2}
template <int POW>
__global__ __launch_bounds__(RED_NT) void partial_sum_kernel(const float* __restrict__ x, int64_t n,
                                                             int64_t per_blk,
                                                             float* __restrict__ partial) {
  __shared__ float red[RED_NT / 64];
  const int64_t lo = (int64_t)blockIdx.x * per_blk;
  int64_t hi = lo + per_blk;
  if (hi > n) hi = n;
  float s = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += RED_NT) {
    const float v = x[i];
    s += POW == 2 ? v * v : v;
  }
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < RED_NT / 64; ++w) t += red[w];
    partial[blockIdx.x] = t;
  }
}

// out[0] = scale * sum(partial) in fixed order; for the clip variant also
// out[1] = min(1, max_norm / (sqrt(sum) + 1e-6)) and out[0] = sqrt(sum).
__global__ void finalize_kernel(const float* __restrict__ partial, int np, float scale,
                                float max_norm, int clip, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double s = 0.0;  // fixed order, wide accumulator
  for (int i = 0; i < np; ++i) s += (double)partial[i];
  if (clip) {
    const float nrm = (float)sqrt(s);
    out[0] = nrm;
    const float coef = max_norm / (nrm + 1e-6f);
    out[1] = coef < 1.f ? coef : 1.f;
    out[2] = 0.f;  // step gate (irc_fault_gate): 0 = apply the update
  } else {
    out[0] = (float)(s * (double)scale);
  }
}

// Adam (torch.optim.Adam, weight_decay 0, amsgrad False) with the clip coefficient
// applied to the gradient: g' = g * coef[1].
// pb (may be null): bf16 shadow of the updated parameters (the MFMA operand copy).
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                            float* __restrict__ m, float* __restrict__ v, int64_t n,
                            const float* __restrict__ coef, float b1, float b2, float step_size,
                            float bc2_sqrt, float eps, unsigned short* __restrict__ pb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (coef && coef[2] != 0.f) return;  // gated: a recurrence timed out in this step
  const float c = coef ? coef[1] : 1.f;
  const float gi = g[i] * c;
  const float mi = m[i] + (1.f - b1) * (gi - m[i]);  // lerp, as torch
  const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  const float np = p[i] - step_size * (mi / denom);
  p[i] = np;
  if (pb) pb[i] = f32_to_bf16(np);
}

// SGD (torch.optim.SGD, dampening 0, nesterov False; the reference's --opt sgd,
// model.py:45-51) with the clip coefficient applied to the gradient:
// d = g * coef[1] + wd * p; buf = first ? d : mom * buf + d; p -= lr * buf.
// pb (may be null): bf16 shadow of the updated parameters.
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                           float* __restrict__ buf, int64_t n, const float* __restrict__ coef,
                           float lr, float mom, float wd, int first, unsigned short* __restrict__ pb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (coef && coef[2] != 0.f) return;  // gated: a recurrence timed out in this step
  const float c = coef ? coef[1] : 1.f;
  const float pi = p[i];
  const float d = g[i] * c + wd * pi;
  const float b = first ? d : buf[i] * mom + d;
  buf[i] = b;
  const float np = pi - lr * b;
  p[i] = np;
  if (pb) pb[i] = f32_to_bf16(np);
}

// The head's output activation (model.py:23-26: nn.Sequential(Linear, eval(f"nn.{act}()")),
// torch's default constructor arguments).  Kind codes: include/irc.h IRC_ACT_*.
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float softplus1(float x) { return x > 20.f ? x : log1pf(expf(x)); }
constexpr float SELU_SCALE = 1.0507009873554804934193349852946f;
constexpr float SELU_ALPHA = 1.6732632423543772848170429916717f;

__device__ __forceinline__ float act_fwd(int k, float u) {
  switch (k) {
    case IRC_ACT_RELU: return u > 0.f ? u : 0.f;
    case IRC_ACT_RELU6: return fminf(fmaxf(u, 0.f), 6.f);
    case IRC_ACT_LEAKY_RELU: return u > 0.f ? u : 0.01f * u;
    case IRC_ACT_ELU:
    case IRC_ACT_CELU: return u > 0.f ? u : expm1f(u);
    case IRC_ACT_SELU: return SELU_SCALE * (u > 0.f ? u : SELU_ALPHA * expm1f(u));
    case IRC_ACT_GELU: return 0.5f * u * (1.f + erff(u * 0.70710678118654752f));
    case IRC_ACT_SILU: return u * sigm(u);
    case IRC_ACT_MISH: return u * tanhf(softplus1(u));
    case IRC_ACT_SIGMOID: return sigm(u);
    case IRC_ACT_TANH: return tanhf(u);
    case IRC_ACT_SOFTPLUS: return softplus1(u);
    case IRC_ACT_SOFTSIGN: return u / (1.f + fabsf(u));
    case IRC_ACT_HARDTANH: return fminf(fmaxf(u, -1.f), 1.f);
    case IRC_ACT_HARDSIGMOID: return fminf(fmaxf(u + 3.f, 0.f), 6.f) / 6.f;
    case IRC_ACT_HARDSWISH: return u * fminf(fmaxf(u + 3.f, 0.f), 6.f) / 6.f;
    case IRC_ACT_TANHSHRINK: return u - tanhf(u);
    default: return u;  // IRC_ACT_IDENTITY
  }
}

// d act / d u at u (torch autograd's conventions at the kinks)
__device__ __forceinline__ float act_grad(int k, float u) {
  switch (k) {
    case IRC_ACT_RELU: return u > 0.f ? 1.f : 0.f;
    case IRC_ACT_RELU6: return (u > 0.f && u < 6.f) ? 1.f : 0.f;
    case IRC_ACT_LEAKY_RELU: return u > 0.f ? 1.f : 0.01f;
    case IRC_ACT_ELU:
    case IRC_ACT_CELU: return u > 0.f ? 1.f : expf(u);
    case IRC_ACT_SELU: return u > 0.f ? SELU_SCALE : SELU_SCALE * SELU_ALPHA * expf(u);
    case IRC_ACT_GELU:
      return 0.5f * (1.f + erff(u * 0.70710678118654752f)) +
             u * 0.39894228040143268f * expf(-0.5f * u * u);
    case IRC_ACT_SILU: {
      const float s = sigm(u);
      return s * (1.f + u * (1.f - s));
    }
    case IRC_ACT_MISH: {
      const float t = tanhf(softplus1(u));
      return t + u * (1.f - t * t) * sigm(u);
    }
    case IRC_ACT_SIGMOID: {
      const float s = sigm(u);
      return s * (1.f - s);
    }
    case IRC_ACT_TANH: {
      const float t = tanhf(u);
      return 1.f - t * t;
    }
    case IRC_ACT_SOFTPLUS: return u > 20.f ? 1.f : sigm(u);
    case IRC_ACT_SOFTSIGN: {
      const float a = 1.f + fabsf(u);
      return 1.f / (a * a);
    }
    case IRC_ACT_HARDTANH: return (u > -1.f && u < 1.f) ? 1.f : 0.f;
    case IRC_ACT_HARDSIGMOID: return (u > -3.f && u < 3.f) ? 1.f / 6.f : 0.f;
    case IRC_ACT_HARDSWISH: return u <= -3.f ? 0.f : (u < 3.f ? u / 3.f + 0.5f : 1.f);
    case IRC_ACT_TANHSHRINK: {
      const float t = tanhf(u);
      return t * t;
    }
    default: return 1.f;
  }
}

__global__ void act_fwd_kernel(int kind, const float* __restrict__ u, float* __restrict__ y,
                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = act_fwd(kind, u[i]);
}

__global__ void act_bwd_kernel(int kind, const float* __restrict__ u, float* __restrict__ g,
                               int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) g[i] *= act_grad(kind, u[i]);
}

__global__ void momentum_kernel(float* __restrict__ pk, const float* __restrict__ pq, int64_t n,
                                float mom, unsigned short* __restrict__ pb,
                                const float* __restrict__ gate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (gate && gate[2] != 0.f) return;
  const float v = pk[i] * mom + pq[i] * (1.f - mom);
  pk[i] = v;
  if (pb) pb[i] = f32_to_bf16(v);
}

// coef[2] = 1 when either sticky fault word (the cluster recurrences' timeout
// words of the query / key encoders) is set: the gated Adam / momentum updates of
// this step then leave every parameter and moment untouched -- no host sync.
__global__ void fault_gate_kernel(const unsigned* __restrict__ a, const unsigned* __restrict__ b,
                                  float* __restrict__ coef) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool f = (a != nullptr && *a != 0u) || (b != nullptr && *b != 0u);
  coef[2] = f ? 1.f : 0.f;
}

// queue[d, ptr + b] = keys[b, d]
__global__ void enqueue_kernel(float* __restrict__ queue, const float* __restrict__ keys,
                               const int64_t* __restrict__ ptr, int D, int K, int B) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)D * B) return;
  const int d = (int)(e / B), b = (int)(e % B);
  queue[(int64_t)d * K + ptr[0] + b] = keys[(int64_t)b * D + d];
}

__global__ void ptr_advance_kernel(int64_t* ptr, int B, int K) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ptr[0] = (ptr[0] + B) % K;
}

__global__ void axpby_kernel(float* __restrict__ out, const float* __restrict__ x,
                             const float* __restrict__ y, float a, float b, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a * x[i] + b * y[i];
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, unsigned short* __restrict__ y,
                                 int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f32_to_bf16(x[i]);
}

// Column sums in two deterministic passes: partial[chunk][c] over a fixed row
// chunk (grid.y), then out[c] (+)= sum over chunks in order.
constexpr int COLSUM_ROWS = 64;
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ x, float* __restrict__ partial,
                                      int64_t R, int C, int64_t ldx) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS;
  int64_t r1 = r0 + COLSUM_ROWS;
  if (r1 > R) r1 = R;
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += ldf(x, r * ldx + c);
  partial[(int64_t)blockIdx.y * C + c] = s;
}

// bf16 rows, C % 8 == 0: each thread sums 8 adjacent columns over the chunk with
// 16-byte loads (a wave covers 512 contiguous columns = 1 KB per row).
__global__ void colsum_partial_vec_kernel(const unsigned short* __restrict__ x,
                                          float* __restrict__ partial, int64_t R, int C,
                                          int64_t ldx) {
  const int c8 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (c8 >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * COLSUM_ROWS;
  int64_t r1 = r0 + COLSUM_ROWS;
  if (r1 > R) r1 = R;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {  // 8 independent 16-byte loads in flight
    u16x8 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const u16x8*>(x + (r + q) * ldx + c8);
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int t = 0; t < 8; ++t) s[t] += bf16_to_f32(v[q][t]);
  }
  for (; r < r1; ++r) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + r * ldx + c8);
#pragma unroll
    for (int t = 0; t < 8; ++t) s[t] += bf16_to_f32(v[t]);
  }
  float* p = partial + (int64_t)blockIdx.y * C + c8;
#pragma unroll
  for (int t = 0; t < 8; ++t) p[t] = s[t];
}

// Batched column sums x[b][r][c] -> out[b * so + c] (the per-layer bias gradients of
// the trainable encoder's deferred weight-gradient pass), deterministic:
// stage 1: block (column group of 512 [bf16] / 256 [fp32], row chunk, batch), 4 waves
// striding the chunk's rows, lanes owning 8 (bf16) or 4 (fp32) adjacent columns,
// folded across waves in fixed order -> partial[b][chunk][c];
// stage 2: out (+)= sum over chunks in order.
constexpr int CSB_ROWS = 256;
template <typename T>
__global__ __launch_bounds__(256) void colsum_b_stage1(const T* __restrict__ x, int64_t R, int C,
                                                       int64_t ldx, int64_t sx,
                                                       float* __restrict__ partial, int nch) {
  constexpr int V = sizeof(T) == 2 ? 8 : 4;  // columns per lane (16 bytes)
  __shared__ float red[4][64 * V];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.z, ch = blockIdx.y;
  const int c0 = (blockIdx.x * 64 + lane) * V;
  const bool ok = c0 < C;
  const T* xb = x + (int64_t)b * sx;
  const int64_t r0 = (int64_t)ch * CSB_ROWS;
  const int64_t r1 = r0 + CSB_ROWS < R ? r0 + CSB_ROWS : R;
  float acc[V];
#pragma unroll
  for (int t = 0; t < V; ++t) acc[t] = 0.f;
  if (ok) {
    int64_t r = r0 + wv;
    for (; r + 12 < r1; r += 16) {  // 4 independent 16-byte loads in flight
      if constexpr (sizeof(T) == 2) {
        u16x8 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = *reinterpret_cast<const u16x8*>(reinterpret_cast<const unsigned short*>(xb) +
                                                 (r + 4 * q) * ldx + c0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] += bf16_to_f32(v[q][t]);
      } else {
        f32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(xb) +
                                                 (r + 4 * q) * ldx + c0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[t] += v[q][t];
      }
    }
    for (; r < r1; r += 4) {
#pragma unroll
      for (int t = 0; t < V; ++t) acc[t] += ldf(xb, r * ldx + c0 + t);
    }
  }
#pragma unroll
  for (int t = 0; t < V; ++t) red[wv][lane * V + t] = acc[t];
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * V; e += 256) {
    const int c = blockIdx.x * 64 * V + e;
    if (c < C)
      partial[((int64_t)b * nch + ch) * C + c] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
  }
}

__global__ void colsum_b_stage2(const float* __restrict__ partial, int nch, int C,
                                float* __restrict__ out, int64_t so, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (c >= C) return;
  const float* p = partial + (int64_t)b * nch * C + c;
  float s = 0.f;
  for (int k = 0; k < nch; ++k) s += p[(int64_t)k * C];
  float* o = out + b * so + c;
  *o = accumulate ? *o + s : s;
}

// W [R][C] fp32 -> W^T [C][R] bf16 through 32x33 LDS tiles (the nn.Linear-layout
// operand of GEMMs that consume W as [K][N]).
// Batched over blockIdx.z: matrix b at x + b * sx, its transpose at y + b * sy.
__global__ void cast_bf16_t_kernel(const float* __restrict__ x, unsigned short* __restrict__ y,
                                   int R, int C, int64_t sx = 0, int64_t sy = 0) {
  __shared__ float tile[32][33];
  x += (int64_t)blockIdx.z * sx;
  y += (int64_t)blockIdx.z * sy;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? x[(int64_t)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[(int64_t)c * R + r] = f32_to_bf16(tile[tx][i]);
  }
}

// 64 columns x 4 chunk segments per block: each thread sums its segment in chunk
// order (8 loads in flight), then the 4 segment sums are added in segment order
// -- a fixed order, so the result is bitwise reproducible.
__global__ void colsum_final_kernel(const float* __restrict__ partial, float* __restrict__ out,
                                    int nchunks, int C, int accumulate) {
  __shared__ float seg[4][64];
  const int cl = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int per = (nchunks + 3) / 4;
  const int k0 = sg * per, k1 = min(nchunks, k0 + per);
  float s = 0.f;
  if (c < C) {
    int k = k0;
    for (; k + 8 <= k1; k += 8) {
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = partial[(int64_t)(k + q) * C + c];
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[q];
    }
    for (; k < k1; ++k) s += partial[(int64_t)k * C + c];
  }
  seg[sg][cl] = s;
  __syncthreads();
  if (sg == 0 && c < C) {
    const float t = ((seg[0][cl] + seg[1][cl]) + seg[2][cl]) + seg[3][cl];
    out[c] = accumulate ? out[c] + t : t;
  }
}

}  // namespace tops
}  // namespace irc

using namespace irc;
using namespace irc::tops;

static inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

extern "C" int irc_mean_rows(int dtype, const void* x, float* out, int64_t B, int64_t L, int64_t C,
                             int64_t ldx, irc_stream_t stream) {
  IRC_REQUIRE(B >= 0 && L >= 1 && C >= 1, "mean_rows: bad sizes");
  if (B == 0) return IRC_OK;
  if (dtype == 0)
    hipLaunchKernelGGL(mean_rows_kernel<unsigned short>, dim3(nblk(B * C)), dim3(256), 0,
                       as_stream(stream), (const unsigned short*)x, out, (int)B, (int)L, (int)C,
                       ldx);
  else
    hipLaunchKernelGGL(mean_rows_kernel<float>, dim3(nblk(B * C)), dim3(256), 0,
                       as_stream(stream), (const float*)x, out, (int)B, (int)L, (int)C, ldx);
  return check_launch("mean_rows");
}

extern "C" int irc_bcast_rows(const float* g, float* y, int64_t B, int64_t L, int64_t C,
                              float scale, irc_stream_t stream) {
  if (B * L * C == 0) return IRC_OK;
  hipLaunchKernelGGL(bcast_rows_kernel, dim3(nblk(B * L * C)), dim3(256), 0, as_stream(stream), g,
                     y, (int)B, (int)L, (int)C, scale);
  return check_launch("bcast_rows");
}

extern "C" int irc_l2norm_fwd(const float* x, float* y, float* nrm, int64_t B, int64_t D,
                              float eps, irc_stream_t stream) {
  if (B == 0) return IRC_OK;
  hipLaunchKernelGGL(l2norm_fwd_kernel, dim3(nblk(B, 4)), dim3(256), 0, as_stream(stream), x, y,
                     nrm, (int)B, (int)D, eps);
  return check_launch("l2norm_fwd");
}

extern "C" int irc_l2norm_bwd(const float* dy, const float* y, const float* nrm, float* dx,
                              int64_t B, int64_t D, float eps, irc_stream_t stream) {
  if (B == 0) return IRC_OK;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3(nblk(B, 4)), dim3(256), 0, as_stream(stream), dy, y,
                     nrm, dx, (int)B, (int)D, eps);
  return check_launch("l2norm_bwd");
}

extern "C" int irc_nce_lse(const float* S, const float* LQ, int64_t N, int64_t K, float T,
                           float* lse, float* loss_row, irc_stream_t stream) {
  IRC_REQUIRE(N >= 1 && K >= 0 && T > 0, "nce_lse: bad sizes");
  hipLaunchKernelGGL(nce_lse_kernel, dim3((unsigned)(2 * N)), dim3(256), 0, as_stream(stream), S,
                     LQ, (int)N, (int)K, 1.f / T, lse, loss_row);
  return check_launch("nce_lse");
}

extern "C" int irc_nce_grads(const float* S, const float* LQ, const float* lse, int64_t N,
                             int64_t K, float T, const float* gscale, float* GS, float* GQ,
                             irc_stream_t stream) {
  IRC_REQUIRE(N >= 1 && K >= 0 && T > 0, "nce_grads: bad sizes");
  const float scale = 0.5f / T;
  hipLaunchKernelGGL(nce_grad_s_kernel, dim3(nblk(4 * N * N)), dim3(256), 0, as_stream(stream), S,
                     lse, GS, (int)N, 1.f / T, scale, gscale);
  int rc = check_launch("nce_grad_s");
  if (rc || K == 0) return rc;
  hipLaunchKernelGGL(nce_grad_q_kernel, dim3(nblk(N * K)), dim3(256), 0, as_stream(stream), LQ,
                     lse, GQ, (int)N, (int)K, 1.f / T, scale, gscale);
  return check_launch("nce_grad_q");
}

// Deterministic sum: out[0] = scale * sum(x).  partial needs >= 1024 floats.
extern "C" int irc_sum(const float* x, int64_t n, float scale, float* partial, float* out,
                       irc_stream_t stream) {
  const int64_t np = n < 1024 * 4096 ? (n + 4095) / 4096 : 1024;
  const int64_t per = np > 0 ? (n + np - 1) / np : 1;
  hipStream_t st = as_stream(stream);
  if (np > 0)
    hipLaunchKernelGGL(partial_sum_kernel<1>, dim3((unsigned)np), dim3(RED_NT), 0, st, x, n, per,
                       partial);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, st, partial, (int)np, scale, 0.f, 0,
                     out);
  return check_launch("sum");
}

// Global grad norm + clip coefficient: out[0] = ||g||, out[1] = min(1, max/(||g||+1e-6)).
extern "C" int irc_grad_norm_clip(const float* g, int64_t n, float max_norm, float* partial,
                                  float* out, irc_stream_t stream) {
  const int64_t np = n < 1024 * 4096 ? (n + 4095) / 4096 : 1024;
  const int64_t per = np > 0 ? (n + np - 1) / np : 1;
  hipStream_t st = as_stream(stream);
  if (np > 0)
    hipLaunchKernelGGL(partial_sum_kernel<2>, dim3((unsigned)np), dim3(RED_NT), 0, st, g, n, per,
                       partial);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, st, partial, (int)np, 1.f, max_norm, 1,
                     out);
  return check_launch("grad_norm_clip");
}

extern "C" int irc_adam_step(float* p, const float* g, float* m, float* v, int64_t n,
                             const float* coef, float b1, float b2, float step_size,
                             float bc2_sqrt, float eps, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), p, g, m, v, n,
                     coef, b1, b2, step_size, bc2_sqrt, eps, nullptr);
  return check_launch("adam");
}

extern "C" int irc_adam_step_bf16(float* p, const float* g, float* m, float* v, int64_t n,
                                  const float* coef, float b1, float b2, float step_size,
                                  float bc2_sqrt, float eps, void* p_bf16, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), p, g, m, v, n,
                     coef, b1, b2, step_size, bc2_sqrt, eps, (unsigned short*)p_bf16);
  return check_launch("adam_bf16");
}

extern "C" int irc_momentum_update_bf16(float* pk, const float* pq, int64_t n, float mom,
                                        void* pk_bf16, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(momentum_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), pk, pq, n,
                     mom, (unsigned short*)pk_bf16, nullptr);
  return check_launch("momentum_bf16");
}

extern "C" int irc_sgd_step(float* p, const float* g, float* buf, int64_t n, const float* coef,
                            float lr, float momentum, float weight_decay, int first_step,
                            void* p_bf16, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(sgd_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), p, g, buf, n,
                     coef, lr, momentum, weight_decay, first_step, (unsigned short*)p_bf16);
  return check_launch("sgd");
}

extern "C" int irc_activation(int kind, const float* u, float* y, int64_t n, irc_stream_t stream) {
  IRC_REQUIRE(kind >= 0 && kind < IRC_ACT_COUNT, "activation: kind %d", kind);
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(act_fwd_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), kind, u, y, n);
  return check_launch("activation");
}

extern "C" int irc_activation_bwd(int kind, const float* u, float* g, int64_t n,
                                  irc_stream_t stream) {
  IRC_REQUIRE(kind >= 0 && kind < IRC_ACT_COUNT, "activation_bwd: kind %d", kind);
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), kind, u, g, n);
  return check_launch("activation_bwd");
}

extern "C" int irc_momentum_update_gated(float* pk, const float* pq, int64_t n, float mom,
                                         const float* gate, void* pk_bf16, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  IRC_REQUIRE(gate != nullptr, "momentum_update_gated: null gate");
  hipLaunchKernelGGL(momentum_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), pk, pq, n,
                     mom, (unsigned short*)pk_bf16, gate);
  return check_launch("momentum_gated");
}

extern "C" int irc_fault_gate(const void* fault_a, const void* fault_b, float* coef,
                              irc_stream_t stream) {
  IRC_REQUIRE(coef != nullptr, "fault_gate: null coef");
  hipLaunchKernelGGL(fault_gate_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                     (const unsigned*)fault_a, (const unsigned*)fault_b, coef);
  return check_launch("fault_gate");
}

extern "C" int irc_momentum_update(float* pk, const float* pq, int64_t n, float mom,
                                   irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(momentum_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), pk, pq, n,
                     mom, nullptr, nullptr);
  return check_launch("momentum");
}

extern "C" int irc_enqueue(float* queue, const float* keys, int64_t* ptr, int64_t D, int64_t K,
                           int64_t B, irc_stream_t stream) {
  IRC_REQUIRE(B >= 1 && K % B == 0, "enqueue: queue_size %% batch != 0 (caller must skip)");
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(enqueue_kernel, dim3(nblk(D * B)), dim3(256), 0, st, queue, keys, ptr,
                     (int)D, (int)K, (int)B);
  hipLaunchKernelGGL(ptr_advance_kernel, dim3(1), dim3(64), 0, st, ptr, (int)B, (int)K);
  return check_launch("enqueue");
}

extern "C" int irc_cast_bf16_t(const float* x, void* y, int64_t R, int64_t C,
                               irc_stream_t stream) {
  if (R == 0 || C == 0) return IRC_OK;
  hipLaunchKernelGGL(cast_bf16_t_kernel, dim3((unsigned)((C + 31) / 32), (unsigned)((R + 31) / 32)),
                     dim3(256), 0, as_stream(stream), x, (unsigned short*)y, (int)R, (int)C);
  return check_launch("cast_bf16_t");
}

// batch matrices [R][C] fp32, sx floats apart -> their transposes [C][R] bf16, sy elements
// apart: one launch for every layer's copy of one weight (the trainable encoder's dX
// operands; 48 launches a step became 4).
extern "C" int irc_cast_bf16_t_batched(const float* x, void* y, int64_t R, int64_t C,
                                       int64_t batch, int64_t sx, int64_t sy,
                                       irc_stream_t stream) {
  IRC_REQUIRE(batch >= 1 && batch < 65536, "cast_bf16_t_batched: batch %lld", (long long)batch);
  if (R == 0 || C == 0) return IRC_OK;
  hipLaunchKernelGGL(cast_bf16_t_kernel,
                     dim3((unsigned)((C + 31) / 32), (unsigned)((R + 31) / 32), (unsigned)batch),
                     dim3(256), 0, as_stream(stream), x, (unsigned short*)y, (int)R, (int)C, sx, sy);
  return check_launch("cast_bf16_t_batched");
}

extern "C" int irc_cast_bf16(const float* x, void* y, int64_t n, irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), x,
                     (unsigned short*)y, n);
  return check_launch("cast_bf16");
}

// partial: workspace of >= ceil(R / 256) * C floats.
extern "C" int irc_colsum(int dtype, const void* x, float* out, int64_t R, int64_t C, int64_t ldx,
                          int accumulate, float* partial, irc_stream_t stream) {
  if (C == 0) return IRC_OK;
  const int64_t nch = (R + COLSUM_ROWS - 1) / COLSUM_ROWS;
  hipStream_t st = as_stream(stream);
  if (nch > 0 && dtype == 0 && C % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0)
    hipLaunchKernelGGL(colsum_partial_vec_kernel, dim3(nblk(C / 8, 64), (unsigned)nch), dim3(64),
                       0, st, (const unsigned short*)x, partial, R, (int)C, ldx);
  else if (nch > 0 && dtype == 0)
    hipLaunchKernelGGL(colsum_partial_kernel<unsigned short>, dim3(nblk(C, 64), (unsigned)nch),
                       dim3(64), 0, st, (const unsigned short*)x, partial, R, (int)C, ldx);
  else if (nch > 0)
    hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3(nblk(C, 64), (unsigned)nch), dim3(64), 0,
                       st, (const float*)x, partial, R, (int)C, ldx);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(nblk(C, 64)), dim3(256), 0, st, partial, out,
                     (int)nch, (int)C, accumulate);
  return check_launch("colsum");
}

extern "C" int irc_axpby(float* out, const float* x, const float* y, float a, float b, int64_t n,
                         irc_stream_t stream) {
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(axpby_kernel, dim3(nblk(n)), dim3(256), 0, as_stream(stream), out, x, y, a, b,
                     n);
  return check_launch("axpby");
}

extern "C" int64_t irc_colsum_batched_workspace(int64_t batch, int64_t R, int64_t C) {
  return batch * ((R + CSB_ROWS - 1) / CSB_ROWS) * C;
}

// out[b * so + c] (+)= sum_r x[b * sx + r * ldx + c]; partial: the workspace above (floats).
extern "C" int irc_colsum_batched(int dtype, const void* x, int64_t batch, int64_t R, int64_t C,
                                  int64_t ldx, int64_t sx, float* out, int64_t so, int accumulate,
                                  float* partial, int64_t partial_floats, irc_stream_t stream) {
  IRC_REQUIRE(dtype == 0 || dtype == 1, "colsum_batched: dtype");
  if (C == 0 || batch == 0) return IRC_OK;
  const int64_t nch = R > 0 ? (R + CSB_ROWS - 1) / CSB_ROWS : 0;
  IRC_REQUIRE(partial_floats >= batch * (nch > 0 ? nch : 1) * C, "colsum_batched: workspace");
  const int V = dtype == 0 ? 8 : 4;
  IRC_REQUIRE(C % V == 0 && ldx % V == 0 && sx % V == 0 && ((uintptr_t)x % 16) == 0,
              "colsum_batched: needs 16-byte aligned rows (C %% %d == 0)", V);
  hipStream_t st = as_stream(stream);
  if (nch > 0) {
    const dim3 g1((unsigned)((C + 64 * V - 1) / (64 * V)), (unsigned)nch, (unsigned)batch);
    if (dtype == 0)
      hipLaunchKernelGGL(colsum_b_stage1<unsigned short>, g1, dim3(256), 0, st,
                         (const unsigned short*)x, R, (int)C, ldx, sx, partial, (int)nch);
    else
      hipLaunchKernelGGL(colsum_b_stage1<float>, g1, dim3(256), 0, st, (const float*)x, R, (int)C,
                         ldx, sx, partial, (int)nch);
  }
  hipLaunchKernelGGL(colsum_b_stage2, dim3(nblk(C, 256), (unsigned)batch), dim3(256), 0, st,
                     partial, (int)nch, (int)C, out, so, accumulate);
  return check_launch("colsum_batched");
}
