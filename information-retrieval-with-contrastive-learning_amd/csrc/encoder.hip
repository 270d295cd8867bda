// BERT-style encoder pieces other than the GEMMs (gfx950):
//  * embed_ln: LN(word[ids] + token_type[0] + position[l]) fused (HF BertEmbeddings,
//    reached from src/contrastor/contrastive_module.py:39, eps 1e-12).
//  * layernorm: y = LN(x) * gamma + beta, one wave per row (BertSelfOutput /
//    BertOutput LayerNorm; the residual add is fused into the producing GEMM).
//  * attention: per (sequence, head) softmax(Q K^T / sqrt(dh) + key mask) V with an
//    online softmax; PAD query rows are computed and kept, as HF does.
// Element type T is bf16 (uint16 bits) or fp32; statistics are always fp32.
#include "irc_common.h"
#include "mx.h"

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

// bf16 embedding gather + LayerNorm for H % 256 == 0: embed_ln_kernel's arithmetic with
// layernorm_vec_kernel's layout (one half-wave per row, 16-byte gathers of the word row,
// position row and token-type row, CPL chunks of 8 per lane).  The 32-lane statistics
// sum in another order than the 64-lane one, so the output can differ from
// embed_ln_kernel's in the last bf16 bit.
template <int CPL>
__global__ __launch_bounds__(256) void embed_ln_vec_kernel(
    const int64_t* __restrict__ ids, const unsigned short* __restrict__ word,
    const unsigned short* __restrict__ pos, const unsigned short* __restrict__ type0,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    unsigned short* __restrict__ y, int64_t rows, int L, float eps) {
  constexpr int H = CPL * 256;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = row < rows;
  const int64_t rr = ok ? row : 0;
  const int64_t id = ids[rr];
  const int l = (int)(rr % L);
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c0 = (i * 32 + hl) * 8;
    const u16x8 w = *reinterpret_cast<const u16x8*>(word + id * H + c0);
    const u16x8 t = *reinterpret_cast<const u16x8*>(type0 + c0);
    const u16x8 p = *reinterpret_cast<const u16x8*>(pos + (int64_t)l * H + c0);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // HF order: (word + token_type) + position
      v[i][e] = (bf16_to_f32(w[e]) + bf16_to_f32(t[e])) + bf16_to_f32(p[e]);
      s += v[i][e];
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[i][e] - mean;
      s2 = __builtin_fmaf(d, d, s2);
    }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
  const float rstd = rsqrtf(s2 / H + eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c0 = (i * 32 + hl) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c0);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c0 + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c0);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + c0 + 4);
    const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
    const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16((v[i][e] - mean) * rstd * gg[e] + bb[e]);
    *reinterpret_cast<u16x8*>(y + row * H + c0) = o;
  }
}

// bf16 LayerNorm for H % 256 == 0 (BERT-base 768, -large 1024): one half-wave
// (32 lanes) per row, 16-byte loads/stores (H/256 chunks of 8 per lane), the
// two half-waves of a wave on consecutive rows; statistics fp32 in the same
// order-independent two-pass form as layernorm_kernel.
// y8 != null: the row is ALSO written as MX-fp8 (e4m3 y8 [rows][H] + E8M0 block scales
// ys in the MX layout, mpad rows): the next fp8 linear layer's A operand, with no
// separate quantisation pass (config C5).  One 32-value block = 4 consecutive
// lanes' chunks of 8.
template <int CPL>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const unsigned short* __restrict__ x,
                                                           unsigned short* __restrict__ y,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           int64_t rows, float eps,
                                                           unsigned char* __restrict__ y8 = nullptr,
                                                           unsigned char* __restrict__ ys = nullptr,
                                                           int64_t mpad = 0) {
  constexpr int H = CPL * 256;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = row < rows;
  const unsigned short* xr = x + (ok ? row : 0) * H;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const u16x8 u = *reinterpret_cast<const u16x8*>(xr + (i * 32 + hl) * 8);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      v[i][t] = bf16_to_f32(u[t]);
      s += v[i][t];
    }
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float d = v[i][t] - mean;
      s2 = __builtin_fmaf(d, d, s2);  // explicit: the same rounding in every LN kernel
    }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
  const float rstd = rsqrtf(s2 / H + eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c0 = (i * 32 + hl) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c0);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c0 + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c0);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + c0 + 4);
    const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
    const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    u16x8 o;
    float r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {  // explicit fma: the same rounding in every variant
      r[t] = __builtin_fmaf((v[i][t] - mean) * rstd, gg[t], bb[t]);
      o[t] = f32_to_bf16(r[t]);
    }
    *reinterpret_cast<u16x8*>(y + row * H + c0) = o;
    if (y8 != nullptr) {  // uniform: one code path, so y is the same bits either way
      // quantise the bf16-rounded values: the fp8 operand is the bf16 activation's
      // quantisation, exactly as the standalone quantiser would produce it
#pragma unroll
      for (int t = 0; t < 8; ++t) r[t] = bf16_to_f32(o[t]);
      uint2 q8;
      const unsigned e8 = gpp::mx_quant8(r, q8);
      *reinterpret_cast<uint2*>(y8 + row * H + c0) = q8;
      if ((hl & 3) == 0) ys[gpp::mx_scale_index(row, c0, mpad)] = (unsigned char)e8;
    }
  }
}

// The bf16 LayerNorm of layernorm_vec_kernel (same per-row arithmetic, bit-identical)
// with R consecutive rows per half-wave: gamma / beta stay in registers across the rows
// and the next row's loads are issued before this row's statistics.
// y8 != null: also the MX-fp8 copy, as layernorm_vec_kernel writes it (config C5).
// Called in place (y == x) by the encoder, so x and y are NOT __restrict__ (aliasing them
// legally): every element is read by the lane that writes it, before it writes it, and a
// half-wave's rows are its own -- the prefetch past the last row re-reads the half-wave's
// own row, whose value is then discarded, never another half-wave's.  The gfx950 code is
// instruction-for-instruction the same as with __restrict__ (hipcc, ROCm 7.2: the next
// row's loads are issued ahead of this row's stores in program order either way).
template <int CPL, int R>
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const unsigned short* x,
                                                            unsigned short* y,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            int64_t rows, float eps,
                                                            unsigned char* __restrict__ y8 = nullptr,
                                                            unsigned char* __restrict__ ys = nullptr,
                                                            int64_t mpad = 0) {
  constexpr int H = CPL * 256;
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t row0 = (((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5)) * R;
  float gg[CPL][8], bb[CPL][8];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c0 = (i * 32 + hl) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c0);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c0 + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(beta + c0);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(beta + c0 + 4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      gg[i][t] = g0[t];
      gg[i][4 + t] = g1[t];
      bb[i][t] = b0[t];
      bb[i][4 + t] = b1[t];
    }
  }
  u16x8 cur[CPL];
  {
    const unsigned short* xr = x + (row0 < rows ? row0 : rows - 1) * H;
#pragma unroll
    for (int i = 0; i < CPL; ++i) cur[i] = *reinterpret_cast<const u16x8*>(xr + (i * 32 + hl) * 8);
  }
#pragma unroll 1
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r;
    u16x8 nxt[CPL];
    if (r + 1 < R) {
      const int64_t rn = row + 1 < rows ? row + 1 : (row < rows ? row : rows - 1);
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        nxt[i] = *reinterpret_cast<const u16x8*>(x + rn * H + (i * 32 + hl) * 8);
    }
    float v[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        v[i][t] = bf16_to_f32(cur[i][t]);
        s += v[i][t];
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / H;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float d = v[i][t] - mean;
        s2 = __builtin_fmaf(d, d, s2);  // explicit: the same rounding in every LN kernel
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    const float rstd = rsqrtf(s2 / H + eps);
    if (row < rows) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        u16x8 o;
#pragma unroll
        for (int t = 0; t < 8; ++t)  // explicit fma: the rounding of layernorm_vec_kernel
          o[t] = f32_to_bf16(__builtin_fmaf((v[i][t] - mean) * rstd, gg[i][t], bb[i][t]));
        const int c0 = (i * 32 + hl) * 8;
        *reinterpret_cast<u16x8*>(y + row * H + c0) = o;
        if (y8 != nullptr) {  // uniform; the bf16-rounded values quantised, as layernorm_vec_kernel
          float rq[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) rq[t] = bf16_to_f32(o[t]);
          uint2 q8;
          const unsigned e8 = gpp::mx_quant8(rq, q8);
          *reinterpret_cast<uint2*>(y8 + row * H + c0) = q8;
          if ((hl & 3) == 0) ys[gpp::mx_scale_index(row, c0, mpad)] = (unsigned char)e8;
        }
      }
    }
    if (r + 1 < R) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) cur[i] = nxt[i];
    }
  }
}

// Attention, any element type / head dim (the fp32 parity mode, head dims other
// than 64): one workgroup per (sequence b, head a, 256 queries).  qkv is the fused
// projection output [B*L, 3H] (cols [0,H)=Q, [H,2H)=K, [2H,3H)=V, head a at a*dh);
// ctx [B*L, H].  Each thread owns one query row (q and the output in registers) and
// runs an online softmax over the unmasked keys in ascending order; K and V are
// streamed through LDS as fp32 tiles of AKT keys, so any L fits (the reference pads
// a batch jointly up to 512 tokens, contrastive_module.py:38).  dh <= 128.
constexpr int AKT = 64;
template <typename T, int DH>
__global__ __launch_bounds__(256) void attention_kernel(const T* __restrict__ qkv,
                                                       const int64_t* __restrict__ mask,
                                                       T* __restrict__ ctx, int L, int H,
                                                       int heads, float scale) {
  __shared__ __attribute__((aligned(16))) float Ks[AKT][DH];
  __shared__ __attribute__((aligned(16))) float Vs[AKT][DH];
  __shared__ int kvis[AKT];
  __shared__ int nvalid;
  const int nqc = (L + 255) / 256;
  const int qc = blockIdx.x % nqc;
  const int a = (blockIdx.x / nqc) % heads, b = blockIdx.x / nqc / heads;
  const int64_t base = (int64_t)b * L;
  const int64_t ld3 = 3LL * H;
  if (threadIdx.x == 0) nvalid = 0;
  __syncthreads();
  int cnt = 0;
  for (int j = threadIdx.x; j < L; j += blockDim.x)
    cnt += (mask == nullptr || mask[base + j] != 0) ? 1 : 0;
  if (cnt) atomicAdd(&nvalid, cnt);
  __syncthreads();
  // all keys masked: HF's finfo.min bias swamps every score -> uniform weights
  const bool uniform = nvalid == 0;
  const int i = qc * 256 + threadIdx.x;
  const bool act = i < L;
  float qv[DH], o[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    qv[d] = act ? ld(qkv, (base + i) * ld3 + a * DH + d) * scale : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < L; j0 += AKT) {
    const int n = min(AKT, L - j0);
    __syncthreads();  // the previous tile's readers are done
    for (int e = threadIdx.x; e < n * DH; e += blockDim.x) {
      const int j = e / DH, d = e % DH;
      Ks[j][d] = ld(qkv, (base + j0 + j) * ld3 + H + a * DH + d);
      Vs[j][d] = ld(qkv, (base + j0 + j) * ld3 + 2 * H + a * DH + d);
    }
    for (int j = threadIdx.x; j < n; j += blockDim.x)
      kvis[j] = (uniform || mask == nullptr || mask[base + j0 + j] != 0) ? 1 : 0;
    __syncthreads();
    if (!act) continue;
    for (int t = 0; t < n; ++t) {
      if (!kvis[t]) continue;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s += qv[d] * Ks[t][d];
      if (uniform) s = 0.f;
      const float mn = fmaxf(m, s);
      const float corr = __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = o[d] * corr + p * Vs[t][d];
      m = mn;
    }
  }
  if (!act) return;
  const float inv = 1.f / l;
#pragma unroll
  for (int d = 0; d < DH; ++d) st(ctx, (base + i) * H + a * DH + d, o[d] * inv);
}

// MFMA attention, bf16, head dim 64, L <= 32*NJ (NJ <= 4, any L: the joint
// padding of a batch gives e.g. L = 72): one workgroup per (sequence, head), one wave
// per block of 32 queries, the NJ waves sharing one V^T image and key-bias row in LDS
// (staged once per (sequence, head); the round-5 form gave each wave its own copy, so
// at NJ = 3 a workgroup of 4 unrelated waves held 53 KB and a CU 12 waves).  Key rows
// past L are read clamped and carry a -3e30 bias (below a
// masked key's -1e30, so an all-masked row still averages its L keys), V rows
// past L are zero in LDS, query rows past L are never stored.
//  * S^T[j][i] = K[j] . Q[i] on v_mfma_f32_32x32x16_bf16 (A = K rows, B = Q rows,
//    both read straight from the fused QKV rows as 16-byte fragments), so lane
//    (i, half) holds query i's scores for the keys j = 32jb + (e&3) + 8(e>>2) + 4*half:
//    the softmax over keys is lane-local plus one exchange with lane ^ 32;
//  * key mask as an additive bias (0 / -1e30: masked keys get exactly zero
//    weight; an all-masked row degrades to a uniform average, as HF's finfo.min
//    bias does), fp32 softmax, probabilities rounded to bf16 (HF bf16 semantics);
//  * O = P . V: P goes straight from registers into the A operand; summing over
//    keys in the lane's permuted key order is matched by reading the V operand
//    from a per-wave transposed V^T copy in LDS (two ds_read_b64 per fragment).
//  * MXO (config C5): ctx leaves as MX-fp8 instead of bf16 -- e4m3 bytes ctx8
//    [B*L][H] and one E8M0 scale per (token, 32 head columns) in the MX layout
//    (cs, mpad rows) -- the out-projection's A operand, no quantisation pass; each
//    block is one half-wave's 32 lanes (the block max by 5 lane exchanges).
template <int NJ, bool MXO = false>
__global__ __launch_bounds__(256) void attention_mfma_kernel(const unsigned short* __restrict__ qkv,
                                                            const int64_t* __restrict__ mask,
                                                            unsigned short* __restrict__ ctx,
                                                            int B, int H, int heads, float scale,
                                                            unsigned char* __restrict__ ctx8 = nullptr,
                                                            unsigned char* __restrict__ cs = nullptr,
                                                            int64_t mpad = 0, int Lr = 32 * NJ) {
  constexpr int L = 32 * NJ, DH = 64, NT = 64 * NJ;
  // V^T row pitch (u16): 8-byte aligned, conflict-free b64 reads
  constexpr int VP = L + 4;
  constexpr int OP = 68;  // MXO: row pitch (floats) of a wave's 32-row O staging
  __shared__ __attribute__((aligned(16))) unsigned short vt[DH][VP];
  __shared__ __attribute__((aligned(16))) float mb[L];
  __shared__ __attribute__((aligned(16))) float ost[MXO ? NJ : 1][MXO ? 32 * OP : 1];
  const int lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
  const int ib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // query block
  const int a = (int)(blockIdx.x % heads), b = (int)(blockIdx.x / heads);
  const int64_t ld3 = 3LL * H;
  const unsigned short* base = qkv + (int64_t)b * Lr * ld3 + a * DH;  // + j*ld3: Q | +H: K | +2H: V
  // key blocks through the sequence's last visible key (visible_key_blocks: the rest add
  // exactly zero; every wave finds the same count); V^T is staged for those only, once
  const int nkb = visible_key_blocks(mask ? mask + (int64_t)b * Lr : nullptr, Lr, NJ, lane);
  for (int p = threadIdx.x; p < nkb * 128; p += NT) {
    const int dc = p & 7, j = (p >> 3) * 2;  // 8-wide d chunk, key pair (j, j+1)
    const u16x8 v0 = j < Lr ? *reinterpret_cast<const u16x8*>(base + (int64_t)j * ld3 + 2 * H + dc * 8)
                            : (u16x8)0;
    const u16x8 v1 =
        j + 1 < Lr ? *reinterpret_cast<const u16x8*>(base + (int64_t)(j + 1) * ld3 + 2 * H + dc * 8)
                   : (u16x8)0;
#pragma unroll
    for (int dd = 0; dd < 8; ++dd)
      *reinterpret_cast<uint32_t*>(&vt[dc * 8 + dd][j]) = (uint32_t)v0[dd] | ((uint32_t)v1[dd] << 16);
  }
  for (int j = threadIdx.x; j < L; j += NT)
    mb[j] = j >= Lr ? -3e30f : ((mask == nullptr || mask[(int64_t)b * Lr + j] != 0) ? 0.f : -1e30f);
  __syncthreads();

  bf16x8 qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    qf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)min(32 * ib + r32, Lr - 1) * ld3 +
                                               16 * kk + 8 * h);
  f32x16 s[NJ];
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    if (jb >= nkb) break;
    s[jb] = (f32x16)0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(
          base + (int64_t)min(32 * jb + r32, Lr - 1) * ld3 + H + 16 * kk + 8 * h);
      s[jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], s[jb], 0, 0, 0);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    if (jb >= nkb) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 bias = *reinterpret_cast<const f32x4*>(&mb[32 * jb + 8 * q + 4 * h]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s[jb][4 * q + r] * scale + bias[r];
        s[jb][4 * q + r] = v;
        mx = fmaxf(mx, v);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    if (jb >= nkb) break;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = __expf(s[jb][e] - mx);
      s[jb][e] = p;
      sum += p;
    }
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;

  f32x16 o[2] = {(f32x16)0.f, (f32x16)0.f};
#pragma unroll
  for (int jb = 0; jb < NJ; ++jb) {
    if (jb >= nkb) break;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      bf16x8 pa;
#pragma unroll
      for (int t = 0; t < 8; ++t) pa[t] = (__bf16)(s[jb][8 * k2 + t] * inv);
      const int j0 = 32 * jb + 16 * k2 + 4 * h;  // keys of slots t<4: j0+t; t>=4: j0+8+t-4
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int d = 32 * db + r32;
        const u16x4 lo = *reinterpret_cast<const u16x4*>(&vt[d][j0]);
        const u16x4 hi = *reinterpret_cast<const u16x4*>(&vt[d][j0 + 8]);
        const u16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, vv), o[db],
                                                        0, 0, 0);
      }
    }
  }
  // O C layout: col = d (lane), row = query 32ib + (e&3) + 8(e>>2) + 4h
  if constexpr (MXO) {
    // O (bf16-rounded like the bf16 path's ctx) goes through the wave's own slot of ost
    // as [32 rows][OP floats] (16-byte rows, h halves 16 banks apart); each lane then
    // owns one MX block (row lane >> 1, 32 columns): lane-local block max, 32 codes in
    // two 16-byte stores, one scale byte.
    float* os = &ost[MXO ? ib : 0][0];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = (e & 3) + 8 * (e >> 2) + 4 * h;
        os[i * OP + 32 * db + r32] = bf16_to_f32(f32_to_bf16(o[db][e]));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int i = lane >> 1, cb = 32 * (lane & 1);
    float v[32];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(&os[i * OP + cb + 4 * t]);
      v[4 * t] = x[0];
      v[4 * t + 1] = x[1];
      v[4 * t + 2] = x[2];
      v[4 * t + 3] = x[3];
    }
    float am = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t) am = fmaxf(am, fabsf(v[t]));
    const int p = gpp::mx_exponent(am);
    const float sc = ldexpf(1.f, -p);
    uint32_t w[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      uint32_t x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * t] * sc, v[4 * t + 1] * sc, 0u, false);
      w[t] = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * t + 2] * sc, v[4 * t + 3] * sc, x, true);
    }
    if (32 * ib + i >= Lr) return;
    const int64_t row = (int64_t)b * Lr + 32 * ib + i;
    uint4* dst = reinterpret_cast<uint4*>(ctx8 + row * H + a * DH + cb);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    cs[gpp::mx_scale_index(row, a * DH + cb, mpad)] = (unsigned char)(p + 127);
    return;
  }
  unsigned short* out = ctx + ((int64_t)b * Lr + 32 * ib) * H + a * DH;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int i = (e & 3) + 8 * (e >> 2) + 4 * h;
      if (32 * ib + i < Lr) out[(int64_t)i * H + 32 * db + r32] = f32_to_bf16(o[db][e]);
    }
}

// Long-sequence MFMA attention (bf16 QKV, head dim 64, any L; attention_mfma_kernel
// holds a whole row of scores in registers and covers L <= 128, this one streams the
// keys, for the joint padding of a batch up to 512 tokens, contrastive_module.py:38).
// One wave per (sequence, head, block of 32 queries), no workgroup barrier; keys in
// tiles of 32 with an online softmax:
//  * S^T tile = K Q^T on v_mfma_f32_32x32x16_bf16 as attention_mfma_kernel: lane
//    (i, half) holds query i's scores for keys (e&3) + 8(e>>2) + 4*half of the tile;
//  * running (max, sum) per query, lane-local plus one exchange with lane ^ 32;
//  * O^T = V^T P^T: P goes from registers into the B operand (lane = query), so the
//    rescale of the accumulator by exp(m_old - m_new) is lane-local; the A operand is
//    the tile's V^T read from this wave's LDS slot in the lanes' permuted key order;
//  * key bias per tile (0 / -1e30 masked / -3e30 past L): masked keys get exactly
//    zero weight, an all-masked row averages its L keys (HF's finfo.min bias);
//  * probabilities rounded to bf16 before P.V (unnormalised, <= 1), O / sum at the end;
//  * the next tile's K fragments and V rows are loaded while this tile computes.
//  * MXO (config C5): the context leaves as MX-fp8 (e4m3 ctx8 [B*L][H], one E8M0
//    scale per (token, 32 head columns) in the MX layout with mpad rows), the values
//    rounded to bf16 first, so the codes equal quantising the bf16 context.
template <bool MXO>
__global__ __launch_bounds__(256) void attention_flash_kernel(
    const unsigned short* __restrict__ qkv, const int64_t* __restrict__ mask,
    unsigned short* __restrict__ ctx, int B, int L, int H, int heads, float scale,
    unsigned char* __restrict__ ctx8, unsigned char* __restrict__ cs, int64_t mpad) {
  constexpr int DH = 64, VP = 36;  // V^T tile row pitch (u16): 8-byte aligned b64 reads
  __shared__ __attribute__((aligned(16))) unsigned short vt[4][DH][VP];
  __shared__ __attribute__((aligned(16))) float mb[4][32];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int nqb = (L + 31) / 32;
  const int64_t item = (int64_t)blockIdx.x * 4 + wv;  // (b, head, ib), ib fastest
  if (item >= (int64_t)B * heads * nqb) return;       // no workgroup barrier below
  const int ib = (int)(item % nqb);
  const int a = (int)(item / nqb % heads);
  const int b = (int)(item / nqb / heads);
  const int64_t ld3 = 3LL * H;
  const unsigned short* base = qkv + (int64_t)b * L * ld3 + a * DH;  // + j*ld3: Q | +H: K | +2H: V
  const int64_t* mrow = mask == nullptr ? nullptr : mask + (int64_t)b * L;

  bf16x8 qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
    qf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)min(32 * ib + r32, L - 1) * ld3 +
                                               16 * kk + 8 * h);
  // tile loads: K fragments (row 32jt + r32, clamped), V rows for the V^T image
  // (lane -> key pair 2*(lane >> 3) + {0, 1} + 16*u, 8-wide d chunk lane & 7), mask
  const int dc = lane & 7, jp = (lane >> 3) * 2;
  bf16x8 kf[4];
  u16x8 vr[2][2];
  float mbias = 0.f;
  auto load_tile = [&](int jt) {
    const int j0 = 32 * jt;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      kf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)min(j0 + r32, L - 1) * ld3 + H +
                                                 16 * kk + 8 * h);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const int j = j0 + 16 * u + jp + w;
        vr[u][w] = j < L ? *reinterpret_cast<const u16x8*>(base + (int64_t)j * ld3 + 2 * H + dc * 8)
                         : (u16x8)0;
      }
    const int jm = j0 + r32;
    mbias = jm >= L ? -3e30f : ((mrow == nullptr || mrow[jm] != 0) ? 0.f : -1e30f);
  };

  f32x16 o[2] = {(f32x16)0.f, (f32x16)0.f};  // O^T: lane = query, rows d
  float m = -INFINITY, l = 0.f;
  const int nkt = (L + 31) / 32;
  load_tile(0);
  for (int jt = 0; jt < nkt; ++jt) {
    // this tile's V^T and key bias into the wave's LDS slot (the previous tile's
    // reads were consumed by its MFMAs: LDS operations of a wave complete in order)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int dd = 0; dd < 8; ++dd)
        *reinterpret_cast<uint32_t*>(&vt[wv][dc * 8 + dd][16 * u + jp]) =
            (uint32_t)vr[u][0][dd] | ((uint32_t)vr[u][1][dd] << 16);
    if (h == 0) mb[wv][r32] = mbias;
    f32x16 s = (f32x16)0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kk], qf[kk], s, 0, 0, 0);
    if (jt + 1 < nkt) load_tile(jt + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    float tmx = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 bias = *reinterpret_cast<const f32x4*>(&mb[wv][8 * q + 4 * h]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s[4 * q + r] * scale + bias[r];
        s[4 * q + r] = v;
        tmx = fmaxf(tmx, v);
      }
    }
    tmx = fmaxf(tmx, __shfl_xor(tmx, 32, 64));
    const float mn = fmaxf(m, tmx);
    const float corr = __expf(m - mn);  // 0 on the first tile (m = -inf)
    float ts = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float p = __expf(s[e] - mn);
      s[e] = p;
      ts += p;
    }
    ts += __shfl_xor(ts, 32, 64);
    l = l * corr + ts;
    m = mn;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) o[db][e] *= corr;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      bf16x8 pb;
#pragma unroll
      for (int t = 0; t < 8; ++t) pb[t] = (__bf16)s[8 * k2 + t];
      const int j0 = 16 * k2 + 4 * h;  // keys of slots t<4: j0+t; t>=4: j0+8+t-4
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const int d = 32 * db + r32;
        const u16x4 lo = *reinterpret_cast<const u16x4*>(&vt[wv][d][j0]);
        const u16x4 hi = *reinterpret_cast<const u16x4*>(&vt[wv][d][j0 + 8]);
        const u16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, vv), pb, o[db],
                                                        0, 0, 0);
      }
    }
  }
  // O^T C layout: lane column = query 32ib + r32; rows d = 32db + 8q + 4h + r (e = 4q + r)
  const int i = 32 * ib + r32;
  const float inv = 1.f / l;
  const int64_t row = (int64_t)b * L + i;
  if constexpr (MXO) {
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      float v[16];
      float am = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        v[e] = bf16_to_f32(f32_to_bf16(o[db][e] * inv));
        am = fmaxf(am, fabsf(v[e]));
      }
      am = fmaxf(am, __shfl_xor(am, 32, 64));  // the 32-column block: both halves
      const int p = gpp::mx_exponent(am);
      const float sc = ldexpf(1.f, -p);
      if (i < L) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q] * sc, v[4 * q + 1] * sc, 0u, false);
          x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * q + 2] * sc, v[4 * q + 3] * sc, x, true);
          *reinterpret_cast<uint32_t*>(ctx8 + row * H + a * DH + 32 * db + 8 * q + 4 * h) = x;
        }
        if (h == 0) cs[gpp::mx_scale_index(row, a * DH + 32 * db, mpad)] = (unsigned char)(p + 127);
      }
    }
    return;
  }
  if (i >= L) return;
  unsigned short* out = ctx + row * H + a * DH;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint2 w;
      w.x = (uint32_t)f32_to_bf16(o[db][4 * q] * inv) | ((uint32_t)f32_to_bf16(o[db][4 * q + 1] * inv) << 16);
      w.y = (uint32_t)f32_to_bf16(o[db][4 * q + 2] * inv) |
            ((uint32_t)f32_to_bf16(o[db][4 * q + 3] * inv) << 16);
      *reinterpret_cast<uint2*>(out + 32 * db + 8 * q + 4 * h) = w;
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
  const bool al = ((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 16) == 0 &&
                  ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0;
  if (dtype == 0 && al && (H == 768 || H == 1024 || H == 512)) {
    hipStream_t st = as_stream(stream);
    prof_begin(st);
    // 4 rows per half-wave: 15.9 vs 17.7 us over [32768, 768] for the one-row
    // layernorm_vec_kernel (6.35 vs 5.70 TB/s, bit-identical; profiles/r04_w_ln_rows.txt)
    const dim3 g32((unsigned)((rows + 31) / 32));
    if (H == 768)
      hipLaunchKernelGGL((enc::layernorm_rows_kernel<3, 4>), g32, dim3(256), 0, st,
                         (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps);
    else if (H == 1024)
      hipLaunchKernelGGL((enc::layernorm_rows_kernel<4, 4>), g32, dim3(256), 0, st,
                         (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps);
    else
      hipLaunchKernelGGL((enc::layernorm_rows_kernel<2, 4>), g32, dim3(256), 0, st,
                         (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps);
    prof_end("layernorm", st, (double)rows * H * 4.0);
    return check_launch("layernorm_vec_kernel");
  }
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

// LayerNorm (bf16, H in {512, 768, 1024}) that also emits the MX-fp8 copy of its
// output (config C5): y bf16 as irc_layernorm, y8 e4m3 [rows][H] and ys E8M0 block
// scales in the MX layout with mpad (>= rows rounded up to 256) rows.
extern "C" int irc_layernorm_mx(const void* x, void* y, const float* gamma, const float* beta,
                                int64_t rows, int64_t H, float eps, void* y8, void* ys,
                                int64_t mpad, irc_stream_t stream) {
  IRC_REQUIRE(H == 512 || H == 768 || H == 1024, "layernorm_mx: H=%lld unsupported", (long long)H);
  IRC_REQUIRE(mpad >= (rows + 255) / 256 * 256, "layernorm_mx: mpad must cover rows rounded to 256");
  IRC_REQUIRE((((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta |
                (uintptr_t)y8) % 16) == 0, "layernorm_mx: 16-byte aligned operands required");
  if (rows == 0) return IRC_OK;
  const dim3 g8((unsigned)((rows + 7) / 8));
  hipStream_t st = as_stream(stream);
  prof_begin(st);
  auto* yy8 = static_cast<unsigned char*>(y8);
  auto* yys = static_cast<unsigned char*>(ys);
  // one row per half-wave: the 4-rows kernel with the MX outputs measured no faster
  // (C5 step 29.2k / 29.2k vs 29.3k / 29.3k pairs/s, profiles/r04_y_ln_mx_rows.txt)
  if (H == 768)
    hipLaunchKernelGGL((enc::layernorm_vec_kernel<3>), g8, dim3(256), 0, st,
                       (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps, yy8,
                       yys, mpad);
  else if (H == 1024)
    hipLaunchKernelGGL((enc::layernorm_vec_kernel<4>), g8, dim3(256), 0, st,
                       (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps, yy8,
                       yys, mpad);
  else
    hipLaunchKernelGGL((enc::layernorm_vec_kernel<2>), g8, dim3(256), 0, st,
                       (const unsigned short*)x, (unsigned short*)y, gamma, beta, rows, eps, yy8,
                       yys, mpad);
  prof_end("layernorm", st, (double)rows * H * 5.0);
  return check_launch("layernorm_mx");
}

// MFMA attention (bf16 QKV, head dim 64, any L) whose context
// leaves as MX-fp8 (ctx8 e4m3 [B*L][H], cs E8M0 scales in the MX layout, mpad rows):
// the fp8 out-projection's A operand (config C5).
extern "C" int irc_attention_mx(const void* qkv, const int64_t* mask, void* ctx8, void* cs,
                                int64_t mpad, int64_t B, int64_t L, int64_t H, int64_t heads,
                                irc_stream_t stream) {
  IRC_REQUIRE(heads >= 1 && H % heads == 0 && H / heads == 64 && L >= 1,
              "attention_mx: head dim 64 required");
  IRC_REQUIRE(mpad >= (B * L + 255) / 256 * 256, "attention_mx: mpad must cover B*L rounded to 256");
  IRC_REQUIRE((uintptr_t)ctx8 % 16 == 0 && H % 16 == 0, "attention_mx: 16-byte aligned ctx8 rows");
  if (B == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const int64_t waves = B * heads * ((L + 31) / 32);
  const dim3 grid((unsigned)((waves + 3) / 4));
  const float sc = 0.125f;
  auto* c8 = static_cast<unsigned char*>(ctx8);
  auto* css = static_cast<unsigned char*>(cs);
  prof_begin(st);
  if (L > 128) {  // keys streamed (online softmax)
    hipLaunchKernelGGL((enc::attention_flash_kernel<true>), grid, dim3(256), 0, st,
                       (const unsigned short*)qkv, mask, (unsigned short*)nullptr, (int)B, (int)L,
                       (int)H, (int)heads, sc, c8, css, mpad);
    prof_end("attention", st, (double)B * L * (3 * H * 2.0 + H));
    return check_launch("attention_mx");
  }
  switch ((L + 31) / 32) {
#define IRC_ATTX(NJ)                                                                             \
  case NJ:                                                                                       \
    hipLaunchKernelGGL((enc::attention_mfma_kernel<NJ, true>), dim3((unsigned)(B * heads)),    \
                       dim3(64 * NJ), 0, st,                                                     \
                       (const unsigned short*)qkv, mask, (unsigned short*)nullptr, (int)B, (int)H, \
                       (int)heads, sc, c8, css, mpad, (int)L);                                   \
    break;
    IRC_ATTX(1) IRC_ATTX(2) IRC_ATTX(3) IRC_ATTX(4)
#undef IRC_ATTX
  }
  prof_end("attention", st, (double)B * L * (3 * H * 2.0 + H));
  return check_launch("attention_mx");
}

extern "C" int irc_embed_ln(int dtype, const int64_t* ids, const void* word, const void* pos,
                            const void* type0, const float* gamma, const float* beta, void* y,
                            int64_t rows, int64_t L, int64_t H, float eps, irc_stream_t stream) {
  IRC_REQUIRE(H >= 1 && H <= 64 * enc::MAXH_PER_LANE, "embed_ln: H=%lld unsupported",
              (long long)H);
  if (rows == 0) return IRC_OK;
  const bool al = ((((uintptr_t)word | (uintptr_t)pos | (uintptr_t)type0 | (uintptr_t)y |
                     (uintptr_t)gamma | (uintptr_t)beta) % 16) == 0);
  if (dtype == 0 && al && (H == 768 || H == 1024)) {
    const dim3 g8((unsigned)((rows + 7) / 8));
    hipStream_t st = as_stream(stream);
    if (H == 768)
      hipLaunchKernelGGL((enc::embed_ln_vec_kernel<3>), g8, dim3(256), 0, st, ids,
                         (const unsigned short*)word, (const unsigned short*)pos,
                         (const unsigned short*)type0, gamma, beta, (unsigned short*)y, rows,
                         (int)L, eps);
    else
      hipLaunchKernelGGL((enc::embed_ln_vec_kernel<4>), g8, dim3(256), 0, st, ids,
                         (const unsigned short*)word, (const unsigned short*)pos,
                         (const unsigned short*)type0, gamma, beta, (unsigned short*)y, rows,
                         (int)L, eps);
    return check_launch("embed_ln_vec_kernel");
  }
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
  const int64_t nqc = (L + 255) / 256;
  hipLaunchKernelGGL((enc::attention_kernel<T, DH>), dim3((unsigned)(B * heads * nqc)), dim3(256), 0,
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
  IRC_REQUIRE(L >= 1, "attention: L=%lld", (long long)L);
  if (B == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  if (dtype == 0 && dh == 64) {  // production shape: MFMA, any L
    const int64_t waves = B * heads * ((L + 31) / 32);
    const dim3 grid((unsigned)((waves + 3) / 4));
    const float sc = 0.125f;  // 1/sqrt(64)
    prof_begin(st);
    if (L > 128) {  // whole score rows no longer fit in registers: keys streamed
      hipLaunchKernelGGL((enc::attention_flash_kernel<false>), grid, dim3(256), 0, st,
                         (const unsigned short*)qkv, mask, (unsigned short*)ctx, (int)B, (int)L,
                         (int)H, (int)heads, sc, (unsigned char*)nullptr, (unsigned char*)nullptr,
                         (int64_t)0);
      prof_end("attention", st, (double)B * L * (3 * H + H) * 2.0);
      return check_launch("attention_flash_kernel");
    }
    switch ((L + 31) / 32) {
#define IRC_ATTB(NJ)                                                                             \
  case NJ:                                                                                       \
    hipLaunchKernelGGL(enc::attention_mfma_kernel<NJ>, dim3((unsigned)(B * heads)), dim3(64 * NJ), \
                       0, st,                                                                    \
                       (const unsigned short*)qkv, mask, (unsigned short*)ctx, (int)B, (int)H,   \
                       (int)heads, sc, (unsigned char*)nullptr, (unsigned char*)nullptr,         \
                       (int64_t)0, (int)L);                                                      \
    break;
      IRC_ATTB(1) IRC_ATTB(2) IRC_ATTB(3) IRC_ATTB(4)
#undef IRC_ATTB
    }
    // algorithmic bytes: QKV read once + ctx written
    prof_end("attention", st, (double)B * L * (3 * H + H) * 2.0);
    return check_launch("attention_mfma_kernel");
  }
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
