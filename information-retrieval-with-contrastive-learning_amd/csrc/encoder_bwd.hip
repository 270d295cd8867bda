// Backward of the BERT-style encoder for the trainable bi-encoder mode
// (`--model BERT`, SURVEY.md 8d: the north star's "encoder forward/backward").
// The reference's encoder is HF BertModel reached from
// src/contrastor/contrastive_module.py:36-41 / 96-99 (run frozen there); these
// kernels are the gradients of exactly that forward (csrc/encoder.hip):
//  * layernorm_bwd: dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma, plus
//    dgamma = sum dy xhat and dbeta = sum dy as deterministic two-pass column sums.
//    The statistics are recomputed from the saved LN input (the residual sum).
//    dy may be broadcast from [rows / bL] rows (the mean-pool backward folded in).
//  * attention_bwd: dQ, dK, dV of softmax(Q K^T * scale + key bias) V per
//    (sequence, head), with P recomputed; MFMA for bf16 head dim 64, L <= 128.
//  * embed_bwd: scatter of the embedding-LN input gradient into the word table
//    (fp32 atomics; the padding row gets none, as nn.Embedding(padding_idx)),
//    position table and token-type row 0 (deterministic fixed-order sums).
#include "irc_common.h"

namespace irc {
namespace encb {

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

constexpr int MAXH_PER_LANE = 32;  // generic kernel: H <= 2048
constexpr int LNB_ROWS = 32;       // rows per block, generic kernel
constexpr int LNV_ROWS = 64;       // rows per block, vector kernel

// ---------------------------------------------------------------- LayerNorm bwd
// Generic: one wave per row, the row in registers (H/64 per lane).
template <typename T, typename TD>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD* __restrict__ dy,
                                                    const T* __restrict__ x,
                                                    const float* __restrict__ gamma,
                                                    T* __restrict__ dx,
                                                    float* __restrict__ partial, int64_t rows,
                                                    int H, float eps, int64_t bL, float dscale) {
  extern __shared__ float sred[];  // [2][H]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int per = (H + 63) / 64;
  float accg[MAXH_PER_LANE], accb[MAXH_PER_LANE];
#pragma unroll
  for (int i = 0; i < MAXH_PER_LANE; ++i) accg[i] = accb[i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * LNB_ROWS;
  for (int rr = wv; rr < LNB_ROWS; rr += 4) {
    const int64_t row = r0 + rr;
    if (row >= rows) break;
    const int64_t drow = bL > 0 ? row / bL : row;
    const float dsc = bL > 0 ? dscale : 1.f;
    float xv[MAXH_PER_LANE], gv[MAXH_PER_LANE];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXH_PER_LANE; ++i) {
      if (i >= per) break;
      const int c = i * 64 + lane;
      xv[i] = c < H ? ld(x, row * H + c) : 0.f;
      s += xv[i];
    }
    const float mean = warp_sum(s) / H;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXH_PER_LANE; ++i) {
      if (i >= per) break;
      const int c = i * 64 + lane;
      const float d = c < H ? xv[i] - mean : 0.f;
      s2 += d * d;
    }
    const float rstd = rsqrtf(warp_sum(s2) / H + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < MAXH_PER_LANE; ++i) {
      if (i >= per) break;
      const int c = i * 64 + lane;
      if (c < H) {
        const float xh = (xv[i] - mean) * rstd;
        const float d = ld(dy, drow * H + c) * dsc;
        accg[i] += d * xh;
        accb[i] += d;
        const float g = d * gamma[c];
        gv[i] = g;
        xv[i] = xh;
        sg += g;
        sgx += g * xh;
      } else {
        gv[i] = 0.f;
        xv[i] = 0.f;
      }
    }
    const float mg = warp_sum(sg) / H, mgx = warp_sum(sgx) / H;
#pragma unroll
    for (int i = 0; i < MAXH_PER_LANE; ++i) {
      if (i >= per) break;
      const int c = i * 64 + lane;
      if (c < H) st(dx, row * H + c, rstd * (gv[i] - mg - xv[i] * mgx));
    }
  }
  // fixed-order block reduction of the column partials (wave 0, 1, 2, 3)
  for (int w = 0; w < 4; ++w) {
    if (wv == w) {
#pragma unroll
      for (int i = 0; i < MAXH_PER_LANE; ++i) {
        if (i >= per) break;
        const int c = i * 64 + lane;
        if (c < H) {
          sred[c] = w == 0 ? accg[i] : sred[c] + accg[i];
          sred[H + c] = w == 0 ? accb[i] : sred[H + c] + accb[i];
        }
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < 2 * H; c += blockDim.x)
    partial[(int64_t)blockIdx.x * 2 * H + c] = sred[c];
}

// bf16, H = 256*CPL: one half-wave per row, 16-byte accesses (layernorm_vec_kernel's
// lane map), each lane owning the same 8*CPL columns on every row so the gamma /
// beta partials stay in registers across the block's 64 rows.
template <int CPL, typename TD>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(const TD* __restrict__ dy,
                                                        const unsigned short* __restrict__ x,
                                                        const float* __restrict__ gamma,
                                                        unsigned short* __restrict__ dx,
                                                        float* __restrict__ partial, int64_t rows,
                                                        float eps, int64_t bL, float dscale) {
  constexpr int H = CPL * 256;
  __shared__ float sred[2 * H];
  const int lane = threadIdx.x & 63, hl = lane & 31, half = lane >> 5, wv = threadIdx.x >> 6;
  float ag[CPL][8], ab[CPL][8], gg[CPL][8];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c0 = (i * 32 + hl) * 8;
    const f32x4 g0 = *reinterpret_cast<const f32x4*>(gamma + c0);
    const f32x4 g1 = *reinterpret_cast<const f32x4*>(gamma + c0 + 4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      gg[i][t] = g0[t];
      gg[i][t + 4] = g1[t];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) ag[i][t] = ab[i][t] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * LNV_ROWS;
  for (int p = 0; p < LNV_ROWS / 8; ++p) {
    const int64_t row = r0 + p * 8 + wv * 2 + half;
    const bool ok = row < rows;
    const int64_t rr = ok ? row : 0;
    const int64_t drow = bL > 0 ? rr / bL : rr;
    const float dsc = bL > 0 ? dscale : 1.f;
    float v[CPL][8], d[CPL][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c0 = (i * 32 + hl) * 8;
      const u16x8 u = *reinterpret_cast<const u16x8*>(x + rr * H + c0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        v[i][t] = bf16_to_f32(u[t]);
        s += v[i][t];
      }
      if constexpr (sizeof(TD) == 2) {
        const u16x8 w = *reinterpret_cast<const u16x8*>(
            reinterpret_cast<const unsigned short*>(dy) + drow * H + c0);
#pragma unroll
        for (int t = 0; t < 8; ++t) d[i][t] = bf16_to_f32(w[t]) * dsc;
      } else {
        const float* dr = reinterpret_cast<const float*>(dy) + drow * H + c0;
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(dr);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(dr + 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          d[i][t] = w0[t] * dsc;
          d[i][t + 4] = w1[t] * dsc;
        }
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
        const float q = v[i][t] - mean;
        s2 += q * q;
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
    const float rstd = rsqrtf(s2 / H + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const float xh = (v[i][t] - mean) * rstd;
        v[i][t] = xh;
        const float g = d[i][t] * gg[i][t];
        sg += g;
        sgx += g * xh;
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      sg += __shfl_xor(sg, o, 64);
      sgx += __shfl_xor(sgx, o, 64);
    }
    const float mg = sg / H, mgx = sgx / H;
    if (ok) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        u16x8 o;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          ag[i][t] += d[i][t] * v[i][t];
          ab[i][t] += d[i][t];
          o[t] = f32_to_bf16(rstd * (d[i][t] * gg[i][t] - mg - v[i][t] * mgx));
        }
        *reinterpret_cast<u16x8*>(dx + row * H + (i * 32 + hl) * 8) = o;
      }
    }
  }
  // the two half-waves own the same columns: fold, then waves in fixed order
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      ag[i][t] += __shfl_xor(ag[i][t], 32, 64);
      ab[i][t] += __shfl_xor(ab[i][t], 32, 64);
    }
  for (int w = 0; w < 4; ++w) {
    if (wv == w && half == 0) {
#pragma unroll
      for (int i = 0; i < CPL; ++i)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int c = (i * 32 + hl) * 8 + t;
          sred[c] = w == 0 ? ag[i][t] : sred[c] + ag[i][t];
          sred[H + c] = w == 0 ? ab[i][t] : sred[H + c] + ab[i][t];
        }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x; c < 2 * H; c += blockDim.x)
    partial[(int64_t)blockIdx.x * 2 * H + c] = sred[c];
}

// Two-stage fixed-order reduction of the per-block partials [nblk][2H]:
// stage 1: partial2[j][c] = sum of rows j*per .. j*per+per-1 (grid (2H/256, S));
// stage 2: dgamma[c] / dbeta[c] (+)= sum_j partial2[j][c] (j ascending).
constexpr int LNF_S = 32;
__global__ void ln_bwd_stage1_kernel(const float* __restrict__ partial, int nblk, int H, int per,
                                     float* __restrict__ partial2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * H) return;
  const int b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  float s = 0.f;
  for (int b = b0; b < b1; ++b) s += partial[(int64_t)b * 2 * H + c];
  partial2[(int64_t)blockIdx.y * 2 * H + c] = s;
}

__global__ void ln_bwd_final_kernel(const float* __restrict__ partial2, int ns, int H,
                                    float* __restrict__ dgamma, float* __restrict__ dbeta,
                                    int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * H) return;
  float s = 0.f;
  for (int j = 0; j < ns; ++j) s += partial2[(int64_t)j * 2 * H + c];
  float* out = c < H ? dgamma + c : dbeta + (c - H);
  *out = accumulate ? *out + s : s;
}

// ---------------------------------------------------------------- attention bwd
// Generic (any element type, DH <= 128, any L): one workgroup per (sequence, head),
// K / V (phase 1) and Q / dO (phase 2) streamed through LDS as fp32 tiles of BKT
// rows, the per-query statistics in dynamic LDS (3 L floats), so nothing L x L is
// stored.  Phase 1, thread = query i: the row max m_i and sum l_i of the softmax with
// the additive key bias (as the forward), D_i = dO_i . O_i, then P_ij, dS_ij = P_ij
// (dO_i . V_j - D_i) and dQ_i = scale sum_j dS_ij K_j.  Phase 2, thread = key j:
// P_ij and dS_ij recomputed from the saved statistics, dK_j = scale sum_i dS_ij Q_i,
// dV_j = sum_i P_ij dO_i.
constexpr int BKT = 32;
constexpr int DH_MF = 64;
template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const T* __restrict__ qkv,
                                                      const int64_t* __restrict__ mask,
                                                      const T* __restrict__ ctx,
                                                      const T* __restrict__ dctx,
                                                      T* __restrict__ dqkv, int L, int H,
                                                      int heads, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float A_s[BKT][DH];  // K (phase 1) / Q (phase 2)
  __shared__ __attribute__((aligned(16))) float B_s[BKT][DH];  // V (phase 1) / dO (phase 2)
  __shared__ float bt[BKT];
  float* mrow = reinterpret_cast<float*>(smem);  // [L]
  float* irow = mrow + L;
  float* drow = irow + L;
  const int b = blockIdx.x / heads, a = blockIdx.x % heads;
  const int64_t base = (int64_t)b * L;
  const int64_t ld3 = 3LL * H;
  const int tid = threadIdx.x;
  // phase 1: queries
  for (int i0 = 0; i0 < L; i0 += blockDim.x) {
    const int i = i0 + tid;
    const bool act = i < L;
    const int ic = act ? i : L - 1;
    float qv[DH], dov[DH], dq[DH];
    float Di = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      qv[d] = ld(qkv, (base + ic) * ld3 + a * DH + d);
      dov[d] = ld(dctx, (base + ic) * H + a * DH + d);
      Di += dov[d] * ld(ctx, (base + ic) * H + a * DH + d);
      dq[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int pass = 0; pass < 3; ++pass) {  // 0: max, 1: sum, 2: dS and dQ
      const float inv = 1.f / l;
      for (int j0 = 0; j0 < L; j0 += BKT) {
        const int n = min(BKT, L - j0);
        __syncthreads();
        for (int e = tid; e < n * DH; e += blockDim.x) {
          const int j = e / DH, d = e % DH;
          A_s[j][d] = ld(qkv, (base + j0 + j) * ld3 + H + a * DH + d);
          if (pass == 2) B_s[j][d] = ld(qkv, (base + j0 + j) * ld3 + 2 * H + a * DH + d);
        }
        for (int j = tid; j < n; j += blockDim.x)
          bt[j] = (mask == nullptr || mask[base + j0 + j] != 0) ? 0.f : -1e30f;
        __syncthreads();
        for (int t = 0; t < n; ++t) {
          float s = 0.f;
#pragma unroll
          for (int d = 0; d < DH; ++d) s += qv[d] * A_s[t][d];
          s = s * scale + bt[t];
          if (pass == 0) {
            m = fmaxf(m, s);
          } else if (pass == 1) {
            l += __expf(s - m);
          } else {
            const float p = __expf(s - m) * inv;
            float dp = 0.f;
#pragma unroll
            for (int d = 0; d < DH; ++d) dp += dov[d] * B_s[t][d];
            const float ds = p * (dp - Di);
#pragma unroll
            for (int d = 0; d < DH; ++d) dq[d] += ds * A_s[t][d];
          }
        }
      }
    }
    if (act) {
      mrow[i] = m;
      irow[i] = 1.f / l;
      drow[i] = Di;
#pragma unroll
      for (int d = 0; d < DH; ++d) st(dqkv, (base + i) * ld3 + a * DH + d, dq[d] * scale);
    }
  }
  // phase 2: keys
  for (int j00 = 0; j00 < L; j00 += blockDim.x) {
    const int j = j00 + tid;
    const bool act = j < L;
    const int jc = act ? j : L - 1;
    float kv[DH], vv[DH], dk[DH], dv[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      kv[d] = ld(qkv, (base + jc) * ld3 + H + a * DH + d);
      vv[d] = ld(qkv, (base + jc) * ld3 + 2 * H + a * DH + d);
      dk[d] = dv[d] = 0.f;
    }
    const float bj = (mask == nullptr || mask[base + jc] != 0) ? 0.f : -1e30f;
    for (int q0 = 0; q0 < L; q0 += BKT) {
      const int n = min(BKT, L - q0);
      __syncthreads();  // phase 1's statistics / the previous tile's readers
      for (int e = tid; e < n * DH; e += blockDim.x) {
        const int r = e / DH, d = e % DH;
        A_s[r][d] = ld(qkv, (base + q0 + r) * ld3 + a * DH + d);
        B_s[r][d] = ld(dctx, (base + q0 + r) * H + a * DH + d);
      }
      __syncthreads();
      for (int t = 0; t < n; ++t) {
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          s += A_s[t][d] * kv[d];
          dp += B_s[t][d] * vv[d];
        }
        const float p = __expf(s * scale + bj - mrow[q0 + t]) * irow[q0 + t];
        const float ds = p * (dp - drow[q0 + t]);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          dk[d] += ds * A_s[t][d];
          dv[d] += p * B_s[t][d];
        }
      }
    }
    if (act) {
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        st(dqkv, (base + j) * ld3 + H + a * DH + d, dk[d] * scale);
        st(dqkv, (base + j) * ld3 + 2 * H + a * DH + d, dv[d]);
      }
    }
  }
}

// Rows (r, r + 1) of column c, held by this lane as v0 / v1 (32x32 accumulator elements e,
// e + 1 for even e), leave as ONE 4-byte store: the DPP neighbour swap (quad_perm
// [1,0,3,2]: lane ^ 1 holds column c ^ 1) gives the even lane columns (c, c + 1) of row r and
// the odd lane those of row r + 1 -- half the store instructions of per-element 2-byte
// stores, same bytes.  row_r points at row r's element of column 0 of the lane's column
// block; ld is the row stride.
// rows_left: rows r, r + 1, ... that exist (Lr - r); a lane whose row does not is not stored
// (the exchange itself needs every lane).
__device__ __forceinline__ void store_row_pair(unsigned short* row_r, int64_t ld, int c, float v0,
                                               float v1, int lane, int rows_left = 2) {
  const uint32_t w = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
  const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, false);
  const int odd = lane & 1;
  const uint32_t v = odd ? ((x >> 16) | (w & 0xFFFF0000u)) : ((w & 0xFFFFu) | (x << 16));
  if (odd < rows_left) *reinterpret_cast<uint32_t*>(row_r + odd * ld + c - odd) = v;
}

// MFMA (bf16, DH = 64, L <= 32*NJ): one workgroup of NJ waves per (sequence, head).
// The 32x32x16 C layout of X^T (rows j, lanes = columns i) is, with the k order
// permuted, the A operand of X (rows i, k over j) -- the forward's P.V trick --
// so the backward needs both orientations:
//  phase A, wave = query block (lanes = queries): S^T = K Q^T -> row softmax
//    (lane-local), saves (max, 1/sum) per query, D_i = dO_i . O_i,
//    dP^T = V dO^T, dS^T = P^T (dP^T - D), dQ = scale dS K (K^T from LDS);
//  phase B, wave = key block (lanes = keys): S = Q K^T, P from the saved row
//    statistics, dP = dO V^T, dS, dV = P^T dO and dK = scale dS^T Q (dO^T, Q^T
//    from LDS).
template <int NJ, bool PART = false>  // PART: L not a multiple of 32 (rows past Lr)
__global__ __launch_bounds__(64 * NJ) void attn_bwd_mfma_kernel(
    const unsigned short* __restrict__ qkv, const int64_t* __restrict__ mask,
    const unsigned short* __restrict__ ctx, const unsigned short* __restrict__ dctx,
    unsigned short* __restrict__ dqkv, int H, int heads, float scale, int Lr = 32 * NJ) {
  constexpr int L = 32 * NJ, DH = 64;
  constexpr int VP = L + 4;  // transposed-tile row pitch (u16)
  __shared__ __attribute__((aligned(16))) unsigned short kT[DH][VP];
  __shared__ __attribute__((aligned(16))) unsigned short qT[DH][VP];
  __shared__ __attribute__((aligned(16))) unsigned short oT[DH][VP];
  __shared__ __attribute__((aligned(16))) float mb[L];
  __shared__ __attribute__((aligned(16))) float mrow[L];
  __shared__ __attribute__((aligned(16))) float irow[L];
  __shared__ __attribute__((aligned(16))) float drow[L];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int b = blockIdx.x / heads, a = blockIdx.x % heads;
  const int64_t ld3 = 3LL * H;
  // Lr <= L rows per sequence (a batch padded to L not a multiple of 32): rows past Lr read
  // as zeros -- keys past Lr carry the -3e30 bias (P = 0), query rows past Lr have dO = 0,
  // so they add exactly nothing to dK / dV -- and are never stored
  const unsigned short* base = qkv + (int64_t)b * Lr * ld3 + a * DH;  // Q | +H: K | +2H: V
  const unsigned short* dob = dctx + (int64_t)b * Lr * H + a * DH;
  const unsigned short* ob = ctx + (int64_t)b * Lr * H + a * DH;
  unsigned short* gb = dqkv + (int64_t)b * Lr * ld3 + a * DH;
  const auto ld8 = [&](const unsigned short* p, int row) {
    if constexpr (PART) return row < Lr ? *reinterpret_cast<const u16x8*>(p) : (u16x8)0;
    return *reinterpret_cast<const u16x8*>(p);
  };
  const auto ldf = [&](const unsigned short* p, int row) {
    if constexpr (PART) return row < Lr ? *reinterpret_cast<const bf16x8*>(p) : (bf16x8)0;
    return *reinterpret_cast<const bf16x8*>(p);
  };
  const auto left = [&](int row) { return PART ? Lr - row : 2; };  // store_row_pair rows

  for (int p = threadIdx.x; p < (L / 2) * 8; p += 64 * NJ) {
    const int dc = p & 7, j = (p >> 3) * 2;
    const u16x8 k0 = ld8(base + (int64_t)j * ld3 + H + dc * 8, j);
    const u16x8 k1 = ld8(base + (int64_t)(j + 1) * ld3 + H + dc * 8, j + 1);
    const u16x8 q0 = ld8(base + (int64_t)j * ld3 + dc * 8, j);
    const u16x8 q1 = ld8(base + (int64_t)(j + 1) * ld3 + dc * 8, j + 1);
    const u16x8 o0 = ld8(dob + (int64_t)j * H + dc * 8, j);
    const u16x8 o1 = ld8(dob + (int64_t)(j + 1) * H + dc * 8, j + 1);
#pragma unroll
    for (int dd = 0; dd < 8; ++dd) {
      *reinterpret_cast<uint32_t*>(&kT[dc * 8 + dd][j]) = (uint32_t)k0[dd] | ((uint32_t)k1[dd] << 16);
      *reinterpret_cast<uint32_t*>(&qT[dc * 8 + dd][j]) = (uint32_t)q0[dd] | ((uint32_t)q1[dd] << 16);
      *reinterpret_cast<uint32_t*>(&oT[dc * 8 + dd][j]) = (uint32_t)o0[dd] | ((uint32_t)o1[dd] << 16);
    }
  }
  for (int j = threadIdx.x; j < L; j += 64 * NJ)
    mb[j] = j >= Lr ? -3e30f : ((mask == nullptr || mask[(int64_t)b * Lr + j] != 0) ? 0.f : -1e30f);
  __syncthreads();

  // ---------------- phase A: this wave's 32 queries
  {
    const int ib = wv;
    const int i = 32 * ib + r32;
    bf16x8 qf[4], df[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      qf[kk] = ldf(base + (int64_t)i * ld3 + 16 * kk + 8 * h, i);
      df[kk] = ldf(dob + (int64_t)i * H + 16 * kk + 8 * h, i);
    }
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u16x8 o8 = ld8(ob + (int64_t)i * H + 32 * h + 8 * c, i);
      const u16x8 d8 = ld8(dob + (int64_t)i * H + 32 * h + 8 * c, i);
#pragma unroll
      for (int t = 0; t < 8; ++t) dsum += bf16_to_f32(o8[t]) * bf16_to_f32(d8[t]);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    f32x16 s[NJ];
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) {
      s[jb] = (f32x16)0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 kf = ldf(base + (int64_t)(32 * jb + r32) * ld3 + H + 16 * kk + 8 * h,
                              32 * jb + r32);
        s[jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], s[jb], 0, 0, 0);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
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
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float p = __expf(s[jb][e] - mx);
        s[jb][e] = p;
        sum += p;
      }
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    if (h == 0) {
      mrow[i] = mx;
      irow[i] = inv;
      drow[i] = dsum;
    }
    // dS^T[j][i] = P^T[j][i] (dP^T[j][i] - D_i), dP^T = V dO^T
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb) {
      f32x16 dp = (f32x16)0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 vf = ldf(base + (int64_t)(32 * jb + r32) * ld3 + 2 * H + 16 * kk + 8 * h,
                              32 * jb + r32);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, df[kk], dp, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) s[jb][e] = s[jb][e] * inv * (dp[e] - dsum);
    }
    // dQ = scale dS K: A = dS (from the C layout of dS^T, permuted k = keys), B = K^T tile
    f32x16 o[2] = {(f32x16)0.f, (f32x16)0.f};
#pragma unroll
    for (int jb = 0; jb < NJ; ++jb)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        bf16x8 pa;
#pragma unroll
        for (int t = 0; t < 8; ++t) pa[t] = (__bf16)s[jb][8 * k2 + t];
        const int j0 = 32 * jb + 16 * k2 + 4 * h;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int d = 32 * db + r32;
          const u16x4 lo = *reinterpret_cast<const u16x4*>(&kT[d][j0]);
          const u16x4 hi = *reinterpret_cast<const u16x4*>(&kT[d][j0 + 8]);
          const u16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, vv),
                                                          o[db], 0, 0, 0);
        }
      }
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; e += 2) {  // rows ii, ii + 1 (e even): one paired store
        const int ii = 32 * ib + (e & 3) + 8 * (e >> 2) + 4 * h;
        store_row_pair(gb + (int64_t)ii * ld3, ld3, 32 * db + r32, o[db][e] * scale,
                       o[db][e + 1] * scale, lane, left(ii));
      }
  }
  __syncthreads();

  // ---------------- phase B: this wave's 32 keys
  {
    const int jb = wv;
    const int j = 32 * jb + r32;
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      kf[kk] = ldf(base + (int64_t)j * ld3 + H + 16 * kk + 8 * h, j);
      vf[kk] = ldf(base + (int64_t)j * ld3 + 2 * H + 16 * kk + 8 * h, j);
    }
    const float bj = mb[j];
    f32x16 dv[2] = {(f32x16)0.f, (f32x16)0.f};
    f32x16 dk[2] = {(f32x16)0.f, (f32x16)0.f};
#pragma unroll
    for (int ib = 0; ib < NJ; ++ib) {
      f32x16 sc = (f32x16)0.f, dp = (f32x16)0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 qa = ldf(base + (int64_t)(32 * ib + r32) * ld3 + 16 * kk + 8 * h,
                              32 * ib + r32);
        const bf16x8 da = ldf(dob + (int64_t)(32 * ib + r32) * H + 16 * kk + 8 * h,
                              32 * ib + r32);
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[kk], sc, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[kk], dp, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r0 = 32 * ib + 8 * q + 4 * h;
        const f32x4 mm = *reinterpret_cast<const f32x4*>(&mrow[r0]);
        const f32x4 iv = *reinterpret_cast<const f32x4*>(&irow[r0]);
        const f32x4 dd = *reinterpret_cast<const f32x4*>(&drow[r0]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 4 * q + r;
          const float p = __expf(sc[e] * scale + bj - mm[r]) * iv[r];
          sc[e] = p;
          dp[e] = p * (dp[e] - dd[r]);
        }
      }
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        bf16x8 pa, sa;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          pa[t] = (__bf16)sc[8 * k2 + t];
          sa[t] = (__bf16)dp[8 * k2 + t];
        }
        const int i0 = 32 * ib + 16 * k2 + 4 * h;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int d = 32 * db + r32;
          const u16x4 olo = *reinterpret_cast<const u16x4*>(&oT[d][i0]);
          const u16x4 ohi = *reinterpret_cast<const u16x4*>(&oT[d][i0 + 8]);
          const u16x8 ov = {olo[0], olo[1], olo[2], olo[3], ohi[0], ohi[1], ohi[2], ohi[3]};
          dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, ov),
                                                           dv[db], 0, 0, 0);
          const u16x4 qlo = *reinterpret_cast<const u16x4*>(&qT[d][i0]);
          const u16x4 qhi = *reinterpret_cast<const u16x4*>(&qT[d][i0 + 8]);
          const u16x8 qv = {qlo[0], qlo[1], qlo[2], qlo[3], qhi[0], qhi[1], qhi[2], qhi[3]};
          dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa, __builtin_bit_cast(bf16x8, qv),
                                                           dk[db], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        const int jj = 32 * jb + (e & 3) + 8 * (e >> 2) + 4 * h;
        store_row_pair(gb + (int64_t)jj * ld3 + H, ld3, 32 * db + r32, dk[db][e] * scale,
                       dk[db][e + 1] * scale, lane, left(jj));
        store_row_pair(gb + (int64_t)jj * ld3 + 2 * H, ld3, 32 * db + r32, dv[db][e],
                       dv[db][e + 1], lane, left(jj));
      }
  }
}

// MFMA (bf16, DH = 64, any L <= 512: the joint padding of a batch, e.g. L = 72 or 300;
// attn_bwd_mfma_kernel takes L <= 128): one workgroup of NW waves per
// (sequence, head), the same two phases with loops over 32-row blocks.  Dynamic LDS:
// the key bias and the per-query statistics [Lp] (Lp = L rounded up to 32), then one
// or two transposed [64][Lp + 4] bf16 images: K^T in phase A, Q^T and dO^T in phase B
// (140 KB at L = 512).
//  phase A, wave = query block: pass 1 the row max / sum (online) over key blocks,
//    pass 2 P, dP^T = V dO^T, dS^T and dQ = scale dS K per key block;
//  phase B, wave = key block: per query block S = Q K^T, P from the saved statistics,
//    dP = dO V^T, dS, dV += P^T dO, dK += scale dS^T Q.
// Rows past L: keys carry a -3e30 bias (P = 0), queries get (m, 1/l, D) = (3e30, 0, 0)
// and zero dO (P = dS = 0); reads are clamped and nothing past L is stored.
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_long_kernel(
    const unsigned short* __restrict__ qkv, const int64_t* __restrict__ mask,
    const unsigned short* __restrict__ ctx, const unsigned short* __restrict__ dctx,
    unsigned short* __restrict__ dqkv, int L, int H, int heads, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lp = (L + 31) & ~31, VP = Lp + 4, nb = Lp / 32;
  float* mb = reinterpret_cast<float*>(smem);
  float* mrow = mb + Lp;
  float* irow = mrow + Lp;
  float* drow = irow + Lp;
  unsigned short* T0 = reinterpret_cast<unsigned short*>(drow + Lp);  // K^T (A) / Q^T (B)
  unsigned short* T1 = T0 + 64 * VP;                                  // dO^T (B)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int b = blockIdx.x / heads, a = blockIdx.x % heads;
  const int64_t ld3 = 3LL * H;
  const unsigned short* base = qkv + (int64_t)b * L * ld3 + a * DH_MF;  // Q | +H: K | +2H: V
  const unsigned short* dob = dctx + (int64_t)b * L * H + a * DH_MF;
  const unsigned short* ob = ctx + (int64_t)b * L * H + a * DH_MF;
  unsigned short* gb = dqkv + (int64_t)b * L * ld3 + a * DH_MF;
  auto stage_t = [&](unsigned short* T, const unsigned short* src, int64_t ld) {
    for (int p = threadIdx.x; p < (Lp / 2) * 8; p += 64 * NW) {
      const int dc = p & 7, j = (p >> 3) * 2;
      const u16x8 v0 = j < L ? *reinterpret_cast<const u16x8*>(src + (int64_t)j * ld + dc * 8) : (u16x8)0;
      const u16x8 v1 =
          j + 1 < L ? *reinterpret_cast<const u16x8*>(src + (int64_t)(j + 1) * ld + dc * 8) : (u16x8)0;
#pragma unroll
      for (int dd = 0; dd < 8; ++dd)
        *reinterpret_cast<uint32_t*>(&T[(dc * 8 + dd) * VP + j]) = (uint32_t)v0[dd] | ((uint32_t)v1[dd] << 16);
    }
  };
  auto frag = [&](const unsigned short* p) { return *reinterpret_cast<const bf16x8*>(p); };
  stage_t(T0, base + H, ld3);
  for (int j = threadIdx.x; j < Lp; j += 64 * NW)
    mb[j] = j >= L ? -3e30f : ((mask == nullptr || mask[(int64_t)b * L + j] != 0) ? 0.f : -1e30f);
  __syncthreads();

  // ---------------- phase A: query blocks
  for (int ib = wv; ib < nb; ib += NW) {
    const int i = 32 * ib + r32, ic = min(i, L - 1);
    bf16x8 qf[4], df[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      qf[kk] = frag(base + (int64_t)ic * ld3 + 16 * kk + 8 * h);
      df[kk] = frag(dob + (int64_t)ic * H + 16 * kk + 8 * h);
    }
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u16x8 o8 = *reinterpret_cast<const u16x8*>(ob + (int64_t)ic * H + 32 * h + 8 * c);
      const u16x8 d8 = *reinterpret_cast<const u16x8*>(dob + (int64_t)ic * H + 32 * h + 8 * c);
#pragma unroll
      for (int t = 0; t < 8; ++t) dsum += bf16_to_f32(o8[t]) * bf16_to_f32(d8[t]);
    }
    dsum += __shfl_xor(dsum, 32, 64);
    auto scores = [&](int jb) {
      f32x16 s = (f32x16)0.f;
      const int jr = min(32 * jb + r32, L - 1);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(base + (int64_t)jr * ld3 + H + 16 * kk + 8 * h),
                                                    qf[kk], s, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 bias = *reinterpret_cast<const f32x4*>(&mb[32 * jb + 8 * q + 4 * h]);
#pragma unroll
        for (int r = 0; r < 4; ++r) s[4 * q + r] = s[4 * q + r] * scale + bias[r];
      }
      return s;
    };
    float m = -INFINITY, l = 0.f;
    for (int jb = 0; jb < nb; ++jb) {
      const f32x16 s = scores(jb);
      float tmx = -INFINITY;
#pragma unroll
      for (int e = 0; e < 16; ++e) tmx = fmaxf(tmx, s[e]);
      tmx = fmaxf(tmx, __shfl_xor(tmx, 32, 64));
      const float mn = fmaxf(m, tmx);
      float ts = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) ts += __expf(s[e] - mn);
      ts += __shfl_xor(ts, 32, 64);
      l = l * __expf(m - mn) + ts;
      m = mn;
    }
    const float inv = 1.f / l;
    if (h == 0) {
      mrow[i] = i < L ? m : 3e30f;
      irow[i] = i < L ? inv : 0.f;
      drow[i] = i < L ? dsum : 0.f;
    }
    f32x16 dq[2] = {(f32x16)0.f, (f32x16)0.f};
    for (int jb = 0; jb < nb; ++jb) {
      f32x16 s = scores(jb);
      f32x16 dp = (f32x16)0.f;
      const int jr = min(32 * jb + r32, L - 1);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(base + (int64_t)jr * ld3 + 2 * H + 16 * kk + 8 * h),
                                                     df[kk], dp, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 16; ++e) s[e] = __expf(s[e] - m) * inv * (dp[e] - dsum);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        bf16x8 pa;
#pragma unroll
        for (int t = 0; t < 8; ++t) pa[t] = (__bf16)s[8 * k2 + t];
        const int j0 = 32 * jb + 16 * k2 + 4 * h;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const unsigned short* tr = T0 + (32 * db + r32) * VP;
          const u16x4 lo = *reinterpret_cast<const u16x4*>(tr + j0);
          const u16x4 hi = *reinterpret_cast<const u16x4*>(tr + j0 + 8);
          const u16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, vv), dq[db], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ii = 32 * ib + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (ii < L) gb[(int64_t)ii * ld3 + 32 * db + r32] = f32_to_bf16(dq[db][e] * scale);
      }
  }
  __syncthreads();  // K^T readers done, statistics complete
  stage_t(T0, base, ld3);
  stage_t(T1, dob, H);
  __syncthreads();

  // ---------------- phase B: key blocks
  for (int jb = wv; jb < nb; jb += NW) {
    const int j = 32 * jb + r32, jc = min(j, L - 1);
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      kf[kk] = frag(base + (int64_t)jc * ld3 + H + 16 * kk + 8 * h);
      vf[kk] = frag(base + (int64_t)jc * ld3 + 2 * H + 16 * kk + 8 * h);
    }
    const float bj = mb[j];
    f32x16 dv[2] = {(f32x16)0.f, (f32x16)0.f};
    f32x16 dk[2] = {(f32x16)0.f, (f32x16)0.f};
    for (int ib = 0; ib < nb; ++ib) {
      const int ir = 32 * ib + r32;
      f32x16 sc = (f32x16)0.f, dp = (f32x16)0.f;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 qa = frag(base + (int64_t)min(ir, L - 1) * ld3 + 16 * kk + 8 * h);
        const bf16x8 da = ir < L ? frag(dob + (int64_t)ir * H + 16 * kk + 8 * h) : (bf16x8)0;
        sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kf[kk], sc, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, vf[kk], dp, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r0 = 32 * ib + 8 * q + 4 * h;
        const f32x4 mm = *reinterpret_cast<const f32x4*>(&mrow[r0]);
        const f32x4 iv = *reinterpret_cast<const f32x4*>(&irow[r0]);
        const f32x4 dd = *reinterpret_cast<const f32x4*>(&drow[r0]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 4 * q + r;
          const float p = __expf(sc[e] * scale + bj - mm[r]) * iv[r];
          sc[e] = p;
          dp[e] = p * (dp[e] - dd[r]);
        }
      }
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        bf16x8 pa, sa;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          pa[t] = (__bf16)sc[8 * k2 + t];
          sa[t] = (__bf16)dp[8 * k2 + t];
        }
        const int i0 = 32 * ib + 16 * k2 + 4 * h;
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          const int d = 32 * db + r32;
          const u16x4 olo = *reinterpret_cast<const u16x4*>(T1 + d * VP + i0);
          const u16x4 ohi = *reinterpret_cast<const u16x4*>(T1 + d * VP + i0 + 8);
          const u16x8 ov = {olo[0], olo[1], olo[2], olo[3], ohi[0], ohi[1], ohi[2], ohi[3]};
          dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, ov), dv[db], 0, 0, 0);
          const u16x4 qlo = *reinterpret_cast<const u16x4*>(T0 + d * VP + i0);
          const u16x4 qhi = *reinterpret_cast<const u16x4*>(T0 + d * VP + i0 + 8);
          const u16x8 qv = {qlo[0], qlo[1], qlo[2], qlo[3], qhi[0], qhi[1], qhi[2], qhi[3]};
          dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa, __builtin_bit_cast(bf16x8, qv), dk[db], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int jj = 32 * jb + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (jj < L) {
          gb[(int64_t)jj * ld3 + H + 32 * db + r32] = f32_to_bf16(dk[db][e] * scale);
          gb[(int64_t)jj * ld3 + 2 * H + 32 * db + r32] = f32_to_bf16(dv[db][e]);
        }
      }
  }
}

static size_t attn_bwd_long_lds(int64_t L) {
  const int64_t Lp = (L + 31) & ~31LL;
  return (size_t)(4 * Lp * 4 + 2 * 64 * (Lp + 4) * 2);
}

// ---------------------------------------------------------------- embedding bwd
// dword[ids[r]] += dx[r] (fp32 atomics; rows holding pad_id skipped: nn.Embedding's
// padding_idx row never receives a gradient).  One wave per row.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_word_kernel(const T* __restrict__ dx,
                                                            const int64_t* __restrict__ ids,
                                                            float* __restrict__ dword,
                                                            int64_t rows, int H, int64_t pad_id) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t id = ids[row];
  if (id == pad_id) return;
  float* dst = dword + id * H;
  for (int c = lane; c < H; c += 64) atomicAdd(dst + c, ld(dx, row * H + c));
}

// ws[l][c] = sum_b dx[b*L + l][c] (b ascending)
template <typename T>
__global__ void embed_bwd_pos_kernel(const T* __restrict__ dx, float* __restrict__ ws, int B,
                                     int L, int H) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = blockIdx.y;
  if (c >= H) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += ld(dx, ((int64_t)b * L + l) * H + c);
  ws[(int64_t)l * H + c] = s;
}

// dpos[l][c] += ws[l][c]; dtype0[c] += sum_l ws[l][c] (l ascending)
__global__ void embed_bwd_final_kernel(const float* __restrict__ ws, float* __restrict__ dpos,
                                       float* __restrict__ dtype0, int L, int H) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= H) return;
  float t = 0.f;
  for (int l = 0; l < L; ++l) {
    const float v = ws[(int64_t)l * H + c];
    if (dpos) dpos[(int64_t)l * H + c] += v;
    t += v;
  }
  if (dtype0) dtype0[c] += t;
}

// y fp32 = (word[id] + type0) + pos[l]: the embedding-LN input (HF summation order)
template <typename T>
__global__ void embed_sum_kernel(const int64_t* __restrict__ ids, const T* __restrict__ word,
                                 const T* __restrict__ pos, const T* __restrict__ type0,
                                 float* __restrict__ y, int64_t rows, int L, int H) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t id = ids[row];
  const int l = (int)(row % L);
  for (int c = lane; c < H; c += 64)
    y[row * H + c] = (ld(word, id * H + c) + ld(type0, c)) + ld(pos, (int64_t)l * H + c);
}

}  // namespace encb
}  // namespace irc

using namespace irc;

static unsigned nblocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// Enough for either kernel (the generic one takes fewer rows per block).
extern "C" int64_t irc_layernorm_bwd_workspace(int64_t rows, int64_t H) {
  const int64_t nb = (rows + encb::LNB_ROWS - 1) / encb::LNB_ROWS;
  return ((nb > 0 ? nb : 1) + encb::LNF_S) * 2 * H;  // block partials + stage-1 partials
}

extern "C" int irc_layernorm_bwd(int dtype, int dy_dtype, const void* dy, const void* x,
                                 const float* gamma, void* dx, float* dgamma, float* dbeta,
                                 float* partial, int64_t partial_floats, int64_t rows, int64_t H,
                                 float eps, int64_t bcast_L, float dy_scale, int accumulate,
                                 irc_stream_t stream) {
  IRC_REQUIRE(H >= 1 && H <= 64 * encb::MAXH_PER_LANE, "layernorm_bwd: H=%lld unsupported",
              (long long)H);
  IRC_REQUIRE(dtype == 0 || dtype == 1, "layernorm_bwd: dtype");
  IRC_REQUIRE(dy_dtype == 0 || dy_dtype == 1, "layernorm_bwd: dy_dtype");
  IRC_REQUIRE(bcast_L >= 0, "layernorm_bwd: bcast_L < 0");
  if (rows == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const bool al = ((uintptr_t)x % 16) == 0 && ((uintptr_t)dx % 16) == 0 &&
                  ((uintptr_t)dy % 16) == 0 && ((uintptr_t)gamma % 16) == 0;
  const bool vec = dtype == 0 && al && (H == 512 || H == 768 || H == 1024);
  const int per = vec ? encb::LNV_ROWS : encb::LNB_ROWS;
  const int64_t nb = (rows + per - 1) / per;
  const int64_t need = ((int64_t)nb + encb::LNF_S) * 2 * H;
  IRC_REQUIRE(partial != nullptr && partial_floats >= need,
              "layernorm_bwd: workspace %lld < %lld floats", (long long)partial_floats,
              (long long)need);
  using u16 = unsigned short;
  prof_begin(st);
  if (vec) {
#define IRC_LNV(CPL)                                                                              \
  if (dy_dtype == 0)                                                                              \
    hipLaunchKernelGGL((encb::ln_bwd_vec_kernel<CPL, u16>), dim3((unsigned)nb), dim3(256), 0, st, \
                       (const u16*)dy, (const u16*)x, gamma, (u16*)dx, partial, rows, eps,        \
                       bcast_L, dy_scale);                                                        \
  else                                                                                            \
    hipLaunchKernelGGL((encb::ln_bwd_vec_kernel<CPL, float>), dim3((unsigned)nb), dim3(256), 0,   \
                       st, (const float*)dy, (const u16*)x, gamma, (u16*)dx, partial, rows, eps,  \
                       bcast_L, dy_scale);
    if (H == 768) {
      IRC_LNV(3)
    } else if (H == 1024) {
      IRC_LNV(4)
    } else {
      IRC_LNV(2)
    }
#undef IRC_LNV
  } else {
    const size_t lds = (size_t)2 * H * sizeof(float);
    if (dtype == 0 && dy_dtype == 0)
      hipLaunchKernelGGL((encb::ln_bwd_kernel<u16, u16>), dim3((unsigned)nb), dim3(256), lds, st,
                         (const u16*)dy, (const u16*)x, gamma, (u16*)dx, partial, rows, (int)H,
                         eps, bcast_L, dy_scale);
    else if (dtype == 0)
      hipLaunchKernelGGL((encb::ln_bwd_kernel<u16, float>), dim3((unsigned)nb), dim3(256), lds,
                         st, (const float*)dy, (const u16*)x, gamma, (u16*)dx, partial, rows,
                         (int)H, eps, bcast_L, dy_scale);
    else if (dy_dtype == 0)
      hipLaunchKernelGGL((encb::ln_bwd_kernel<float, u16>), dim3((unsigned)nb), dim3(256), lds,
                         st, (const u16*)dy, (const float*)x, gamma, (float*)dx, partial, rows,
                         (int)H, eps, bcast_L, dy_scale);
    else
      hipLaunchKernelGGL((encb::ln_bwd_kernel<float, float>), dim3((unsigned)nb), dim3(256), lds,
                         st, (const float*)dy, (const float*)x, gamma, (float*)dx, partial, rows,
                         (int)H, eps, bcast_L, dy_scale);
  }
  int rc = check_launch("layernorm_bwd");
  if (rc) return rc;
  const int per2 = (int)((nb + encb::LNF_S - 1) / encb::LNF_S);
  const int ns = (int)((nb + per2 - 1) / per2);
  float* partial2 = partial + nb * 2 * H;
  hipLaunchKernelGGL(encb::ln_bwd_stage1_kernel, dim3(nblocks(2 * H, 256), (unsigned)ns),
                     dim3(256), 0, st, partial, (int)nb, (int)H, per2, partial2);
  hipLaunchKernelGGL(encb::ln_bwd_final_kernel, dim3(nblocks(2 * H, 256)), dim3(256), 0, st,
                     partial2, ns, (int)H, dgamma, dbeta, accumulate);
  prof_end("layernorm_bwd", st, (double)rows * H * (dtype == 0 ? 2.0 : 4.0) * 3.0);
  return check_launch("layernorm_bwd_final");
}

template <typename T, int DH>
static int attn_bwd_launch(const void* qkv, const int64_t* mask, const void* ctx, const void* dctx,
                           void* dqkv, int64_t B, int64_t L, int64_t H, int64_t heads,
                           hipStream_t st) {
  const size_t lds = (size_t)3 * L * 4;  // per-query statistics (the tiles are static)
  hipLaunchKernelGGL((encb::attn_bwd_kernel<T, DH>), dim3((unsigned)(B * heads)), dim3(256), lds,
                     st, (const T*)qkv, mask, (const T*)ctx, (const T*)dctx, (T*)dqkv, (int)L,
                     (int)H, (int)heads, 1.0f / sqrtf((float)DH));
  return check_launch("attention_bwd_kernel");
}

extern "C" int irc_attention_bwd(int dtype, const void* qkv, const int64_t* mask, const void* ctx,
                                 const void* dctx, void* dqkv, int64_t B, int64_t L, int64_t H,
                                 int64_t heads, irc_stream_t stream) {
  IRC_REQUIRE(heads >= 1 && H % heads == 0, "attention_bwd: H %% heads != 0");
  const int64_t dh = H / heads;
  IRC_REQUIRE(dh == 16 || dh == 32 || dh == 64 || dh == 128, "attention_bwd: head dim %lld",
              (long long)dh);
  IRC_REQUIRE(dtype == 0 || dtype == 1, "attention_bwd: dtype");
  if (B == 0 || L == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  using u16 = unsigned short;
  if (dtype == 0 && dh == 64 && L > 128) {
    IRC_REQUIRE(L <= 512, "attention_bwd: L=%lld > 512 (BERT's position table)", (long long)L);
    const size_t lds = encb::attn_bwd_long_lds(L);
    const dim3 grid((unsigned)(B * heads));
    prof_begin(st);
    hipLaunchKernelGGL(encb::attn_bwd_long_kernel<8>, grid, dim3(512), lds, st, (const u16*)qkv,
                       mask, (const u16*)ctx, (const u16*)dctx, (u16*)dqkv, (int)L, (int)H,
                       (int)heads, 0.125f);
    prof_end("attention_bwd", st, (double)B * L * (3 * H + 2 * H + 3 * H) * 2.0);
    return check_launch("attention_bwd_long_kernel");
  }
  // L <= 128: whole rows in registers, L rounded up to 32-row blocks (rows past L read as
  // zeros, never stored).  At L = 65 / 72 (32k tokens) 419 / 400 us in the blocked long
  // kernel this replaced there, against 169 / 185 us at 64 / 96 (profiles/r06_u/).
  if (dtype == 0 && dh == 64) {
    const float sc = 0.125f;
    const dim3 grid((unsigned)(B * heads));
    prof_begin(st);
#define IRC_ABW(NJ, P)                                                                        \
  hipLaunchKernelGGL((encb::attn_bwd_mfma_kernel<NJ, P>), grid, dim3(64 * NJ), 0, st,            \
                     (const u16*)qkv, mask, (const u16*)ctx, (const u16*)dctx, (u16*)dqkv, (int)H, \
                     (int)heads, sc, (int)L)
    const bool part = L % 32 != 0;
    switch ((L + 31) / 32) {
      case 1: if (part) IRC_ABW(1, true); else IRC_ABW(1, false); break;
      case 2: if (part) IRC_ABW(2, true); else IRC_ABW(2, false); break;
      case 3: if (part) IRC_ABW(3, true); else IRC_ABW(3, false); break;
      default: if (part) IRC_ABW(4, true); else IRC_ABW(4, false); break;
    }
#undef IRC_ABW
    // algorithmic bytes: QKV, ctx, dctx read, dQKV written
    prof_end("attention_bwd", st, (double)B * L * (3 * H + 2 * H + 3 * H) * 2.0);
    return check_launch("attention_bwd_mfma_kernel");
  }
  IRC_REQUIRE((size_t)3 * L * 4 <= (size_t)IRC_LDS_BYTES / 2,
              "attention_bwd: L=%lld too long for the per-query statistics", (long long)L);
#define IRC_ATTB(DH)                                                                          \
  if (dh == DH)                                                                               \
    return dtype == 0                                                                         \
               ? attn_bwd_launch<u16, DH>(qkv, mask, ctx, dctx, dqkv, B, L, H, heads, st)     \
               : attn_bwd_launch<float, DH>(qkv, mask, ctx, dctx, dqkv, B, L, H, heads, st);
  IRC_ATTB(16)
  IRC_ATTB(32)
  IRC_ATTB(64)
  IRC_ATTB(128)
#undef IRC_ATTB
  return IRC_E_INVALID;
}

extern "C" int irc_embed_bwd(int dtype, const void* dx, const int64_t* ids, float* dword,
                             float* dpos, float* dtype0, float* workspace, int64_t ws_floats,
                             int64_t B, int64_t L, int64_t H, int64_t pad_id,
                             irc_stream_t stream) {
  IRC_REQUIRE(dtype == 0 || dtype == 1, "embed_bwd: dtype");
  IRC_REQUIRE(B >= 0 && L >= 1 && H >= 1, "embed_bwd: bad sizes");
  if (B == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const int64_t rows = B * L;
  using u16 = unsigned short;
  if (dword) {
    if (dtype == 0)
      hipLaunchKernelGGL(encb::embed_bwd_word_kernel<u16>, dim3(nblocks(rows, 4)), dim3(256), 0,
                         st, (const u16*)dx, ids, dword, rows, (int)H, pad_id);
    else
      hipLaunchKernelGGL(encb::embed_bwd_word_kernel<float>, dim3(nblocks(rows, 4)), dim3(256), 0,
                         st, (const float*)dx, ids, dword, rows, (int)H, pad_id);
    int rc = check_launch("embed_bwd_word");
    if (rc) return rc;
  }
  if (dpos || dtype0) {
    IRC_REQUIRE(workspace != nullptr && ws_floats >= L * H, "embed_bwd: workspace < L*H floats");
    const dim3 g(nblocks(H, 256), (unsigned)L);
    if (dtype == 0)
      hipLaunchKernelGGL(encb::embed_bwd_pos_kernel<u16>, g, dim3(256), 0, st, (const u16*)dx,
                         workspace, (int)B, (int)L, (int)H);
    else
      hipLaunchKernelGGL(encb::embed_bwd_pos_kernel<float>, g, dim3(256), 0, st, (const float*)dx,
                         workspace, (int)B, (int)L, (int)H);
    hipLaunchKernelGGL(encb::embed_bwd_final_kernel, dim3(nblocks(H, 256)), dim3(256), 0, st,
                       workspace, dpos, dtype0, (int)L, (int)H);
  }
  return check_launch("embed_bwd");
}

extern "C" int irc_embed_sum(int dtype, const int64_t* ids, const void* word, const void* pos,
                             const void* type0, float* y, int64_t rows, int64_t L, int64_t H,
                             irc_stream_t stream) {
  IRC_REQUIRE(dtype == 0 || dtype == 1, "embed_sum: dtype");
  IRC_REQUIRE(L >= 1 && H >= 1, "embed_sum: bad sizes");
  if (rows == 0) return IRC_OK;
  using u16 = unsigned short;
  if (dtype == 0)
    hipLaunchKernelGGL(encb::embed_sum_kernel<u16>, dim3(nblocks(rows, 4)), dim3(256), 0,
                       as_stream(stream), ids, (const u16*)word, (const u16*)pos,
                       (const u16*)type0, y, rows, (int)L, (int)H);
  else
    hipLaunchKernelGGL(encb::embed_sum_kernel<float>, dim3(nblocks(rows, 4)), dim3(256), 0,
                       as_stream(stream), ids, (const float*)word, (const float*)pos,
                       (const float*)type0, y, rows, (int)L, (int)H);
  return check_launch("embed_sum");
}
