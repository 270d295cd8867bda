// General MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M, N] (=|+=) alpha * op(A)[M, K] . op(B)[K, N]  (+ bias[N]) (-> GELU) (+ R[M, N])
//
// Replaces the cuBLAS GEMMs the reference reaches through nn.Linear /
// torch.matmul: BERT QKV / out-proj / FFN (HF modeling_bert, called from
// src/contrastor/contrastive_module.py:39), the LSTM input projections and their
// backward products (src/model.py:16-26, 39-40), the BiLSTM head's Linear
// 512->128, and the InfoNCE logits (src/contrastor/contrastive_loss.py:61-62,79).
//
// Operand layouts (all row-major in memory):
//   A: ROW = [M][K] (lda)            COL = [K][M] (lda)
//   B: NK  = [N][K] (ldb, nn.Linear) KN  = [K][N] (ldb)
// Input types: bf16 (v_mfma_f32_32x32x16_bf16, fp32 accumulate) or fp32
// (v_mfma_f32_32x32x2_f32: exact fp32 products, the parity mode).
//
// Structure: 128x128 block tile, 4 waves (2x2) of 64x64, BK k-slab staged
// global -> registers -> LDS (double buffered; the next slab's global loads are
// issued before the current slab's MFMAs).  LDS rows are padded by 16 B so the
// row-wise ds_read_b128 fragment reads are conflict free.  K-major (ROW / NK)
// slabs move as 16-byte vectors; the transposed layouts (COL / KN) are loaded
// along M/N and scattered into the [row][k] LDS image.  Blocks are remapped so
// each XCD walks a contiguous band of output tiles (neighbours share A/B panels
// in that XCD's L2).
#include "gemm_pp.h"

#include <algorithm>
#include <atomic>

// Grouped output-tile order of the GEMM kernels' tiles (see gemm_group_m; 0 = row-major).
#ifndef IRC_GEMM_GROUP_M
#define IRC_GEMM_GROUP_M 0
#endif

namespace irc {
namespace gemm {

enum Layout { ROW = 0, COL = 1 };  // A: ROW=[M][K], COL=[K][M]; B: ROW=[N][K] (NK), COL=[K][N] (KN)
// EPI_DGELU: C = alpha acc * gelu'(R)  (GELU backward; R = saved pre-activation)
// EPI_BIAS_GELU_SAVE: C = gelu(alpha acc + bias) and R <- alpha acc + bias (R is a
// second OUTPUT here: the pre-activation the GELU backward needs)
enum Epi {
  EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RESID = 3, EPI_RESID = 4,
  EPI_DGELU = 5, EPI_BIAS_GELU_SAVE = 6
};
__host__ __device__ constexpr bool epi_has_bias(int e) {
  return e == EPI_BIAS || e == EPI_BIAS_GELU || e == EPI_BIAS_RESID || e == EPI_BIAS_GELU_SAVE;
}

constexpr int BM = 128, BN = 128, NT = 256;

template <typename T>
struct TT;
template <>
struct TT<unsigned short> {  // bf16
  static constexpr int BK = 32;
  static constexpr int VEC = 8;  // elements per 16-byte vector
  static constexpr int PITCH = BK * 2 + 16;  // bytes per LDS row (64 + 16 pad)
};
template <>
struct TT<float> {
  static constexpr int BK = 16;
  static constexpr int VEC = 4;
  static constexpr int PITCH = BK * 4 + 16;  // 64 + 16 pad
};

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// GELU(x) = 0.5 x (1 + erf(x / sqrt 2)) with erf from Abramowitz & Stegun 7.1.26
// (|error| <= 1.5e-7 absolute, i.e. below fp32 resolution of the (1 + erf) sum
// for |x| >~ 1): ~15 branch-free VALU ops against the library erff's ~40, which
// matters when the epilogue is not hidden behind MFMA work (big-tile path).
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
  float p = 1.061405429f;
  p = p * t - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const float e = 1.0f - p * t * __expf(-az * az);
  return 0.5f * x * (1.0f + copysignf(e, z));
}

// d/dx GELU(x) = Phi(x) + x phi(x), Phi via the same A&S 7.1.26 erf as gelu_fast.
__device__ __forceinline__ float gelu_grad_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
  float p = 1.061405429f;
  p = p * t - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const float ez = __expf(-az * az);
  const float e = 1.0f - p * t * ez;
  return 0.5f * (1.0f + copysignf(e, z)) + x * 0.3989422804014327f * ez;
}
__device__ __forceinline__ float gelu_grad_erf(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) +
         x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

struct Args {
  const void* A;
  const void* B;
  void* C;
  const float* bias;
  const void* R;  // residual, same type/ld as C
  int M, N, K;
  int64_t lda, ldb, ldc, ldr;
  int64_t sA, sB, sC, sR, sBias;  // batch strides (elements)
  float alpha;
  int accumulate;  // C += result (fp32 C only)
  int vec_a, vec_b;  // operand rows 16-byte aligned: vector staging allowed
  int vec_c;         // C (and R) rows 16-byte aligned and N % 8 == 0: vector epilogue
  int kchunk;        // split-K: K range of one blockIdx.z slice (multiple of BK)
  float* P;          // split-K partials [batch][split][M][N] (raw sums), or null
  int group_m;       // big-tile kernel: grouped tile order (irc_common.h); 0 = row-major
  LnArgs ln;         // LayerNorm fold (big-tile kernel, bf16 C, vectorised epilogue)
};

// bf16 K-outer (COL / KN) slabs are kept k-major in LDS: [BK=32 k][128 rows]
// bf16 = 256-byte k-rows with the XOR chunk swizzle of the guide's dual-use image
// (b), and MFMA fragments come from ds_read_b64_tr_b16 (hardware transpose: a
// 16-lane group reads 4 k-rows x 16 columns and each lane receives its column),
// instead of scattering 2-byte LDS writes.
__device__ __forceinline__ int kimg_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4s ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(p));
}
// 32x32x16 operand fragment (lane r32 = column, half h = k 8h..8h+7) of the 32
// columns starting at col0, k-step ks, from a k-major image.
__device__ __forceinline__ bf16x8 kimg_frag(const char* img, int col0, int ks, int lane) {
  const int g = lane >> 4, j = lane & 15, q = j >> 2, p = j & 3;
  const int c = col0 + 16 * (g & 1);
  const int k0 = ks * 16 + 8 * (g >> 1);
  const int cb = c / 8 + (p >> 1), b8 = 8 * (p & 1);
  const v4s lo = ds_tr16(img + kimg_off(k0 + q, cb) + b8);
  const v4s hi = ds_tr16(img + kimg_off(k0 + 4 + q, cb) + b8);
  const v4s both[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, both);
}

// Load one [rows x BK] slab of an operand into registers (as 16-byte vectors).
// For K-major storage (ROW) each vector = 8 (bf16) / 4 (f32) consecutive k of one
// row; for transposed storage (COL) each vector = consecutive rows at one k.
template <typename T, int LAYOUT>
struct Slab {
  static constexpr int BK = TT<T>::BK;
  static constexpr int VEC = TT<T>::VEC;
  static constexpr int NVEC = (128 * BK) / VEC;  // vectors per slab
  static constexpr int PER_T = NVEC / NT;
  u16x8 v[PER_T];

  // vec: rows start 16-byte aligned (ld and base), so whole 16-byte vectors may
  // be loaded; otherwise every element is loaded on its own.
  __device__ __forceinline__ void load(const T* base, int64_t ld, int row0, int nrows, int k0,
                                       int K, bool vec) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int e = i * NT + tid;
      int r, kk;
      if (LAYOUT == ROW) {
        r = e / (BK / VEC);
        kk = (e % (BK / VEC)) * VEC;
      } else {
        kk = e / (128 / VEC);
        r = (e % (128 / VEC)) * VEC;
      }
      const int gr = row0 + r, gk = k0 + kk;
      u16x8 val = (u16x8)0;
      if (LAYOUT == ROW) {
        if (vec && gr < nrows && gk + VEC <= K) {
          val = *reinterpret_cast<const u16x8*>(base + (int64_t)gr * ld + gk);
        } else if (gr < nrows) {
          T tmp[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) tmp[j] = (gk + j < K) ? base[(int64_t)gr * ld + gk + j] : T(0);
          val = *reinterpret_cast<u16x8*>(tmp);
        }
      } else {
        if (vec && gk < K && gr + VEC <= nrows) {
          val = *reinterpret_cast<const u16x8*>(base + (int64_t)gk * ld + gr);
        } else if (gk < K) {
          T tmp[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            tmp[j] = (gr + j < nrows) ? base[(int64_t)gk * ld + gr + j] : T(0);
          val = *reinterpret_cast<u16x8*>(tmp);
        }
      }
      v[i] = val;
    }
  }

  __device__ __forceinline__ void store(char* lds) const {
    const int tid = threadIdx.x;
    constexpr int PITCH = TT<T>::PITCH;
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int e = i * NT + tid;
      if (LAYOUT == ROW) {
        const int r = e / (BK / VEC);
        const int kk = (e % (BK / VEC)) * VEC;
        *reinterpret_cast<u16x8*>(lds + r * PITCH + kk * (int)sizeof(T)) = v[i];
      } else if constexpr (sizeof(T) == 2) {
        const int kk = e / (128 / VEC);
        const int r = (e % (128 / VEC)) * VEC;
        *reinterpret_cast<u16x8*>(lds + kimg_off(kk, r / 8)) = v[i];  // k-major image
      } else {
        const int kk = e / (128 / VEC);
        const int r = (e % (128 / VEC)) * VEC;
        const T* t = reinterpret_cast<const T*>(&v[i]);
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          *reinterpret_cast<T*>(lds + (r + j) * PITCH + kk * (int)sizeof(T)) = t[j];
      }
    }
  }
};

template <typename TI, typename TO, int LA, int LB, int EPI>
__global__ __launch_bounds__(NT) void gemm_kernel(Args g) {
  constexpr int BK = TT<TI>::BK;
  constexpr int PITCH = TT<TI>::PITCH;
  constexpr int SLAB = 128 * PITCH;
  __shared__ __attribute__((aligned(16))) char lds[2][2][SLAB];  // [buf][A/B]

  const int tiles_m = (g.M + BM - 1) / BM;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  // XCD-aware bijective remap of the linear block id (blocks b and b+8 share an XCD)
  int bid = blockIdx.x;
  {
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int batch = blockIdx.y;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const TI* A = reinterpret_cast<const TI*>(g.A) + batch * g.sA;
  const TI* B = reinterpret_cast<const TI*>(g.B) + batch * g.sB;
  TO* C = reinterpret_cast<TO*>(g.C) + batch * g.sC;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, r32 = lane & 31;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16)0.0f;

  Slab<TI, LA> sa;
  Slab<TI, LB> sb;
  const int nk = (kend - kbeg + BK - 1) / BK;
  sa.load(A, g.lda, m0, g.M, kbeg, kend, g.vec_a);
  sb.load(B, g.ldb, n0, g.N, kbeg, kend, g.vec_b);
  sa.store(lds[0][0]);
  sb.store(lds[0][1]);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      sa.load(A, g.lda, m0, g.M, kbeg + (kt + 1) * BK, kend, g.vec_a);
      sb.load(B, g.ldb, n0, g.N, kbeg + (kt + 1) * BK, kend, g.vec_b);
    }
    const char* la = lds[cur][0];
    const char* lb = lds[cur][1];
    if constexpr (sizeof(TI) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wm * 64 + i * 32 + r32;
          if constexpr (LA == COL)
            fa[i] = kimg_frag(la, wm * 64 + i * 32, ks, lane);
          else
            fa[i] = *reinterpret_cast<const bf16x8*>(la + row * PITCH + (ks * 16 + 8 * h) * 2);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wn * 64 + j * 32 + r32;
          if constexpr (LB == COL)
            fb[j] = kimg_frag(lb, wn * 64 + j * 32, ks, lane);
          else
            fb[j] = *reinterpret_cast<const bf16x8*>(lb + row * PITCH + (ks * 16 + 8 * h) * 2);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // fp32: lane half h owns k = 8h .. 8h+7 of the 16-deep slab (same k pairing
      // for A and B), read as two 16-byte vectors; 8 MFMAs of K=2 (one k-slot per half).
      f32x4 fa[2][2], fb[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + r32;
        fa[i][0] = *reinterpret_cast<const f32x4*>(la + row * PITCH + (8 * h) * 4);
        fa[i][1] = *reinterpret_cast<const f32x4*>(la + row * PITCH + (8 * h + 4) * 4);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn * 64 + j * 32 + r32;
        fb[j][0] = *reinterpret_cast<const f32x4*>(lb + row * PITCH + (8 * h) * 4);
        fb[j][1] = *reinterpret_cast<const f32x4*>(lb + row * PITCH + (8 * h + 4) * 4);
      }
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk >> 2][kk & 3],
                                                             fb[j][kk >> 2][kk & 3], acc[i][j],
                                                             0, 0, 0);
    }
    if (kt + 1 < nk) {
      __syncthreads();  // everyone done reading the other buffer
      sa.store(lds[cur ^ 1][0]);
      sb.store(lds[cur ^ 1][1]);
      __syncthreads();
    }
  }

  // Epilogue: acc[i][j] reg e -> row = m0 + wm*64 + i*32 + (e&3) + 8(e>>2) + 4h,
  //                              col = n0 + wn*64 + j*32 + r32.
  if (g.P) {  // split-K slice: raw partial sums, reduced in a fixed order afterwards
    float* P = g.P + ((int64_t)batch * gridDim.z + blockIdx.z) * g.M * g.N;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 64 + j * 32 + r32;
      if (col >= g.N) continue;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (row < g.M) P[(int64_t)row * g.N + col] = acc[i][j][e];
        }
    }
    return;
  }
  const float* bias = g.bias ? g.bias + batch * g.sBias : nullptr;
  const TO* R = g.R ? reinterpret_cast<const TO*>(g.R) + batch * g.sR : nullptr;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + r32;
    if (col >= g.N) continue;
    const float bv = epi_has_bias(EPI) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= g.M) continue;
        float v = acc[i][j][e] * g.alpha + bv;
        // bf16 outputs: the same GELU as every other bf16 epilogue (the kernel choice
        // must not change the result beyond fp32 reassociation)
        if (EPI == EPI_BIAS_GELU) v = sizeof(TO) == 2 ? gelu_lite(v) : gelu_erf(v);
        if (EPI == EPI_BIAS_GELU_SAVE) {
          TO* pre = const_cast<TO*>(R) + (int64_t)row * g.ldr + col;
          if constexpr (sizeof(TO) == 2)
            *reinterpret_cast<unsigned short*>(pre) = f32_to_bf16(v);
          else
            *reinterpret_cast<float*>(pre) = v;
          v = gelu_erf(v);
        }
        if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
          float r;
          if constexpr (sizeof(TO) == 2)
            r = bf16_to_f32(reinterpret_cast<const unsigned short*>(R)[(int64_t)row * g.ldr + col]);
          else
            r = reinterpret_cast<const float*>(R)[(int64_t)row * g.ldr + col];
          v = EPI == EPI_DGELU ? v * gelu_grad_erf(r) : v + r;
        }
        TO* dst = C + (int64_t)row * g.ldc + col;
        if constexpr (sizeof(TO) == 2) {
          *reinterpret_cast<unsigned short*>(dst) = f32_to_bf16(v);
        } else {
          if (g.accumulate)
            *reinterpret_cast<float*>(dst) += v;
          else
            *reinterpret_cast<float*>(dst) = v;
        }
      }
    }
  }
}

// C[b][m][n] (=|+=) alpha * sum_s P[b][s][m][n] (+ bias[b][n])  (s ascending:
// deterministic; the bias is the EPI_BIAS epilogue of an fp32 GEMM that was split)
__global__ void splitk_reduce_kernel(const float* __restrict__ P, float* __restrict__ C, int M,
                                     int N, int S, int64_t ldc, int64_t sC, int batch,
                                     float alpha, int accumulate,
                                     const float* __restrict__ bias = nullptr,
                                     int64_t sBias = 0) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t mn = (int64_t)M * N;
  if (e >= mn * batch) return;
  const int b = (int)(e / mn);
  const int64_t r = e % mn;
  const float* p = P + (int64_t)b * S * mn + r;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += p[k * mn];
  float v = alpha * s;
  if (bias) v += bias[b * sBias + (r % N)];
  float* dst = C + b * sC + (r / N) * ldc + (r % N);
  *dst = accumulate ? *dst + v : v;
}

// Split-K count: only when the output tile grid cannot fill the chip and each
// slice keeps >= 512 of K (bf16) / >= 128 of K (fp32: the exact-fp32 MFMA runs at
// 1/16 of the bf16 rate, so a 128-deep slice is already 8 K-steps of real work --
// the InfoNCE / scaling-layer GEMMs of the heads' step ran on 2-4 workgroups for
// 50-100 us each before).  Restricted to fp32 C with no fused epilogue.
// budget: the largest number of split-K blocks, in 256 x 256-tile units (two 128 x 128
// blocks each); 256 = one wave on MI355X.
inline int split_count(int TIbytes, int out_f32, int epi, int64_t M, int64_t N, int64_t K,
                       int64_t batch, int64_t budget = 256) {
  if (!out_f32 || !(epi == EPI_NONE || (epi == EPI_BIAS && TIbytes == 4))) return 1;
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * batch;
  const int bk = TIbytes == 2 ? TT<unsigned short>::BK : TT<float>::BK;
  int64_t s = (2 * budget + tiles - 1) / tiles;
  const int64_t smax = K / (TIbytes == 2 ? 512 : 128);
  if (s > smax) s = smax;
  if (s > (TIbytes == 2 ? 32 : 64)) s = TIbytes == 2 ? 32 : 64;
  if (s < 2) return 1;
  // equalise slices on BK boundaries; drop empty trailing slices
  const int64_t chunk = ((K + s - 1) / s + bk - 1) / bk * bk;
  return (int)((K + chunk - 1) / chunk);
}

// ---------------------------------------------------------------------------
// Large-tile bf16 path for K-contiguous operands (A [M][K], B [N][K]: the BERT
// and LSTM-projection GEMMs).  256 x (128*WNB) x 64 block tile, 8 waves as
// 2(M) x 4(N), 128 x 32*WNB per wave = 4 x WNB blocks of v_mfma_f32_32x32x16_bf16.
// WNB = 3 (256x384) when N % 384 == 0 -- every BERT-base N (768, 2304, 3072), so
// M = 32768 gives whole waves of tiles over 256 CUs -- else WNB = 2 (256x256).
// Both tiles move global -> LDS by global_load_lds_dwordx4 (no VGPR staging),
// double buffered (2 x 80 KB at WNB=3): tile k+1 is in flight while tile k is
// consumed.  LDS rows are 128 B (64 k); the 16-byte chunk c of row r is stored at
// chunk c ^ ((r >> 1) & 7) (big::chunk_key) so the row-wise ds_read_b128 fragment reads
// are conflict free -- applied on the SOURCE address, since the DMA destination is
// lane-linear.  Rows past M / N load a clamped valid row and are never stored.
// Requires K % 64 == 0, lda/ldb % 8 == 0 and 16-byte aligned bases.
// Algorithmic HBM bytes of one bf16 GEMM launch: both operands read once, C written
// once (read too when accumulating), the residual / saved pre-activation read (or,
// for the GELU-save epilogue, written) once; bias vectors ignored.
inline double gemm_alg_bytes(int out_f32, int epi, int accumulate, int64_t M, int64_t N,
                             int64_t K, int64_t batch) {
  const double ob = out_f32 ? 4.0 : 2.0;
  double b = 2.0 * (double)(M + N) * K + ob * (double)M * N * (accumulate ? 2 : 1);
  if (epi >= 3) b += ob * (double)M * N;
  return b * batch;
}

namespace big {
constexpr int BM = 256, BK = 64, NW = 8, NT = NW * 64;
constexpr int ROW_BYTES = BK * 2;  // 128

// The 16-byte chunk c of tile row r sits in slot c ^ chunk_key(r).  ds_read_b128 serves a
// wave in four 16-lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32), and two
// 128-byte rows share one 256-byte bank line, so a group's 16 reads are conflict free iff
// its 8 even and 8 odd rows each get 8 distinct slots.  (r >> 1) & 7 does that for every
// fragment row set used here (row offsets are multiples of 16); the round-2 key r & 7
// repeats inside every group (rows r, r + 8 / r + 24) and made every fragment read 2-way
// conflicted: 47-49% of the LDS-array cycles (profiles/r03_lds_y_before.txt).
__device__ __forceinline__ int chunk_key(int r) {
  return (r >> 1) & 7;
}

// rows [0, nrows_tile) of one operand tile: nrows_tile*8 16-byte chunks, NT per pass.
// ls > 0 (the sequence-slot layout of qkv_attn_kernel, slots of 2^sh rows): tile row t
// is token min(t mod 2^sh, ls - 1) of sequence (r0 + t) >> sh, sequences of ls rows
// stored contiguously (r0 a multiple of 2^sh); ls = 0: tile row t is row r0 + t.
template <int ROWS>
__device__ __forceinline__ void stage(const unsigned short* __restrict__ X, int64_t ld, int r0,
                                      int nrows, int k0, char* lds_tile, int wave, int lane,
                                      int ls = 0, int sh = 6) {
  constexpr int PASSES = ROWS * 8 / NT;
#pragma unroll
  for (int i = 0; i < PASSES; ++i) {
    const int p = (i * NW + wave) * 64 + lane;  // 16-byte LDS chunk index (lane-linear)
    const int row = p >> 3;
    const int c = (p & 7) ^ chunk_key(row);     // logical k-chunk stored at this slot
    int gr = ls == 0 ? r0 + row
                     : ((r0 + row) >> sh) * ls + min(row & ((1 << sh) - 1), ls - 1);
    gr = gr < nrows ? gr : nrows - 1;
    glds16(X + (int64_t)gr * ld + k0 + c * 8, lds_tile + (i * NW + wave) * 1024);
  }
}
// pass i of stage<ROWS> (i uniform; constant after unrolling)
template <int ROWS>
__device__ __forceinline__ void stage_one(int i, const unsigned short* __restrict__ X, int64_t ld,
                                          int r0, int nrows, int k0, char* lds_tile, int wave,
                                          int lane) {
  const int p = (i * NW + wave) * 64 + lane;
  const int row = p >> 3;
  const int c = (p & 7) ^ chunk_key(row);
  int gr = r0 + row;
  gr = gr < nrows ? gr : nrows - 1;
  glds16(X + (int64_t)gr * ld + k0 + c * 8, lds_tile + (i * NW + wave) * 1024);
}
// passes [P0, P1) of stage<ROWS> (spreading one K-tile's DMA over the k-steps)
template <int ROWS, int P0, int P1>
__device__ __forceinline__ void stage_part(const unsigned short* __restrict__ X, int64_t ld,
                                           int r0, int nrows, int k0, char* lds_tile, int wave,
                                           int lane) {
#pragma unroll
  for (int i = P0; i < P1; ++i) {
    const int p = (i * NW + wave) * 64 + lane;
    const int row = p >> 3;
    const int c = (p & 7) ^ chunk_key(row);
    int gr = r0 + row;
    gr = gr < nrows ? gr : nrows - 1;
    glds16(X + (int64_t)gr * ld + k0 + c * 8, lds_tile + (i * NW + wave) * 1024);
  }
}
// Ring form (RING = true): 32-deep K-tiles in 4 LDS slots (64-byte rows, 40 KB a
// slot at 256 x 384), three in flight: K-tile kt + 3 is issued into the slot K-tile
// kt - 1 used, right after the one barrier of iteration kt (every wave is past its
// reads of kt - 1 there), and waited for by a counted vmcnt three iterations later,
// so the DMA has three K-tiles of MFMAs to land instead of one (the 2-slot form waits
// vmcnt(0) at the end of every 64-deep K-tile: FFN2 181 -> 126 us with no DMA at all,
// profiles/r03_big_q_*).  Chunk c of row r sits in slot c ^ ((r >> 2) & 3), so the 8
// lanes of each ds_read_b128 phase (rows r0 .. r0 + 7) hit 8 distinct 16-byte bank
// slots.  Same MFMAs in the same k order as the 2-slot form: bit-identical results.
constexpr int BK4 = 32, ROW4 = BK4 * 2, NST = 4;
template <int ROWS>
__device__ __forceinline__ void stage4(const unsigned short* __restrict__ X, int64_t ld, int r0,
                                       int nrows, int k0, char* lds_tile, int wave, int lane) {
  constexpr int CH = ROWS * 4;  // 16-byte chunks (4 per 64-byte row)
  static_assert(CH % NT == 0, "whole passes");
#pragma unroll
  for (int i = 0; i < CH / NT; ++i) {
    const int p = (i * NW + wave) * 64 + lane;  // lane-linear LDS chunk
    const int row = p >> 2;
    const int c = (p & 3) ^ ((row >> 2) & 3);
    int gr = r0 + row;
    gr = gr < nrows ? gr : nrows - 1;
    glds16(X + (int64_t)gr * ld + k0 + c * 8, lds_tile + (i * NW + wave) * 1024);
  }
}

#ifdef IRC_BIG_STAMPS  // diagnostic build: per-K-tile phase stamps of block 0, wave 0
// [kt][phase]: s_memtime (shader clock) and s_memrealtime (100 MHz) after each phase of
// mainloop_mf16 -- 0 loop top, 1 DMA issued, 2 fragment reads + MFMAs issued, 3 vmcnt(0)
// returned, 4 barrier passed.  Read by irc_big_dbg_stamps (this build only).
__device__ uint64_t big_stamps[64][5][2];
#define BSTAMP(kt, i)                                                                      \
  do {                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (kt) < 64) {                               \
      uint64_t c_, r_;                                                                     \
      asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"            \
                   : "=s"(c_), "=s"(r_)::"memory");                                        \
      *(volatile uint64_t*)&big_stamps[(kt)][(i)][0] = c_;                                 \
      *(volatile uint64_t*)&big_stamps[(kt)][(i)][1] = r_;                                 \
    }                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                     \
  } while (0)
#else
#define BSTAMP(kt, i) \
  do {                \
  } while (0)
#endif

// The 2-slot K loop in its 16x16x32 form (gemm_big_kernel MF16, qkv_attn_kernel) over
// the 256 x (128 WNB) tile at (m0, n0): wave (wm, wn) = (wave >> 2, wave & 3) accumulates
// acc4[i][j] element e = C[m0 + 128 wm + 16 i + 4 (lane >> 4) + e][n0 + 32 WNB wn + 16 j +
// (lane & 15)].  The chunk key (r >> 1) & 7 stays conflict free for the 16x16x32 fragment
// reads (lane l: row l & 15, chunk 4 s + (l >> 4): each 16-lane group covers 16 distinct
// 16-byte bank slots).  Ends with every wave past its last LDS read (LDS free).
// ls > 0: A rows in the sequence-slot layout of stage() (qkv_attn_kernel at L = ls < 64).
template <int WNB>
__device__ __forceinline__ void mainloop_mf16(const unsigned short* A, int64_t lda,
                                              const unsigned short* B, int64_t ldb, int m0,
                                              int n0, int M, int N, int K, char* lds, int wave,
                                              int lane, f32x4 (&acc4)[8][2 * WNB], int ls = 0,
                                              int sh = 6) {
  constexpr int BN = 128 * WNB;
  constexpr int A_BYTES = BM * ROW_BYTES, STAGE = A_BYTES + BN * ROW_BYTES;
  const int wm = wave >> 2, wn = wave & 3;
  const int nk = K / BK;
  stage<BM>(A, lda, m0, M, 0, lds, wave, lane, ls, sh);
  stage<BN>(B, ldb, n0, N, 0, lds + A_BYTES, wave, lane);
  wait_vmcnt<0>();
  __syncthreads();
  const int l16 = lane & 15, q4 = lane >> 4;
  const int key = chunk_key(l16);  // rows 16 i + l16: (row >> 1) & 7 = (l16 >> 1) & 7
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
#ifdef IRC_PP_DIAG_NODMA  // diagnostic build: only K-tile 0 is loaded
    const bool more = kt + 1 < nk && kt < 0;
#else
    const bool more = kt + 1 < nk;
#endif
    BSTAMP(kt, 0);
    char* nxt = lds + (cur ^ 1) * STAGE;
    if (more) {
      // the DMA addresses are re-derived per K-tile (kept live through the loop they
      // would push the 16x16 fragments into spills)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      stage<BM>(A, lda, m0, M, (kt + 1) * BK, nxt, wave, ln, ls, sh);
      stage<BN>(B, ldb, n0, N, (kt + 1) * BK, nxt + A_BYTES, wave, ln);
    }
    BSTAMP(kt, 1);
    const char* la = lds + cur * STAGE;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int coff = (((4 * s2 + q4) ^ key) * 16);
      bf16x8 fa[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(la + (wm * 128 + i * 16 + l16) * 128 + coff);
#pragma unroll
      for (int j = 0; j < 2 * WNB; ++j) {
        const bf16x8 fb =
            *reinterpret_cast<const bf16x8*>(lb + (wn * 32 * WNB + j * 16 + l16) * 128 + coff);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc4[i][j], 0, 0, 0);
      }
    }
    BSTAMP(kt, 2);
    wait_vmcnt<0>();
    BSTAMP(kt, 3);
    __syncthreads();
    BSTAMP(kt, 4);
  }
}
}  // namespace big

// The 4-slot ring of gemm_big_kernel: off (within noise of the 2-slot loop on every BERT
// shape and 1.4% slower on the C2 step, profiles/r03_ring_r_*); irc_gemm_set_big_ring
// switches it at run time (the tests compare both bit for bit).
inline std::atomic<int>& big_ring_mode() {
  static std::atomic<int> on{0};
  return on;
}
inline bool big_ring() { return big_ring_mode().load(std::memory_order_relaxed) != 0; }

// The 16x16x32 MFMA form of gemm_big_kernel is the default (irc_gemm_set_big_mf16 selects
// the 32x32x16 form at run time; the tests compare both).  Measured on MI355X,
// interleaved (profiles/r04_f_*): out-proj 48.6 / 48.4 vs 53.1 / 50.3 us, FFN2 156.7 /
// 152.9 vs 163.5 / 164.2 us, the C2 step 27.3k vs 26.7k pairs/s.
inline std::atomic<int>& big_mf16_mode() {
  static std::atomic<int> on{1};
  return on;
}
inline bool big_mf16() { return big_mf16_mode().load(std::memory_order_relaxed) != 0; }

// MF16: v_mfma_f32_16x16x32_bf16 instead of 32x32x16 (2-slot form only): the same
// 256 x 128 WNB tile and LDS image, 8 x 2 WNB accumulators of 16 x 16 per wave, one
// k32 step per half K-tile.  The chunk key (r >> 1) & 7 stays conflict free for the
// 16x16x32 fragment reads too (lane l: row l & 15, chunk 4 s + (l >> 4): each 16-lane
// group covers 16 distinct 16-byte bank slots).  On MI355X the 16x16x32 loop runs at
// a higher clock for the same work (MI355X_MICROARCH.md, bf16 MFMA shapes).
//
// LN: the LayerNorm-fold instantiation (irc_gemm_ln, 16x16x32 form only; see LnArgs) --
// a template flag so the other instantiations keep their register allocation.
template <typename TO, int EPI, int WNB, bool RING = false, bool MF16 = false, bool LN = false>
__global__ __launch_bounds__(big::NT, 1) void gemm_big_kernel(Args g) {
  static_assert(!(RING && MF16), "the 16x16x32 form is 2-slot only");
  static_assert(!LN || (MF16 && sizeof(TO) == 2), "the LayerNorm fold: 16x16x32 form, bf16 C");
  using big::BK;
  using big::NT;
  using big::NW;
  constexpr int BM = big::BM, BN = 128 * WNB;
  constexpr int A_BYTES = BM * big::ROW_BYTES, B_BYTES = BN * big::ROW_BYTES;
  constexpr int STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char lds[2 * STAGE];  // [stage][A | B]
  const int tiles_m = (g.M + BM - 1) / BM;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap: blocks sharing an XCD walk consecutive tiles
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  int tm, tn;
  grouped_tile(bid, tiles_m, tiles_n, g.group_m, tm, tn);
  const int batch = blockIdx.y;
  const unsigned short* A = reinterpret_cast<const unsigned short*>(g.A) + batch * g.sA;
  const unsigned short* B = reinterpret_cast<const unsigned short*>(g.B) + batch * g.sB;
  TO* C = reinterpret_cast<TO*>(g.C) + batch * g.sC;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int h = lane >> 5, r32 = lane & 31;

  f32x16 acc[4][WNB];
  f32x4 acc4[8][2 * WNB];  // MF16: element e -> row 16 i + 4 (lane >> 4) + e, col 16 j + (lane & 15)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WNB; ++j) acc[i][j] = (f32x16)0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * WNB; ++j) acc4[i][j] = (f32x4)0.0f;

  if constexpr (RING) {
    using big::BK4;
    using big::ROW4;
    constexpr int A4 = BM * ROW4, STG4 = A4 + BN * ROW4;
    static_assert(big::NST * STG4 <= 2 * STAGE, "ring fits the 2-slot allocation");
    constexpr int PPT = (BM * 4 + BN * 4) / NT;  // DMA wave-instructions per K-tile per wave
    const int nk = g.K / BK4;
#pragma unroll
    for (int s0 = 0; s0 < big::NST - 1; ++s0)
      if (s0 < nk) {
        big::stage4<BM>(A, g.lda, m0, g.M, s0 * BK4, lds + s0 * STG4, wave, lane);
        big::stage4<BN>(B, g.ldb, n0, g.N, s0 * BK4, lds + s0 * STG4 + A4, wave, lane);
      }
    const int sw4 = (r32 >> 2) & 3;
    for (int kt = 0; kt < nk; ++kt) {
      // K-tiles kt + 1, kt + 2 may still be in flight (issued after kt)
      const int after = nk - 1 - kt;
      if (after >= 2) wait_vmcnt<2 * PPT>();
      else if (after == 1) wait_vmcnt<PPT>();
      else wait_vmcnt<0>();
      wg_barrier();  // every wave's share of kt landed; every wave done reading kt - 1
      if (kt + 3 < nk) {
        char* nxt = lds + ((kt + 3) & 3) * STG4;
        big::stage4<BM>(A, g.lda, m0, g.M, (kt + 3) * BK4, nxt, wave, lane);
        big::stage4<BN>(B, g.ldb, n0, g.N, (kt + 3) * BK4, nxt + A4, wave, lane);
      }
      const char* la = lds + (kt & 3) * STG4;
      const char* lb = la + A4;
#pragma unroll
      for (int kk = 0; kk < BK4 / 16; ++kk) {
        const int coff = ((2 * kk + h) ^ sw4) * 16;
        bf16x8 fa[4], fb[WNB];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = *reinterpret_cast<const bf16x8*>(la + (wm * 128 + i * 32 + r32) * ROW4 + coff);
#pragma unroll
        for (int j = 0; j < WNB; ++j)
          fb[j] = *reinterpret_cast<const bf16x8*>(lb + (wn * 32 * WNB + j * 32 + r32) * ROW4 + coff);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WNB; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();  // the epilogue's staging rows overlap the ring
  } else if constexpr (MF16) {
    big::mainloop_mf16<WNB>(A, g.lda, B, g.ldb, m0, n0, g.M, g.N, g.K, lds, wave, lane, acc4);
  } else {
  const int nk = g.K / BK;
  big::stage<BM>(A, g.lda, m0, g.M, 0, lds, wave, lane);
  big::stage<BN>(B, g.ldb, n0, g.N, 0, lds + A_BYTES, wave, lane);
  wait_vmcnt<0>();
  __syncthreads();
  const int swz = big::chunk_key(r32);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
#ifdef IRC_PP_DIAG_NODMA  // diagnostic build: only K-tile 0 is loaded
    const bool more = kt + 1 < nk && kt < 0;
#else
    const bool more = kt + 1 < nk;
#endif
    if (more) {
      char* nxt = lds + (cur ^ 1) * STAGE;
      big::stage<BM>(A, g.lda, m0, g.M, (kt + 1) * BK, nxt, wave, lane);
      big::stage<BN>(B, g.ldb, n0, g.N, (kt + 1) * BK, nxt + A_BYTES, wave, lane);
    }
    const char* la = lds + cur * STAGE;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int coff = (((2 * kk + h) ^ swz) * 16);
      bf16x8 fa[4], fb[WNB];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(la + (wm * 128 + i * 32 + r32) * 128 + coff);
#pragma unroll
      for (int j = 0; j < WNB; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(lb + (wn * 32 * WNB + j * 32 + r32) * 128 + coff);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WNB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    wait_vmcnt<0>();
    __syncthreads();
  }
  }  // 2-slot form

#ifdef IRC_PP_DIAG_NOEPI  // diagnostic build: main loop only (every accumulator kept live)
  {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < WNB; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) t += acc[i][j][e];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 2 * WNB; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) t += acc4[i][j][e];
    if (t == 1234.5f) reinterpret_cast<float*>(g.C)[threadIdx.x] = t;
    return;
  }
#endif
  const float* bias = g.bias ? g.bias + batch * g.sBias : nullptr;
  const TO* R = g.R ? reinterpret_cast<const TO*>(g.R) + batch * g.sR : nullptr;
  constexpr int WCOLS = 32 * WNB;  // columns per wave
  if (g.vec_c) {
    // Staged epilogue: the wave's 128 x WCOLS fp32 tile goes through LDS in four
    // 32-row passes (row pitch WCOLS+8 floats: rows r and r+4 of the two
    // half-waves land 128 B apart in bank space, so the ds_write_b32 are
    // conflict free) and leaves as coalesced 16-byte row pieces; bias / GELU
    // before, residual / accumulate after, all fp32 (one rounding).
    constexpr int PITCH = WCOLS + 8;
    float* st = reinterpret_cast<float*>(lds) + wave * (32 * PITCH);
    const int rbase0 = m0 + wm * 128;
    const int cbase = n0 + wn * WCOLS;
    // LayerNorm fold (bf16 C; uniform flags): see LnArgs (gemm_pp.h)
    constexpr bool LNOK = LN;
    const bool lnfold = LNOK && g.ln.fold_s != nullptr;
    const bool lnres = LNOK && g.ln.gamma != nullptr;
    const bool lnout = LNOK && g.ln.st_out != nullptr;
    float* lst = reinterpret_cast<float*>(lds) + 8 * 32 * PITCH;  // [256 rows][2] partials
    static_assert((8 * 32 * PITCH + 512) * 4 <= 2 * STAGE, "LN partials fit the LDS");
    if (lnout) {
      lst[threadIdx.x] = 0.f;  // 512 threads, 512 floats
      __syncthreads();
    }
    float bv[WNB], bv16[2 * WNB];
#pragma unroll
    for (int j = 0; j < WNB; ++j) {
      const int col = cbase + j * 32 + r32;
      bv[j] = !MF16 && epi_has_bias(EPI) && col < g.N ? bias[col] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 2 * WNB; ++j) {
      const int col = cbase + j * 16 + (lane & 15);
      bv16[j] = MF16 && epi_has_bias(EPI) && col < g.N ? bias[col] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (MF16) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int j = 0; j < 2 * WNB; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int rl = 16 * ii + 4 * (lane >> 4) + e;
              float v = acc4[2 * i + ii][j][e] * g.alpha + (lnfold ? 0.f : bv16[j]);
              if (EPI == EPI_BIAS_GELU && !lnfold) v = sizeof(TO) == 2 ? gelu_lite(v) : gelu_fast(v);
              st[rl * PITCH + j * 16 + (lane & 15)] = v;
            }
      } else {
#pragma unroll
      for (int j = 0; j < WNB; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rl = (e & 3) + 8 * (e >> 2) + 4 * h;
          float v = acc[i][j][e] * g.alpha + (lnfold ? 0.f : bv[j]);
          if (EPI == EPI_BIAS_GELU && !lnfold) v = sizeof(TO) == 2 ? gelu_lite(v) : gelu_fast(v);
          st[rl * PITCH + j * 32 + r32] = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int rbase = rbase0 + i * 32;
      if constexpr (sizeof(TO) == 2) {
        constexpr int CPR = WCOLS / 8;  // 16-byte bf16 chunks per row
#pragma unroll
        for (int it = 0; it < 32 * CPR / 64; ++it) {
          const int c = it * 64 + lane;
          const int rl = c / CPR, c8 = (c % CPR) * 8;
          const int row = rbase + rl, col = cbase + c8;
          if (row >= g.M || col >= g.N) continue;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(&st[rl * PITCH + c8]);
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(&st[rl * PITCH + c8 + 4]);
          float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
            if (lnfold) {  // y = r acc + (-r mu) s + t, then GELU
              float mu, rs;
              ln_row_stats(g.ln, row, mu, rs);
              const float nrm = -rs * mu;
              const float* sc = g.ln.fold_s + col;
              const float* tc = bias + col;
              const f32x4 s0 = *reinterpret_cast<const f32x4*>(sc), s1 = *reinterpret_cast<const f32x4*>(sc + 4);
              const f32x4 t0 = *reinterpret_cast<const f32x4*>(tc), t1 = *reinterpret_cast<const f32x4*>(tc + 4);
              const float ss[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
              const float tt[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
              for (int t = 0; t < 8; ++t) v[t] = __builtin_fmaf(rs, v[t], __builtin_fmaf(nrm, ss[t], tt[t]));
              if (EPI == EPI_BIAS_GELU) {
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = gelu_lite(v[t]);
              }
            }
          }
          if (EPI == EPI_BIAS_RESID && lnres) {  // residual = LN(R) as the LN kernel writes it
            const u16x8 rr = *reinterpret_cast<const u16x8*>(
                reinterpret_cast<const unsigned short*>(R) + (int64_t)row * g.ldr + col);
            float mu, rs;
            ln_row_stats(g.ln, row, mu, rs);
            const f32x4 g0 = *reinterpret_cast<const f32x4*>(g.ln.gamma + col);
            const f32x4 g1 = *reinterpret_cast<const f32x4*>(g.ln.gamma + col + 4);
            const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.ln.beta + col);
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.ln.beta + col + 4);
            const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
            const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
            for (int t = 0; t < 8; ++t)
              v[t] += bf16_to_f32(f32_to_bf16(__builtin_fmaf((bf16_to_f32(rr[t]) - mu) * rs, gg[t], bb[t])));
          } else if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
            const u16x8 rr = *reinterpret_cast<const u16x8*>(
                reinterpret_cast<const unsigned short*>(R) + (int64_t)row * g.ldr + col);
#pragma unroll
            for (int t = 0; t < 8; ++t)
              v[t] = EPI == EPI_DGELU ? v[t] * gelu_grad_fast(bf16_to_f32(rr[t]))
                                      : v[t] + bf16_to_f32(rr[t]);
          }
          if (EPI == EPI_BIAS_GELU_SAVE) {
            u16x8 pre;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              pre[t] = f32_to_bf16(v[t]);
              v[t] = gelu_fast(v[t]);
            }
            *reinterpret_cast<u16x8*>(const_cast<unsigned short*>(
                reinterpret_cast<const unsigned short*>(R)) + (int64_t)row * g.ldr + col) = pre;
          }
          u16x8 o;
#pragma unroll
          for (int t = 0; t < 8; ++t) o[t] = f32_to_bf16(v[t]);
          if (lnout) {  // row partials of the bf16 output (this tile's columns)
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const float x = bf16_to_f32(o[t]);
              s1 += x;
              s2 = __builtin_fmaf(x, x, s2);
            }
            const int lr = row - m0;
            atomicAdd(&lst[2 * lr], s1);
            atomicAdd(&lst[2 * lr + 1], s2);
          }
#ifdef IRC_PP_DIAG_NOSTORE  // diagnostic build: the epilogue without its C stores
          if (o[0] == 0x7fc1 && o[7] == 0x7fc3)
#endif
          *reinterpret_cast<u16x8*>(reinterpret_cast<unsigned short*>(C) + (int64_t)row * g.ldc +
                                    col) = o;
        }
      } else {
        constexpr int CPR = WCOLS / 4;  // 16-byte fp32 chunks per row
#pragma unroll
        for (int it = 0; it < 32 * CPR / 64; ++it) {
          const int c = it * 64 + lane;
          const int rl = c / CPR, c4 = (c % CPR) * 4;
          const int row = rbase + rl, col = cbase + c4;
          if (row >= g.M || col >= g.N) continue;
          f32x4 v = *reinterpret_cast<const f32x4*>(&st[rl * PITCH + c4]);
          if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
            const f32x4 r = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(R) +
                                                            (int64_t)row * g.ldr + col);
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = EPI == EPI_DGELU ? v[t] * gelu_grad_fast(r[t]) : v[t] + r[t];
          }
          if (EPI == EPI_BIAS_GELU_SAVE) {
            *reinterpret_cast<f32x4*>(const_cast<float*>(reinterpret_cast<const float*>(R)) +
                                      (int64_t)row * g.ldr + col) = v;
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = gelu_fast(v[t]);
          }
          float* dst = reinterpret_cast<float*>(C) + (int64_t)row * g.ldc + col;
          if (g.accumulate) v += *reinterpret_cast<const f32x4*>(dst);
          *reinterpret_cast<f32x4*>(dst) = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (lnout) {  // this tile's (sum, sum of squares) of every row, one pair per tile column
      lds_barrier();
      const int lr = threadIdx.x >> 1, row = m0 + lr;
      if (row < g.M)
        g.ln.st_out[((int64_t)row * g.ln.nt_out + tn) * 2 + (threadIdx.x & 1)] = lst[threadIdx.x];
    }
    return;
  }
  constexpr int NJ = MF16 ? 2 * WNB : WNB, NI = MF16 ? 8 : 4, NE = MF16 ? 4 : 16;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = MF16 ? n0 + wn * WCOLS + j * 16 + (lane & 15) : n0 + wn * WCOLS + j * 32 + r32;
    if (col >= g.N) continue;
    const float bv = epi_has_bias(EPI) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int row = MF16 ? m0 + wm * 128 + i * 16 + 4 * (lane >> 4) + e
                             : m0 + wm * 128 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= g.M) continue;
        float v = (MF16 ? acc4[i % 8][j % (2 * WNB)][e % 4] : acc[i % 4][j % WNB][e % 16]) * g.alpha +
                  bv;
        if (EPI == EPI_BIAS_GELU) v = sizeof(TO) == 2 ? gelu_lite(v) : gelu_fast(v);
        if (EPI == EPI_BIAS_GELU_SAVE) {
          TO* pre = const_cast<TO*>(R) + (int64_t)row * g.ldr + col;
          if constexpr (sizeof(TO) == 2)
            *reinterpret_cast<unsigned short*>(pre) = f32_to_bf16(v);
          else
            *reinterpret_cast<float*>(pre) = v;
          v = gelu_fast(v);
        }
        if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
          float r;
          if constexpr (sizeof(TO) == 2)
            r = bf16_to_f32(reinterpret_cast<const unsigned short*>(R)[(int64_t)row * g.ldr + col]);
          else
            r = reinterpret_cast<const float*>(R)[(int64_t)row * g.ldr + col];
          v = EPI == EPI_DGELU ? v * gelu_grad_fast(r) : v + r;
        }
        TO* dst = C + (int64_t)row * g.ldc + col;
        if constexpr (sizeof(TO) == 2) {
          *reinterpret_cast<unsigned short*>(dst) = f32_to_bf16(v);
        } else {
          if (g.accumulate)
            *reinterpret_cast<float*>(dst) += v;
          else
            *reinterpret_cast<float*>(dst) = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// QKV projection + self-attention in one launch: the frozen encoder's BertSelfAttention
// (modeling_bert, reached from contrastive_module.py:36-41) at L <= 128, head dim 64.
// The Wqkv rows are permuted so that output tile column block n (384 wide) holds
// [Q | K | V] of heads 2n and 2n + 1 (64 columns each), and a 256-row tile holds whole
// sequences, each in a slot of SL rows: four of 64 (L <= 64) or two of 128 (L <= 128).
// At L < SL (the joint padding of a batch) the slot's rows past L repeat token L - 1,
// their keys carry the -3e30 past-L bias and their queries are never stored, as in
// attention_mfma_kernel; the QKV activation then never leaves the CU.  Main loop: the big-tile
// kernel's 16x16x32 2-slot loop (WNB = 3).  Epilogue, per 128-row half (the waves with
// wm == half own its accumulators): those 4 waves write bf16(acc + bias) into LDS
// [128][392] (the same bf16 values the unfused GEMM stores), then all 8 waves run its
// attention, one (sequence, head, 32 queries) each, with attention_mfma_kernel's
// arithmetic (encoder.hip: S^T by 32x32x16 MFMAs, scale, mask bias, max / exp / sum,
// P rounded to bf16, P.V), so the
// context equals the unfused QKV GEMM + irc_attention output bit for bit wherever the
// unfused QKV runs on this main loop (the big-tile shapes).  The halves run one after
// the other; every wave first packs its accumulators to bf16 pairs (96 VGPRs), so the
// waiting half's values and the attention's registers fit side by side.
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
struct QaArgs {
  const unsigned short* x;  // [M][K] layer input
  const unsigned short* w;  // [3H][K] head-pair-permuted Wqkv
  const float* bias;        // [3H] permuted bias
  const int64_t* mask;      // [M / L][L], nonzero = key visible; null = all visible
  unsigned short* ctx;      // [M][H] (row stride ldc)
  int M, K, H;
  int64_t ldx, ldc;
  float scale;
  int L;                    // sequence length, 1..128
  int group_m;              // grouped tile order (grouped_tile; 0 = row-major)
};

//
// SL = 0, the packed form (any L <= 128; launched where it takes fewer waves of tiles, see
// irc_qkv_attention): a 256-row tile holds 256 / L whole sequences as contiguous rows (L =
// 80: three, where 128-row slots take two), and the epilogue stages one head at a time for all
// 256 rows -- T [256][264]: that head's Q | K | V columns, 135 KB -- because a sequence now
// straddles the 128-row halves.  Per head the 8 waves take (sequence, 32 queries) items in
// turn, with the same per-item arithmetic, so the context is again bit-identical to the
// unfused form.  Key and query rows past the tile's 256 (a last sequence's last key block)
// are read from row 255: finite values whose probabilities the -3e30 past-L bias zeroes,
// and whose queries are not stored.
template <int SL>
__global__ __launch_bounds__(big::NT, 1) void qkv_attn_kernel(QaArgs g) {
  constexpr bool PACK = SL == 0;
  constexpr int WNB = 3, BM = big::BM, BN = 128 * WNB, TP = BN + 8;
  constexpr int SLX = PACK ? 128 : SL;  // key rows of a sequence, at most
  constexpr int SH = SLX == 64 ? 6 : 7;
  constexpr int NJM = SLX / 32;         // key blocks of 32 per sequence, at most
  __shared__ __attribute__((aligned(1024))) char lds[2 * (BM + BN) * big::ROW_BYTES];
  static_assert(128 * TP * 2 + 8 * SLX * 4 <= 2 * (BM + BN) * big::ROW_BYTES,
                "staged half and mask biases fit the LDS");
  const int nseq = g.M / g.L;
  // sequences per tile: 4 (SL = 64), 2 (SL = 128) or 256 / L (packed)
  const int spt = PACK ? BM / g.L : BM / SLX;
  const int ls = PACK || g.L == SL ? 0 : g.L;  // 0: contiguous rows
  const int tiles_m = (nseq + spt - 1) / spt;
  const int tiles_n = 3 * g.H / BN;
  const int ntiles = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap, as gemm_big_kernel
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  int tm, tn;
  grouped_tile(bid, tiles_m, tiles_n, g.group_m, tm, tn);
  // packed: first token row of the tile's first sequence; slots: first slot row
  const int m0 = PACK ? tm * spt * g.L : tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  f32x4 acc4[8][2 * WNB];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * WNB; ++j) acc4[i][j] = (f32x4)0.0f;
  big::mainloop_mf16<WNB>(g.x, g.ldx, g.w, g.K, m0, n0, g.M, 3 * g.H, g.K, lds, wave, lane, acc4,
                          ls, SH);

  unsigned short* T = reinterpret_cast<unsigned short*>(lds);    // [128][TP] staged half
  float* mbw = reinterpret_cast<float*>(lds + 128 * TP * 2) + SL * wave;  // this wave's key bias
  // acc + bias -> bf16 pairs (rows e, e + 1 of one column) in registers:
  // 96 VGPRs instead of 192 live while the halves take turns through the LDS
  uint32_t pk[8][2 * WNB][2];
#pragma unroll
  for (int j = 0; j < 2 * WNB; ++j) {
    const int col = n0 + wn * 32 * WNB + 16 * j + (lane & 15);
    const float bvj = g.bias[col];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        f32x2_t v;
#pragma unroll
        for (int u = 0; u < 2; ++u) v[u] = acc4[i][j][2 * e2 + u] * 1.0f + bvj;
        // one v_cvt_pk_bf16_f32 per pair (RNE, as f32_to_bf16); opaque, so the compiler
        // cannot forward the unpacked values to the staging stores and keep 192 live
        uint32_t w = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_v));
        asm volatile("" : "+v"(w));
        pk[i][j][e2] = w;
      }
  }
  const int h = lane >> 5, r32 = lane & 31;
  const int nj = (g.L + 31) / 32;  // key (and query) blocks of 32 of a sequence
  if constexpr (PACK) {
    constexpr int TQ = 264;  // 192 columns + pad: a 132-dword row stride, as TP's 196 = 4 mod 64
    static_assert(BM * TQ * 2 + 8 * 128 * 4 <= 2 * (BM + BN) * big::ROW_BYTES,
                  "staged head and mask biases fit the LDS");
    unsigned short* Tq = reinterpret_cast<unsigned short*>(lds);  // [256][TQ] one head
    float* mb = reinterpret_cast<float*>(lds + BM * TQ * 2) + 128 * wave;
    const int odd = lane & 1;
    const int nsq = min(spt, nseq - tm * spt);  // sequences in this tile
    const int nit = nsq * nj;                   // (sequence, query block) items per head
#pragma unroll
    for (int hd = 0; hd < 2; ++hd) {
      // this head's columns of every wave's accumulators -> Tq (Q at 0, K at 64, V at 128);
      // tile column b of a 16-column group: part b >> 7, head (b >> 6) & 1
#pragma unroll
      for (int j = 0; j < 2 * WNB; ++j) {
        const int b = wn * 32 * WNB + 16 * j;
        if (((b >> 6) & 1) != hd) continue;
        const int tc = 64 * (b >> 7) + (b & 63) + (lane & 14);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            const uint32_t w = pk[i][j][e2];
            const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, false);
            const uint32_t v = odd ? ((x >> 16) | (w & 0xFFFF0000u)) : ((w & 0xFFFFu) | (x << 16));
            const int rl = 128 * wm + 16 * i + 4 * (lane >> 4) + 2 * e2 + odd;
            *reinterpret_cast<uint32_t*>(&Tq[rl * TQ + tc]) = v;
          }
      }
      __syncthreads();  // the head is staged
      for (int it = wave; it < nit; it += 8) {
        const int s = it / nj, ib = it - s * nj;
        const int t0 = s * g.L;                  // the sequence's first tile row
        const int r0 = (tm * spt + s) * g.L;     // its first token
#pragma unroll
        for (int j = lane; j < 128; j += 64)
          mb[j] = j >= g.L ? -3e30f
                           : ((g.mask == nullptr || g.mask[r0 + j] != 0) ? 0.f : -1e30f);
        const int nkb = visible_key_blocks(g.mask ? g.mask + r0 : nullptr, g.L, nj, lane);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned short* Q = Tq;
        const unsigned short* Kp = Tq + 64;
        const unsigned short* V = Tq + 128;
        unsigned short* out = g.ctx + (int64_t)r0 * g.ldc + (2 * tn + hd) * 64;
        bf16x8 qf[4];
        const int qr = min(t0 + 32 * ib + r32, BM - 1);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          qf[kk] = *reinterpret_cast<const bf16x8*>(Q + qr * TQ + 16 * kk + 8 * h);
        f32x16 sc[NJM];
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          sc[jb] = (f32x16)0.f;
          if (jb < nkb) {
            const int kr = min(t0 + 32 * jb + r32, BM - 1);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
              const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Kp + kr * TQ + 16 * kk + 8 * h);
              sc[jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], sc[jb], 0, 0, 0);
            }
          }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 bias = *reinterpret_cast<const f32x4*>(&mb[32 * jb + 8 * q + 4 * h]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = sc[jb][4 * q + r] * g.scale + bias[r];
              sc[jb][4 * q + r] = v;
              mx = fmaxf(mx, v);
            }
          }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float sum = 0.f;
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float p = __expf(sc[jb][e] - mx);
            sc[jb][e] = p;
            sum += p;
          }
        }
        sum += __shfl_xor(sum, 32, 64);
        const float inv = 1.f / sum;
        f32x16 o[2] = {(f32x16)0.f, (f32x16)0.f};
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) {
            bf16x8 pa;
#pragma unroll
            for (int t = 0; t < 8; ++t) pa[t] = (__bf16)(sc[jb][8 * k2 + t] * inv);
            const int j0 = 32 * jb + 16 * k2 + 4 * h;
            const int i16 = lane & 15;
            const int vr = t0 + j0 + (i16 >> 2);
#pragma unroll
            for (int db = 0; db < 2; ++db) {
              const int vc = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
              const v4s lo = ds_tr16(reinterpret_cast<const char*>(V + min(vr, BM - 1) * TQ + vc));
              const v4s hi =
                  ds_tr16(reinterpret_cast<const char*>(V + min(vr + 8, BM - 1) * TQ + vc));
              const v4s both[2] = {lo, hi};
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, both),
                                                              o[db], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int i = 32 * ib + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (i < g.L) out[(int64_t)i * g.ldc + 32 * db + r32] = f32_to_bf16(o[db][e]);
          }
      }
      if (hd == 0) __syncthreads();  // every wave is done with head 0's Tq
    }
    return;
  }
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    if (wm == hf) {  // this half's accumulators -> T [128][TP]
      // a lane holds rows (r, r + 1) of its column; swapping with the neighbour lane
      // (DPP quad_perm [1,0,3,2]) gives the even lane columns (c, c + 1) of row r and the
      // odd lane those of row r + 1: one 4-byte store per pair instead of two 2-byte ones
      const int odd = lane & 1;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2 * WNB; ++j)
#pragma unroll
          for (int e2 = 0; e2 < 2; ++e2) {
            const uint32_t w = pk[i][j][e2];
            const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, false);
            const uint32_t v = odd ? ((x >> 16) | (w & 0xFFFF0000u)) : ((w & 0xFFFFu) | (x << 16));
            const int rl = 16 * i + 4 * (lane >> 4) + 2 * e2 + odd;
            *reinterpret_cast<uint32_t*>(&T[rl * TP + wn * 32 * WNB + 16 * j + (lane & 14)]) = v;
          }
    }
    __syncthreads();  // the half is staged
    // every wave: 32 queries of one (sequence, head) of this half (the other half's
    // waves hold their packed values meanwhile).  SL = 64: two sequences per half,
    // wave = (query block wm, sequence wn >> 1, head wn & 1); SL = 128: one sequence,
    // wave = (query block wave >> 1, head wave & 1)
    const int sl = SL == 64 ? wn >> 1 : 0, hh = SL == 64 ? wn & 1 : wave & 1;
    const int ib = SL == 64 ? wm : wave >> 1;
    const int seq = spt * tm + (SL == 64 ? 2 * hf + sl : hf);
    const int r0 = seq * g.L;  // first token of the sequence
    if (seq < nseq && ib < nj) {
#pragma unroll
      for (int j = lane; j < SL; j += 64)
        mbw[j] = j >= g.L ? -3e30f
                          : ((g.mask == nullptr || g.mask[r0 + j] != 0) ? 0.f : -1e30f);
      // key blocks through the sequence's last visible key (the rest add exactly zero)
      const int nkb = visible_key_blocks(g.mask ? g.mask + r0 : nullptr, g.L, nj, lane);
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned short* Ts = T + 64 * sl * TP;
      const unsigned short* Q = Ts + hh * 64;
      const unsigned short* Kp = Ts + 128 + hh * 64;
      const unsigned short* V = Ts + 256 + hh * 64;
      unsigned short* out = g.ctx + (int64_t)r0 * g.ldc + (2 * tn + hh) * 64;
      {
        bf16x8 qf[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          qf[kk] = *reinterpret_cast<const bf16x8*>(Q + (32 * ib + r32) * TP + 16 * kk + 8 * h);
        // the key blocks jb < nj, in order: attention_mfma_kernel<nj>'s arithmetic
        f32x16 sc[NJM];
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          sc[jb] = (f32x16)0.f;
          if (jb < nkb) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
              const bf16x8 kf =
                  *reinterpret_cast<const bf16x8*>(Kp + (32 * jb + r32) * TP + 16 * kk + 8 * h);
              sc[jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kk], sc[jb], 0, 0, 0);
            }
          }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 bias = *reinterpret_cast<const f32x4*>(&mbw[32 * jb + 8 * q + 4 * h]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = sc[jb][4 * q + r] * g.scale + bias[r];
              sc[jb][4 * q + r] = v;
              mx = fmaxf(mx, v);
            }
          }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float sum = 0.f;
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float p = __expf(sc[jb][e] - mx);
            sc[jb][e] = p;
            sum += p;
          }
        }
        sum += __shfl_xor(sum, 32, 64);
        const float inv = 1.f / sum;
        f32x16 o[2] = {(f32x16)0.f, (f32x16)0.f};
#pragma unroll
        for (int jb = 0; jb < NJM; ++jb) {
          if (jb >= nkb) break;
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) {
            bf16x8 pa;
#pragma unroll
            for (int t = 0; t < 8; ++t) pa[t] = (__bf16)(sc[jb][8 * k2 + t] * inv);
            const int j0 = 32 * jb + 16 * k2 + 4 * h;  // keys: t < 4: j0 + t; else j0 + 8 + t - 4
#pragma unroll
            for (int db = 0; db < 2; ++db) {
              // V^T fragment by two transposed LDS reads: 16-lane group g (d half g & 1)
              // addresses keys j0 + (l >> 2) and 4 columns 4 (l & 3) of its 16; lane l of
              // the group receives column l of those 4 keys (then keys + 8)
              const int i16 = lane & 15;
              const unsigned short* vp =
                  V + (j0 + (i16 >> 2)) * TP + 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
              const v4s lo = ds_tr16(reinterpret_cast<const char*>(vp));
              const v4s hi = ds_tr16(reinterpret_cast<const char*>(vp + 8 * TP));
              const v4s both[2] = {lo, hi};
              o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, __builtin_bit_cast(bf16x8, both),
                                                              o[db], 0, 0, 0);
            }
          }
        }
        // O: col = d (32 db + r32), row = query 32 ib + (e & 3) + 8 (e >> 2) + 4 h
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int i = 32 * ib + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (i < g.L) out[(int64_t)i * g.ldc + 32 * db + r32] = f32_to_bf16(o[db][e]);
          }
      }
    }
    if (hf == 0) __syncthreads();  // the half's readers are done with T
  }
}

// The large-tile path applies: bf16 in, A [M][K] and B [N][K], aligned, K % 64,
// and enough tiles to occupy the chip.  Returns the per-wave N blocks (0: no).
inline int big_wnb(const Args& g, int batch, int la, int lb) {
  if (la != ROW || lb != ROW || !g.vec_a || !g.vec_b) return 0;
  if (g.K % big::BK != 0 || g.K == 0) return 0;
  const int wnb = g.N % 384 == 0 ? 3 : 2;
  const int64_t tiles = (int64_t)((g.M + 255) / 256) * ((g.N + 128 * wnb - 1) / (128 * wnb)) * batch;
  return tiles >= 128 ? wnb : 0;
}

template <typename TO, int EPI, bool LN = false>
static int launch_big(const Args& g, int batch, int wnb, hipStream_t st) {
  const int bn = 128 * wnb;
  const int tiles = ((g.M + big::BM - 1) / big::BM) * ((g.N + bn - 1) / bn);
  prof_begin(st);
  const bool ring = big_ring() && g.K % big::BK4 == 0;
  if constexpr (LN) {
    if (wnb == 3)
      hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 3, false, true, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 2, false, true, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  } else if (big_mf16() && !ring) {
    if (wnb == 3)
      hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 3, false, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
    else
      hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 2, false, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  } else if (wnb == 3 && ring)
    hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 3, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  else if (wnb == 3)
    hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 3>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  else if (ring)
    hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 2, true>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  else
    hipLaunchKernelGGL((gemm_big_kernel<TO, EPI, 2>), dim3(tiles, batch), dim3(big::NT), 0, st, g);
  prof_end("gemm_bf16", st, 2.0 * g.M * g.N * g.K * batch);
  prof_work("gemm_bf16_bytes", gemm_alg_bytes(sizeof(TO) == 4, EPI, g.accumulate, g.M, g.N, g.K,
                                               batch));
  return check_launch("gemm_big_kernel");
}

template <typename TI, typename TO, int LA, int LB, int EPI>
static int launch(const Args& g0, int batch, int splits, hipStream_t st) {
  if constexpr (sizeof(TI) == 2) {
    if (splits == 1) {
      const int wnb = big_wnb(g0, batch, LA, LB);
      if (wnb) return launch_big<TO, EPI>(g0, batch, wnb, st);
    }
  }
  Args g = g0;
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  constexpr int bk = TT<TI>::BK;
  g.kchunk = splits > 1 ? ((g.K + splits - 1) / splits + bk - 1) / bk * bk : (g.K > 0 ? g.K : 1);
  prof_begin(st);
  hipLaunchKernelGGL((gemm_kernel<TI, TO, LA, LB, EPI>), dim3(tiles, batch, splits), dim3(NT), 0,
                     st, g);
  if (splits > 1) {
    const int64_t n = (int64_t)g.M * g.N * batch;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       g.P, reinterpret_cast<float*>(g.C), g.M, g.N, splits, g.ldc, g.sC, batch,
                       g.alpha, g.accumulate, EPI == EPI_BIAS ? g.bias : nullptr, g.sBias);
  }
  prof_end(sizeof(TI) == 2 ? "gemm_bf16" : "gemm_f32", st, 2.0 * g.M * g.N * g.K * batch);
  if (sizeof(TI) == 2)
    prof_work("gemm_bf16_bytes", gemm_alg_bytes(sizeof(TO) == 4, EPI, g.accumulate, g.M, g.N, g.K,
                                                 batch));
  return check_launch("gemm_kernel");
}

template <typename TI, typename TO, int LA, int LB>
static int by_epi(int epi, const Args& g, int batch, int splits, hipStream_t st) {
  switch (epi) {
    case EPI_NONE: return launch<TI, TO, LA, LB, EPI_NONE>(g, batch, splits, st);
    case EPI_BIAS:  // split only for fp32 operands (split_count); the reduce adds the bias
      return launch<TI, TO, LA, LB, EPI_BIAS>(g, batch, sizeof(TI) == 4 ? splits : 1, st);
    case EPI_BIAS_GELU: return launch<TI, TO, LA, LB, EPI_BIAS_GELU>(g, batch, 1, st);
    case EPI_BIAS_RESID: return launch<TI, TO, LA, LB, EPI_BIAS_RESID>(g, batch, 1, st);
    case EPI_RESID: return launch<TI, TO, LA, LB, EPI_RESID>(g, batch, 1, st);
    case EPI_DGELU: return launch<TI, TO, LA, LB, EPI_DGELU>(g, batch, 1, st);
    case EPI_BIAS_GELU_SAVE: return launch<TI, TO, LA, LB, EPI_BIAS_GELU_SAVE>(g, batch, 1, st);
  }
  set_error("gemm: bad epilogue %d", epi);
  return IRC_E_INVALID;
}

template <typename TI, typename TO>
static int by_layout(int la, int lb, int epi, const Args& g, int batch, int splits,
                     hipStream_t st) {
  if (la == ROW && lb == ROW) return by_epi<TI, TO, ROW, ROW>(epi, g, batch, splits, st);
  if (la == ROW && lb == COL) return by_epi<TI, TO, ROW, COL>(epi, g, batch, splits, st);
  if (la == COL && lb == ROW) return by_epi<TI, TO, COL, ROW>(epi, g, batch, splits, st);
  return by_epi<TI, TO, COL, COL>(epi, g, batch, splits, st);
}

}  // namespace gemm
}  // namespace irc

using namespace irc;

// Grouped output-tile order of the 256-row GEMM kernels (row tiles per group, rows walked
// fastest inside a group; 0 = row-major): the tiles an XCD has in flight then share a few
// column tiles of B, which stays in that XCD's 4 MB L2 across the group, instead of every
// wave of row tiles streaming all of B again.  Taken where a launch has at least 12 column
// tiles of its kernel's width bn (BERT-large FFN1, N = 4096, whose 8 MB weight streamed once per wave of row
// tiles: 606 MB read per launch against 75 MB algorithmic, profiles/r06_g_pmc.log).  With 8
// rows per group for every launch: C4 step 11.17-11.20k -> 11.31-11.34k pairs/s and C4 GEMM
// traffic 460 -> 407 MB per launch, C2 step 31.87-31.94k -> 31.81-31.88k (its widest launch
// has 8 column tiles; profiles/r06_h/), hence the threshold.  IRC_GEMM_GROUP_M (build
// flag) forces one value for every launch.
static int gemm_group_m(int64_t N, int64_t bn) {
  if (IRC_GEMM_GROUP_M != 0) return IRC_GEMM_GROUP_M;
  return (N + bn - 1) / bn >= 12 ? 8 : 0;
}

// IRC_GEMM_PP=0 disables the ping-pong path (A/B experiments; read once).
static bool pp_enabled() {
  static const bool on = [] {
    const char* e = getenv("IRC_GEMM_PP");
    return !(e && e[0] == '0');
  }();
  return on;
}

constexpr int64_t SPLIT_BLOCKS_DEFAULT = 256;  // split-K budget: one wave of 256 x 256 blocks
// max_blocks > 0: the split-K budget; < 0: a grid cap of -max_blocks workgroups on an
// unsplit launch (the split-K budget stays the default); 0: neither.
static inline int64_t split_budget(int64_t max_blocks) {
  return max_blocks > 0 ? max_blocks : SPLIT_BLOCKS_DEFAULT;
}
static inline int64_t grid_cap(int64_t max_blocks) { return max_blocks < 0 ? -max_blocks : 0; }

extern "C" int64_t irc_gemm_workspace_ex(int in_dtype, int out_dtype, int epilogue, int64_t M,
                                         int64_t N, int64_t K, int64_t batch, int64_t max_blocks) {
  const int64_t bud = split_budget(max_blocks);
  int s = gemm::split_count(in_dtype == 0 ? 2 : 4, out_dtype == 1, epilogue, M, N, K, batch, bud);
  if (in_dtype == 0 && pp_enabled()) {
    const int sp = gpp::splits_for(out_dtype == 1, epilogue, M, N, K, batch, bud);
    if (sp > s) s = sp;
  }
  int64_t bytes = s > 1 ? (int64_t)s * M * N * batch * (int64_t)sizeof(float) : 0;
  return bytes;
}

extern "C" int64_t irc_gemm_workspace(int in_dtype, int out_dtype, int epilogue, int64_t M,
                                      int64_t N, int64_t K, int64_t batch) {
  return irc_gemm_workspace_ex(in_dtype, out_dtype, epilogue, M, N, K, batch, 0);
}

// LayerNorm-fold GEMM of the BERT encoder (include/irc.h irc_gemm_ln): bf16 A [M][K],
// B [N][K], bf16 C; routed like irc_gemm (ping-pong 256 x 256 where it qualifies, else the
// big-tile kernel in its 16x16x32 form), never split or persistent.
extern "C" int irc_gemm_ln(int epilogue, int64_t M, int64_t N, int64_t K, const void* A,
                           int64_t lda, const void* B, int64_t ldb, const float* bias,
                           const void* R, int64_t ldr, void* C, int64_t ldc,
                           const float* ln_stats, int ln_nt, const float* ln_gamma,
                           const float* ln_beta, float ln_eps, int64_t ln_h,
                           const float* fold_colsum, float* stats_out, int* stats_nt_out,
                           irc_stream_t stream) {
  using namespace irc::gemm;
  IRC_REQUIRE(epilogue == EPI_BIAS || epilogue == EPI_BIAS_GELU || epilogue == EPI_BIAS_RESID,
              "gemm_ln: epilogue must be 1 (fold), 2 (fold + GELU) or 3 (residual)");
  IRC_REQUIRE(M > 0 && N > 0 && K > 0 && M < (1ll << 31) && N < (1ll << 31), "gemm_ln: bad sizes");
  IRC_REQUIRE(bias != nullptr, "gemm_ln: bias required");
  const bool fold = epilogue != EPI_BIAS_RESID;
  IRC_REQUIRE(!fold || (ln_stats && fold_colsum && ln_nt > 0 && ln_h > 0),
              "gemm_ln: the fold needs the input statistics and the column sums");
  IRC_REQUIRE(fold || R != nullptr, "gemm_ln: epilogue 3 needs the residual");
  IRC_REQUIRE(fold || ln_gamma == nullptr || (ln_stats && ln_beta && ln_nt > 0 && ln_h > 0),
              "gemm_ln: the residual LayerNorm needs statistics, gamma and beta");
  IRC_REQUIRE(stats_out == nullptr || stats_nt_out != nullptr, "gemm_ln: stats_nt_out required");
  IRC_REQUIRE(K % 64 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
                  (R == nullptr || ldr % 8 == 0) &&
                  (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)R) % 16) == 0,
              "gemm_ln: needs K %% 64 == 0, N %% 8 == 0 and 16-byte aligned rows");
  LnArgs ln{};
  ln.st = ln_stats;
  ln.nt = ln_nt;
  ln.inv_h = ln_h > 0 ? 1.0f / (float)ln_h : 0.f;
  ln.eps = ln_eps;
  ln.gamma = fold ? nullptr : ln_gamma;
  ln.beta = fold ? nullptr : ln_beta;
  ln.fold_s = fold ? fold_colsum : nullptr;
  ln.st_out = stats_out;
  hipStream_t st = as_stream(stream);
  const double flops = 2.0 * M * N * K;
  Args g{A, B, C, bias, R, (int)M, (int)N, (int)K, lda, ldb, ldc, ldr, 0, 0, 0, 0, 0, 1.0f, 0, 1, 1,
         1, 0, nullptr, gemm_group_m(N, 384)};
  const int wnb = big_wnb(g, 1, ROW, ROW);
  // the 256 x 256 kernel unless the big-tile one is preferred and applies (small shapes
  // that neither kernel's heuristics take also run 256 x 256)
  if ((pp_enabled() && gpp::qualifies(0, 0, M, N, K, A, lda, 0, B, ldb, 0, 1, 1)) || wnb == 0) {
    gpp::PArgs pa{static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), C,
                  bias, R, nullptr, (int)M, (int)N, (int)K, (int)K, lda, ldb, ldc, ldr, 0, 0, 0, 0,
                  0, 1.0f, 0, 1};
    pa.group_m = gemm_group_m(N, 256);
    ln.nt_out = (int)((N + 255) / 256);
    pa.ln = ln;
    if (stats_nt_out) *stats_nt_out = ln.nt_out;
    prof_begin(st);
    gpp::run_ln(epilogue, pa, st);
    prof_end("gemm_bf16", st, flops);
    prof_work("gemm_bf16_bytes", gemm_alg_bytes(0, epilogue, 0, M, N, K, 1));
    return check_launch("gemm_pp_kernel(ln)");
  }
  ln.nt_out = (int)((N + 128 * wnb - 1) / (128 * wnb));
  g.ln = ln;
  if (stats_nt_out) *stats_nt_out = ln.nt_out;
  switch (epilogue) {
    case EPI_BIAS: return launch_big<unsigned short, EPI_BIAS, true>(g, 1, wnb, st);
    case EPI_BIAS_GELU: return launch_big<unsigned short, EPI_BIAS_GELU, true>(g, 1, wnb, st);
    default: return launch_big<unsigned short, EPI_BIAS_RESID, true>(g, 1, wnb, st);
  }
}

// QKV projection + attention in one launch (include/irc.h irc_qkv_attention; see
// qkv_attn_kernel): L <= 128, head dim 64, H % 128 == 0.
extern "C" int irc_qkv_attention(int64_t M, int64_t H, int64_t heads, int64_t L, const void* x,
                                 int64_t ldx, const void* wqkv_perm, const float* bias_perm,
                                 const int64_t* mask, void* ctx, int64_t ldc,
                                 irc_stream_t stream) {
  using namespace irc::gemm;
  IRC_REQUIRE(L >= 1 && L <= 128 && heads * 64 == H && H % 128 == 0,
              "qkv_attention: needs L <= 128, head dim 64 and H %% 128 == 0");
  IRC_REQUIRE(M > 0 && M % L == 0 && M < (1ll << 31), "qkv_attention: M must be a multiple of L");
  IRC_REQUIRE(H % 64 == 0 && ldx % 8 == 0 && ldx >= H && ldc >= H, "qkv_attention: bad strides");
  IRC_REQUIRE((((uintptr_t)x | (uintptr_t)wqkv_perm) % 16) == 0 && ((uintptr_t)ctx % 2) == 0,
              "qkv_attention: operands must be 16-byte aligned");
  IRC_REQUIRE(bias_perm != nullptr, "qkv_attention: bias required");
  QaArgs a{static_cast<const unsigned short*>(x), static_cast<const unsigned short*>(wqkv_perm),
           bias_perm, mask, static_cast<unsigned short*>(ctx), (int)M, (int)H, (int)H, ldx, ldc,
           0.125f, (int)L, IRC_GEMM_GROUP_M};
  // Row-major tile order here even where Wqkv exceeds an XCD's 4 MB L2 (C4: 6 MB): grouped
  // (8 rows) measured 11.35-11.39k against 11.38-11.43k pairs/s on the C4 leg, GEMM traffic
  // 407 vs 415 MB per launch (profiles/r06_n/)
  hipStream_t st = as_stream(stream);
  // Sequences per 256-row tile: 64- or 128-row slots, or packed (256 / L) where that takes
  // fewer waves of tiles over the CUs.  Packed tiles pay an attention round per 8 (sequence,
  // query block) items of a head (~5 us a tile each), so at equal waves the slots stay.
  // B = 512 (a C2 / C4 micro-batch), fused us per layer, slots -> packed where it applies
  // (profiles/r06_k/): L = 16: 116-122 -> 49-50, L = 32: 75-76 (packed in both), L = 34:
  // 115 -> 91-92, L = 72: 236-239 -> 222-223, L = 85: 238-239 -> 225-226; L = 48 keeps slots
  // (120-122 against 130-131 packed: both 3 waves).
  const int64_t nseq = M / L, tiles_n = 3 * H / 384;
  const int slot = L <= 64 ? 4 : 2;
  const int64_t ncu = std::max(1, gpp::cu_count() > 0 ? gpp::cu_count() : 256);
  const auto waves = [&](int64_t s) { return ((nseq + s - 1) / s * tiles_n + ncu - 1) / ncu; };
  const bool packed = 256 / L > slot && waves(256 / L) < waves(slot);
  const int spt = packed ? (int)(256 / L) : slot;
  const int tiles = (int)(((nseq + spt - 1) / spt) * tiles_n);
  prof_begin(st);
  if (packed)
    hipLaunchKernelGGL(qkv_attn_kernel<0>, dim3(tiles), dim3(big::NT), 0, st, a);
  else if (L <= 64)
    hipLaunchKernelGGL(qkv_attn_kernel<64>, dim3(tiles), dim3(big::NT), 0, st, a);
  else
    hipLaunchKernelGGL(qkv_attn_kernel<128>, dim3(tiles), dim3(big::NT), 0, st, a);
  // priced as the QKV GEMM alone (its flops; bytes x, Wqkv, ctx): the attention in its
  // epilogue is extra work the GEMM family's rate does not credit
  prof_end("gemm_bf16", st, 2.0 * M * 3 * H * H);
  prof_work("gemm_bf16_bytes", 2.0 * (double)M * H + 2.0 * 3 * H * H + 2.0 * (double)M * H);
  return check_launch("qkv_attn_kernel");
}

#ifdef IRC_BIG_STAMPS
extern "C" int irc_big_dbg_stamps(uint64_t* out /* [64][5][2] */) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(irc::gemm::big::big_stamps),
                             sizeof(irc::gemm::big::big_stamps)) == hipSuccess ? 0 : -1;
}
#endif

// 16x16x32 (1) or 32x32x16 (0) MFMAs in the big-tile kernel's 2-slot loop; returns the
// previous setting.
extern "C" int irc_gemm_set_big_mf16(int on) {
  return irc::gemm::big_mf16_mode().exchange(on ? 1 : 0);
}

// 4-slot ring (1) or 2-slot loop (0, the default: the ring measured no faster on
// the BERT shapes, profiles/r03_ring_r_*) of the 256-row big-tile GEMM; returns the
// previous setting.
extern "C" int irc_gemm_set_big_ring(int on) {
  return irc::gemm::big_ring_mode().exchange(on ? 1 : 0);
}

// dtype codes: 0 = bf16, 1 = fp32
extern "C" int irc_gemm_ex(int in_dtype, int out_dtype, int a_layout, int b_layout, int epilogue,
                           int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                           int64_t strideA, const void* B, int64_t ldb, int64_t strideB,
                           const float* bias, int64_t strideBias, const void* R, int64_t ldr,
                           int64_t strideR, void* C, int64_t ldc, int64_t strideC, int accumulate,
                           int64_t batch, void* workspace, int64_t workspace_bytes,
                           int64_t max_blocks, irc_stream_t stream) {
  const int64_t bud = split_budget(max_blocks);
  IRC_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "gemm: bad sizes");
  IRC_REQUIRE(M < (1ll << 31) && N < (1ll << 31) && K < (1ll << 31), "gemm: size too large");
  IRC_REQUIRE(in_dtype == 0 || in_dtype == 1, "gemm: in_dtype must be 0 (bf16) or 1 (fp32)");
  IRC_REQUIRE(out_dtype == 0 || out_dtype == 1, "gemm: out_dtype must be 0 (bf16) or 1 (fp32)");
  IRC_REQUIRE(!(accumulate && out_dtype == 0), "gemm: accumulate needs fp32 C");
  IRC_REQUIRE(epilogue >= 0 && epilogue <= 6, "gemm: bad epilogue");
  IRC_REQUIRE(!gemm::epi_has_bias(epilogue) || bias, "gemm: epilogue needs bias");
  IRC_REQUIRE(!(epilogue >= 3 && epilogue != 1 && epilogue != 2) || R,
              "gemm: epilogue needs R (residual / pre-activation)");
  IRC_REQUIRE(!(accumulate && epilogue >= 5), "gemm: accumulate with a GELU epilogue");
  // 16-byte vector staging needs every row start 16-byte aligned; otherwise the
  // operand is staged element by element (same results, slower).
  const int vec = in_dtype == 0 ? 8 : 4;
  const int vec_a = lda % vec == 0 && strideA % vec == 0 && ((uintptr_t)A % 16) == 0;
  const int vec_b = ldb % vec == 0 && strideB % vec == 0 && ((uintptr_t)B % 16) == 0;
  if (M == 0 || N == 0) return IRC_OK;
  // split-K when the caller provided the workspace irc_gemm_workspace asked for
  int splits = gemm::split_count(in_dtype == 0 ? 2 : 4, out_dtype == 1, epilogue, M, N, K, batch, bud);
  if (splits > 1 && (workspace == nullptr ||
                     workspace_bytes < (int64_t)splits * M * N * batch * (int64_t)sizeof(float)))
    splits = 1;
  const int cvec = out_dtype == 0 ? 8 : 4;
  const int vec_c = N % 8 == 0 && ldc % cvec == 0 && strideC % cvec == 0 &&
                    ((uintptr_t)C % 16) == 0 &&
                    (R == nullptr || (ldr % cvec == 0 && strideR % cvec == 0 &&
                                      ((uintptr_t)R % 16) == 0));
  gemm::Args g{A, B, C, bias, R, (int)M, (int)N, (int)K, lda, ldb, ldc, ldr,
               strideA, strideB, strideC, strideR, strideBias, alpha, accumulate, vec_a, vec_b,
               vec_c, 0, splits > 1 ? static_cast<float*>(workspace) : nullptr,
               gemm_group_m(N, 384)};
  hipStream_t st = as_stream(stream);
  const int nb = (int)batch;
  if (in_dtype == 0 && pp_enabled()) {
    int sp = gpp::splits_for(out_dtype == 1, epilogue, M, N, K, batch, bud);
    if (sp > 1 && (workspace == nullptr ||
                   workspace_bytes < (int64_t)sp * M * N * batch * (int64_t)sizeof(float)))
      sp = 1;
    if (gpp::qualifies(a_layout, b_layout, M, N, K, A, lda, strideA, B, ldb, strideB, batch, sp)) {
      gpp::PArgs pa{static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B),
                    C, bias, R, sp > 1 ? static_cast<float*>(workspace) : nullptr, (int)M, (int)N,
                    (int)K, sp > 1 ? (int)(((K + sp - 1) / sp + 63) / 64 * 64) : (int)K,
                    lda, ldb, ldc, ldr, strideA, strideB, strideC, strideR, strideBias, alpha,
                    accumulate, vec_c};
      pa.group_m = gemm_group_m(N, 256);
      prof_begin(st);
      gpp::run(out_dtype == 1, a_layout, b_layout, epilogue, pa, batch, sp, st, grid_cap(max_blocks));
      if (sp > 1) {
        const int64_t n = M * N * batch;
        hipLaunchKernelGGL(gemm::splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256),
                           0, st, pa.P, static_cast<float*>(C), (int)M, (int)N, sp, ldc, strideC,
                           nb, alpha, accumulate);
      }
      prof_end("gemm_bf16", st, 2.0 * M * N * K * batch);
      prof_work("gemm_bf16_bytes",
                gemm::gemm_alg_bytes(out_dtype, epilogue, accumulate, M, N, K, batch));
      return check_launch("gemm_pp_kernel");
    }
  }
  if (in_dtype == 0 && out_dtype == 0)
    return gemm::by_layout<unsigned short, unsigned short>(a_layout, b_layout, epilogue, g, nb,
                                                           1, st);
  if (in_dtype == 0 && out_dtype == 1)
    return gemm::by_layout<unsigned short, float>(a_layout, b_layout, epilogue, g, nb, splits, st);
  if (in_dtype == 1 && out_dtype == 1)
    return gemm::by_layout<float, float>(a_layout, b_layout, epilogue, g, nb, splits, st);
  set_error("gemm: fp32 inputs with bf16 output is not supported");
  return IRC_E_INVALID;
}

extern "C" int irc_gemm(int in_dtype, int out_dtype, int a_layout, int b_layout, int epilogue,
                        int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                        int64_t strideA, const void* B, int64_t ldb, int64_t strideB,
                        const float* bias, int64_t strideBias, const void* R, int64_t ldr,
                        int64_t strideR, void* C, int64_t ldc, int64_t strideC, int accumulate,
                        int64_t batch, void* workspace, int64_t workspace_bytes,
                        irc_stream_t stream) {
  return irc_gemm_ex(in_dtype, out_dtype, a_layout, b_layout, epilogue, M, N, K, alpha, A, lda,
                     strideA, B, ldb, strideB, bias, strideBias, R, ldr, strideR, C, ldc, strideC,
                     accumulate, batch, workspace, workspace_bytes, 0, stream);
}
