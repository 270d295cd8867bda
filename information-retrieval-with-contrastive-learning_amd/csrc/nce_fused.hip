// Fused InfoNCE (NT-Xent + MoCo queue) for the LSTM-head embedding width (D <= 256).
//
// Reference: NCELoss._compute_info_loss (src/contrastor/contrastive_loss.py:56-93):
// F = [q; k] [2N, D]; row r's logits are F_r . F_c / T for c != r (the positive is
// c = (r + N) mod 2N) and, with the queue, q_{r mod N} . queue_j / T (the k-rows
// REUSE q's queue logits); loss = sum_r CE_r / 2.
//
// The logits never land in HBM (the unfused path materialises S [2N, 2N] and
// LQ [N, K]): a workgroup streams 32-column tiles of [F ; queue^T] through a
// double-buffered LDS tile, each of its 4 waves against its own block of 32 rows
// (held in registers) on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32: products and sums
// in fp32, as the reference's CPU path) and keeps an online (max, sum exp) per
// row; a combine kernel turns the per-chunk partials into lse / loss rows.  The
// backward recomputes each logit tile and folds it straight into dF:
//   dF_u = sum_{v != u} (G_uv + G_vu) F_v  +  [u < N] sum_j (P_uj + P_{u+N,j}) queue_j
//   G_uv = (exp(s_uv / T - lse_u) - [v == pos_u]) * g / (2T),  P_rj = exp(lq_j / T - lse_r) * g / (2T)
// -- a second fp32 MFMA on the same registers (the coefficient tile is the MFMA's
// B operand as it stands: its column is the lane, and the 16 accumulator
// registers give the k-steps).  The rows of any pair range [p_lo, p_hi) (q rows
// p_lo.. and their k rows N + p_lo..) can be computed on their own given every
// row's lse: a data-parallel rank computes only its local pairs' rows (SURVEY.md
// 8e) after an all-gather of lse.  Partials are reduced in a fixed order, so the
// results are deterministic.
//
// Tile geometry of v_mfma_f32_32x32x2_f32 used here (S^T = X . F_u^T):
//   A (32 x 2): lane (r = l & 31, h = l >> 5) holds X[v0 + r][d]   (X = F or queue^T)
//   B (2 x 32): lane (r, h)                 holds F[u0 + r][d]
//   for the d pairs of each 8-wide group t: d = 8t + 4h + s, s = 0..3 (one MFMA per s)
//   C: lane (r, h) register e = S^T[v0 + (e & 3) + 8 (e >> 2) + 4 h][u0 + r]
// so the lane owns ROW u0 + r of the logits: the row reductions are lane-local
// plus one exchange with lane ^ 32.
#include "irc_common.h"

#include <algorithm>

namespace irc {
namespace ncef {

constexpr int NT = 256;    // 4 waves per workgroup: 4 u-blocks of 32 rows (128 rows)
constexpr int MAXD = 256;  // D <= 256 (the u-block's B fragments: D / 2 VGPRs)
constexpr int TC = 32;     // columns per tile

struct Args {
  const float* F;      // [2N][D]
  const float* queue;  // [D][K] (key columns), or null
  int N, D, K;
  float invT;
  // rows computed: the pairs [p_lo, p_hi), i.e. q rows p_lo.. and k rows N + p_lo..
  // (all 2N rows when the range is [0, N); else 32-aligned, N % 32 == 0).  Local
  // row index: q rows 0 .. P-1, k rows P .. 2P-1 (P = p_hi - p_lo).
  int p_lo, p_hi;
  int C;  // 32-column tiles per chunk
  // work items (one per workgroup): 128-row groups of the in-batch row ranges
  // [b_lo[i], b_lo[i] + b_len[i]) x chunks_b, then of the queue row range
  // [q_lo, q_lo + q_len) x chunks_q
  int nr, b_lo[2], b_len[2], q_lo, q_len, chunks_b, chunks_q;
  // forward
  float2* part_b;      // [chunks_b][2N]  (max, sum exp) over in-batch chunk
  float2* part_q;      // [chunks_q][N]   over queue chunk (q rows)
  float* pos;          // [2N] positive logit (/T)
  // backward
  const float* lse;    // [2N] (all rows)
  const float* gscale; // [1] upstream gradient (device), or null = 1
  float* dpart;        // [chunks][local rows][D] partial dF of the computed rows
};

__device__ __forceinline__ bool full_range(const Args& a) { return a.p_lo == 0 && a.p_hi == a.N; }
__device__ __forceinline__ int local_rows(const Args& a) { return 2 * (a.p_hi - a.p_lo); }
// absolute row u -> local row (or -1 when u is not computed here)
__device__ __forceinline__ int local_of(const Args& a, int u) {
  if (u < 0 || u >= 2 * a.N) return -1;
  const int P = a.p_hi - a.p_lo;
  if (u < a.N) return (u >= a.p_lo && u < a.p_hi) ? u - a.p_lo : -1;
  const int k = u - a.N;
  return (k >= a.p_lo && k < a.p_hi) ? P + k - a.p_lo : -1;
}
__device__ __forceinline__ int abs_of(const Args& a, int lr) {
  const int P = a.p_hi - a.p_lo;
  return lr < P ? a.p_lo + lr : a.N + a.p_lo + (lr - P);
}
// workgroup item -> (first row of its 128-row group, end of the row range, chunk
// index in [0, chunks_b + chunks_q), queue part?)
__device__ __forceinline__ bool decode(const Args& a, int item, int& row0, int& row_end, int& ch,
                                       bool& qpart) {
  int it = item;
  for (int i = 0; i < a.nr; ++i) {
    const int ng = (a.b_len[i] + 127) / 128;
    if (it < ng * a.chunks_b) {
      row0 = a.b_lo[i] + (it / a.chunks_b) * 128;
      row_end = a.b_lo[i] + a.b_len[i];
      ch = it % a.chunks_b;
      qpart = false;
      return true;
    }
    it -= ng * a.chunks_b;
  }
  const int ng = (a.q_len + 127) / 128;
  if (it < ng * a.chunks_q) {
    row0 = a.q_lo + (it / a.chunks_q) * 128;
    row_end = a.q_lo + a.q_len;
    ch = a.chunks_b + it % a.chunks_q;
    qpart = true;
    return true;
  }
  return false;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ int pos_of(int u, int N) { return u < N ? u + N : u - N; }

// A 32-column tile X [32][D] (X = rows of F, or queue^T) staged in LDS with row
// pitch D + 4 floats: the logit product reads rows (ds_read_b128 at d = 8t + 4h),
// the backward's dF product reads columns (32 lanes = 32 consecutive d of one row).
// Every thread holds D / 32 float4 of the tile between the global load and the
// LDS write, so the next tile's loads are in flight during this tile's MFMAs.
template <int D>
struct Stage {
  static constexpr int P = D + 4;
  static constexpr int NV = D / 32;  // float4 per thread
  f32x4 v[NV];
  __device__ __forceinline__ void load(const Args& a, bool qpart, int v0) {
    const int t = threadIdx.x;
    if (!qpart) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = t + NT * i;
        const int row = f / (D / 4), c4 = f % (D / 4);
        const int vr = min(v0 + row, 2 * a.N - 1);
        v[i] = ld4(a.F + (int64_t)vr * D + 4 * c4);
      }
    } else {
      const bool vec = (a.K & 3) == 0 && v0 + TC <= a.K;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = t + NT * i;
        const int d = f / 8, j = v0 + 4 * (f % 8);
        const float* src = a.queue + (int64_t)d * a.K + j;
        if (vec) {
          v[i] = ld4(src);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) v[i][s] = j + s < a.K ? src[s] : 0.f;
        }
      }
    }
  }
  __device__ __forceinline__ void store(float* xs, bool qpart) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = t + NT * i;
      if (!qpart) {
        const int row = f / (D / 4), c4 = f % (D / 4);
        *reinterpret_cast<f32x4*>(xs + row * P + 4 * c4) = v[i];
      } else {
        const int d = f / 8, j4 = f % 8;
#pragma unroll
        for (int s = 0; s < 4; ++s) xs[(4 * j4 + s) * P + d] = v[i][s];
      }
    }
  }
};

// The wave's u-block as MFMA B fragments: lane (r, h) holds F[u0 + r][8t + 4h .. + 4].
template <int D>
__device__ __forceinline__ void load_u(const Args& a, int u0, int lane, f32x4 (&fu)[D / 8]) {
  const int u = min(u0 + (lane & 31), 2 * a.N - 1);
  const float* p = a.F + (int64_t)u * D + 4 * (lane >> 5);
#pragma unroll
  for (int t = 0; t < D / 8; ++t) fu[t] = ld4(p + 8 * t);
}

// S^T tile [v0 + 32][u0 + 32] = X . F_u^T over all D (exact fp32 MFMA).
template <int D>
__device__ __forceinline__ f32x16 logit_tile(const float* xs, const f32x4 (&fu)[D / 8], int lane) {
  const float* row = xs + (lane & 31) * Stage<D>::P + 4 * (lane >> 5);
  f32x16 acc = (f32x16)0.0f;
#pragma unroll
  for (int t = 0; t < D / 8; ++t) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(row + 8 * t);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], fu[t][s], acc, 0, 0, 0);
  }
  return acc;
}

// ---- forward: per (128-row group, column chunk) the online (max, sum exp) -------
template <int D>
__global__ __launch_bounds__(NT) void fwd_partial_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) float xsm[];  // [2][TC * P]
  auto xs = [&](int i) { return xsm + i * (TC * Stage<D>::P); };
  int row0, row_end, ch;
  bool qpart;
  if (!decode(a, blockIdx.x, row0, row_end, ch, qpart)) return;
  const int cq = qpart ? ch - a.chunks_b : ch;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int u0 = row0 + 32 * (threadIdx.x >> 6);
  const bool active = u0 < row_end;  // wave-uniform (ranges are 32-aligned or end at 2N)
  const int n2 = 2 * a.N;
  const int u = u0 + r;
  const int ncols = qpart ? a.K : n2;
  const int t_lo = cq * a.C;
  const int t_hi = min(t_lo + a.C, (ncols + TC - 1) / TC);
  f32x4 fu[D / 8];
  if (active) load_u<D>(a, u0, lane, fu);
  Stage<D> st;
  st.load(a, qpart, t_lo * TC);
  st.store(xs(0), qpart);
  __syncthreads();
  float m = -INFINITY, s = 0.f;
  for (int tt = t_lo; tt < t_hi; ++tt) {
    const int bi = (tt - t_lo) & 1;
    const bool more = tt + 1 < t_hi;
    if (more) st.load(a, qpart, (tt + 1) * TC);
    if (active) {
      const int v0 = tt * TC;
      const f32x16 acc = logit_tile<D>(xs(bi), fu, lane);
      float x[16];
      float tm = -INFINITY;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int v = v0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        x[e] = acc[e] * a.invT;
        const bool ok = v < ncols && (qpart || v != u);
        if (!qpart && v == pos_of(u, a.N) && u < n2) a.pos[u] = x[e];
        x[e] = ok ? x[e] : -INFINITY;
        tm = fmaxf(tm, x[e]);
      }
      const float mn = fmaxf(m, tm);
      if (mn != -INFINITY) {
        float add = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) add += __expf(x[e] - mn);
        s = s * __expf(m - mn) + add;
        m = mn;
      }
    }
    if (more) st.store(xs(bi ^ 1), qpart);
    __syncthreads();
  }
  if (!active) return;
  // combine with the other half-wave (same row, the other 16 columns of each tile)
  const float m2 = __shfl_xor(m, 32, 64), s2 = __shfl_xor(s, 32, 64);
  const float mm = fmaxf(m, m2);
  const float ss = mm == -INFINITY ? 0.f : s * __expf(m - mm) + s2 * __expf(m2 - mm);
  if (h == 0 && u < row_end) {
    if (qpart) {
      a.part_q[(int64_t)cq * a.N + u] = make_float2(mm, ss);
    } else {
      a.part_b[(int64_t)cq * n2 + u] = make_float2(mm, ss);
    }
  }
}

// lse[r], loss_row[r] for the computed rows: one wave per row, lane l combining
// chunks l, l + 64, ... in order, then a fixed xor tree (deterministic).
__global__ __launch_bounds__(256) void fwd_combine_kernel(Args a, float* __restrict__ lse,
                                                          float* __restrict__ loss_row) {
  const int lr = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (lr >= (full_range(a) ? 2 * a.N : local_rows(a))) return;
  const int r = full_range(a) ? lr : abs_of(a, lr);
  const int n2 = 2 * a.N;
  const int cb = a.chunks_b, cq = a.K > 0 ? a.chunks_q : 0;
  const int n = r % a.N;
  auto part = [&](int c) {
    return c < cb ? a.part_b[(int64_t)c * n2 + r] : a.part_q[(int64_t)(c - cb) * a.N + n];
  };
  float m = -INFINITY;
  for (int c = lane; c < cb + cq; c += 64) m = fmaxf(m, part(c).x);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float s = 0.f;
  for (int c = lane; c < cb + cq; c += 64) {
    const float2 p = part(c);
    if (p.x != -INFINITY) s += p.y * __expf(p.x - m);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) {
    const float l = m + logf(s);
    lse[r] = l;
    loss_row[r] = l - a.pos[r];
  }
}

// ---- backward: dF partial of one (128-row group, column chunk) -----------------
// The coefficient tile C^T[v][u] (registers = v, lane = u) is the B operand of
// dF^T[d][u] += sum_v X[v][d] C^T[v][u]: MFMA step e pairs k = 0 (lanes h = 0) with
// v = v0 + (e & 3) + 8 (e >> 2) and k = 1 (h = 1) with that v + 4, so the A operand
// of step e is lane (r, h) <- X[v_e(h)][32 b + r], a column read of the LDS tile.
template <int D>
__global__ __launch_bounds__(NT) void bwd_partial_kernel(Args a) {
  constexpr int ND = D / 32;
  constexpr int P = Stage<D>::P;
  extern __shared__ __attribute__((aligned(16))) float xsm[];  // [2][TC * P]
  auto xs = [&](int i) { return xsm + i * (TC * P); };
  int row0, row_end, ch;
  bool qpart;
  if (!decode(a, blockIdx.x, row0, row_end, ch, qpart)) return;
  const int cq = qpart ? ch - a.chunks_b : ch;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int u0 = row0 + 32 * (threadIdx.x >> 6);
  const bool active = u0 < row_end;
  const int n2 = 2 * a.N;
  const int u = u0 + r;
  const bool uok = u < row_end;
  const float scale = 0.5f * a.invT * (a.gscale ? a.gscale[0] : 1.f);
  const int ncols = qpart ? a.K : n2;
  const float lse_u = a.lse[min(u, n2 - 1)];
  const float lse_k = qpart ? a.lse[min(u + a.N, n2 - 1)] : 0.f;  // the k-row sharing q's queue logits
  const int pu = pos_of(u, a.N);
  const int t_lo = cq * a.C;
  const int t_hi = min(t_lo + a.C, (ncols + TC - 1) / TC);
  f32x4 fu[D / 8];
  if (active) load_u<D>(a, u0, lane, fu);
  f32x16 dacc[ND];
#pragma unroll
  for (int b = 0; b < ND; ++b) dacc[b] = (f32x16)0.0f;
  Stage<D> st;
  st.load(a, qpart, t_lo * TC);
  st.store(xs(0), qpart);
  __syncthreads();
  for (int tt = t_lo; tt < t_hi; ++tt) {
    const int bi = (tt - t_lo) & 1;
    const bool more = tt + 1 < t_hi;
    if (more) st.load(a, qpart, (tt + 1) * TC);
    if (active) {
      const int v0 = tt * TC;
      const f32x16 acc = logit_tile<D>(xs(bi), fu, lane);
      float coef[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int v = v0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const float z = acc[e] * a.invT;
        float c = 0.f;
        if (v < ncols && uok) {
          if (qpart) {
            c = __expf(z - lse_u) + __expf(z - lse_k);
          } else if (v != u) {
            c = __expf(z - lse_u) - (v == pu ? 1.f : 0.f);                  // G_uv
            c += __expf(z - a.lse[v]) - (u == pos_of(v, a.N) ? 1.f : 0.f);  // G_vu
          }
        }
        coef[e] = c * scale;
      }
      // dF^T[d][u] += X[v][d] coef[v][u]
      const float* col = xs(bi) + 4 * h * P + r;
#pragma unroll
      for (int b = 0; b < ND; ++b) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int vl = (e & 3) + 8 * (e >> 2);
          dacc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(col[vl * P + 32 * b], coef[e], dacc[b], 0,
                                                         0, 0);
        }
      }
    }
    if (more) st.store(xs(bi ^ 1), qpart);
    __syncthreads();
  }
  if (!active) return;
  // dacc[b] C layout: lane (r, h) register e = dF^T[32 b + (e & 3) + 8 (e >> 2) + 4 h][u0 + r]
  const int lr = full_range(a) ? (u < n2 ? u : -1) : local_of(a, u);
  const int nloc = full_range(a) ? n2 : local_rows(a);
  if (uok && lr >= 0) {
    float* out = a.dpart + ((int64_t)ch * nloc + lr) * D;
#pragma unroll
    for (int b = 0; b < ND; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(out + 32 * b + 8 * g + 4 * h) =
            (f32x4){dacc[b][4 * g], dacc[b][4 * g + 1], dacc[b][4 * g + 2], dacc[b][4 * g + 3]};
  }
}

// dF[r] = sum over chunks (fixed order) of the partials that cover row r.
__global__ void bwd_reduce_kernel(const float* __restrict__ dpart, int rows, int D, int chunks_b,
                                  int chunks_q, int q_rows, float* __restrict__ dF) {
  const int64_t e4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  if (e4 * 4 >= (int64_t)rows * D) return;
  const int row = (int)(e4 * 4 / D);
  const f32x4* p = reinterpret_cast<const f32x4*>(dpart) + e4;
  const int64_t cs = (int64_t)rows * D / 4;
  const int nc = chunks_b + (row < q_rows ? chunks_q : 0);
  // 8 independent sums (chunk c into sum c % 8, in chunk order), then added in a
  // fixed order: deterministic, and 8 loads in flight per thread
  f32x4 s8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s8[j] = (f32x4)0.f;
  int c = 0;
  for (; c + 8 <= nc; c += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) s8[j] += p[(c + j) * cs];
  for (int j = 0; c + j < nc; ++j) s8[j] += p[(c + j) * cs];
  const f32x4 s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  reinterpret_cast<f32x4*>(dF)[e4] = s;
}

}  // namespace ncef
}  // namespace irc

using namespace irc;

namespace {
// Tiles per chunk.  Forward: about 1024 workgroups (4 per CU; the (max, sum exp)
// partials are 8 bytes per row and chunk).  Backward: also bounded so that the dF
// partials (D floats per row and chunk) stay <= 48 MB.
int pick_chunk(int64_t N, int64_t D, int64_t K, int64_t rows_b, int64_t rows_q, bool bwd) {
  const int64_t tb = (2 * N + 31) / 32, tq = (K + 31) / 32;
  const int64_t groups = ((rows_b + 127) / 128) * tb + ((rows_q + 127) / 128) * tq;
  int64_t c = (groups + 1023) / 1024;
  if (c < 2) c = 2;  // >= 2 tiles per workgroup: the row block's loads amortised
  if (bwd) {
    const int64_t part1 = (rows_b * tb + rows_q * tq) * D * 4;
    const int64_t cb = (part1 + (48ll << 20) - 1) / (48ll << 20);
    if (cb > c) c = cb;
  }
  return (int)(c < 1 ? 1 : c);
}

// Plan of the work items; false when the pair range is not supported.
bool plan(ncef::Args& a, int64_t N, int64_t D, int64_t K, int64_t p_lo, int64_t p_hi, bool bwd) {
  a.p_lo = (int)p_lo;
  a.p_hi = (int)p_hi;
  if (p_lo == 0 && p_hi == N) {  // every row: one range, no alignment needed
    a.nr = 1;
    a.b_lo[0] = 0;
    a.b_len[0] = (int)(2 * N);
    a.q_lo = 0;
    a.q_len = K > 0 ? (int)N : 0;
  } else {
    if (N % 32 || p_lo % 32 || p_hi % 32 || p_lo < 0 || p_hi > N || p_lo >= p_hi) return false;
    a.nr = 2;
    a.b_lo[0] = (int)p_lo;
    a.b_lo[1] = (int)(N + p_lo);
    a.b_len[0] = a.b_len[1] = (int)(p_hi - p_lo);
    a.q_lo = (int)p_lo;
    a.q_len = K > 0 ? (int)(p_hi - p_lo) : 0;
  }
  const int64_t rows_b = a.nr == 1 ? a.b_len[0] : 2 * (int64_t)a.b_len[0];
  a.C = pick_chunk(N, D, K, rows_b, a.q_len, bwd);
  a.chunks_b = (int)(((2 * N + 31) / 32 + a.C - 1) / a.C);
  a.chunks_q = K > 0 ? (int)(((K + 31) / 32 + a.C - 1) / a.C) : 0;
  return true;
}
int64_t n_items(const ncef::Args& a) {
  int64_t n = (int64_t)((a.q_len + 127) / 128) * a.chunks_q;
  for (int i = 0; i < a.nr; ++i) n += (int64_t)((a.b_len[i] + 127) / 128) * a.chunks_b;
  return n;
}
int64_t local_rows(int64_t N, int64_t p_lo, int64_t p_hi) {
  return (p_lo == 0 && p_hi == N) ? 2 * N : 2 * (p_hi - p_lo);
}
}  // namespace

extern "C" int64_t irc_nce_fused_workspace(int64_t N, int64_t D, int64_t K, int64_t p_lo,
                                           int64_t p_hi) {
  ncef::Args a{}, b{};
  if (!plan(a, N, D, K, p_lo, p_hi, false) || !plan(b, N, D, K, p_lo, p_hi, true)) return 0;
  const int64_t fwd = ((int64_t)a.chunks_b * 2 * N + (int64_t)a.chunks_q * N) * 8 + 2 * N * 4;
  const int64_t bwd = (int64_t)(b.chunks_b + b.chunks_q) * local_rows(N, p_lo, p_hi) * D * 4;
  return (fwd > bwd ? fwd : bwd) + 256;
}

extern "C" int irc_nce_fused_fwd(const float* F, const float* queue, int64_t N, int64_t D,
                                 int64_t K, float T, int64_t p_lo, int64_t p_hi, void* ws,
                                 int64_t ws_bytes, float* lse, float* loss_row,
                                 irc_stream_t stream) {
  IRC_REQUIRE(N >= 1 && D >= 32 && D <= ncef::MAXD && D % 32 == 0 && K >= 0 && T > 0 &&
                  (K == 0 || queue != nullptr),
              "nce_fused: 32 <= D <= 256, D %% 32 == 0 (D=%lld)", (long long)D);
  ncef::Args a{};
  IRC_REQUIRE(plan(a, N, D, K, p_lo, p_hi, false),
              "nce_fused: pairs [%lld, %lld) must be [0, N) or 32-aligned with N %% 32 == 0",
              (long long)p_lo, (long long)p_hi);
  IRC_REQUIRE(ws_bytes >= irc_nce_fused_workspace(N, D, K, p_lo, p_hi), "nce_fused: workspace");
  a.F = F;
  a.queue = queue;
  a.N = (int)N;
  a.D = (int)D;
  a.K = (int)K;
  a.invT = 1.f / T;
  char* w = static_cast<char*>(ws);
  a.part_b = reinterpret_cast<float2*>(w);
  a.part_q = a.part_b + (int64_t)a.chunks_b * 2 * N;
  a.pos = reinterpret_cast<float*>(a.part_q + (int64_t)a.chunks_q * N);
  const int64_t items = n_items(a);
  const int64_t rows = local_rows(N, p_lo, p_hi);
  hipStream_t st = as_stream(stream);
  prof_begin(st);
  const dim3 gf((unsigned)items);
  const size_t lds = (size_t)2 * ncef::TC * (D + 4) * sizeof(float);
  switch (D / 32) {
#define IRC_NCEF(ND)                                                                \
  case ND:                                                                          \
    hipLaunchKernelGGL(ncef::fwd_partial_kernel<32 * ND>, gf, dim3(ncef::NT), lds, st, a); \
    break;
    IRC_NCEF(1) IRC_NCEF(2) IRC_NCEF(3) IRC_NCEF(4) IRC_NCEF(5) IRC_NCEF(6) IRC_NCEF(7) IRC_NCEF(8)
#undef IRC_NCEF
  }
  hipLaunchKernelGGL(ncef::fwd_combine_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st,
                     a, lse, loss_row);
  prof_end("nce_fused", st, 2.0 * rows * D * (2.0 * N) + 2.0 * (rows / 2) * D * K);
  return check_launch("nce_fused_fwd");
}

extern "C" int irc_nce_fused_bwd(const float* F, const float* queue, const float* lse, int64_t N,
                                 int64_t D, int64_t K, float T, const float* gscale, int64_t p_lo,
                                 int64_t p_hi, void* ws, int64_t ws_bytes, float* dF,
                                 irc_stream_t stream) {
  IRC_REQUIRE(N >= 1 && D >= 32 && D <= ncef::MAXD && D % 32 == 0 && K >= 0 && T > 0 &&
                  (K == 0 || queue != nullptr),
              "nce_fused: 32 <= D <= 256, D %% 32 == 0");
  ncef::Args a{};
  IRC_REQUIRE(plan(a, N, D, K, p_lo, p_hi, true), "nce_fused: bad pair range");
  IRC_REQUIRE(ws_bytes >= irc_nce_fused_workspace(N, D, K, p_lo, p_hi), "nce_fused: workspace");
  a.F = F;
  a.queue = queue;
  a.N = (int)N;
  a.D = (int)D;
  a.K = (int)K;
  a.invT = 1.f / T;
  a.lse = lse;
  a.gscale = gscale;
  a.dpart = static_cast<float*>(ws);
  const int64_t items = n_items(a);
  const int64_t rows = local_rows(N, p_lo, p_hi);
  const int q_rows = (int)(rows / 2);
  hipStream_t st = as_stream(stream);
  prof_begin(st);
  const dim3 gb((unsigned)items);
  const size_t lds = (size_t)2 * ncef::TC * (D + 4) * sizeof(float);
  switch (D / 32) {
#define IRC_NCEB(ND)                                                                     \
  case ND:                                                                               \
    hipLaunchKernelGGL(ncef::bwd_partial_kernel<32 * ND>, gb, dim3(ncef::NT), lds, st, a); \
    break;
    IRC_NCEB(1) IRC_NCEB(2) IRC_NCEB(3) IRC_NCEB(4) IRC_NCEB(5) IRC_NCEB(6) IRC_NCEB(7) IRC_NCEB(8)
#undef IRC_NCEB
  }
  const int64_t tot4 = rows * D / 4;
  hipLaunchKernelGGL(ncef::bwd_reduce_kernel, dim3((unsigned)((tot4 + 255) / 256)), dim3(256), 0,
                     st, a.dpart, (int)rows, (int)D, a.chunks_b, a.q_len > 0 ? a.chunks_q : 0,
                     q_rows, dF);
  prof_end("nce_fused", st, 4.0 * rows * D * (2.0 * N) + 4.0 * (rows / 2) * D * K);
  return check_launch("nce_fused_bwd");
}
