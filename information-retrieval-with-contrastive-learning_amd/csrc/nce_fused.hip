// Fused InfoNCE (NT-Xent + MoCo queue) for the LSTM-head embedding width (D <= 256).
//
// Reference: NCELoss._compute_info_loss (src/contrastor/contrastive_loss.py:56-93):
// F = [q; k] [2N, D]; row r's logits are F_r . F_c / T for c != r (the positive is
// c = (r + N) mod 2N) and, with the queue, q_{r mod N} . queue_j / T (the k-rows
// REUSE q's queue logits); loss = sum_r CE_r / 2.
//
// The logits never land in HBM (the unfused path materialises S [2N, 2N] and
// LQ [N, K]): each wave streams 32-column tiles of [F ; queue^T] against a block
// of 32 rows on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32: products and sums
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

constexpr int NT = 256;       // 4 waves per workgroup, one work item each
constexpr int MAXD = 256;     // D <= 256 (8 d-blocks of 32 accumulate in 128 VGPRs)

struct Args {
  const float* F;      // [2N][D]
  const float* queue;  // [D][K] (key columns), or null
  int N, D, K;
  float invT;
  // rows computed: the pairs [p_lo, p_hi), i.e. q rows p_lo.. and k rows N + p_lo..
  // (all 2N rows when the range is [0, N); else 32-aligned, N % 32 == 0).  Local
  // row index: q rows 0 .. P-1, k rows P .. 2P-1 (P = p_hi - p_lo).
  int p_lo, p_hi;
  int tiles_per_item;  // 32-column tiles per wave
  // work items: u-blocks of the (one or two) row ranges x chunks
  int nr, ub_lo[2], n_ub[2], q_ub_lo, q_n_ub, chunks_b, chunks_q;
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
__device__ __forceinline__ int local_q_rows(const Args& a) { return a.p_hi - a.p_lo; }
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
// work item -> (u-block, chunk index in [0, chunks_b + chunks_q), queue part?)
__device__ __forceinline__ bool decode(const Args& a, int item, int& ub, int& ch, bool& qpart) {
  int it = item;
  for (int i = 0; i < a.nr; ++i) {
    const int n = a.n_ub[i] * a.chunks_b;
    if (it < n) {
      ub = a.ub_lo[i] + it / a.chunks_b;
      ch = it % a.chunks_b;
      qpart = false;
      return true;
    }
    it -= n;
  }
  if (it < a.q_n_ub * a.chunks_q) {
    ub = a.q_ub_lo + it / a.chunks_q;
    ch = a.chunks_b + it % a.chunks_q;
    qpart = true;
    return true;
  }
  return false;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// One 32 x 32 tile of S^T = X . F_u^T over all D (D % 8 == 0).  qcol: X is
// queue^T (column j of the [D][K] queue), else rows of F.  Rows / cols past the
// valid range read a clamped row (never used).
// qlds != null (backward, queue part): the queue tile X[j][d] is also kept in LDS as
// qlds[d * 33 + (j - v0)] for the dF product's transposed reads (pitch 33: the 32
// lanes of one d-column read 32 distinct banks).
__device__ __forceinline__ f32x16 logit_tile(const Args& a, int u0, int v0, bool qcol, int lane,
                                             float* qlds = nullptr) {
  const int r = lane & 31, h = lane >> 5;
  const int u = min(u0 + r, 2 * a.N - 1);
  const float* fu = a.F + (int64_t)u * a.D;
  f32x16 acc = (f32x16)0.0f;
  if (!qcol) {
    const int v = min(v0 + r, 2 * a.N - 1);
    const float* fv = a.F + (int64_t)v * a.D;
    for (int t = 0; t < a.D / 8; ++t) {
      const f32x4 x = ld4(fv + 8 * t + 4 * h);
      const f32x4 y = ld4(fu + 8 * t + 4 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s], y[s], acc, 0, 0, 0);
    }
  } else {
    const int j = min(v0 + r, a.K - 1);
    const float* qc = a.queue + j;
    for (int t = 0; t < a.D / 8; ++t) {
      const f32x4 y = ld4(fu + 8 * t + 4 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float x = qc[(int64_t)(8 * t + 4 * h + s) * a.K];
        if (qlds) qlds[(8 * t + 4 * h + s) * 33 + r] = x;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y[s], acc, 0, 0, 0);
      }
    }
  }
  return acc;
}

__device__ __forceinline__ int pos_of(int u, int N) { return u < N ? u + N : u - N; }

// ---- forward: per (32-row block, column chunk) the online (max, sum exp) --------
// item = blockIdx.x * 4 + wave over [in-batch items | queue items]
__global__ __launch_bounds__(NT) void fwd_partial_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  int ub, ch;
  bool qpart;
  if (!decode(a, blockIdx.x * 4 + (threadIdx.x >> 6), ub, ch, qpart)) return;
  if (qpart) ch -= a.chunks_b;
  const int n2 = 2 * a.N;
  const int u0 = ub * 32, r = lane & 31, h = lane >> 5;
  const int u = u0 + r;
  const int ncols = qpart ? a.K : n2;
  float m = -INFINITY, s = 0.f;
  for (int tt = 0; tt < a.tiles_per_item; ++tt) {
    const int v0 = (ch * a.tiles_per_item + tt) * 32;
    if (v0 >= ncols) break;
    const f32x16 acc = logit_tile(a, u0, v0, qpart, lane);
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
  // combine with the other half-wave (same row, the other 16 columns of each tile)
  const float m2 = __shfl_xor(m, 32, 64), s2 = __shfl_xor(s, 32, 64);
  const float mm = fmaxf(m, m2);
  const float ss = mm == -INFINITY ? 0.f : s * __expf(m - mm) + s2 * __expf(m2 - mm);
  if (h == 0) {
    if (qpart) {
      if (u < a.N) a.part_q[(int64_t)ch * a.N + u] = make_float2(mm, ss);
    } else if (u < n2) {
      a.part_b[(int64_t)ch * n2 + u] = make_float2(mm, ss);
    }
  }
}

// lse[r], loss_row[r] for the computed rows: partials combined in chunk order.
__global__ void fwd_combine_kernel(Args a, float* __restrict__ lse, float* __restrict__ loss_row) {
  const int lr = blockIdx.x * blockDim.x + threadIdx.x;
  if (lr >= (full_range(a) ? 2 * a.N : local_rows(a))) return;
  const int r = full_range(a) ? lr : abs_of(a, lr);
  const int n2 = 2 * a.N;
  const int chunks_q = a.K > 0 ? a.chunks_q : 0;
  float m = -INFINITY;
  for (int c = 0; c < a.chunks_b; ++c) m = fmaxf(m, a.part_b[(int64_t)c * n2 + r].x);
  const int n = r % a.N;
  for (int c = 0; c < chunks_q; ++c) m = fmaxf(m, a.part_q[(int64_t)c * a.N + n].x);
  float s = 0.f;
  for (int c = 0; c < a.chunks_b; ++c) {
    const float2 p = a.part_b[(int64_t)c * n2 + r];
    if (p.x != -INFINITY) s += p.y * __expf(p.x - m);
  }
  for (int c = 0; c < chunks_q; ++c) {
    const float2 p = a.part_q[(int64_t)c * a.N + n];
    if (p.x != -INFINITY) s += p.y * __expf(p.x - m);
  }
  const float l = m + logf(s);
  lse[r] = l;
  loss_row[r] = l - a.pos[r];
}

// ---- backward: dF partial of one (32-row block, column chunk) ------------------
// The coefficient tile C^T[v][u] (registers = v, lane = u) is the B operand of
// dF^T[d][u] += sum_v F_v[d] C^T[v][u]: MFMA step e pairs k = 0 (lanes h = 0) with
// v = v0 + (e & 3) + 8 (e >> 2) and k = 1 (h = 1) with that v + 4, so the A operand
// of step e is lane (r, h) <- X[v_e(h)][d0 + r].
template <int ND>
__global__ __launch_bounds__(NT) void bwd_partial_kernel(Args a) {
  extern __shared__ float qsh[];  // [4 waves][D][33] queue tiles
  const int lane = threadIdx.x & 63;
  float* qlds = qsh + (threadIdx.x >> 6) * a.D * 33;
  int ub, ch;
  bool qpart;
  if (!decode(a, blockIdx.x * 4 + (threadIdx.x >> 6), ub, ch, qpart)) return;
  const int n2 = 2 * a.N;
  const int u0 = ub * 32, r = lane & 31, h = lane >> 5;
  const int u = u0 + r;
  const float scale = 0.5f * a.invT * (a.gscale ? a.gscale[0] : 1.f);
  const int ncols = qpart ? a.K : n2;
  const float lse_u = a.lse[min(u, n2 - 1)];
  const float lse_k = qpart ? a.lse[min(u + a.N, n2 - 1)] : 0.f;  // the k-row sharing q's queue logits
  const int pu = pos_of(u, a.N);
  f32x16 dacc[ND];
#pragma unroll
  for (int b = 0; b < ND; ++b) dacc[b] = (f32x16)0.0f;
  const int cb = qpart ? ch - a.chunks_b : ch;
  for (int tt = 0; tt < a.tiles_per_item; ++tt) {
    const int v0 = (cb * a.tiles_per_item + tt) * 32;
    if (v0 >= ncols) break;
    const f32x16 acc = logit_tile(a, u0, v0, qpart, lane, qpart ? qlds : nullptr);
    if (qpart) __builtin_amdgcn_wave_barrier();  // the wave's own LDS tile: no workgroup sync
    float coef[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int v = v0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      const float z = acc[e] * a.invT;
      float c = 0.f;
      if (v < ncols && u < n2) {
        if (qpart) {
          c = __expf(z - lse_u) + __expf(z - lse_k);
        } else if (v != u) {
          c = __expf(z - lse_u) - (v == pu ? 1.f : 0.f);       // G_uv
          c += __expf(z - a.lse[v]) - (u == pos_of(v, a.N) ? 1.f : 0.f);  // G_vu
        }
      }
      coef[e] = c * scale;
    }
    // dF^T[d][u] += X[v][d] coef[v][u]
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      const int d = 32 * b + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int vl = (e & 3) + 8 * (e >> 2) + 4 * h;
        const float x = qpart ? qlds[d * 33 + vl]
                              : a.F[(int64_t)min(v0 + vl, n2 - 1) * a.D + d];
        dacc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, coef[e], dacc[b], 0, 0, 0);
      }
    }
    if (qpart) __builtin_amdgcn_wave_barrier();  // reads done before the next tile's writes
  }
  // dacc[b] C layout: lane (r, h) register e = dF^T[32 b + (e & 3) + 8 (e >> 2) + 4 h][u0 + r]
  const int lr = full_range(a) ? (u < n2 ? u : -1) : local_of(a, u);
  const int nloc = full_range(a) ? n2 : local_rows(a);
  if (lr >= 0) {
    float* out = a.dpart + ((int64_t)ch * nloc + lr) * a.D;
#pragma unroll
    for (int b = 0; b < ND; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) out[32 * b + (e & 3) + 8 * (e >> 2) + 4 * h] = dacc[b][e];
  }
}

// dF[r] = sum over chunks (fixed order) of the partials that cover row r.
__global__ void bwd_reduce_kernel(const float* __restrict__ dpart, int rows, int D, int chunks_b,
                                  int chunks_q, int q_rows, float* __restrict__ dF) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)rows * D) return;
  const int row = (int)(e / D);
  float s = 0.f;
  for (int c = 0; c < chunks_b; ++c) s += dpart[(int64_t)c * rows * D + e];
  if (row < q_rows)
    for (int c = 0; c < chunks_q; ++c) s += dpart[(int64_t)(chunks_b + c) * rows * D + e];
  dF[e] = s;
}

}  // namespace ncef
}  // namespace irc

using namespace irc;

namespace {
constexpr int TPI = 4;  // 32-column tiles per work item (wave)

// Plan of the work items; false when the pair range is not supported.
bool plan(ncef::Args& a, int64_t N, int64_t K, int64_t p_lo, int64_t p_hi) {
  a.p_lo = (int)p_lo;
  a.p_hi = (int)p_hi;
  a.tiles_per_item = TPI;
  a.chunks_b = (int)((2 * N + 32 * TPI - 1) / (32 * TPI));
  a.chunks_q = K > 0 ? (int)((K + 32 * TPI - 1) / (32 * TPI)) : 0;
  if (p_lo == 0 && p_hi == N) {  // every row: one range, no alignment needed
    a.nr = 1;
    a.ub_lo[0] = 0;
    a.n_ub[0] = (int)((2 * N + 31) / 32);
    a.q_ub_lo = 0;
    a.q_n_ub = K > 0 ? (int)((N + 31) / 32) : 0;
    return true;
  }
  if (N % 32 || p_lo % 32 || p_hi % 32 || p_lo < 0 || p_hi > N || p_lo >= p_hi) return false;
  a.nr = 2;
  a.ub_lo[0] = (int)(p_lo / 32);
  a.ub_lo[1] = (int)((N + p_lo) / 32);
  a.n_ub[0] = a.n_ub[1] = (int)((p_hi - p_lo) / 32);
  a.q_ub_lo = a.ub_lo[0];
  a.q_n_ub = K > 0 ? a.n_ub[0] : 0;
  return true;
}
int64_t n_items(const ncef::Args& a) {
  int64_t n = (int64_t)a.q_n_ub * a.chunks_q;
  for (int i = 0; i < a.nr; ++i) n += (int64_t)a.n_ub[i] * a.chunks_b;
  return n;
}
int64_t local_rows(int64_t N, int64_t p_lo, int64_t p_hi) {
  return (p_lo == 0 && p_hi == N) ? 2 * N : 2 * (p_hi - p_lo);
}
}  // namespace

extern "C" int64_t irc_nce_fused_workspace(int64_t N, int64_t D, int64_t K, int64_t p_lo,
                                           int64_t p_hi) {
  ncef::Args a{};
  if (!plan(a, N, K, p_lo, p_hi)) return 0;
  const int64_t fwd = ((int64_t)a.chunks_b * 2 * N + (int64_t)a.chunks_q * N) * 8 + 2 * N * 4;
  const int64_t bwd = (int64_t)(a.chunks_b + a.chunks_q) * local_rows(N, p_lo, p_hi) * D * 4;
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
  IRC_REQUIRE(plan(a, N, K, p_lo, p_hi),
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
  hipLaunchKernelGGL(ncef::fwd_partial_kernel, dim3((unsigned)((items + 3) / 4)), dim3(ncef::NT),
                     0, st, a);
  hipLaunchKernelGGL(ncef::fwd_combine_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                     st, a, lse, loss_row);
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
  IRC_REQUIRE(plan(a, N, K, p_lo, p_hi), "nce_fused: bad pair range");
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
  const dim3 gb((unsigned)((items + 3) / 4));
  const size_t lds = (size_t)4 * D * 33 * sizeof(float);
  switch (D / 32) {
#define IRC_NCEB(ND)                                                                      \
  case ND:                                                                                \
    hipLaunchKernelGGL(ncef::bwd_partial_kernel<ND>, gb, dim3(ncef::NT), lds, st, a); \
    break;
    IRC_NCEB(1) IRC_NCEB(2) IRC_NCEB(3) IRC_NCEB(4) IRC_NCEB(5) IRC_NCEB(6) IRC_NCEB(7) IRC_NCEB(8)
#undef IRC_NCEB
  }
  const int64_t tot = rows * D;
  hipLaunchKernelGGL(ncef::bwd_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                     a.dpart, (int)rows, (int)D, a.chunks_b, a.q_n_ub > 0 ? a.chunks_q : 0, q_rows,
                     dF);
  prof_end("nce_fused", st, 4.0 * rows * D * (2.0 * N) + 4.0 * (rows / 2) * D * K);
  return check_launch("nce_fused_bwd");
}
