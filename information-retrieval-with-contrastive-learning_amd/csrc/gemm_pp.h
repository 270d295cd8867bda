// Host interface of the ping-pong bf16 GEMM (gemm_pp.hip), used by irc_gemm.
#pragma once
#include "irc_common.h"

namespace irc {

// LayerNorm fold of the BERT encoder: a pre-LN activation h is kept
// with per-row statistics as partial (sum, sum of squares) pairs over disjoint column
// tiles, stats[row][tile][2], written by the epilogue that produces h.  A GEMM whose
// input is LN(h) = (h - mu) r gamma + beta runs on h itself with the folded weight
// W' = W diag(gamma) and the epilogue  y = r acc + (-r mu) s_n + t_n  (s_n = sum_k W'_nk,
// t_n = b_n + sum_k beta_k W_nk); a residual LN(h) is recomputed in the epilogue as the
// LayerNorm kernel would write it (bf16 of fma((h - mu) r, gamma, beta)).
struct LnArgs {
  const float* st;  // input statistics [M][nt][2] (fold: of A's rows; else of R's rows)
  int nt;
  float inv_h, eps;
  const float* gamma;  // residual recompute (EPI_BIAS_RESID): LN weight / bias of R
  const float* beta;
  const float* fold_s;  // fold (EPI_BIAS / EPI_BIAS_GELU): column sums of the folded weight
  float* st_out;        // output statistics [M][nt_out][2] of C's bf16 values, or null
  int nt_out;
};

__device__ __forceinline__ void ln_row_stats(const LnArgs& l, int row, float& mu, float& r) {
  const float2* p = reinterpret_cast<const float2*>(l.st) + (int64_t)row * l.nt;
  float s = 0.f, q = 0.f;
  for (int t = 0; t < l.nt; ++t) {
    const float2 v = p[t];
    s += v.x;
    q += v.y;
  }
  mu = s * l.inv_h;
  const float var = fmaxf(q * l.inv_h - mu * mu, 0.f);
  r = rsqrtf(var + l.eps);
}

namespace gpp {

struct PArgs {
  const unsigned short* A;
  const unsigned short* B;
  void* C;
  const float* bias;
  const void* R;
  float* P;  // split-K slabs [batch][split][M][N] or null
  int M, N, K, kchunk;
  int64_t lda, ldb, ldc, ldr;
  int64_t sA, sB, sC, sR, sBias;
  float alpha;
  int accumulate;
  int vec_c;
  // scan-filter epilogue (EPI_SCAN): survivors key >= thr[q] of C[q][doc] go to
  // keys[(tn * qpad + q) * cap + slot] (cap >= 256: a doc tile never overflows),
  // their count to counts[tn * qpad + q]; doc global index = idx_base + doc * stride
  const uint64_t* thr;
  uint64_t* keys;
  uint32_t* counts;
  int64_t cap;
  int qpad;
  int stride;
  uint32_t idx_base;
  // scan filter lists (EPI_SCAN with lists != null, no threshold): the 4 largest keys
  // of each (256-doc tile tn, query q) go to lists[(q * ls + tn) * 4 + i], in
  // descending order, 0 for empty slots (the single pass: select_dense reads them;
  // the threshold sample: lists_kth_kernel)
  uint64_t* lists;
  int ls;
  // fp8 linear layers (F8, non-scan epilogues): C = alpha * (A8 . B8^T) * sa[row]
  // * sb[col] (+ bias ...): per-row dequantisation scales of both e4m3 operands
  const float* sa;
  const float* sb;
  // grouped tile order (grouped_tile in irc_common.h); 0 / 1 = row-major
  int group_m;
  // MX-fp8 linear layers (run_mx): E8M0 block scales of A / B in the MX layout
  // [K8/128][rows padded to 256][4] (mpad / npad = the padded row counts), and,
  // when cx != null, an MX-fp8 OUTPUT: C holds e4m3 bytes (ldc in bytes) and cx
  // its block scales ([N/128][mpad][4]); else C is bf16.
  const unsigned char* sax;
  const unsigned char* sbx;
  int mpad, npad;
  unsigned char* cx;
  // LayerNorm fold (bf16 C, vectorised epilogue, non-persistent): ln.st == null = off
  LnArgs ln;
};

constexpr int EPI_SCAN = 7;

int splits_for(int out_f32, int epi, int64_t M, int64_t N, int64_t K, int64_t batch,
               int64_t budget = 256);
// CUs of the current device (256 when the query fails)
int device_cu_count();
// compute units of the current device (cached per device; 0 if unknown)
int cu_count();
bool qualifies(int la, int lb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
               int64_t sA, const void* B, int64_t ldb, int64_t sB, int64_t batch, int splits);
// max_grid > 0: at most that many workgroups -- a launch of more tiles runs as a static
// persistent tile loop over a grid of max_grid (same per-tile arithmetic: bit-identical)
void run(int out_f32, int la, int lb, int epi, const PArgs& a, int64_t batch, int splits,
         hipStream_t st, int64_t max_grid = 0);
// scan filter: A = queries [M=Q][K=D], B = docs [N][D] (row stride ldb), EPI_SCAN;
// fp8: e4m3 operands, K / lda / ldb in 2-byte units (D/2)
void run_scan(const PArgs& a, hipStream_t st, bool fp8 = false);
// raw fp32 C = A . B^T of e4m3 operands (K, lda, ldb in 2-byte units; vec_c layout)
void run_scores_fp8(const PArgs& a, hipStream_t st);
// e4m3 linear layer: bf16 C = (A8 . B8^T) * sa[m] * sb[n] (+ bias / GELU / residual);
// both operands K-major, K / lda / ldb in 2-byte units, vec_c layout required
void run_fp8(int epi, const PArgs& a, hipStream_t st);
// MX-fp8 linear layer: C = (A8 . B8^T with per-32-k E8M0 block scales) (+ bias /
// GELU / residual); bf16 C, or MX-fp8 C when a.cx != null (epilogues 1, 2 only)
void run_mx(int epi, const PArgs& a, hipStream_t st);
// LayerNorm-fold linear layer (irc_gemm_ln): bf16 K-major operands, bf16 vec_c C,
// epilogues 1-3 with a.ln set (see LnArgs)
void run_ln(int epi, const PArgs& a, hipStream_t st);

}  // namespace gpp
}  // namespace irc
