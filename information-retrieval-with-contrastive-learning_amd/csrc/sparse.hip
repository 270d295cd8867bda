// Hashed n-gram TF-IDF retrieval on the GPU: the reference's actual predict path
// (SURVEY.md 8f rank 2).
//
//  * irc_csr_union_count / irc_csr_union_emit -- documents_filtering
//    (src/evaluation.py:57-81): the docs with a nonzero in any of a claim's
//    hashed n-gram rows of the inverted count matrix, `np.unique(
//    count_matrix[wids_unique].nonzero()[1])` = sorted ascending.  One bitmap
//    per query (atomicOr marks), per-chunk popcounts, an ordered compaction.
//  * irc_csr_spmv_f64 -- TfidfDocRanker.closest_docs' `spvec * doc_mat`
//    (preprocessing/drqa/retriever/tfidf_doc_ranker.py:64-65): per query the
//    rows are applied in ascending hash order, one at a time, each product and
//    sum rounded separately in fp64 (no FMA) -- scipy's csr_matmat order, so the
//    scores are bit-identical to the reference's.
//  * irc_topk_f64 -- the top-k of the nonzero scores (:67-73): the k-th largest
//    score by an exact radix select on the orderable 64-bit patterns, ties at
//    the boundary resolved to the lower doc index (the build's rule; numpy's
//    argpartition leaves it unspecified), then a (score desc, index asc) sort.
//
// Integer / fp64 gather-scatter work, HBM- and latency-bound: no MFMA.
#include "irc_common.h"

namespace irc {
namespace sparse {

constexpr int NT = 256;
constexpr int64_t CHUNK_WORDS = 1024;  // bitmap words per compaction chunk (32 K docs): a
// dense union emits up to 32 docs per word serially, so chunks are kept small for
// parallelism (7 workgroups per query at 200k docs instead of 1)

// grid (pairs, SEG): block (pair, s) ORs the doc bits of segment s of the pair's
// row -- long (Zipf-head) rows are spread over SEG workgroups.
constexpr int SEG = 16;
__global__ __launch_bounds__(NT) void union_mark_kernel(const int64_t* __restrict__ indptr,
                                                        const int32_t* __restrict__ indices,
                                                        const int64_t* __restrict__ q_off,
                                                        const int64_t* __restrict__ q_rows,
                                                        int64_t Q, int64_t words,
                                                        uint32_t* __restrict__ bitmaps) {
  const int64_t pair = blockIdx.x;
  // query of this pair: binary search in q_off (Q + 1 entries)
  int64_t lo = 0, hi = Q;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (q_off[mid] <= pair) lo = mid; else hi = mid;
  }
  const int64_t q = lo;
  const int64_t r = q_rows[pair];
  uint32_t* bm = bitmaps + q * words;
  const int64_t b = indptr[r], len = indptr[r + 1] - b;
  const int64_t j0 = b + len * blockIdx.y / SEG, j1 = b + len * (blockIdx.y + 1) / SEG;
  // A row's doc indices ascend, so a wave's 64 docs fall in a few bitmap words:
  // OR the bits of each run of equal words across lanes (segmented suffix scan,
  // run head = first lane of the run) and let only run heads issue the atomic.
  // Any order stays correct: a lane only ever merges bits of its own word.
  const int lane = threadIdx.x & 63;
  for (int64_t base = j0; base < j1; base += NT) {  // uniform trip count
    const int64_t j = base + threadIdx.x;
    const bool valid = j < j1;
    const uint32_t d = valid ? (uint32_t)indices[j] : 0u;
    const uint32_t word = valid ? d >> 5 : 0xffffffffu;
    uint32_t bits = valid ? 1u << (d & 31) : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t w2 = __shfl_down(word, o, 64);
      const uint32_t b2 = __shfl_down(bits, o, 64);
      if (lane + o < 64 && w2 == word) bits |= b2;
    }
    const uint32_t prev = __shfl_up(word, 1, 64);
    if (valid && (lane == 0 || prev != word)) atomicOr(&bm[word], bits);
  }
}

// grid (chunks, Q): popcount of one chunk of one query's bitmap.
__global__ __launch_bounds__(NT) void union_count_kernel(const uint32_t* __restrict__ bitmaps,
                                                         int64_t words, int64_t nchunks,
                                                         int64_t* __restrict__ chunk_sums) {
  __shared__ int64_t part[NT / 64];
  const int64_t q = blockIdx.y, c = blockIdx.x;
  const uint32_t* bm = bitmaps + q * words;
  const int64_t w0 = c * CHUNK_WORDS;
  const int64_t w1 = w0 + CHUNK_WORDS < words ? w0 + CHUNK_WORDS : words;
  int64_t s = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += NT) s += __popc(bm[w]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int i = 0; i < NT / 64; ++i) t += part[i];
    chunk_sums[q * nchunks + c] = t;
  }
}

// grid (chunks, Q): writes the chunk's doc indices in ascending order at
// out_off[q] + (sum of the query's earlier chunks) -- a deterministic compaction.
__global__ __launch_bounds__(NT) void union_emit_kernel(const uint32_t* __restrict__ bitmaps,
                                                        int64_t words, int64_t nchunks,
                                                        const int64_t* __restrict__ chunk_sums,
                                                        const int64_t* __restrict__ out_off,
                                                        int32_t* __restrict__ out_idx) {
  __shared__ int64_t wsum[NT / 64];
  const int64_t q = blockIdx.y, c = blockIdx.x;
  const uint32_t* bm = bitmaps + q * words;
  int64_t base = out_off[q];
  for (int64_t i = 0; i < c; ++i) base += chunk_sums[q * nchunks + i];
  constexpr int WPT = CHUNK_WORDS / NT;  // 4 consecutive words per thread
  const int64_t w0 = c * CHUNK_WORDS + (int64_t)threadIdx.x * WPT;
  int64_t mine = 0;
  for (int i = 0; i < WPT; ++i)
    if (w0 + i < words) mine += __popc(bm[w0 + i]);
  // block exclusive scan of `mine` (thread order = word order)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int64_t pos = base + incl - mine;
  for (int w = 0; w < wave; ++w) pos += wsum[w];
  for (int i = 0; i < WPT; ++i) {
    if (w0 + i >= words) break;
    uint32_t b = bm[w0 + i];
    while (b) {
      const int t = __builtin_ctz(b);
      b &= b - 1;
      out_idx[pos++] = (int32_t)(((w0 + i) << 5) + t);
    }
  }
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t lo,
                                                   int64_t hi, int32_t x) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// grid (DR doc ranges, Q): dense[q][doc] += w_r * A[r][doc] for the query's rows
// in the given (ascending) order.  Each doc belongs to one workgroup (its doc
// range; CSR rows are index-sorted, so a range is a binary-searched slice of
// every row), and a barrier between rows orders the updates of a doc two rows
// share -- every doc sees its products in row order.  fp64 multiply and add
// rounded separately.
constexpr int DR = 32;
__global__ __launch_bounds__(NT) void spmv_f64_kernel(const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ indices,
                                                      const double* __restrict__ data,
                                                      const int64_t* __restrict__ q_off,
                                                      const int64_t* __restrict__ q_rows,
                                                      const double* __restrict__ q_w,
                                                      int64_t n_cols,
                                                      double* __restrict__ dense) {
#pragma clang fp contract(off)  // a separately rounded product and sum, as scipy
  const int64_t q = blockIdx.y;
  double* row_out = dense + q * n_cols;
  const int32_t d0 = (int32_t)(n_cols * blockIdx.x / DR);
  const int32_t d1 = (int32_t)(n_cols * (blockIdx.x + 1) / DR);
  for (int64_t p = q_off[q]; p < q_off[q + 1]; ++p) {
    const int64_t r = q_rows[p];
    const double w = q_w[p];
    const int64_t lo = lower_bound_i32(indices, indptr[r], indptr[r + 1], d0);
    const int64_t hi = lower_bound_i32(indices, lo, indptr[r + 1], d1);
    for (int64_t j = lo + threadIdx.x; j < hi; j += NT) {
      const int32_t d = indices[j];
      const double prod = w * data[j];
      row_out[d] = row_out[d] + prod;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint64_t orderable_f64(double x) {
  uint64_t u = __double_as_longlong(x);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

constexpr int TK_MAX = 1024;
// 1024 threads per query: the candidate passes are dependent gathers
// (row[cand[i]]), latency-bound, and only Q workgroups exist -- 16 waves per
// query keep 4x the loads in flight of a 256-thread block.
constexpr int TNT = 1024;
constexpr int TK_STAGE = 8192;  // 64 KB of LDS keys
constexpr int TK_U = 8;          // score loads in flight per thread

// One workgroup per query over its candidate docs (ascending indices) with
// nonzero scores: exact k-th largest score, boundary ties to the lower index,
// then a (score desc, index asc) bitonic sort in LDS.  Writes out_n[q] valid
// entries (fewer than k when fewer docs scored), the rest (0, -1).
__global__ __launch_bounds__(TNT) void topk_f64_kernel(const double* __restrict__ dense,
                                                      int64_t n_cols,
                                                      const int32_t* __restrict__ cand,
                                                      const int64_t* __restrict__ cand_off,
                                                      int k, double* __restrict__ out_score,
                                                      int64_t* __restrict__ out_idx,
                                                      int32_t* __restrict__ out_n) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_key[TK_MAX];
  __shared__ int32_t s_idx[TK_MAX];
  __shared__ uint64_t c_key[TK_STAGE];  // keys of the selected bucket, once they fit
  // 0: nonzero count, 1: kr, 2: digit, 3: collect ctr, 4: selected bucket size,
  // 5: staged count
  __shared__ uint32_t s_misc[6];
  __shared__ int64_t s_wsum[TNT / 64];
  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* row = dense + q * n_cols;
  // cand == nullptr: every doc of the row is a candidate (a dense union reads the
  // row contiguously instead of gathering through the candidate list)
  const bool all_docs = cand == nullptr;
  const int64_t c0 = all_docs ? 0 : cand_off[q], c1 = all_docs ? n_cols : cand_off[q + 1];
  auto doc = [&](int64_t i) -> int64_t { return all_docs ? i : (int64_t)cand[i]; };
  // Unordered pass over the candidates' scores, TK_U loads in flight per thread
  // (one load per iteration left each thread waiting out a full memory latency).
  auto each_score = [&](auto&& f) {
    for (int64_t b = c0 + tid; b < c1; b += (int64_t)TNT * TK_U) {
      double v[TK_U];
#pragma unroll
      for (int u = 0; u < TK_U; ++u) {
        const int64_t i = b + (int64_t)u * TNT;
        v[u] = i < c1 ? row[doc(i)] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < TK_U; ++u)
        if (v[u] != 0.0) f(v[u], b + (int64_t)u * TNT);
    }
  };
  if (tid == 0) {
    s_misc[0] = 0;
    s_misc[3] = 0;
    s_misc[5] = 0;
  }
  if (tid < 256) hist[tid] = 0;
  __syncthreads();
  // first pass: nonzero count and the top digit's histogram together
  uint32_t nz = 0;
  each_score([&](double s, int64_t) {
    ++nz;
    atomicAdd(&hist[orderable_f64(s) >> 56], 1u);
  });
  atomicAdd(&s_misc[0], nz);
  __syncthreads();
  const uint32_t M = s_misc[0];
  const int cnt = (int)(M < (uint32_t)k ? M : (uint32_t)k);
  // k-th largest orderable key among nonzero scores (exact, 8 x 8-bit digits).
  // Once the selected bucket (the keys matching the prefix so far) fits
  // TK_STAGE, one more gather stages it in LDS and the later digits read LDS.
  uint64_t kth = 0, pmask = 0, prefix = 0;
  if (M > (uint32_t)k) {
    uint32_t kr = (uint32_t)k;
    uint32_t nsel = M;
    bool staged = false;
    for (int shift = 56; shift >= 0; shift -= 8) {
      if (shift != 56) {
        if (!staged && nsel <= (uint32_t)TK_STAGE) {
          each_score([&](double s, int64_t) {
            const uint64_t key = orderable_f64(s);
            if ((key & pmask) == prefix) c_key[atomicAdd(&s_misc[5], 1u)] = key;
          });
          staged = true;
        }
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        if (staged) {
          const int ns = (int)s_misc[5];
          for (int i = tid; i < ns; i += TNT) {
            const uint64_t key = c_key[i];
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
          }
        } else {
          each_score([&](double s, int64_t) {
            const uint64_t key = orderable_f64(s);
            if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
          });
        }
        __syncthreads();
      }
      if (wave == 0) {
        uint32_t bb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bb[j] = hist[4 * lane + j];
        const uint32_t c4 = bb[0] + bb[1] + bb[2] + bb[3];
        uint32_t suf = c4;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_down(suf, o, 64);
          if (lane + o < 64) suf += t;
        }
        const uint32_t above = suf - c4;
        if (suf >= kr && above < kr) {
          uint32_t acc = above;
          int sel = 4 * lane;
          uint32_t bsz = bb[0];
          for (int j = 3; j >= 0; --j) {
            if (acc + bb[j] >= kr) {
              sel = 4 * lane + j;
              bsz = bb[j];
              break;
            }
            acc += bb[j];
          }
          s_misc[2] = (uint32_t)sel;
          s_misc[1] = kr - acc;
          s_misc[4] = bsz;
        }
      }
      __syncthreads();
      prefix |= (uint64_t)s_misc[2] << shift;
      pmask |= (uint64_t)0xff << shift;
      kr = s_misc[1];
      nsel = s_misc[4];
      __syncthreads();
    }
    kth = prefix;  // the exact k-th largest key; kr = how many of the ties to take
    // keys > kth: all taken; keys == kth: the lowest `need` indices (ordered scan)
    const uint32_t need = kr;
    // nsel = the last digit's bucket = the keys equal to kth. When all of them
    // are taken, nothing depends on the order: one unordered pass.
    const bool all_eq = nsel == need;
    if (all_eq)
      each_score([&](double s, int64_t i) {
        const uint64_t key = orderable_f64(s);
        if (key >= kth) {
          const uint32_t slot = atomicAdd(&s_misc[3], 1u);
          s_key[slot] = key;
          s_idx[slot] = (int32_t)doc(i);
        }
      });
    int64_t taken_eq_before = 0;
    for (int64_t b0 = all_eq ? c1 : c0; b0 < c1; b0 += TNT) {
      const int64_t i = b0 + tid;
      uint64_t key = 0;
      bool gt = false, eq = false;
      if (i < c1) {
        const double s = row[doc(i)];
        if (s != 0.0) {
          key = orderable_f64(s);
          gt = key > kth;
          eq = key == kth;
        }
      }
      // ordered rank of this thread's eq among the block's eq flags
      const uint64_t bal = __ballot(eq);
      const int64_t r_in_wave = __popcll(bal & ((1ull << lane) - 1));
      if (lane == 0) s_wsum[wave] = __popcll(bal);
      __syncthreads();
      int64_t r_eq = taken_eq_before + r_in_wave;
      int64_t blk_eq = 0;
      for (int w = 0; w < TNT / 64; ++w) {
        if (w < wave) r_eq += s_wsum[w];
        blk_eq += s_wsum[w];
      }
      if (gt || (eq && r_eq < (int64_t)need)) {
        const uint32_t slot = atomicAdd(&s_misc[3], 1u);
        s_key[slot] = key;
        s_idx[slot] = (int32_t)doc(i);
      }
      taken_eq_before += blk_eq;
      __syncthreads();
    }
  } else {
    each_score([&](double s, int64_t i) {
      const uint32_t slot = atomicAdd(&s_misc[3], 1u);
      s_key[slot] = orderable_f64(s);
      s_idx[slot] = (int32_t)doc(i);
    });
  }
  __syncthreads();
  // bitonic sort of cnt entries by (key desc, idx asc)
  int npow = 1;
  while (npow < cnt) npow <<= 1;
  for (int i = cnt + tid; i < npow; i += TNT) {
    s_key[i] = 0;
    s_idx[i] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < npow; i += TNT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint64_t ki = s_key[i], kj = s_key[j];
          const int32_t ii = s_idx[i], ij = s_idx[j];
          // "i before j" in the final order: larger key, then lower index
          const bool i_first = ki > kj || (ki == kj && ii < ij);
          if (desc ? !i_first : i_first) {
            s_key[i] = kj;
            s_key[j] = ki;
            s_idx[i] = ij;
            s_idx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += TNT) {
    double sc = 0.0;
    int64_t id = -1;
    if (i < cnt) {
      const uint64_t key = s_key[i];
      const uint64_t u = (key >> 63) ? (key & ~(1ull << 63)) : ~key;
      sc = __longlong_as_double((long long)u);
      id = s_idx[i];
    }
    out_score[q * k + i] = sc;
    out_idx[q * k + i] = id;
  }
  if (tid == 0) out_n[q] = cnt;
}

}  // namespace sparse
}  // namespace irc

using namespace irc;
using namespace irc::sparse;

extern "C" int64_t irc_csr_union_chunks(int64_t n_cols) {
  const int64_t words = (n_cols + 31) / 32;
  return (words + CHUNK_WORDS - 1) / CHUNK_WORDS;
}

extern "C" int irc_csr_union_count(const int64_t* indptr, const int32_t* indices, int64_t n_cols,
                                   const int64_t* q_off, const int64_t* q_rows, int64_t Q,
                                   int64_t n_pairs, uint32_t* bitmaps, int64_t* chunk_sums,
                                   irc_stream_t stream) {
  IRC_REQUIRE(n_cols >= 0 && Q >= 0 && n_pairs >= 0, "csr_union: negative size");
  IRC_REQUIRE(n_cols < (1ll << 31), "csr_union: n_cols must fit int32 doc indices");
  if (Q == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const int64_t words = (n_cols + 31) / 32;
  const int64_t nchunks = irc_csr_union_chunks(n_cols);
  if (words > 0 && hipMemsetAsync(bitmaps, 0, (size_t)Q * words * 4, st) != hipSuccess)
    return check_launch("csr_union memset");
  if (n_pairs > 0)
    hipLaunchKernelGGL(union_mark_kernel, dim3((unsigned)n_pairs, SEG), dim3(NT), 0, st, indptr,
                       indices, q_off, q_rows, Q, words, bitmaps);
  if (int rc = check_launch("union_mark_kernel")) return rc;
  if (nchunks > 0)
    hipLaunchKernelGGL(union_count_kernel, dim3((unsigned)nchunks, (unsigned)Q), dim3(NT), 0, st,
                       bitmaps, words, nchunks, chunk_sums);
  return check_launch("union_count_kernel");
}

extern "C" int irc_csr_union_emit(const uint32_t* bitmaps, int64_t n_cols, int64_t Q,
                                  const int64_t* chunk_sums, const int64_t* out_off,
                                  int32_t* out_idx, irc_stream_t stream) {
  IRC_REQUIRE(n_cols >= 0 && Q >= 0, "csr_union_emit: negative size");
  if (Q == 0 || n_cols == 0) return IRC_OK;
  const int64_t words = (n_cols + 31) / 32;
  const int64_t nchunks = irc_csr_union_chunks(n_cols);
  hipLaunchKernelGGL(union_emit_kernel, dim3((unsigned)nchunks, (unsigned)Q), dim3(NT), 0,
                     as_stream(stream), bitmaps, words, nchunks, chunk_sums, out_off, out_idx);
  return check_launch("union_emit_kernel");
}

extern "C" int irc_csr_spmv_f64(const int64_t* indptr, const int32_t* indices, const double* data,
                                int64_t n_cols, const int64_t* q_off, const int64_t* q_rows,
                                const double* q_w, int64_t Q, double* dense,
                                irc_stream_t stream) {
  IRC_REQUIRE(n_cols >= 0 && Q >= 0, "csr_spmv_f64: negative size");
  if (Q == 0) return IRC_OK;
  hipLaunchKernelGGL(spmv_f64_kernel, dim3(DR, (unsigned)Q), dim3(NT), 0, as_stream(stream),
                     indptr, indices, data, q_off, q_rows, q_w, n_cols, dense);
  return check_launch("spmv_f64_kernel");
}

extern "C" int irc_topk_f64(const double* dense, int64_t n_cols, const int32_t* cand,
                            const int64_t* cand_off, int64_t Q, int64_t k, double* out_score,
                            int64_t* out_idx, int32_t* out_n, irc_stream_t stream) {
  IRC_REQUIRE(k >= 1 && k <= TK_MAX, "topk_f64: k=%lld outside [1, %d]", (long long)k, TK_MAX);
  IRC_REQUIRE(Q >= 0, "topk_f64: negative Q");
  IRC_REQUIRE(cand != nullptr || n_cols < (1ll << 31), "topk_f64: n_cols must fit int32 doc ids");
  IRC_REQUIRE(cand == nullptr || cand_off != nullptr, "topk_f64: cand without cand_off");
  if (Q == 0) return IRC_OK;
  hipLaunchKernelGGL(topk_f64_kernel, dim3((unsigned)Q), dim3(TNT), 0, as_stream(stream), dense,
                     n_cols, cand, cand_off, (int)k, out_score, out_idx, out_n);
  return check_launch("topk_f64_kernel");
}
