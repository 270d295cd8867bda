/*
 * irc.h -- C ABI of libirc_hip.so, the MI355X (gfx950 / CDNA4) kernels behind the
 * contrastive-training + dense-retrieval hot path of
 * PM25/Information-Retrieval-with-Contrastive-Learning.
 *
 * The reference is pure Python over torch/transformers and has no FFI of its own
 * (SURVEY.md 2.1); each entry point below names the reference call site whose
 * device work it replaces.  The Python host layer (irc_amd/_lib.py) binds these
 * with ctypes -- plain pointers and sizes, no torch types.
 *
 * Conventions
 *  - Every call is stream-ordered on `stream` (a hipStream_t) and never
 *    synchronises the host.  Device buffers are owned by the caller (the PyTorch
 *    caching allocator); scratch is passed in explicitly as `workspace`.
 *  - Return value: 0 on success, otherwise a hipError_t or an IRC_E_* code;
 *    irc_last_error() returns a thread-local message for the last failure.
 *  - bf16 buffers are raw uint16 bit patterns; all matrices are row-major and
 *    contiguous unless a leading dimension is given.
 */
#ifndef IRC_H_
#define IRC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* irc_stream_t; /* hipStream_t */

#define IRC_OK 0
#define IRC_E_INVALID 1001   /* bad argument / unsupported shape */
#define IRC_E_WORKSPACE 1002 /* workspace too small */
#define IRC_E_LAUNCH 1003    /* kernel launch failed */

const char* irc_last_error(void);
int irc_abi_version(void);

/* ------------------------------------------------------------------ retrieval
 * Corpus-wide cosine top-k.  Replaces the dense scoring that
 * src/evaluation.py:110-112 sketches ((clm_vec * evdn_vec).sum(-1) over
 * ctx2vec outputs) with the ordering of
 * preprocessing/drqa/retriever/tfidf_doc_ranker.py:60-75 (closest_docs: top-k by
 * descending score).  Ties: lower global doc index first.
 *
 * queries [Q, D] bf16, docs [N, D] bf16 (one shard; global index = doc_offset +
 * row, must stay < 2^32).  Outputs out_score [Q, k] fp32 and out_idx [Q, k]
 * int64, sorted; slots beyond min(k, N) are (-inf, -1).  D % 64 == 0,
 * 1 <= k <= 1024.  Exact: the result is the top-k of the fp32 scores the MFMA
 * produced, never an approximation (sample threshold + exact radix select).
 */
int64_t irc_scan_topk_workspace(int64_t Q, int64_t N, int64_t D, int64_t k);
int irc_scan_topk(const void* queries, const void* docs, int64_t Q, int64_t N, int64_t D,
                  int64_t k, int64_t doc_offset, void* workspace, int64_t workspace_bytes,
                  float* out_score, int64_t* out_idx, irc_stream_t stream);

/* Merge P per-shard sorted top-k lists, in_score/in_idx [P, Q, kin] (global
 * indices, -1 = empty), into out [Q, kout] with the same (score desc, idx asc)
 * rule -- the reduce step of the sharded scan. kout <= 1024. */
int irc_topk_merge(const float* in_score, const int64_t* in_idx, int64_t P, int64_t Q,
                   int64_t kin, int64_t kout, float* out_score, int64_t* out_idx,
                   irc_stream_t stream);

/* Raw score tile for tests / diagnostics: out[Q, N] fp32 = queries . docs^T
 * using the same MFMA path as irc_scan_topk. */
int irc_scan_scores(const void* queries, const void* docs, int64_t Q, int64_t N, int64_t D,
                    float* out, irc_stream_t stream);

/* ------------------------------------------------------------------ profiling
 * HIP-event timing of the dominant kernel of each entry point, recorded on the
 * caller's stream (bench.py's roofline "achieved" figure).  Names: "scan_filter". */
int irc_prof_enable(int on);
int irc_prof_query(const char* name, double* total_ms, int64_t* count);
int irc_prof_reset(void);

#ifdef __cplusplus
}
#endif

#endif /* IRC_H_ */
