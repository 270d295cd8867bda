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
 * produced, never an approximation (sample threshold + exact radix select).  A
 * shard larger than one pass of the GEMM filter's plan (Q >= 192: over 1M docs, or
 * a survivor workspace over IRC_SCAN_PP_MAX_GB) is scanned in equal doc chunks
 * whose top-k lists are merged in the same launch sequence; same result.
 */
int64_t irc_scan_topk_workspace(int64_t Q, int64_t N, int64_t D, int64_t k);
int irc_scan_topk(const void* queries, const void* docs, int64_t Q, int64_t N, int64_t D,
                  int64_t k, int64_t doc_offset, void* workspace, int64_t workspace_bytes,
                  float* out_score, int64_t* out_idx, irc_stream_t stream);

/* `batches` bf16 query batches of one shape [Q][D] (queries[b]) against one shard, with
 * `depth` (<= 16) of them in flight: batch b runs as irc_scan_topk on streams[b % depth]
 * with workspaces[b % depth] (each of workspace_bytes, irc_scan_topk_workspace) and writes
 * rows [b Q, (b + 1) Q) of out_score / out_idx ([batches Q][k]).  Every stream first waits
 * for the work queued on `origin`, and `origin` then waits for every stream, so the
 * results are ready in `origin`'s order.  The serving loop of search_many in one call (the
 * reference's predict() takes its claims batch by batch, src/evaluation.py:98-112);
 * results identical to the per-batch calls. */
int irc_scan_topk_many(const void* const* queries, int64_t batches, const void* docs, int64_t Q,
                       int64_t N, int64_t D, int64_t k, int64_t doc_offset,
                       void* const* workspaces, int64_t workspace_bytes, int64_t depth,
                       float* out_score, int64_t* out_idx, const irc_stream_t* streams,
                       irc_stream_t origin);

/* Rescan statistics of the single-pass scan (Q <= 64): out[0] = queries whose
 * exact select had to rescan a worker's docs (a truncated 4-key list could hide
 * a winner), out[1] = workers rescanned, since the last reset.  out is a HOST
 * pointer to 2 uint64; the call synchronises the device.  Test / diagnostic aid,
 * no reference counterpart. */
int irc_scan_rescan_stats(uint64_t* out, int reset);

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

/* Smallest query batch Q for which irc_scan_topk / irc_scan_topk_fp8 run the
 * single-pass GEMM filter (Q in [q, 256]: the 4 largest keys of every (256-doc tile,
 * query) kept in the filter's epilogue, then an exact select over those lists that
 * rescans any tile whose 4th key reaches the k-th; no threshold sample pass).  q > 256
 * selects the sampled-threshold pipeline for every Q.  Same top-k either way (exact);
 * env IRC_SCAN_PPL_MINQ sets the initial value (default: off, 2^30), IRC_SCAN_PPL=0
 * turns it off.  Returns the previous value.  Replaces nothing in the reference: it selects
 * between two exact implementations of evaluation.py:110-112 / tfidf_doc_ranker.py:60-75. */
int irc_scan_set_ppl_min_q(int q);

/* fp8 (e4m3fn) corpus scan: the same exact top-k as irc_scan_topk over e4m3
 * queries [Q][D] and docs [N][D] (16-byte aligned rows), products exact, fp32
 * accumulation; returned scores are the raw dot products times score_scale (a
 * power of two, e.g. 1/(s_q*s_d) for quantisation scales s_q, s_d), so the
 * ranking is that of the quantised embeddings.  The fp8 form of BASELINE
 * config C5 ("fp8 ... 5M docs"); replaces the same dense scoring
 * (src/evaluation.py:110-112, tfidf_doc_ranker.py:60-75 ranking) as
 * irc_scan_topk. */
int64_t irc_scan_topk_fp8_workspace(int64_t Q, int64_t N, int64_t D, int64_t k);
int irc_scan_topk_fp8(const void* queries, const void* docs, int64_t Q, int64_t N, int64_t D,
                      int64_t k, int64_t doc_offset, float score_scale, void* workspace,
                      int64_t workspace_bytes, float* out_score, int64_t* out_idx,
                      irc_stream_t stream);
/* raw fp32 dot products of e4m3 queries and docs (the fp8 filter's arithmetic) */
int irc_scan_scores_fp8(const void* queries, const void* docs, int64_t Q, int64_t N, int64_t D,
                        float* out, irc_stream_t stream);
/* out[i] = e4m3fn(round-to-nearest-even(x[i] * scale)), saturated to +-448;
 * in_dtype 0 = bf16, 1 = fp32.  Used to store a corpus shard and its queries
 * in fp8 (ShardedDenseIndex(dtype="fp8")). */
int irc_quantize_fp8(int in_dtype, const void* x, int64_t n, float scale, void* out,
                     irc_stream_t stream);

/* ---------------------------------------------------------------- GEMM
 * C[M,N] (=|+=) alpha * op(A) . op(B) (+bias[N]) (->GELU) (+R[M,N]), batched.
 * Replaces the cuBLAS GEMMs behind nn.Linear / torch.matmul on the path: BERT
 * QKV/out/FFN (contrastive_module.py:39 -> HF modeling_bert), the LSTM
 * projections and the head Linear (src/model.py:16-26, 39-40), and the InfoNCE
 * logits (contrastive_loss.py:61-62, 79).
 * in_dtype/out_dtype: 0 = bf16, 1 = fp32 (fp32 inputs use the exact f32 MFMA).
 * a_layout: 0 = A is [M][K], 1 = A is [K][M];  b_layout: 0 = B is [N][K]
 * (nn.Linear weight), 1 = B is [K][N].  epilogue: 0 none, 1 +bias, 2 +bias->GELU(erf),
 * 3 +bias+R, 4 +R, 5 *gelu'(R) (GELU backward, R = saved pre-activation),
 * 6 +bias->GELU with the pre-activation ALSO written to R (R is an output here;
 * the forward of the trainable encoder's FFN1, saving what epilogue 5 needs).
 * accumulate (fp32 C only, epilogues 0-4): C += result. */
int irc_gemm(int in_dtype, int out_dtype, int a_layout, int b_layout, int epilogue, int64_t M,
             int64_t N, int64_t K, float alpha, const void* A, int64_t lda, int64_t strideA,
             const void* B, int64_t ldb, int64_t strideB, const float* bias, int64_t strideBias,
             const void* R, int64_t ldr, int64_t strideR, void* C, int64_t ldc, int64_t strideC,
             int accumulate, int64_t batch, void* workspace, int64_t workspace_bytes,
             irc_stream_t stream);
/* Bytes of device workspace irc_gemm would use for a deterministic split-K of
 * this shape (0: no split).  Split-K is taken only for fp32 C without a fused
 * epilogue when the output tiles cannot fill the chip (e.g. the LSTM weight
 * gradients, K = B*L); passing a smaller/NULL workspace disables it. */
int64_t irc_gemm_workspace(int in_dtype, int out_dtype, int epilogue, int64_t M, int64_t N,
                           int64_t K, int64_t batch);
/* irc_gemm / irc_gemm_workspace with a cap on the split-K launch: at most max_blocks
 * 256 x 256-tile blocks (0 = the default, 256 = one wave on the chip).  A smaller cap
 * gives fewer, longer splits: slower alone, but a GEMM that runs beside other work
 * (the LSTM weight gradients on their side stream) takes fewer CUs from it.  Pass the
 * same max_blocks to both calls; results stay deterministic for a given cap.  The cap
 * never limits an unsplit launch.  A negative max_blocks is a grid cap instead (no
 * split-K cap): an unsplit 256 x 256-tile launch of more tiles than -max_blocks (batch 1,
 * A [M][K]) runs as a static persistent tile loop over -max_blocks workgroups,
 * bit-identical to the uncapped launch. */
int irc_gemm_ex(int in_dtype, int out_dtype, int a_layout, int b_layout, int epilogue, int64_t M,
                int64_t N, int64_t K, float alpha, const void* A, int64_t lda, int64_t strideA,
                const void* B, int64_t ldb, int64_t strideB, const float* bias, int64_t strideBias,
                const void* R, int64_t ldr, int64_t strideR, void* C, int64_t ldc, int64_t strideC,
                int accumulate, int64_t batch, void* workspace, int64_t workspace_bytes,
                int64_t max_blocks, irc_stream_t stream);
int64_t irc_gemm_workspace_ex(int in_dtype, int out_dtype, int epilogue, int64_t M, int64_t N,
                              int64_t K, int64_t batch, int64_t max_blocks);
/* Persistent tile loop of the 256x256 bf16 GEMM, for launches of more output tiles
 * than CUs (batch 1, no split-K, aligned C): mode 0 = one workgroup per tile (the
 * default); 1 = each workgroup takes tiles from a tile counter and DMAs the next
 * tile's first K-tile while this tile's epilogue runs; 2 = static waves of tiles
 * with that prestage; 3 = static waves without it.  Same arithmetic per tile, so
 * the results are bit-identical in every mode (env IRC_GEMM_PERSIST sets the
 * initial mode).  Returns the previous mode. */
int irc_gemm_set_persistent(int mode);
/* K loop of the 256 x 384 / 256 x 256 big-tile bf16 GEMM (QKV, out-proj, FFN2, the
 * LSTM input projections): 1 = a 4-slot ring of 32-deep K-tiles with three in flight,
 * 0 = two 64-deep slots (the default).  Same MFMAs in the same k order, so the
 * results are bit-identical (env IRC_BIG_RING sets the initial value).  Returns the
 * previous setting. */
int irc_gemm_set_big_ring(int on);
/* LayerNorm-fold GEMM of the BERT encoder forward (bf16; HF BertLayer's
 * attention.output / intermediate / output sublayers, contrastive_module.py:39 ->
 * modeling_bert): the encoder keeps each pre-LayerNorm activation h with per-row
 * statistics -- partial (sum, sum of squares) pairs over column tiles,
 * stats[row][nt][2] -- instead of materialising LN(h).
 *   epilogue 1 / 2 (fold): C = r (A . B^T) + (-r mu) colsum + bias (-> GELU), where A = h,
 *     B = W diag(gamma) (bf16), colsum[n] = sum_k B[n][k], bias = b + W beta, and mu, r =
 *     1 / sqrt(var + eps) come from ln_stats (ln_nt pairs per row, row length ln_h):
 *     = LN(h) . W^T + b (HF: LayerNorm then Linear).
 *   epilogue 3: C = A . B^T + bias + residual, the residual taken as LN(R) recomputed from
 *     R = h, ln_stats, ln_gamma, ln_beta (bf16-rounded, as irc_layernorm writes it) when
 *     ln_gamma != NULL, else R itself.
 * stats_out (optional): the partials of C's bf16 values, *stats_nt_out pairs per row.
 * A [M][K], B [N][K], C / R [M][N]-strided bf16; K % 64 == 0, N % 8 == 0, 16-byte rows.
 * Not bit-reproducible: each tile's row partials are summed with LDS float atomics in
 * arrival order, so stats_out (and the LayerNorm that later reads it) can differ in the
 * last bits from run to run.  The default encoder path (separate LayerNorm kernels,
 * IRC_LN_FOLD unset) does not use it and is deterministic. */
int irc_gemm_ln(int epilogue, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                const void* B, int64_t ldb, const float* bias, const void* R, int64_t ldr,
                void* C, int64_t ldc, const float* ln_stats, int ln_nt, const float* ln_gamma,
                const float* ln_beta, float ln_eps, int64_t ln_h, const float* fold_colsum,
                float* stats_out, int* stats_nt_out, irc_stream_t stream);
/* MFMA shape of the big-tile kernel's 2-slot loop: 1 = v_mfma_f32_16x16x32_bf16 (the
 * default), 0 = v_mfma_f32_32x32x16_bf16.  Same products; the fp32 accumulation order
 * within a k32 step differs, so results agree within fp32 reassociation (env
 * IRC_BIG_MF16 sets the initial value).  Returns the previous setting. */
int irc_gemm_set_big_mf16(int on);

/* ------------------------------------------------------------- BERT encoder
 * Frozen BERT forward pieces (contrastive_module.py:36-41 -> HF BertModel):
 * fused embedding gather + LayerNorm, LayerNorm (residual fused in the GEMM),
 * masked multi-head self-attention over the fused [B*L, 3H] QKV projection.
 * dtype: 0 = bf16 activations/tables, 1 = fp32.  gamma/beta fp32. */
int irc_embed_ln(int dtype, const int64_t* ids, const void* word, const void* pos,
                 const void* type0, const float* gamma, const float* beta, void* y, int64_t rows,
                 int64_t L, int64_t H, float eps, irc_stream_t stream);
int irc_layernorm(int dtype, const void* x, void* y, const float* gamma, const float* beta,
                  int64_t rows, int64_t H, float eps, irc_stream_t stream);
int irc_attention(int dtype, const void* qkv, const int64_t* mask, void* ctx, int64_t B,
                  int64_t L, int64_t H, int64_t heads, irc_stream_t stream);
/* QKV projection + self-attention in one launch (replaces irc_gemm(QKV) + irc_attention
 * for the bf16 frozen encoder at L <= 128, head dim 64, H % 128 == 0): ctx [M = B*L][H]
 * (row stride ldc) = attention(x . Wqkv^T + b) with the same arithmetic as the unfused
 * pair.  wqkv_perm / bias_perm: Wqkv [3H][H] and its bias with the rows permuted so that
 * each 384-row block n holds the Q, K, V rows of heads 2n and 2n + 1 (64 each, in that
 * order) -- the QKV activation never leaves the CU.  x [M][H] (row stride ldx), mask
 * [M / L][L] int64 (nonzero = visible) or NULL.  A 256-row tile holds 4 (L <= 64) or 2
 * sequences in fixed slots, or 256 / L packed sequences where that takes fewer waves of
 * tiles over the device's CUs. */
int irc_qkv_attention(int64_t M, int64_t H, int64_t heads, int64_t L, const void* x, int64_t ldx,
                      const void* wqkv_perm, const float* bias_perm, const int64_t* mask,
                      void* ctx, int64_t ldc, irc_stream_t stream);

/* ----------------------------------------------------- BERT encoder backward
 * Gradients of the forward above for the trainable bi-encoder (`--model BERT`,
 * the north star's encoder fwd/bwd; the reference runs the same HF BertModel
 * frozen at contrastive_module.py:36-41).
 * irc_layernorm_bwd: x = the LN input (recomputed statistics), dy [rows, H]
 *   (dy_dtype 0 bf16 / 1 fp32; with bcast_L > 0 row r reads dy[r / bcast_L] *
 *   dy_scale -- the mean-pool backward folded in), dx in dtype; dgamma/dbeta fp32
 *   (+)= deterministic column sums; partial: irc_layernorm_bwd_workspace floats.
 * irc_attention_bwd: qkv / mask / ctx as the forward, dctx [B*L, H] -> dqkv
 *   [B*L, 3H] (same fused layout as qkv).  P is recomputed (additive key bias).
 * irc_embed_bwd: dx = gradient of the embedding sum [B*L, H] -> dword[ids] +=
 *   (fp32 atomics; rows with pad_id skipped, as nn.Embedding(padding_idx)),
 *   dpos[l] += sum_b, dtype0 += sum over all rows (fixed order); workspace L*H
 *   floats; any of dword/dpos/dtype0 may be NULL. */
int64_t irc_layernorm_bwd_workspace(int64_t rows, int64_t H);
int irc_layernorm_bwd(int dtype, int dy_dtype, const void* dy, const void* x, const float* gamma,
                      void* dx, float* dgamma, float* dbeta, float* partial,
                      int64_t partial_floats, int64_t rows, int64_t H, float eps, int64_t bcast_L,
                      float dy_scale, int accumulate, irc_stream_t stream);
int irc_attention_bwd(int dtype, const void* qkv, const int64_t* mask, const void* ctx,
                      const void* dctx, void* dqkv, int64_t B, int64_t L, int64_t H,
                      int64_t heads, irc_stream_t stream);
/* y fp32 [rows, H] = word[ids] + type0 + pos[row % L]: the embedding-LN input
 * (irc_embed_ln fuses it away in the forward; the backward rebuilds it). */
int irc_embed_sum(int dtype, const int64_t* ids, const void* word, const void* pos,
                  const void* type0, float* y, int64_t rows, int64_t L, int64_t H,
                  irc_stream_t stream);
int irc_embed_bwd(int dtype, const void* dx, const int64_t* ids, float* dword, float* dpos,
                  float* dtype0, float* workspace, int64_t ws_floats, int64_t B, int64_t L,
                  int64_t H, int64_t pad_id, irc_stream_t stream);

/* --------------------------------------------------------------- BiLSTM head
 * nn.LSTM recurrences (src/model.py:16-22, 39), gate order i,f,g,o, zero state,
 * padded sequences processed as is.  xp = x W_ih^T + b_ih + b_hh comes from
 * irc_gemm.  dtype: type of W_hh / h (0 bf16, 1 fp32); state math is fp32.
 * lstm_fwd saves activated gates, c and the consumed h_{t-1} for BPTT (any of
 * gsave/csave/hprev may be NULL for the no-grad momentum encoder);
 * lstm_bwd turns dL/dh (dy) into dL/d(gate pre-activations). */
int irc_lstm_fwd(int dtype, const float* xp, const void* whh, void* hout, float* gsave,
                 float* csave, void* hprev, int64_t B, int64_t L, int64_t H, int64_t ndir,
                 irc_stream_t stream);
int irc_lstm_bwd(int dtype, const float* dy, const void* whh, const float* gsave,
                 const float* csave, float* dgates, int64_t B, int64_t L, int64_t H,
                 int64_t ndir, irc_stream_t stream);

/* MFMA recurrences (bf16 operands, fp32 gates/state) for the production head
 * width H = 256: per step gates[32 x 4H] = xp_t + h_{t-1} W_hh^T on
 * v_mfma_f32_32x32x16_bf16 with h in LDS and W_hh streamed from L2.
 * irc_lstm_pack: W_ih (fp32 [ndir*4H][In]) -> bf16 with the gate columns of each
 *   unit interleaved (packed column 4u+g <- original g*H+u) plus the matching
 *   b_ih + b_hh, and W_hh -> bf16 B-operand fragments for the forward and the
 *   backward recurrence (4H*H elements per direction each; private layout).
 *   whh_bf16 and whhT_bf16 may both be NULL (W_ih / bias pack only: the cluster
 *   recurrence packs W_hh itself with irc_lstm_coop_pack).
 * irc_lstm_fwd_mfma: xp_packed = x . wih_packed^T + bias_packed (irc_gemm, fp32),
 *   hout bf16 [B*L][ndir*H]; gsave/csave (sizes from irc_lstm_mfma_save_floats,
 *   which 0 = gates, 1 = c; a layout private to these two kernels) and hprev bf16
 *   [ndir][B*L][H] may be NULL for the no-grad key encoder.
 * irc_lstm_bwd_mfma: dy fp32 [B*L][ndir*H] -> dgates bf16 [B*L][ndir*4H], each
 *   direction's 4H columns in the ORIGINAL gate order (weight-gradient GEMM
 *   operand; dx of the layer is one GEMM against [W_ih fwd; W_ih rev]). */
int irc_lstm_mfma_supported(int64_t H);
int64_t irc_lstm_mfma_save_floats(int64_t B, int64_t L, int64_t H, int64_t ndir, int which);
int irc_lstm_pack(const float* wih, const float* bih, const float* bhh, const float* whh,
                  int64_t In, int64_t H, int64_t ndir, void* wih_packed, float* bias_packed,
                  void* whh_bf16, void* whhT_bf16, irc_stream_t stream);
int irc_lstm_fwd_mfma(const float* xp_packed, const void* whh_bf16, void* hout, float* gsave,
                      float* csave, void* hprev, int64_t B, int64_t L, int64_t H, int64_t ndir,
                      irc_stream_t stream);
int irc_lstm_bwd_mfma(const float* dy, const void* whhT_bf16, const float* gsave,
                      const float* csave, void* dgates, int64_t B, int64_t L, int64_t H,
                      int64_t ndir, irc_stream_t stream);
/* hprev bf16 [ndir][B*L][H] = h_{t-1} of each direction (0 at its first step). */
int irc_lstm_hprev(const void* hout, void* hprev, int64_t B, int64_t L, int64_t H, int64_t ndir,
                   irc_stream_t stream);

/* Multi-CU recurrences (csrc/lstm_coop.hip), H = 256: each (32-sequence group,
 * direction) is a cluster of 4 workgroups on 4 CUs, each holding a quarter of
 * W_hh resident in LDS; the hidden state (forward) / partial dh (backward) is
 * exchanged through L2 every step (write-through stores + flags, bounded spins).
 * irc_lstm_coop_sizes(which): 0 gates floats, 1 c floats, 2 forward exchange
 *   bytes, 3 backward exchange bytes, 4 sync bytes (flags + timeout word).
 * irc_lstm_coop_pack: W_hh fp32 [ndir][4H][H] -> wf, wb bf16 (4H*H per dir each).
 * irc_lstm_fwd_coop: xp_packed as irc_lstm_fwd_mfma; gsave/csave (NULL for the
 *   no-grad encoder) in a layout private to the coop pair; hprev (may be NULL)
 *   as irc_lstm_hprev's output, written by the recurrence itself.  sync is zeroed by the
 *   call; its last word is nonzero after a cluster timed out (never expected: the
 *   launch is sized from the device's CU count so both encoders' clusters are
 *   co-resident).  On a timeout the call itself overwrites its output (hout /
 *   dgates) with NaN on the device, so no caller can consume stale state.
 * irc_lstm_bwd_coop: dy fp32 [B*L][ndir*H] -> dgates bf16 [B*L][ndir*4H].
 * irc_lstm_coop_fault: *fault (uint32, device) |= the call's timeout word, on
 *   the stream without a host sync; the head keeps one sticky word per encoder
 *   and the train loop reads it at its existing sync points.
 * IRC_LSTM_COOP_SPIN_MAX (environment, read per call) bounds the spins of every
 *   cross-CU wait (debug knob; 0 = time out at the first unsatisfied wait). */
int irc_lstm_coop_supported(int64_t H);
int64_t irc_lstm_coop_sizes(int64_t B, int64_t L, int64_t H, int64_t ndir, int which);
int irc_lstm_coop_pack(const float* whh, int64_t H, int64_t ndir, void* wf, void* wb,
                       irc_stream_t stream);
int irc_lstm_fwd_coop(const float* xp_packed, const void* wf, void* hout, float* gsave,
                      float* csave, void* hprev, void* xch, void* sync, int64_t B, int64_t L,
                      int64_t H, int64_t ndir, irc_stream_t stream);
int irc_lstm_bwd_coop(const float* dy, const void* wb, const float* gsave, const float* csave,
                      void* dgates, void* xch, void* sync, int64_t B, int64_t L, int64_t H,
                      int64_t ndir, irc_stream_t stream);
int irc_lstm_coop_fault(const void* sync, int64_t B, int64_t ndir, void* fault,
                        irc_stream_t stream);

/* ------------------------------------------------- seq2vec tail + InfoNCE + optimizer
 * seq2vec mean-over-L (PAD included) + F.normalize (contrastive_module.py:102-112);
 * InfoNCE row log-sum-exp / NLL and softmax gradients (contrastive_loss.py:56-93,
 * the k-rows reuse q's queue logits); deterministic sums; clip_grad_norm_ +
 * Adam (train.py:155-165, model.py:52-57); momentum update and enqueue
 * (contrastive_module.py:43-68); casts and column sums for bias gradients. */
int irc_mean_rows(int dtype, const void* x, float* out, int64_t B, int64_t L, int64_t C,
                  int64_t ldx, irc_stream_t stream);
int irc_bcast_rows(const float* g, float* y, int64_t B, int64_t L, int64_t C, float scale,
                   irc_stream_t stream);
int irc_l2norm_fwd(const float* x, float* y, float* nrm, int64_t B, int64_t D, float eps,
                   irc_stream_t stream);
int irc_l2norm_bwd(const float* dy, const float* y, const float* nrm, float* dx, int64_t B,
                   int64_t D, float eps, irc_stream_t stream);
int irc_nce_lse(const float* S, const float* LQ, int64_t N, int64_t K, float T, float* lse,
                float* loss_row, irc_stream_t stream);
int irc_nce_grads(const float* S, const float* LQ, const float* lse, int64_t N, int64_t K,
                  float T, const float* gscale, float* GS, float* GQ, irc_stream_t stream);
/* Fused InfoNCE for D in {32, 64, ..., 256} (the LSTM head's embedding width):
 * NCELoss._compute_info_loss (src/contrastor/contrastive_loss.py:56-93) without
 * materialising S = F F^T [2N, 2N] or q . queue [N, K] in HBM.  F = [q; k] fp32
 * [2N][D], queue fp32 [D][K] (K = 0: no queue).  Exact-fp32 MFMA logits, online
 * row max / sum exp, fixed-order partial reductions (deterministic).
 * The rows computed are those of the pairs [p_lo, p_hi): q rows p_lo .. p_hi-1 and
 * k rows N + p_lo .. N + p_hi-1 -- all 2N rows for [0, N) (any N); a sub-range (a
 * data-parallel rank's local pairs) needs N, p_lo, p_hi multiples of 32.
 * irc_nce_fused_fwd: lse[r], loss_row[r] = lse_r - logit_{r, pos(r)} for the rows
 *   computed (lse / loss_row indexed by absolute row, [2N]).
 * irc_nce_fused_bwd: dF [2P][D] (P = p_hi - p_lo; q rows then k rows) = d(loss) /
 *   d(F rows) with loss = sum over ALL 2N rows of loss_row / 2, times *gscale;
 *   needs every row's lse (a sub-range caller all-gathers them first).
 * workspace: irc_nce_fused_workspace bytes (the same for both calls). */
int64_t irc_nce_fused_workspace(int64_t N, int64_t D, int64_t K, int64_t p_lo, int64_t p_hi);
int irc_nce_fused_fwd(const float* F, const float* queue, int64_t N, int64_t D, int64_t K,
                      float T, int64_t p_lo, int64_t p_hi, void* ws, int64_t ws_bytes, float* lse,
                      float* loss_row, irc_stream_t stream);
int irc_nce_fused_bwd(const float* F, const float* queue, const float* lse, int64_t N, int64_t D,
                      int64_t K, float T, const float* gscale, int64_t p_lo, int64_t p_hi,
                      void* ws, int64_t ws_bytes, float* dF, irc_stream_t stream);
int irc_sum(const float* x, int64_t n, float scale, float* partial, float* out,
            irc_stream_t stream);
int irc_grad_norm_clip(const float* g, int64_t n, float max_norm, float* partial, float* out /* >= 3 */,
                       irc_stream_t stream);
int irc_adam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* coef,
                  float b1, float b2, float step_size, float bc2_sqrt, float eps,
                  irc_stream_t stream);
int irc_momentum_update(float* pk, const float* pq, int64_t n, float mom, irc_stream_t stream);
/* Same updates that also refresh a bf16 shadow of the parameters (the trainable
 * encoder's MFMA operand copy) in the same pass. */
int irc_adam_step_bf16(float* p, const float* g, float* m, float* v, int64_t n, const float* coef,
                       float b1, float b2, float step_size, float bc2_sqrt, float eps,
                       void* p_bf16, irc_stream_t stream);
int irc_momentum_update_bf16(float* pk, const float* pq, int64_t n, float mom, void* pk_bf16,
                             irc_stream_t stream);
/* SGD step (the reference's --opt sgd: torch.optim.SGD(lr, momentum, weight_decay),
 * src/model.py:45-51), clip coefficient / gate read from coef (NULL: none) as in
 * irc_adam_step: d = g * coef[1] + weight_decay * p; buf = first_step ? d :
 * momentum * buf + d; p -= lr * buf.  p_bf16 (NULL: none): bf16 shadow of p. */
int irc_sgd_step(float* p, const float* g, float* buf, int64_t n, const float* coef, float lr,
                 float momentum, float weight_decay, int first_step, void* p_bf16,
                 irc_stream_t stream);
/* The head's output activation (src/model.py:23-26, eval(f"nn.{act}()") with torch's
 * default arguments): y = act(u) elementwise; the backward scales g by act'(u) in
 * place.  fp32. */
enum {
  IRC_ACT_IDENTITY = 0, IRC_ACT_RELU, IRC_ACT_RELU6, IRC_ACT_LEAKY_RELU, IRC_ACT_ELU,
  IRC_ACT_CELU, IRC_ACT_SELU, IRC_ACT_GELU, IRC_ACT_SILU, IRC_ACT_MISH, IRC_ACT_SIGMOID,
  IRC_ACT_TANH, IRC_ACT_SOFTPLUS, IRC_ACT_SOFTSIGN, IRC_ACT_HARDTANH, IRC_ACT_HARDSIGMOID,
  IRC_ACT_HARDSWISH, IRC_ACT_TANHSHRINK, IRC_ACT_COUNT
};
int irc_activation(int kind, const float* u, float* y, int64_t n, irc_stream_t stream);
int irc_activation_bwd(int kind, const float* u, float* g, int64_t n, irc_stream_t stream);
/* Fault gate of a training step (no host sync; replaces nothing in the reference,
 * whose cuDNN LSTM cannot time out): coef[2] = 1 when *fault_a or *fault_b (uint32
 * sticky timeout words of irc_lstm_coop_fault; either may be NULL) is set, else 0.
 * coef is irc_grad_norm_clip's output (>= 3 floats; it sets coef[2] = 0).  The
 * Adam steps skip every element while coef[2] != 0, and so does
 * irc_momentum_update_gated (train.py:150-169's update, momentum:
 * contrastive_module.py:43-53), so a step whose recurrence timed out (its
 * outputs NaN-poisoned) leaves the parameters, moments and key encoder as they
 * were.  pk_bf16 may be NULL. */
int irc_fault_gate(const void* fault_a, const void* fault_b, float* coef, irc_stream_t stream);
int irc_momentum_update_gated(float* pk, const float* pq, int64_t n, float mom, const float* gate,
                              void* pk_bf16, irc_stream_t stream);
int irc_enqueue(float* queue, const float* keys, int64_t* ptr, int64_t D, int64_t K, int64_t B,
                irc_stream_t stream);
int irc_cast_bf16(const float* x, void* y, int64_t n, irc_stream_t stream);
/* y bf16 [C][R] = transpose of x fp32 [R][C] (weights as the NK GEMM operand). */
int irc_cast_bf16_t(const float* x, void* y, int64_t R, int64_t C, irc_stream_t stream);
/* irc_cast_bf16_t over `batch` matrices: x + b * sx (floats) -> y + b * sy (bf16 elements). */
int irc_cast_bf16_t_batched(const float* x, void* y, int64_t R, int64_t C, int64_t batch,
                            int64_t sx, int64_t sy, irc_stream_t stream);
int irc_axpby(float* out, const float* x, const float* y, float a, float b, int64_t n,
              irc_stream_t stream);
/* column sums of x [R][C] (dtype 0 bf16, 1 fp32) into fp32 out; partial holds
 * ceil(R/64)*C floats of scratch (deterministic two-pass order). */
int irc_colsum(int dtype, const void* x, float* out, int64_t R, int64_t C, int64_t ldx,
               int accumulate, float* partial, irc_stream_t stream);

/* Batched column sums: out[b * so + c] (+)= sum_r x[b * sx + r * ldx + c] for b < batch
 * (dtype 0 bf16 / 1 fp32 rows, 16-byte aligned) -- the per-layer bias gradients of
 * the trainable encoder's layer-batched weight-gradient pass; deterministic
 * (fixed-order two-pass).  partial: irc_colsum_batched_workspace floats. */
int64_t irc_colsum_batched_workspace(int64_t batch, int64_t R, int64_t C);
int irc_colsum_batched(int dtype, const void* x, int64_t batch, int64_t R, int64_t C, int64_t ldx,
                       int64_t sx, float* out, int64_t so, int accumulate, float* partial,
                       int64_t partial_floats, irc_stream_t stream);

/* ------------------------------------------------- fp8 encoder weights (csrc/fp8_linear.hip)
 * BASELINE config C5 ("fp8 (CDNA4 MFMA) encoder weights"): the frozen BERT's
 * nn.Linear layers (contrastive_module.py:36-41 -> HF modeling_bert) on e4m3.
 * irc_quantize_rows_fp8: x bf16 (in_dtype 0) / fp32 (1) [M][ldx] -> out e4m3
 *   [M][ldo], scale[m] = amax|x[m]| / 448 (1 for a zero row), out = e4m3(RNE(x /
 *   scale)) saturated; used per output channel for weights, per token for inputs.
 * irc_gemm_fp8: C bf16 [M][ldc] = (A8 [M][lda] . B8 [N][ldb]^T) * sa[m] * sb[n]
 *   (+ bias) (epi 1) / -> GELU (2) / + residual R bf16 [M][ldr] (3); K % 128 == 0. */
int irc_quantize_rows_fp8(int in_dtype, const void* x, int64_t ldx, int64_t M, int64_t K,
                          void* out, int64_t ldo, float* scale, irc_stream_t stream);
int irc_gemm_fp8(const void* A8, int64_t lda, const float* sa, const void* B8, int64_t ldb,
                 const float* sb, int64_t M, int64_t N, int64_t K, const float* bias,
                 const void* R, int64_t ldr, void* C, int64_t ldc, int epi, irc_stream_t stream);

/* MX-fp8: the CDNA4-native form of the same layers.  An MX-fp8 matrix [rows][K]
 * is e4m3 codes [rows][ld] plus one E8M0 scale (2^(byte - 127)) per 32 consecutive
 * values of a row, the smallest power of two for which the block's max / scale
 * <= 448 (no saturation; 2^0 for an all-zero block).  The scales live in the "MX
 * layout": K/128 records of mpad * 4 bytes (mpad = rows rounded up to 256), each
 * 256-row block's 1 KB ordered [row bit 7][k-block][row bits 0-3][row bits 4-6]
 * (csrc/mx.h mx_scale_index), which the GEMM DMAs into LDS with its K-tiles.
 * irc_quantize_mx_fp8: x bf16 (0) / fp32 (1) [M][ldx] -> out [M][ldo], scales.
 * irc_gemm_mx: C = A . B^T with both operands' block scales applied inside
 *   v_mfma_scale_f32_16x16x128_f8f6f4 (+ bias / GELU / residual as irc_gemm_fp8);
 *   C bf16 [M][ldc], or, when cx != NULL, MX-fp8 (C = e4m3 bytes, ldc in bytes, cx
 *   its scales with mpad rows: the FFN1 + GELU output feeding FFN2).  K % 128, N % 32.
 * irc_layernorm_mx: irc_layernorm (bf16, H 512 / 768 / 1024) that also writes the
 *   MX-fp8 copy y8 / ys of its bf16 output (the next projection's A operand).
 * irc_attention_mx: irc_attention's MFMA path (head dim 64, L % 32 == 0, L <= 128)
 *   with the context written as MX-fp8 only (ctx8 / cs) for the out-projection.
 * Producers quantise their bf16-rounded outputs, so each MX operand equals
 * irc_quantize_mx_fp8 of the bf16 tensor the bf16 path would have produced. */
int irc_quantize_mx_fp8(int in_dtype, const void* x, int64_t ldx, int64_t M, int64_t K, void* out,
                        int64_t ldo, void* scales, int64_t mpad, irc_stream_t stream);
int irc_gemm_mx(const void* A8, int64_t lda, const void* sa, int64_t mpad, const void* B8,
                int64_t ldb, const void* sb, int64_t npad, int64_t M, int64_t N, int64_t K,
                const float* bias, const void* R, int64_t ldr, void* C, int64_t ldc, void* cx,
                int epi, irc_stream_t stream);
int irc_layernorm_mx(const void* x, void* y, const float* gamma, const float* beta, int64_t rows,
                     int64_t H, float eps, void* y8, void* ys, int64_t mpad, irc_stream_t stream);
int irc_attention_mx(const void* qkv, const int64_t* mask, void* ctx8, void* cs, int64_t mpad,
                     int64_t B, int64_t L, int64_t H, int64_t heads, irc_stream_t stream);

/* ------------------------------------------------- device corpus (csrc/corpus.hip)
 * The training corpus tokenised once and resident in HBM, so a micro-batch is
 * the sampler's sentence indices only (replaces the DataLoader string batches of
 * src/dataset.py:89-101, 159-182 and the per-batch tokenizer call of
 * src/contrastor/contrastive_module.py:36-41).
 * irc_corpus_pack: rows of irc_wordpiece's tok [n][max_tokens] (tok_len valid
 *   ids each) -> flat int32 at offsets[i] (int64 [n+1], the exclusive scan of
 *   tok_len).
 * irc_pair_batch: ids / mask int64 [rows][L] = [CLS] flat[offsets[sel[r]] ..]
 *   (truncated to L - 2) [SEP] [PAD]..., mask 1 on [CLS] .. [SEP]: the output of
 *   bert_tokenizer(sentences, padding=True, truncation=True) for the selected
 *   sentences when L = min(max length, 510) + 2. */
int irc_corpus_pack(const int* tok, const int* tok_len, int64_t n, int64_t max_tokens,
                    const int64_t* offsets, int* flat, irc_stream_t stream);
int irc_pair_batch(const int* flat, const int64_t* offsets, const int64_t* sel, int64_t rows,
                   int64_t L, int64_t cls_id, int64_t sep_id, int64_t pad_id, int64_t* ids,
                   int64_t* mask, irc_stream_t stream);
/* Host function (no device work): the uniform pair draw of DocDataset.__getitem__
 * (src/dataset.py:89-101: np.random.choice(len(doc), 2, replace=False) on numpy's
 * global legacy RandomState) for n documents at once.  mt_key[624] / *mt_pos are
 * numpy's MT19937 state (np.random.get_state()), advanced in place exactly as the
 * n calls would; first / second [n] = doc_start[docs[t]] + the two drawn sentences. */
int irc_pair_sample(uint32_t* mt_key, int* mt_pos, const int64_t* doc_start,
                    const int64_t* docs, int64_t n, int64_t* first, int64_t* second);

/* ------------------------------------------------- input pipeline (csrc/wordpiece.hip)
 * BERT WordPiece tokenisation + joint padding on the device: replaces the
 * reference's per-micro-batch host call bert_tokenizer(d1 + d2, padding=True,
 * truncation=True) (src/contrastor/contrastive_module.py:36-41, 96-100).
 * irc_wordpiece: n sentences as UTF-8 bytes (offsets int64 [n+1]); cmap uint32
 *   [0x110000] (normaliser output per code point: kind 0 drop, 1 single cp << 8,
 *   2 (pool offset << 8 | len << 2)), cpool uint32, cls uint8 [0x110000]
 *   (1 whitespace, 2 punctuation); vocab as an open-addressing FNV-1a table
 *   (htab_id int32 / htab_hash uint32, power-of-two size) with the pieces' code
 *   points (vocab_off int32 [V+1], vocab_cps uint32, vocab_cont uint8 [V]) ->
 *   tok int32 [n][max_tokens], tok_len int32 [n], *max_len = max row length + 2.
 * irc_wordpiece_pad: ids / mask int64 [n][L] = [CLS] tokens [SEP] [PAD]... */
int irc_wordpiece(const void* bytes, const int64_t* offsets, int64_t n, const void* cmap,
                  const void* cpool, const void* cls, const int* htab_id, const void* htab_hash,
                  int64_t htab_size, const int* vocab_off, const void* vocab_cps,
                  const void* vocab_cont, int64_t max_piece, int64_t unk_id, int64_t max_tokens,
                  int* tok, int* tok_len, int* max_len, irc_stream_t stream);
int irc_wordpiece_pad(const int* tok, const int* tok_len, int64_t n, int64_t max_tokens,
                      int64_t L, int64_t cls_id, int64_t sep_id, int64_t pad_id, int64_t* ids,
                      int64_t* mask, irc_stream_t stream);

/* ------------------------------------------------------------------ profiling
 * HIP-event timing of the dominant kernel of each entry point, recorded on the
 * caller's stream (bench.py's roofline "achieved" figure), with the launches'
 * algorithmic work (flops or bytes).  Names: "scan_filter" (bytes), "gemm_bf16",
 * "gemm_f32" (flops). */
int irc_prof_enable(int on);
int irc_prof_query(const char* name, double* total_ms, int64_t* count, double* work);
int irc_prof_reset(void);

/* ---- Sparse hashed n-gram TF-IDF retrieval ----------
 * The reference's real predict path.  A CSR matrix [hash_size rows][n_cols docs]
 * (indptr int64 [rows+1], indices int32, data fp64), resident on the device;
 * queries are lists of (row, weight) in ascending row order, flattened with
 * offsets q_off [Q+1] (n_pairs = q_off[Q]).
 *
 * documents_filtering (src/evaluation.py:57-81): the sorted unique docs with a
 * nonzero in any of a query's rows.  irc_csr_union_count marks one bitmap per
 * query (bitmaps: Q * ceil(n_cols/32) words) and writes per-chunk counts
 * (chunk_sums: Q * irc_csr_union_chunks(n_cols)); the caller sums a query's
 * chunks into out_off [Q+1] and irc_csr_union_emit writes the indices. */
int64_t irc_csr_union_chunks(int64_t n_cols);
int irc_csr_union_count(const int64_t* indptr, const int32_t* indices, int64_t n_cols,
                        const int64_t* q_off, const int64_t* q_rows, int64_t Q, int64_t n_pairs,
                        uint32_t* bitmaps, int64_t* chunk_sums, irc_stream_t stream);
int irc_csr_union_emit(const uint32_t* bitmaps, int64_t n_cols, int64_t Q,
                       const int64_t* chunk_sums, const int64_t* out_off, int32_t* out_idx,
                       irc_stream_t stream);
/* TfidfDocRanker.closest_docs' spvec * doc_mat
 * (preprocessing/drqa/retriever/tfidf_doc_ranker.py:64-65): dense [Q][n_cols]
 * (zeroed by the caller) += w * row, rows in the given order (CSR indices sorted
 * within each row), fp64 multiply and
 * add rounded separately -- scipy's accumulation order, bit-identical scores. */
int irc_csr_spmv_f64(const int64_t* indptr, const int32_t* indices, const double* data,
                     int64_t n_cols, const int64_t* q_off, const int64_t* q_rows,
                     const double* q_w, int64_t Q, double* dense, irc_stream_t stream);
/* Top-k of the nonzero dense[q][cand] over each query's candidate docs (cand,
 * ascending, offsets cand_off [Q+1]): (score desc, doc index asc), k <= 1024;
 * out_n[q] = number of valid entries, the rest (0, -1)
 * (tfidf_doc_ranker.py:67-73). cand == NULL (cand_off unused): every doc of the
 * row is a candidate -- the same result over a dense buffer that is zero outside
 * the union (what irc_csr_spmv_f64 leaves in a zeroed buffer), read contiguously. */
int irc_topk_f64(const double* dense, int64_t n_cols, const int32_t* cand,
                 const int64_t* cand_off, int64_t Q, int64_t k, double* out_score,
                 int64_t* out_idx, int32_t* out_n, irc_stream_t stream);

/* ---- ProtoNCE / HProtoNCE ----------------------------
 * NCELoss._compute_proto_loss (src/contrastor/contrastive_loss.py:95-135):
 * logits [B][C] (C >= B prototypes, row i's positive is column i), column
 * temperatures temp [C]; row_loss[i] = CE(logits[i] / temp, i) (optional) and
 * dlogits = gscale * (softmax - onehot) / temp (optional; gscale a device
 * scalar or NULL = 1). */
int irc_proto_ce(const float* logits, const float* temp, int64_t B, int64_t C, float* row_loss,
                 float* dlogits, const float* gscale, irc_stream_t stream);
/* run_kmeans (src/contrastor/utils.py:50-110; faiss Clustering in the reference):
 * idx[r] = argmax_j S[r][j] + bias[j] (lowest j on ties), val[r] the maximum --
 * nearest centroid with S = x . c^T and bias = -|c|^2 / 2. */
int irc_argmax_bias(const float* S, const float* bias, int64_t rows, int64_t k, int64_t* idx,
                    float* val, irc_stream_t stream);
/* sums[assign[r]] += x[r], counts[assign[r]] += 1 (fp32 atomics) */
int irc_centroid_accumulate(const float* x, const int64_t* assign, int64_t n, int64_t D,
                            float* sums, float* counts, irc_stream_t stream);
/* centroids = sums / counts where counts > 0 (else unchanged); bias = -|c|^2 / 2 */
int irc_centroid_finalize(const float* sums, const float* counts, int64_t k, int64_t D,
                          float* centroids, float* bias, irc_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* IRC_H_ */
