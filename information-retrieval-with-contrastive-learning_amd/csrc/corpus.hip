// Device-resident tokenised sentence corpus and the training pair batch built
// from it.  Replaces, per micro-batch, the reference's
// DataLoader workers pickling sentence strings to the main process
// (src/dataset.py:89-101, 159-182) and the host tokenizer call on them
// (src/contrastor/contrastive_module.py:36-41): the corpus is WordPiece-tokenised
// ONCE (irc_wordpiece) and packed here into CSR form (ids int32, offsets int64);
// a micro-batch is then just the sentence indices the sampler drew, gathered and
// jointly padded on the device ([CLS] ids [SEP] [PAD]..., as the tokenizer with
// padding=True, truncation=True emits them).
#include "irc_common.h"

namespace irc {
namespace corpus {

// Row i of tok [n][max_tokens] (tok_len[i] valid ids) -> flat[off[i] .. off[i] + len).
__global__ __launch_bounds__(256) void pack_kernel(const int* __restrict__ tok,
                                                   const int* __restrict__ tlen, int64_t n,
                                                   int max_tokens, const int64_t* __restrict__ off,
                                                   int* __restrict__ flat) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  const int len = tlen[i];
  const int* src = tok + i * max_tokens;
  int* dst = flat + off[i];
  for (int t = threadIdx.x; t < len; t += blockDim.x) dst[t] = src[t];
}

// One 64-lane wave per output row r: sentence sel[r] -> ids[r] = [CLS] tokens
// (truncated to L - 2) [SEP] [PAD]..., mask 1 on the real tokens.
__global__ __launch_bounds__(256) void pair_batch_kernel(const int* __restrict__ flat,
                                                         const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ sel, int64_t rows,
                                                         int L, int cls_id, int sep_id, int pad_id,
                                                         int64_t* __restrict__ ids,
                                                         int64_t* __restrict__ mask) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int64_t s = sel[r];
  const int64_t o = off[s];
  int len = (int)(off[s + 1] - o);
  if (len > L - 2) len = L - 2;
  int64_t* ir = ids + r * L;
  int64_t* mr = mask + r * L;
  for (int t = lane; t < L; t += 64) {
    int v;
    if (t == 0) v = cls_id;
    else if (t <= len) v = flat[o + t - 1];
    else if (t == len + 1) v = sep_id;
    else v = pad_id;
    ir[t] = v;
    mr[t] = t <= len + 1 ? 1 : 0;
  }
}

}  // namespace corpus
}  // namespace irc

using namespace irc;

extern "C" int irc_corpus_pack(const int* tok, const int* tok_len, int64_t n, int64_t max_tokens,
                               const int64_t* offsets, int* flat, irc_stream_t stream) {
  IRC_REQUIRE(n >= 0 && max_tokens >= 1, "corpus_pack: bad sizes");
  if (n == 0) return IRC_OK;
  hipLaunchKernelGGL(corpus::pack_kernel, dim3((unsigned)n), dim3(256), 0, as_stream(stream), tok,
                     tok_len, n, (int)max_tokens, offsets, flat);
  return check_launch("corpus_pack");
}

extern "C" int irc_pair_batch(const int* flat, const int64_t* offsets, const int64_t* sel,
                              int64_t rows, int64_t L, int64_t cls_id, int64_t sep_id,
                              int64_t pad_id, int64_t* ids, int64_t* mask, irc_stream_t stream) {
  IRC_REQUIRE(L >= 2 && L <= 512, "pair_batch: L=%lld", (long long)L);
  if (rows == 0) return IRC_OK;
  hipLaunchKernelGGL(corpus::pair_batch_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     as_stream(stream), flat, offsets, sel, rows, (int)L, (int)cls_id, (int)sep_id,
                     (int)pad_id, ids, mask);
  return check_launch("pair_batch");
}
