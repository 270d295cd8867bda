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

#include <utility>
#include <vector>

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

// ---------------------------------------------------------------- host: pair sampler
// DocDataset.__getitem__'s uniform draw (src/dataset.py:89-101):
// np.random.choice(len(doc), 2, replace=False) on numpy's global legacy RandomState,
// i.e. permutation(n)[:2] = a Fisher-Yates shuffle of arange(n) from i = n-1 down to 1
// with j = random_interval(i) (MT19937 32-bit draws masked to the smallest 2^k - 1 >=
// i, rejected above i).  Restated here in C so the sampler costs ~0.1 us per pair
// instead of ~20 us of Python per np.random.choice call; the MT19937 state (key[624],
// pos) is read from and written back to numpy's, so the stream continues exactly.
namespace {
struct MT {
  uint32_t* key;
  int pos;
  void gen() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
      key[i] = key[i + 397] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; i < 623; ++i) {
      const uint32_t y = (key[i] & 0x80000000u) | (key[i + 1] & 0x7fffffffu);
      key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    const uint32_t y = (key[623] & 0x80000000u) | (key[0] & 0x7fffffffu);
    key[623] = key[396] ^ (y >> 1) ^ mag01[y & 1u];
    pos = 0;
  }
  uint32_t next32() {
    if (pos >= 624) gen();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  uint32_t interval(uint32_t max) {  // numpy random_interval, max < 2^32
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > max) {
    }
    return v;
  }
};
}  // namespace

extern "C" int irc_pair_sample(uint32_t* mt_key, int* mt_pos, const int64_t* doc_start,
                               const int64_t* docs, int64_t n, int64_t* first,
                               int64_t* second) {
  IRC_REQUIRE(mt_key != nullptr && mt_pos != nullptr && *mt_pos >= 0 && *mt_pos <= 624,
              "pair_sample: bad MT19937 state");
  MT mt{mt_key, *mt_pos};
  std::vector<int64_t> perm;
  for (int64_t t = 0; t < n; ++t) {
    const int64_t d = docs[t];
    const int64_t len = doc_start[d + 1] - doc_start[d];
    IRC_REQUIRE(len >= 2, "pair_sample: document %lld has %lld sentences", (long long)d,
                (long long)len);
    perm.resize((size_t)len);
    for (int64_t i = 0; i < len; ++i) perm[i] = i;
    for (int64_t i = len - 1; i >= 1; --i) {  // one draw per i >= 1, as the shuffle
      const int64_t j = mt.interval((uint32_t)i);
      std::swap(perm[i], perm[j]);
    }
    first[t] = doc_start[d] + perm[0];
    second[t] = doc_start[d] + perm[1];
  }
  *mt_pos = mt.pos;
  return IRC_OK;
}
