// BERT WordPiece tokenisation + joint padding on the GPU.
//
// Reference: the reference tokenises every micro-batch on the host,
// bert_tokenizer(d1 + d2, padding=True, truncation=True) (src/contrastor/
// contrastive_module.py:36-41, 96-100) with BertTokenizer('bert-base-uncased'),
// whose pipeline in this environment is the `tokenizers` one: BertNormalizer
// (clean text, CJK spacing, NFD accent strip, lowercase -- all per character),
// BertPreTokenizer (split on whitespace, isolate punctuation), WordPiece
// (greedy longest match, "##" continuations, a word of more than 100 characters
// or with an unmatchable remainder -> [UNK]), [CLS] ... [SEP], truncation to
// max_length, padding to the longest row of the batch.
//
// Here one thread tokenises one sentence straight from its UTF-8 bytes:
//   decode -> cmap (the normaliser's per-character output, built on the host
//   from the tokenizer itself) -> cls (whitespace / punctuation of the
//   pre-tokeniser) -> word buffer in LDS -> greedy longest match with prefix
//   FNV-1a hashes probed in an open-addressing vocab table (exact compare
//   against the vocab's code points) -> token ids.
// A second launch writes the padded [n, L] ids / attention mask once the host
// has read L = max row length (a 4-byte read on the tokeniser's own stream).
// The work is tiny next to a training step (a few thousand waves of integer
// work per batch), so the kernels favour simplicity over occupancy.
#include "irc_common.h"

namespace irc {
namespace wp {

constexpr int NT = 32;            // threads (sentences) per workgroup (13 KB LDS: fits beside a GEMM workgroup)
constexpr int MAXW = 100;         // max_input_chars_per_word
constexpr int MAXP = 64;          // longest vocab piece handled (host-checked)
constexpr unsigned FNV_P = 16777619u;
constexpr unsigned SEED_WORD = 2166136261u;
constexpr unsigned SEED_CONT = 0x9E3779B9u;

struct Tables {
  const unsigned* cmap;   // [0x110000]: kind 0 drop, 1 single (cp << 8), 2 multi (off << 8 | len << 2)
  const unsigned* cpool;  // multi-cp outputs
  const unsigned char* cls;  // [0x110000]: 1 whitespace, 2 punctuation
  const int* htab_id;     // [mask + 1], -1 empty
  const unsigned* htab_hash;
  unsigned hmask;
  const int* voff;        // [V + 1] offsets into vcps
  const unsigned* vcps;   // vocab pieces' code points (without "##")
  const unsigned char* vcont;  // [V] 1: "##" continuation piece
  int max_piece;
  int unk;
};

__device__ __forceinline__ unsigned fnv(unsigned h, unsigned cp) { return (h ^ cp) * FNV_P; }

__device__ __forceinline__ int lookup(const Tables& T, unsigned h, const unsigned* w, int a, int b,
                                      int cont) {
  unsigned idx = h & T.hmask;
  for (;;) {
    const int id = T.htab_id[idx];
    if (id < 0) return -1;
    if (T.htab_hash[idx] == h && (int)T.vcont[id] == cont && T.voff[id + 1] - T.voff[id] == b - a) {
      const unsigned* p = T.vcps + T.voff[id];
      bool eq = true;
      for (int i = 0; i < b - a && eq; ++i) eq = p[i] == w[a + i];
      if (eq) return id;
    }
    idx = (idx + 1) & T.hmask;
  }
}

struct Out {
  int* row;
  int n, cap;
  __device__ __forceinline__ bool full() const { return n >= cap; }
  __device__ __forceinline__ void put(int id) {
    if (n < cap) row[n] = id;
    ++n;
  }
};

// WordPiece of one word w[0..len) (len <= MAXW): greedy longest match.
__device__ void word_pieces(const Tables& T, const unsigned* w, int len, Out& o) {
  // first pass: does the whole word split? (ids are emitted only if it does)
  int ids[MAXW];
  int nid = 0;
  for (int start = 0; start < len;) {
    const int cont = start > 0;
    int lim = len - start < T.max_piece ? len - start : T.max_piece;
    unsigned ph[MAXP + 1];
    ph[0] = cont ? SEED_CONT : SEED_WORD;
    for (int i = 0; i < lim; ++i) ph[i + 1] = fnv(ph[i], w[start + i]);
    int got = -1, end = start;
    for (int l = lim; l >= 1; --l) {
      const int id = lookup(T, ph[l], w, start, start + l, cont);
      if (id >= 0) {
        got = id;
        end = start + l;
        break;
      }
    }
    if (got < 0) {
      o.put(T.unk);
      return;
    }
    ids[nid++] = got;
    start = end;
  }
  for (int i = 0; i < nid; ++i) o.put(ids[i]);
}

__device__ __forceinline__ unsigned decode_utf8(const unsigned char* s, int64_t& i, int64_t end) {
  const unsigned c0 = s[i];
  if (c0 < 0x80) { i += 1; return c0; }
  int n = c0 >= 0xF0 ? 3 : c0 >= 0xE0 ? 2 : 1;
  unsigned cp = c0 & (0x3F >> n);
  for (int k = 1; k <= n && i + k < end; ++k) cp = (cp << 6) | (s[i + k] & 0x3F);
  i += n + 1;
  return cp < 0x110000 ? cp : 0xFFFD;
}

__global__ __launch_bounds__(NT) void wordpiece_kernel(const unsigned char* __restrict__ bytes,
                                                       const int64_t* __restrict__ offs, int n,
                                                       Tables T, int cap, int* __restrict__ tok,
                                                       int* __restrict__ tok_len, int* max_len) {
  __shared__ unsigned wbuf[NT][MAXW + 1];
  const int s = blockIdx.x * NT + threadIdx.x;
  if (s >= n) return;
  unsigned* w = wbuf[threadIdx.x];
  Out o{tok + (int64_t)s * cap, 0, cap};
  int wl = 0;  // current word length (may exceed MAXW: then the word is [UNK])
  auto flush = [&]() {
    if (wl > MAXW) o.put(T.unk);
    else if (wl > 0) word_pieces(T, w, wl, o);
    wl = 0;
  };
  auto feed = [&](unsigned cp) {
    const unsigned char c = T.cls[cp];
    if (c == 1) {
      flush();
    } else if (c == 2) {
      flush();
      w[0] = cp;
      wl = 1;
      flush();
    } else {
      if (wl < MAXW + 1) w[wl] = cp;
      ++wl;
    }
  };
  const int64_t end = offs[s + 1];
  for (int64_t i = offs[s]; i < end && !o.full();) {
    const unsigned cp = decode_utf8(bytes, i, end);
    const unsigned m = T.cmap[cp];
    const unsigned kind = m & 3u;
    if (kind == 1) {
      feed(m >> 8);
    } else if (kind == 2) {
      const unsigned off = m >> 8, len = (m >> 2) & 15u;
      for (unsigned k = 0; k < len; ++k) feed(T.cpool[off + k]);
    }
  }
  if (!o.full()) flush();
  const int len = o.n < cap ? o.n : cap;
  tok_len[s] = len;
  atomicMax(max_len, len + 2);
}

// ids / mask [n][L]: [CLS] tokens [SEP] [PAD]...  (int64, as the tokenizer's tensors)
__global__ void pad_kernel(const int* __restrict__ tok, const int* __restrict__ tok_len, int n,
                           int cap, int L, int cls_id, int sep_id, int pad_id,
                           int64_t* __restrict__ ids, int64_t* __restrict__ mask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * L) return;
  const int s = (int)(e / L), j = (int)(e % L);
  const int len = tok_len[s];
  int64_t id = pad_id, m = 0;
  if (j == 0) { id = cls_id; m = 1; }
  else if (j <= len) { id = tok[(int64_t)s * cap + j - 1]; m = 1; }
  else if (j == len + 1) { id = sep_id; m = 1; }
  ids[e] = id;
  mask[e] = m;
}

}  // namespace wp
}  // namespace irc

using namespace irc;

extern "C" int irc_wordpiece(const void* bytes, const int64_t* offsets, int64_t n,
                             const void* cmap, const void* cpool, const void* cls,
                             const int* htab_id, const void* htab_hash, int64_t htab_size,
                             const int* vocab_off, const void* vocab_cps, const void* vocab_cont,
                             int64_t max_piece, int64_t unk_id, int64_t max_tokens, int* tok,
                             int* tok_len, int* max_len, irc_stream_t stream) {
  IRC_REQUIRE(n >= 0 && max_tokens >= 0, "wordpiece: n=%lld max_tokens=%lld", (long long)n,
              (long long)max_tokens);
  IRC_REQUIRE(htab_size > 0 && (htab_size & (htab_size - 1)) == 0,
              "wordpiece: hash table size %lld is not a power of two", (long long)htab_size);
  IRC_REQUIRE(max_piece >= 1 && max_piece <= wp::MAXP, "wordpiece: longest vocab piece %lld > %d",
              (long long)max_piece, wp::MAXP);
  hipStream_t st = as_stream(stream);
  hipMemsetAsync(max_len, 0, sizeof(int), st);
  if (n == 0) return IRC_OK;
  wp::Tables T{(const unsigned*)cmap, (const unsigned*)cpool, (const unsigned char*)cls, htab_id,
               (const unsigned*)htab_hash, (unsigned)(htab_size - 1), vocab_off,
               (const unsigned*)vocab_cps, (const unsigned char*)vocab_cont, (int)max_piece,
               (int)unk_id};
  hipLaunchKernelGGL(wp::wordpiece_kernel, dim3((unsigned)((n + wp::NT - 1) / wp::NT)),
                     dim3(wp::NT), 0, st, (const unsigned char*)bytes, offsets, (int)n, T,
                     (int)max_tokens, tok, tok_len, max_len);
  return check_launch("wordpiece");
}

extern "C" int irc_wordpiece_pad(const int* tok, const int* tok_len, int64_t n, int64_t max_tokens,
                                 int64_t L, int64_t cls_id, int64_t sep_id, int64_t pad_id,
                                 int64_t* ids, int64_t* mask, irc_stream_t stream) {
  IRC_REQUIRE(L >= 2 && L <= max_tokens + 2, "wordpiece_pad: L=%lld", (long long)L);
  if (n == 0) return IRC_OK;
  const int64_t tot = n * L;
  hipLaunchKernelGGL(wp::pad_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), tok, tok_len, (int)n, (int)max_tokens, (int)L, (int)cls_id,
                     (int)sep_id, (int)pad_id, ids, mask);
  return check_launch("wordpiece_pad");
}
