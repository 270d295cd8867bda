// Corpus-wide query x document cosine top-k for gfx950 (MI355X).
//
// Replaces the dense scoring sketched at src/evaluation.py:110-112 with the
// ranking semantics of preprocessing/drqa/retriever/tfidf_doc_ranker.py:60-75
// (top-k by descending score); ties -> lower global doc index.
//
// Design (DESIGN.md "scan"):
//  * scan_tile_kernel: queries are STATIONARY in registers (each wave owns 32
//    queries' full-D B fragments of v_mfma_f32_32x32x16_bf16); the corpus shard
//    STREAMS once from HBM through a 2-3 deep LDS ring filled by
//    global_load_lds_dwordx4 (XOR-swizzled via the per-lane source address so the
//    row-wise ds_read_b128 fragment reads are bank-conflict free).  Each score is
//    turned into a distinct 64-bit key (score, ~gidx) and kept only if it is >=
//    the query's threshold key; survivors go to a per-(worker, query) region of
//    the workspace with an LDS slot counter (no global atomics).
//  * The threshold is the EXACT k-th largest key of a strided sample of the
//    corpus (a lower bound of the true k-th key), so the survivors always contain
//    the exact top-k and the result is exact for any input, ties included.
//  * select_kernel: one workgroup per query, exact radix select (8 x 8-bit
//    digits) of the k-th key, then a bitonic sort of the k winners.
#include <stdio.h>

#include "irc_common.h"

namespace irc {
namespace scan {

constexpr int TD = 32;  // docs per tile (M of the 32x32x16 MFMA)

template <int D>
struct Geo {
  static constexpr int CH = D / 8;                   // 16-byte chunks per row
  static constexpr int LOWBIT = CH & (-CH);
  static constexpr int SWZ = (LOWBIT < 16 ? LOWBIT : 16) - 1;
  static constexpr int TILE_BYTES = TD * D * 2;
  static constexpr int GLDS_PER_TILE = TD * CH / 64;  // wave-instructions per tile
  static constexpr int NBUF = ((IRC_LDS_BYTES - 2048) / TILE_BYTES) >= 3 ? 3 : 2;
  static constexpr int KK = D / 16;                  // MFMA k-steps
};

enum Mode { KEYS = 0, SCORES = 1 };

// grid: x = worker (contiguous range of tiles), y = query block of NW*32 queries.
template <int D, int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void scan_tile_kernel(
    const unsigned short* __restrict__ queries, const unsigned short* __restrict__ docs, int Q,
    int Qpad, int64_t NS, int64_t stride, int tiles_per_worker, uint32_t idx_base,
    const uint64_t* __restrict__ thr, uint64_t* __restrict__ keys, uint32_t* __restrict__ counts,
    int64_t cap, float* __restrict__ scores_out) {
  using G = Geo<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + G::NBUF * G::TILE_BYTES);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int r32 = lane & 31;
  const int worker = blockIdx.x;
  const int q = blockIdx.y * (NW * 32) + wave * 32 + r32;

  const int64_t ntiles_total = (NS + TD - 1) / TD;
  const int64_t t_begin = (int64_t)worker * tiles_per_worker;
  int64_t t_end = t_begin + tiles_per_worker;
  if (t_end > ntiles_total) t_end = ntiles_total;
  const int my_tiles = t_end > t_begin ? (int)(t_end - t_begin) : 0;

  if (MODE == KEYS && threadIdx.x < NW * 32) lds_cnt[threadIdx.x] = 0;

  // Stage one tile of TD logical docs into LDS buffer `buf` (lane-linear image;
  // swizzle applied on the global source address, read with the same XOR).
  auto issue_tile = [&](int64_t tile, int buf) {
    char* base = smem + buf * G::TILE_BYTES;
#pragma unroll
    for (int i0 = 0; i0 < G::GLDS_PER_TILE; i0 += NW) {
      const int i = i0 + wave;
      if (G::GLDS_PER_TILE % NW == 0 || i < G::GLDS_PER_TILE) {
        const int p = i * 64 + lane;
        const int row = p / G::CH;
        const int cp = p % G::CH;
        const int c = cp ^ (row & G::SWZ);
        int64_t s = tile * TD + row;
        if (s >= NS) s = NS - 1;  // clamp: rows past the end are loaded but never kept
        const unsigned short* src = docs + (s * stride) * (int64_t)D + c * 8;
        glds16(src, base + i * 1024);
      }
    }
  };

  // Prologue: start the LDS ring before touching the query fragments.
  constexpr int PW = (G::GLDS_PER_TILE + NW - 1) / NW;  // glds per wave per tile (upper bound)
#pragma unroll
  for (int b = 0; b < G::NBUF - 1; ++b)
    if (b < my_tiles) issue_tile(t_begin + b, b);

  // Stationary B fragments: lane holds Q[q][kk*16 + 8h .. +8] for every k-step.
  bf16x8 bq[G::KK];
  {
    const bool qv = q < Q;
    const unsigned short* qrow = queries + (int64_t)(qv ? q : 0) * D + 8 * h;
#pragma unroll
    for (int kk = 0; kk < G::KK; ++kk) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + kk * 16);
      if (!qv) v = (u16x8)0;
      bq[kk] = __builtin_bit_cast(bf16x8, v);
    }
  }
  const uint64_t qthr = (MODE == KEYS && thr != nullptr) ? thr[q] : 0ull;

  for (int it = 0; it < my_tiles; ++it) {
    const int64_t tile = t_begin + it;
    if (it + G::NBUF - 1 < my_tiles) issue_tile(tile + G::NBUF - 1, (it + G::NBUF - 1) % G::NBUF);
    // Wait for THIS wave's DMA of tile `it`: later tiles' DMAs may stay in flight.
    const int after = my_tiles - 1 - it;
    if (G::NBUF == 3 && after >= 2)
      wait_vmcnt<2 * PW>();
    else if (after >= 1)
      wait_vmcnt<PW>();
    else
      wait_vmcnt<0>();
    wg_barrier();  // every wave's share of the tile has landed

    const char* tb = smem + (it % G::NBUF) * G::TILE_BYTES;
    f32x16 acc = (f32x16)0.0f;
#pragma unroll
    for (int kk = 0; kk < G::KK; ++kk) {
      const int c = kk * 2 + h;
      const int off = r32 * (G::CH * 16) + ((c ^ (r32 & G::SWZ)) * 16);
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(tb + off);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bq[kk], acc, 0, 0, 0);
    }

    // Epilogue: C[doc row][query col]; col = lane&31, row = (j&3) + 8(j>>2) + 4h.
    if (q < Q) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * h;
        const int64_t s = tile * TD + row;
        if (s < NS) {
          if (MODE == SCORES) {
            scores_out[(int64_t)q * NS + s] = acc[j];
          } else {
            const uint32_t gidx = idx_base + (uint32_t)(s * stride);
            const uint64_t key = make_key(acc[j], gidx);
            if (key >= qthr) {
              const uint32_t slot = atomicAdd(&lds_cnt[wave * 32 + r32], 1u);
              keys[((int64_t)worker * Qpad + q) * cap + slot] = key;
            }
          }
        }
      }
    }
    wg_barrier();  // all reads of this buffer done before it is refilled
  }

  if (MODE == KEYS) {
    __syncthreads();
    if (threadIdx.x < NW * 32) {
      const int qq = blockIdx.y * (NW * 32) + threadIdx.x;
      counts[(int64_t)worker * Qpad + qq] = lds_cnt[threadIdx.x];
    }
  }
}

// ----------------------------------------------------------------- selection
// Key sources for the select kernel.
struct RegionSource {  // scan workspace: G regions per query, counts[g][q]
  const uint64_t* keys;
  const uint32_t* counts;
  int G;
  int Qpad;
  int64_t cap;
  template <class F>
  __device__ __forceinline__ void for_each(int q, int tid, int nt, F&& f) const {
    for (int g = tid; g < G; g += nt) {
      const uint32_t n = counts[(int64_t)g * Qpad + q];
      const uint64_t* p = keys + ((int64_t)g * Qpad + q) * cap;
      for (uint32_t j = 0; j < n; ++j) f(p[j]);
    }
  }
};

struct ListSource {  // merge input: [P][Q][kin] scores + global idx (-1 = empty)
  const float* score;
  const int64_t* idx;
  int P;
  int Q;
  int kin;
  template <class F>
  __device__ __forceinline__ void for_each(int q, int tid, int nt, F&& f) const {
    const int64_t M = (int64_t)P * kin;
    for (int64_t i = tid; i < M; i += nt) {
      const int p = (int)(i / kin), j = (int)(i % kin);
      const int64_t off = ((int64_t)p * Q + q) * kin + j;
      const int64_t id = idx[off];
      if (id >= 0) f(make_key(score[off], (uint32_t)id));
    }
  }
};

constexpr int SEL_NT = 256;
constexpr int SEL_NW = SEL_NT / 64;
constexpr int SEL_MAXK = 1024;

enum SelMode { SEL_THRESHOLD = 0, SEL_FINAL = 1 };

template <class Src>
__global__ __launch_bounds__(SEL_NT) void select_kernel(Src src, int k, int mode,
                                                         uint64_t* __restrict__ thr_out,
                                                         float* __restrict__ out_score,
                                                         int64_t* __restrict__ out_idx) {
  __shared__ uint32_t hist[SEL_NW][256];
  __shared__ uint64_t cand[SEL_MAXK];
  __shared__ uint32_t s_misc[4];  // 0: total count, 1: kr, 2: selected digit, 3: collect ctr

  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  // total candidate count
  if (tid == 0) {
    s_misc[0] = 0;
    s_misc[3] = 0;
  }
  __syncthreads();
  {
    uint32_t c = 0;
    src.for_each(q, tid, SEL_NT, [&](uint64_t) { ++c; });
    atomicAdd(&s_misc[0], c);
  }
  __syncthreads();
  const uint32_t M = s_misc[0];

  uint64_t kth = 0;  // 0 = keep everything
  if (M > (uint32_t)k) {
    if (tid == 0) s_misc[1] = (uint32_t)k;
    uint64_t prefix = 0, pmask = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
      for (int i = tid; i < SEL_NW * 256; i += SEL_NT) (&hist[0][0])[i] = 0;
      __syncthreads();
      src.for_each(q, tid, SEL_NT, [&](uint64_t key) {
        if ((key & pmask) == prefix) atomicAdd(&hist[wave][(key >> shift) & 255], 1u);
      });
      __syncthreads();
      if (wave == 0) {
        // lane covers digits 4*lane .. 4*lane+3; suffix-scan from the top digit.
        uint32_t b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t s = 0;
#pragma unroll
          for (int w = 0; w < SEL_NW; ++w) s += hist[w][4 * lane + j];
          b[j] = s;
        }
        const uint32_t mine = b[0] + b[1] + b[2] + b[3];
        uint32_t suf = mine;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_down(suf, o, 64);
          if (lane + o < 64) suf += t;
        }
        const uint32_t kr = s_misc[1];
        const uint32_t above = suf - mine;  // count in digits of higher lanes
        if (suf >= kr && above < kr) {
          uint32_t acc = above;
          int sel = 4 * lane;
          for (int j = 3; j >= 0; --j) {
            if (acc + b[j] >= kr) {
              sel = 4 * lane + j;
              break;
            }
            acc += b[j];
          }
          s_misc[2] = (uint32_t)sel;
          s_misc[1] = kr - acc;
        }
      }
      __syncthreads();
      prefix |= (uint64_t)s_misc[2] << shift;
      pmask |= (uint64_t)0xff << shift;
    }
    kth = prefix;
  }

  if (mode == SEL_THRESHOLD) {
    if (tid == 0) thr_out[q] = kth;
    return;
  }

  // collect the (exactly min(M, k)) keys >= kth
  const int cnt = (int)(M < (uint32_t)k ? M : (uint32_t)k);
  int npow = 1;
  while (npow < cnt) npow <<= 1;
  for (int i = tid; i < npow; i += SEL_NT) cand[i] = 0;
  __syncthreads();
  src.for_each(q, tid, SEL_NT, [&](uint64_t key) {
    if (key >= kth) {
      const uint32_t slot = atomicAdd(&s_misc[3], 1u);
      if (slot < (uint32_t)SEL_MAXK) cand[slot] = key;
    }
  });
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < npow; i += SEL_NT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool desc = ((i & size) == 0);
          const uint64_t a = cand[i], b = cand[j];
          if (desc ? (a < b) : (a > b)) {
            cand[i] = b;
            cand[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += SEL_NT) {
    float s = -__builtin_huge_valf();
    int64_t id = -1;
    if (i < cnt) {
      const uint64_t key = cand[i];
      s = unorderable_f32((uint32_t)(key >> 32));
      id = (int64_t)(uint32_t)(~(uint32_t)key);
    }
    out_score[(int64_t)q * k + i] = s;
    out_idx[(int64_t)q * k + i] = id;
  }
}

// ------------------------------------------------------------------ planning
struct Plan {
  int nw;
  int qpad;
  int gy;
  bool two_phase;
  int64_t stride;  // sample stride
  int64_t S;       // sample size
  int g_s, tpw_s;
  int64_t cap_s;
  int g_f, tpw_f;
  int64_t cap_f;
  size_t off_thr, off_cnt, off_keys, bytes;
};

static int pick_nw(int64_t D, int64_t Q) {
  int nw = D <= 256 ? 8 : 4;  // B fragments: D/16 * 4 VGPRs per lane
  int need = (int)((Q + 31) / 32);
  int p = 1;
  while (p < need && p < nw) p <<= 1;
  return p < nw ? p : nw;
}

static void plan_workers(int64_t ntiles, int gy, int* g, int* tpw) {
  const int64_t target = 256 * 2;  // ~2 waves of workgroups over 256 CUs
  int64_t want = (target + gy - 1) / gy;
  if (want < 1) want = 1;
  if (want > ntiles) want = ntiles > 0 ? ntiles : 1;
  int64_t per = (ntiles + want - 1) / want;
  if (per < 1) per = 1;
  *tpw = (int)per;
  *g = (int)((ntiles + per - 1) / per);
  if (*g < 1) *g = 1;
}

static Plan make_plan(int64_t Q, int64_t N, int64_t D, int64_t k) {
  Plan p{};
  p.nw = pick_nw(D, Q);
  const int qb = p.nw * 32;
  p.gy = (int)((Q + qb - 1) / qb);
  if (p.gy < 1) p.gy = 1;
  p.qpad = p.gy * qb;
  int64_t s_target = 16 * k;
  if (N / 16 > s_target) s_target = N / 16;
  p.stride = s_target > 0 ? N / s_target : 1;
  if (p.stride < 1) p.stride = 1;
  p.two_phase = p.stride > 1;
  p.S = p.two_phase ? (N + p.stride - 1) / p.stride : N;
  plan_workers((p.S + TD - 1) / TD, p.gy, &p.g_s, &p.tpw_s);
  p.cap_s = (int64_t)p.tpw_s * TD;
  plan_workers((N + TD - 1) / TD, p.gy, &p.g_f, &p.tpw_f);
  p.cap_f = (int64_t)p.tpw_f * TD;
  const int gmax = p.g_s > p.g_f ? p.g_s : p.g_f;
  int64_t kmax = (int64_t)p.g_s * p.cap_s;
  if (p.two_phase && (int64_t)p.g_f * p.cap_f > kmax) kmax = (int64_t)p.g_f * p.cap_f;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  p.off_thr = 0;
  p.off_cnt = al(p.off_thr + (size_t)p.qpad * 8);
  p.off_cnt = al(p.off_cnt);
  p.off_keys = al(p.off_cnt + (size_t)gmax * p.qpad * 4);
  p.bytes = al(p.off_keys + (size_t)kmax * p.qpad * 8);
  return p;
}

template <int D, int NW, int MODE>
static void launch_tile(const Plan& p, dim3 grid, const unsigned short* qs,
                        const unsigned short* docs, int Q, int64_t NS, int64_t stride, int tpw,
                        uint32_t idx_base, const uint64_t* thr, uint64_t* keys, uint32_t* counts,
                        int64_t cap, float* scores, hipStream_t st) {
  using G = Geo<D>;
  const size_t lds = (size_t)G::NBUF * G::TILE_BYTES + NW * 32 * 4;
  hipLaunchKernelGGL((scan_tile_kernel<D, NW, MODE>), grid, dim3(NW * 64), lds, st, qs, docs, Q,
                     p.qpad, NS, stride, tpw, idx_base, thr, keys, counts, cap, scores);
}

template <int MODE>
static int dispatch_tile(int64_t D, const Plan& p, dim3 grid, const unsigned short* qs,
                         const unsigned short* docs, int Q, int64_t NS, int64_t stride, int tpw,
                         uint32_t idx_base, const uint64_t* thr, uint64_t* keys, uint32_t* counts,
                         int64_t cap, float* scores, hipStream_t st) {
#define IRC_SCAN_CASE(DD)                                                                       \
  case DD:                                                                                      \
    switch (p.nw) {                                                                             \
      case 1:                                                                                   \
        launch_tile<DD, 1, MODE>(p, grid, qs, docs, Q, NS, stride, tpw, idx_base, thr, keys,   \
                                 counts, cap, scores, st);                                      \
        break;                                                                                  \
      case 2:                                                                                   \
        launch_tile<DD, 2, MODE>(p, grid, qs, docs, Q, NS, stride, tpw, idx_base, thr, keys,   \
                                 counts, cap, scores, st);                                      \
        break;                                                                                  \
      case 4:                                                                                   \
        launch_tile<DD, 4, MODE>(p, grid, qs, docs, Q, NS, stride, tpw, idx_base, thr, keys,   \
                                 counts, cap, scores, st);                                      \
        break;                                                                                  \
      default:                                                                                  \
        if (DD <= 256)                                                                          \
          launch_tile<DD, (DD <= 256 ? 8 : 4), MODE>(p, grid, qs, docs, Q, NS, stride, tpw,     \
                                                     idx_base, thr, keys, counts, cap, scores,  \
                                                     st);                                       \
        break;                                                                                  \
    }                                                                                           \
    break;
  switch (D) {
    IRC_SCAN_CASE(64)
    IRC_SCAN_CASE(128)
    IRC_SCAN_CASE(256)
    IRC_SCAN_CASE(384)
    IRC_SCAN_CASE(512)
    IRC_SCAN_CASE(768)
    IRC_SCAN_CASE(1024)
    default:
      set_error("scan: unsupported D=%lld (supported: 64,128,256,384,512,768,1024)",
                (long long)D);
      return IRC_E_INVALID;
  }
#undef IRC_SCAN_CASE
  return check_launch("scan_tile_kernel");
}

static bool supported_d(int64_t D) {
  return D == 64 || D == 128 || D == 256 || D == 384 || D == 512 || D == 768 || D == 1024;
}

}  // namespace scan
}  // namespace irc

using namespace irc;
using namespace irc::scan;

extern "C" int64_t irc_scan_topk_workspace(int64_t Q, int64_t N, int64_t D, int64_t k) {
  if (Q <= 0 || N <= 0 || k <= 0) return 256;
  return (int64_t)make_plan(Q, N, D, k).bytes;
}

extern "C" int irc_scan_topk(const void* queries, const void* docs, int64_t Q, int64_t N,
                             int64_t D, int64_t k, int64_t doc_offset, void* workspace,
                             int64_t workspace_bytes, float* out_score, int64_t* out_idx,
                             irc_stream_t stream) {
  IRC_REQUIRE(Q >= 0 && N >= 0, "scan_topk: negative size");
  IRC_REQUIRE(k >= 1 && k <= SEL_MAXK, "scan_topk: k=%lld outside [1, %d]", (long long)k,
              SEL_MAXK);
  IRC_REQUIRE(supported_d(D), "scan_topk: unsupported D=%lld", (long long)D);
  IRC_REQUIRE(doc_offset >= 0 && doc_offset + N <= (int64_t)0xFFFFFFFFll,
              "scan_topk: global doc index must fit 32 bits");
  IRC_REQUIRE(Q < (1 << 24), "scan_topk: Q too large");
  hipStream_t st = as_stream(stream);
  if (Q == 0) return IRC_OK;
  if (N == 0) {
    // nothing to rank: every slot empty
    IRC_REQUIRE(workspace_bytes >= 0, "bad workspace");
    ListSource src{out_score, out_idx, 0, (int)Q, 1};
    hipLaunchKernelGGL((select_kernel<ListSource>), dim3(Q), dim3(SEL_NT), 0, st, src, (int)k,
                       (int)SEL_FINAL, nullptr, out_score, out_idx);
    return check_launch("select_kernel(empty)");
  }
  const Plan p = make_plan(Q, N, D, k);
  IRC_REQUIRE(workspace != nullptr && workspace_bytes >= (int64_t)p.bytes,
              "scan_topk: workspace %lld < required %lld bytes", (long long)workspace_bytes,
              (long long)p.bytes);
  char* ws = static_cast<char*>(workspace);
  uint64_t* thr = reinterpret_cast<uint64_t*>(ws + p.off_thr);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ws + p.off_cnt);
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + p.off_keys);
  const unsigned short* qs = static_cast<const unsigned short*>(queries);
  const unsigned short* ds = static_cast<const unsigned short*>(docs);
  const uint32_t base = (uint32_t)doc_offset;
  int rc;
  if (p.two_phase) {
    rc = dispatch_tile<KEYS>(D, p, dim3(p.g_s, p.gy), qs, ds, (int)Q, p.S, p.stride, p.tpw_s,
                             base, nullptr, keys, cnt, p.cap_s, nullptr, st);
    if (rc) return rc;
    RegionSource s1{keys, cnt, p.g_s, p.qpad, p.cap_s};
    hipLaunchKernelGGL((select_kernel<RegionSource>), dim3(Q), dim3(SEL_NT), 0, st, s1, (int)k,
                       (int)SEL_THRESHOLD, thr, nullptr, nullptr);
    if ((rc = check_launch("select_kernel(threshold)"))) return rc;
  }
  prof_begin(st);
  rc = dispatch_tile<KEYS>(D, p, dim3(p.g_f, p.gy), qs, ds, (int)Q, N, 1, p.tpw_f, base,
                           p.two_phase ? thr : nullptr, keys, cnt, p.cap_f, nullptr, st);
  prof_end("scan_filter", st);
  if (rc) return rc;
  RegionSource s2{keys, cnt, p.g_f, p.qpad, p.cap_f};
  hipLaunchKernelGGL((select_kernel<RegionSource>), dim3(Q), dim3(SEL_NT), 0, st, s2, (int)k,
                     (int)SEL_FINAL, nullptr, out_score, out_idx);
  return check_launch("select_kernel(final)");
}

extern "C" int irc_topk_merge(const float* in_score, const int64_t* in_idx, int64_t P, int64_t Q,
                              int64_t kin, int64_t kout, float* out_score, int64_t* out_idx,
                              irc_stream_t stream) {
  IRC_REQUIRE(P >= 1 && Q >= 0 && kin >= 1, "topk_merge: bad sizes");
  IRC_REQUIRE(kout >= 1 && kout <= SEL_MAXK, "topk_merge: kout outside [1, %d]", SEL_MAXK);
  if (Q == 0) return IRC_OK;
  ListSource src{in_score, in_idx, (int)P, (int)Q, (int)kin};
  hipLaunchKernelGGL((select_kernel<ListSource>), dim3(Q), dim3(SEL_NT), 0, as_stream(stream),
                     src, (int)kout, (int)SEL_FINAL, nullptr, out_score, out_idx);
  return check_launch("select_kernel(merge)");
}

extern "C" int irc_scan_scores(const void* queries, const void* docs, int64_t Q, int64_t N,
                               int64_t D, float* out, irc_stream_t stream) {
  IRC_REQUIRE(Q >= 0 && N >= 0, "scan_scores: negative size");
  IRC_REQUIRE(supported_d(D), "scan_scores: unsupported D=%lld", (long long)D);
  if (Q == 0 || N == 0) return IRC_OK;
  Plan p = make_plan(Q, N, D, 1);
  return dispatch_tile<SCORES>(D, p, dim3(p.g_f, p.gy), static_cast<const unsigned short*>(queries),
                               static_cast<const unsigned short*>(docs), (int)Q, N, 1, p.tpw_f, 0,
                               nullptr, nullptr, nullptr, 0, out, as_stream(stream));
}
