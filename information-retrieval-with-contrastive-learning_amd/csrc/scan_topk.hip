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
#include <math.h>
#include <stdio.h>

#include <atomic>
#include <cmath>

#include "gemm_pp.h"

#ifndef IRC_SCAN_AUX
#define IRC_SCAN_AUX 0  // cache policy of the corpus stream (0: default)
#endif
#ifndef IRC_SCAN_SEL_STOP
#define IRC_SCAN_SEL_STOP -1  // diagnostic builds: the final select returns at stage N
#endif
// 1: the DMA of tile it + NBUF is issued into tile it's ring slot as soon as every
// wave holds tile it's A fragments in registers (one extra barrier), so NBUF tiles
// are in flight during the MFMAs and the epilogue instead of NBUF - 1 (0: the
// round-2 order, the next DMA at the top of each iteration).
#define IRC_SCAN_EARLY_ISSUE 1
// 1: that DMA is issued piece by piece between the tile's MFMAs instead of all at once
// ahead of them, so a piece whose issue waits on a full memory queue no longer holds the
// MFMAs back.  C3 shard (250k x 768), filter: Q = 48 / 64 / 96 / 128 single pass
// 92.6-95.4 / 92.9-93.1 / 108.6-109.0 / 111.0-111.7 -> 87.5-88.5 / 88.0-88.4 / 105.0-105.2 /
// 108.1-108.6 us, the sampled pipeline at Q = 64 84.6 -> 79.5-79.9 us, Q <= 16 within
// +-1 us (two interleaved runs, profiles/r06_e_*); same results (0: the all-at-once form).
#ifndef IRC_SCAN_IL
#define IRC_SCAN_IL 1
#endif

namespace irc {
namespace scan {

constexpr int TD = 32;  // docs per tile (M of the 32x32x16 MFMA)

#ifdef IRC_SCAN_STAMPS  // diagnostic build: phase timestamps of block 0 (s_memrealtime, 100 MHz)
__device__ uint64_t dbg_stamps[4][32];
#define STAMP(slot, i)                                                                   \
  do {                                                                                   \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                           \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                              \
      volatile uint64_t* p_ = &dbg_stamps[slot][(i) + (int)(threadIdx.x & 0)];            \
      *p_ = t_;                                                                          \
    }                                                                                    \
  } while (0)
// every block's start / end of the filter launch (LTOP or KEYS-with-threshold)
__device__ uint64_t dbg_blk[2 * 8192];
#define BLK_STAMP(i)                                                                     \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 8192 && (MODE == LTOP || thr != nullptr)) {     \
      volatile uint64_t* p_ = &dbg_blk[2 * blockIdx.x + (i)];                            \
      *p_ = __builtin_amdgcn_s_memrealtime();                                            \
    }                                                                                    \
  } while (0)
#else
#define STAMP(slot, i) \
  do {                 \
  } while (0)
#define BLK_STAMP(i) \
  do {               \
  } while (0)
#endif

// Tile geometry for embeddings of D elements of EB bytes (2: bf16, 1: fp8 e4m3).
// The chunk XOR is confined to the low bits that divide a k-slice's chunk count,
// so the per-slice read offsets stay base + immediate.
// KSX = k-slices (waves sharing one 32-query group): 1 for D <= 512, 2 above, and 4
// for the single-pass scan of at most 64 queries at D = 768 / 1024 (LTOP_KS4).
template <int D, int EB = 2, int KSX = (D > 512 ? 2 : 1)>
struct Geo {
  static constexpr int KS = KSX;
  static constexpr int CH = D * EB / 16;             // 16-byte chunks per row
  static constexpr int LOWBIT = (CH / KS) & (-(CH / KS));
  static constexpr int SWZ = (LOWBIT < 16 ? LOWBIT : 16) - 1;
  static constexpr int TILE_BYTES = TD * D * EB;
  static constexpr int GLDS_PER_TILE = TD * CH / 64;  // wave-instructions per tile
  // k-slice exchange: KS = 2, NQ <= 4 (8 floats per lane per wave); KS = 4, NQ <= 2
  // (the butterfly's 8-float rounds)
  static constexpr int XBUF_BYTES = (KSX > 1) ? 4 * 4096 : 0;
  // ring depth: 3 x 48 KB for bf16 D=768; fp8 tiles are half as large, so the
  // ring goes deeper (same bytes in flight)
  static constexpr int NBMAX = EB == 1 ? 5 : 3;
  static constexpr int NFIT = (IRC_LDS_BYTES - XBUF_BYTES) / TILE_BYTES;
  static constexpr int NBUF = NFIT >= NBMAX ? NBMAX : (NFIT >= 3 ? 3 : 2);
  static constexpr int KK = D / 16;                  // MFMA k-steps (K = 16 for both types)
};

// KEYS: every key >= the threshold survives.  GMAX (the sample pass): each lane
// keeps only the largest key of the JPW docs it finishes per tile -- the k-th
// largest of these group maxima is still a lower bound of the true k-th key
// (k distinct docs reach it), with 8-16x fewer keys to store and select.
// LTOP (single pass, no threshold): each lane keeps the 4 largest keys of the
// docs it finishes (its "list": one (worker, query, slice)), in registers, and
// writes them densely at the end; select_dense then finds the k-th key of all
// lists and rescans, exactly, the workers whose truncated lists could hide a
// winner.
enum Mode { KEYS = 0, SCORES = 1, GMAX = 2, LTOP = 3 };
constexpr int LT_M = 4;  // keys per LTOP list

// Opaque copy: stops LICM from hoisting per-lane address math out of the tile
// loop (keeping 12+ 64-bit DMA addresses live costs more VGPRs than recomputing).
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// grid (1-D): G workers x GY query blocks, decoded XCD-aware so the GY blocks
// that scan the SAME doc range are consecutive in dispatch order on the same XCD
// (blocks b and b+8 share an XCD under round-robin placement): the corpus tile is
// fetched from HBM once and re-read from that XCD's L2 by the partner block.
// Placement only affects speed, never results.
//
// Waves: NQ query groups (32 queries each) x KS k-slices.  Wave (g, kh) keeps
// the B fragments of its 32 queries for dims [kh*D/KS, (kh+1)*D/KS) in VGPRs;
// with KS = 2 the partial 32x32 accumulators of the two k-slices are exchanged
// through LDS (each wave finishes half of the 16 accumulator rows).
//
// Survivors: lane (r32, h) of wave (g, kh) finishes rows {(j&3) + 8(j>>2) + 4h}
// for j in its half of [0, 16) of every tile, for query (g, r32).  It owns the
// private slice (kh*2 + h) of the (worker, query) region and counts in a
// register -- no atomics, nothing that could drain the LDS-DMA ring.
// EB = 1: e4m3 embeddings on v_mfma_f32_32x32x16_fp8_fp8.  A 16-byte chunk then
// holds two k-steps (low 8 bytes: step 2c, high: step 2c+1); queries and docs use
// the same k order, so the dot product is unchanged.
template <int D, int NQ, int KS, int MODE, int EB = 2>
__global__ __launch_bounds__(NQ * KS * 64) __attribute__((amdgpu_waves_per_eu(1, 4)))
void scan_tile_kernel(
    const unsigned char* __restrict__ queries, const unsigned char* __restrict__ docs, int Q,
    int Qpad, int GY, int NS, int stride, int tiles_per_worker, uint32_t idx_base,
    const uint64_t* __restrict__ thr, uint64_t* __restrict__ keys, uint32_t* __restrict__ counts,
    int64_t cap, float* __restrict__ scores_out) {
  using G = Geo<D, EB, KS>;
  static_assert(KS != 4 || ((MODE == LTOP || MODE == SCORES) && NQ <= 2),
                "four k-slices: the single-pass scan (and scan_scores on the same plan) only");
  constexpr int NW = NQ * KS;
  constexpr int KKW = G::KK / KS;  // k-steps per wave
  constexpr int NCW = KKW * EB / 2;  // 16-byte fragment chunks per wave per tile
  constexpr int JPW = 16 / KS;     // accumulator registers each wave finishes
  constexpr int PW = (G::GLDS_PER_TILE + NW - 1) / NW;  // glds per wave per tile (upper bound)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* xbuf = reinterpret_cast<float*>(smem + G::NBUF * G::TILE_BYTES);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave % NQ;
  const int kh = wave / NQ;
  const int h = lane >> 5;
  const int r32 = lane & 31;
  const int b = blockIdx.x;
  const int qblock = (b >> 3) % GY;
  const int worker = ((b >> 3) / GY) * 8 + (b & 7);
  const int q = qblock * (NQ * 32) + g * 32 + r32;

  STAMP(thr == nullptr ? 2 : 3, 0);
  BLK_STAMP(0);
  const int ntiles_total = (NS + TD - 1) / TD;
  const int t_begin = worker * tiles_per_worker;
  int t_end = t_begin + tiles_per_worker;
  if (t_end > ntiles_total) t_end = ntiles_total;
  const int my_tiles = t_end > t_begin ? t_end - t_begin : 0;

  // Per-lane byte offsets (within a tile) of this wave's PW DMA pieces; a piece
  // i covers LDS bytes [1024 i, 1024 i + 1024) of the lane-linear image, lane l
  // the 16 bytes at 1024 i + 16 l, sourced from (row, chunk ^ (row & SWZ)).
  const int64_t row_bytes = (int64_t)stride * D * EB;
  uint32_t goff[PW];
  int grow[PW];
#pragma unroll
  for (int t = 0; t < PW; ++t) {
    const int i = t * NW + wave;
    const int p = i * 64 + lane;
    const int row = p / G::CH;
    const int cp = p - row * G::CH;
    const int c = cp ^ (row & G::SWZ);
    grow[t] = row;
    goff[t] = (uint32_t)(row * row_bytes + c * 16);
  }
  // piece t (of PW) of this wave's share of tile `tile`'s DMA into ring slot `buf`
  auto issue_piece = [&](int tile, int buf, int t) {
    char* base = smem + buf * G::TILE_BYTES;
    const char* src0 = reinterpret_cast<const char*>(docs) + (int64_t)tile * TD * row_bytes;
    const bool tail = (tile + 1) * TD > NS;  // uniform
    const int i = t * NW + wave;
    if (G::GLDS_PER_TILE % NW == 0 || i < G::GLDS_PER_TILE) {
      uint32_t off = goff[t];
      if (tail && tile * TD + grow[t] >= NS)  // clamp: loaded but never kept
        off -= (uint32_t)((tile * TD + grow[t] - (NS - 1)) * row_bytes);
      glds16_pol<IRC_SCAN_AUX>(src0 + off, base + i * 1024);
    }
  };
  auto issue_tile = [&](int tile, int buf) {
    char* base = smem + buf * G::TILE_BYTES;
    const char* src0 = reinterpret_cast<const char*>(docs) + (int64_t)tile * TD * row_bytes;
    const bool tail = (tile + 1) * TD > NS;  // uniform
#pragma unroll
    for (int t = 0; t < PW; ++t) {
      const int i = t * NW + wave;
      if (G::GLDS_PER_TILE % NW == 0 || i < G::GLDS_PER_TILE) {
        uint32_t off = goff[t];
        if (tail && tile * TD + grow[t] >= NS)  // clamp: loaded but never kept
          off -= (uint32_t)((tile * TD + grow[t] - (NS - 1)) * row_bytes);
        glds16_pol<IRC_SCAN_AUX>(src0 + off, base + i * 1024);
      }
    }
  };

  constexpr int PRE = IRC_SCAN_EARLY_ISSUE ? G::NBUF : G::NBUF - 1;  // tiles issued up front
#pragma unroll
  for (int bb = 0; bb < PRE; ++bb)
    if (bb < my_tiles) issue_tile(t_begin + bb, bb);

  // Stationary B fragments: lane holds chunk 2c + h of its query row (of its
  // k-slice) for every c -- the same chunks it reads of each doc row.
  u16x8 bq[NCW];
  {
    const bool qv = q < Q;
    const unsigned char* qrow =
        queries + (int64_t)(qv ? q : 0) * D * EB + 16 * h + kh * (D * EB / KS);
#pragma unroll
    for (int c = 0; c < NCW; ++c) {
      u16x8 v = *reinterpret_cast<const u16x8*>(qrow + c * 32);
      if (!qv) v = (u16x8)0;
      bq[c] = v;
    }
  }
  // LTOP list (descending; 0 = empty slot: real keys are >= 1) and the float
  // prefilter of its last slot
  uint64_t lt0 = 0, lt1 = 0, lt2 = 0, lt3 = 0;
  float ltf = q < Q ? -__builtin_huge_valf() : __builtin_huge_valf();
  const uint64_t qthr = (MODE == KEYS && thr != nullptr && q < Q) ? thr[q] : 0ull;
  const uint32_t qthr_hi = (uint32_t)(qthr >> 32);
  const float qtf = q >= Q ? __builtin_huge_valf()
                           : (qthr_hi == 0 ? -__builtin_huge_valf() : unorderable_f32(qthr_hi));
  // LDS read offsets: chunk c = 2kk + h of row r32 lives at 16*(c ^ (r32 & SWZ));
  // the XOR only touches the low 4 bits, so 8 per-lane offsets + an immediate
  // 256*(kk>>3) cover all k-steps.
  int lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int cj = 2 * j + h;
    lo[j] = r32 * (G::CH * 16) + (((cj & 15) ^ (r32 & G::SWZ)) * 16);
  }
  uint32_t nsurv = 0;
  uint64_t sb0 = 0, sb1 = 0, sb2 = 0, sb3 = 0;  // survivor shift buffer (KEYS mode)
  int sbn = 0;
  // Survivor store instructions issued by this wave in each of the last NBUF-1
  // tiles, one byte per tile (wave-uniform).  They sit between the ring's DMAs in
  // vmcnt order, so the wait for tile `it` allows them as extra younger operations.
  uint64_t nst_hist = 0;
  const int slice = kh * 2 + h;  // private output slice (of 2*KS)
  uint64_t* myreg = keys + ((int64_t)worker * Qpad + q) * cap + slice * (cap / (2 * KS));

  for (int it = 0; it < my_tiles; ++it) {
    const int tile = t_begin + it;
    if (!IRC_SCAN_EARLY_ISSUE && it + G::NBUF - 1 < my_tiles)
      issue_tile(tile + G::NBUF - 1, (it + G::NBUF - 1) % G::NBUF);
    const int after = my_tiles - 1 - it;
    const int ahead = after < G::NBUF - 1 ? after : G::NBUF - 1;
    // survivor stores younger than tile it's DMA: those of the iterations after
    // the one that issued it (PRE of them)
    int extra = 0;
#pragma unroll
    for (int t = 0; t < PRE; ++t) extra += (int)((nst_hist >> (8 * t)) & 0xff);
    extra = extra < 15 ? extra : 15;  // smaller = safe
    wait_vmcnt_n(__builtin_amdgcn_readfirstlane(ahead == 0 ? 0 : ahead * PW + extra));
    wg_barrier();  // every wave's share of the tile has landed

#ifdef IRC_SCAN_DMA_ONLY  // diagnostic build: the corpus stream alone
    wg_barrier();
    if (IRC_SCAN_EARLY_ISSUE && it + G::NBUF < my_tiles)
      issue_tile(tile + G::NBUF, it % G::NBUF);
    continue;
#endif
    const char* tb = smem + (it % G::NBUF) * G::TILE_BYTES + kh * (D * EB / KS);
    f32x16 acc = (f32x16)0.0f;
    {
      // every A fragment of the tile first (one LDS latency, not NCW of them:
      // with one wave per SIMD nothing else hides it), then the MFMA chain
      u16x8 af[NCW];
#pragma unroll
      for (int c = 0; c < NCW; ++c)
        af[c] = *reinterpret_cast<const u16x8*>(tb + lo[c & 7] + 256 * (c >> 3));
      if (IRC_SCAN_EARLY_ISSUE) {
        // the slot is free once every wave's fragment reads have returned
        lds_barrier();
        if (!IRC_SCAN_IL && it + G::NBUF < my_tiles) issue_tile(tile + G::NBUF, it % G::NBUF);
      }
#pragma unroll
      for (int c = 0; c < NCW; ++c) {
        if constexpr (EB == 2) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[c]),
                                                        __builtin_bit_cast(bf16x8, bq[c]), acc,
                                                        0, 0, 0);
        } else {
          typedef long l2 __attribute__((ext_vector_type(2)));
          const l2 a2 = __builtin_bit_cast(l2, af[c]), b2 = __builtin_bit_cast(l2, bq[c]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a2[0], b2[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a2[1], b2[1], acc, 0, 0, 0);
        }
        if (IRC_SCAN_IL && IRC_SCAN_EARLY_ISSUE && it + G::NBUF < my_tiles) {
          // the next DMA spread over the MFMA chain: a piece whose issue stalls on a full
          // memory queue then no longer holds back the MFMAs behind it
#pragma unroll
          for (int t = 0; t < PW; ++t)
            if (t * NCW / PW == c) issue_piece(tile + G::NBUF, it % G::NBUF, t);
        }
      }
    }
#ifdef IRC_SCAN_MFMA_ONLY  // diagnostic build
    if (acc[0] == 12345.f) myreg[0] = 1;  // keep the MFMAs alive
    wg_barrier();
    continue;
#endif
    if (KS == 4) {
      // Butterfly reduce-scatter of the four k-slice partial sums: round 1 with
      // wave kh ^ 2 (keep half kh >> 1 of the 16 registers, send the other), round 2
      // with wave kh ^ 1 (keep quarter kh & 1 of that half).  Every wave's registers
      // end as fl(fl(s0 + s2) + fl(s1 + s3)) whatever its kh (fp32 addition is
      // commutative), the order rescore_docs reproduces.  Round 2 writes into the
      // slot this wave alone read in round 1, so it needs no barrier before it.
      float* s1 = xbuf + ((g * 4 + kh) * 64 + lane) * 8;
      float* s2 = xbuf + ((g * 4 + (kh ^ 2)) * 64 + lane) * 8;
      float* s3 = xbuf + ((g * 4 + (kh ^ 3)) * 64 + lane) * 8;  // wave kh ^ 1's round-2 slot
      f32x4 o0, o1, k0, k1;
      if ((kh >> 1) == 0) {
        o0 = (f32x4){acc[8], acc[9], acc[10], acc[11]};
        o1 = (f32x4){acc[12], acc[13], acc[14], acc[15]};
        k0 = (f32x4){acc[0], acc[1], acc[2], acc[3]};
        k1 = (f32x4){acc[4], acc[5], acc[6], acc[7]};
      } else {
        o0 = (f32x4){acc[0], acc[1], acc[2], acc[3]};
        o1 = (f32x4){acc[4], acc[5], acc[6], acc[7]};
        k0 = (f32x4){acc[8], acc[9], acc[10], acc[11]};
        k1 = (f32x4){acc[12], acc[13], acc[14], acc[15]};
      }
      reinterpret_cast<f32x4*>(s1)[0] = o0;
      reinterpret_cast<f32x4*>(s1)[1] = o1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the raw barrier does not wait
      wg_barrier();
      k0 += reinterpret_cast<const f32x4*>(s2)[0];
      k1 += reinterpret_cast<const f32x4*>(s2)[1];
      const f32x4 keep = (kh & 1) ? k1 : k0;
      reinterpret_cast<f32x4*>(s2)[0] = (kh & 1) ? k0 : k1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wg_barrier();
      const f32x4 fq = keep + reinterpret_cast<const f32x4*>(s3)[0];
      // the finished quarter kh (rows of registers 4 kh .. 4 kh + 3) in registers 0-3
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] = fq[e];
    } else if (KS == 2) {
      // exchange: wave kh sends the half it does NOT finish, adds the partner's.
      float* xo = xbuf + ((g * 2 + kh) * 64 + lane) * 8;
      float* xi = xbuf + ((g * 2 + (kh ^ 1)) * 64 + lane) * 8;
      f32x4 s0, s1;
      if (kh == 0) {
        s0 = (f32x4){acc[8], acc[9], acc[10], acc[11]};
        s1 = (f32x4){acc[12], acc[13], acc[14], acc[15]};
      } else {
        s0 = (f32x4){acc[0], acc[1], acc[2], acc[3]};
        s1 = (f32x4){acc[4], acc[5], acc[6], acc[7]};
      }
      reinterpret_cast<f32x4*>(xo)[0] = s0;
      reinterpret_cast<f32x4*>(xo)[1] = s1;
      // the raw barrier does not wait for LDS writes: without this wait the partner
      // wave can read the slot before the write lands (seen on MI355X with the
      // four-slice exchange, whose round 2 also overwrites a slot another wave wrote)
      lds_barrier();
      const f32x4 t0 = reinterpret_cast<const f32x4*>(xi)[0];
      const f32x4 t1 = reinterpret_cast<const f32x4*>(xi)[1];
      if (kh == 0) {
        acc[0] += t0[0]; acc[1] += t0[1]; acc[2] += t0[2]; acc[3] += t0[3];
        acc[4] += t1[0]; acc[5] += t1[1]; acc[6] += t1[2]; acc[7] += t1[3];
      } else {
        acc[8] += t0[0]; acc[9] += t0[1]; acc[10] += t0[2]; acc[11] += t0[3];
        acc[12] += t1[0]; acc[13] += t1[1]; acc[14] += t1[2]; acc[15] += t1[3];
      }
    }

#ifdef IRC_SCAN_NO_EPI  // diagnostic build
    if (acc[0] == 12345.f) myreg[0] = 1;
    wg_barrier();
    continue;
#endif
    // Epilogue: C[doc row][query col]; col = lane&31, row = (j&3) + 8(j>>2) + 4h.
    // The wave finishes registers jj + joff of acc (joff: wave-uniform half).
    int nst = 0;
    const int s0row = tile * TD;
    f32x16 fin = acc;
    int joff = 0;
    if (KS == 2 && kh == 1) {  // uniform branch: move the upper half down
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) fin[jj] = acc[jj + 8];
      joff = 8;
    }
    if (KS == 4) joff = 4 * kh;  // the exchange left quarter kh in registers 0-3
    // Survivors wait in a per-lane 4-key shift buffer and leave 4 at a time: a
    // store is older than the DMAs issued after it and vmcnt retires in order,
    // so every store episode delays a later tile's wait by its write-ack
    // latency -- 4x fewer episodes.  Called by the whole wave (ballot).
    auto push = [&](bool keep, uint64_t key) {
      if (keep) {
        sb3 = sb2;
        sb2 = sb1;
        sb1 = sb0;
        sb0 = key;
        ++sbn;
      }
      if (__ballot(sbn == 4)) {
        nst += 4;
        if (sbn == 4) {
          myreg[nsurv] = sb0;
          myreg[nsurv + 1] = sb1;
          myreg[nsurv + 2] = sb2;
          myreg[nsurv + 3] = sb3;
          nsurv += 4;
          sbn = 0;
        }
      }
    };
    if (MODE == SCORES) {
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) {
        const int j = jj + joff;
        const int s = s0row + (j & 3) + 8 * (j >> 2) + 4 * h;
        if (q < Q && s < NS) scores_out[(int64_t)q * NS + s] = fin[jj];
      }
    } else if (MODE == GMAX) {
      // the largest score of the lane's docs (first of equals) -> one real key
      float bv = -__builtin_huge_valf();
      int bs = -1;
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) {
        const int j = jj + joff;
        const int s = s0row + (j & 3) + 8 * (j >> 2) + 4 * h;
        const bool better = (q < Q) && (s < NS) && fin[jj] > bv;
        bv = better ? fin[jj] : bv;
        bs = better ? s : bs;
      }
      push(bs >= 0, make_key(bv, idx_base + (uint32_t)bs * (uint32_t)stride));
    } else if (MODE == LTOP) {
      // candidates: scores >= the list's last score; one per lane per round
      // (rounds = the wave's largest candidate count; after the first tiles
      // mostly 0-2).  Measured alternatives on MI355X: one insertion step per slot
      // with any candidate (the select chain saved, more steps at Q >= 16), a
      // select tree + position-compare insertion (more instructions) and a floor
      // shared with the h-partner lane (select_dense slower) were slower; a fixed
      // merge network (sorted 4-runs + top-4 merges) for tiles where some lane has
      // 3+ candidates gave C2 calls of 55.3 / 55.8 / 56.5 / 59.6 us at Q = 1 / 16 /
      // 32 / 64 against 51.4 / 56.5 / 58.4 / 61.9 with rounds only -- not kept.
      uint32_t pm = 0;
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) pm |= (uint32_t)(!(fin[jj] < ltf)) << jj;
      while (__ballot(pm != 0)) {
#if defined(IRC_SCAN_STAMPS) && !defined(IRC_SCAN_NO_ROUNDS)  // diagnostic: LTOP rounds (wave 0 of blocks < 256)
        if (wave == 0 && lane == 0 && blockIdx.x < 256)
          atomicAdd((unsigned long long*)&dbg_stamps[3][28], 1ull);
#endif
        const int b = pm != 0 ? __builtin_ctz(pm) : 0;
        const bool cand = pm != 0;
        pm &= pm - 1;
        float v = fin[0];
#pragma unroll
        for (int jj = 1; jj < JPW; ++jj) v = b == jj ? fin[jj] : v;
        const int j = b + joff;
        const int s = s0row + (j & 3) + 8 * (j >> 2) + 4 * h;
        const uint64_t key = make_key(v, idx_base + (uint32_t)s * (uint32_t)stride);
        if (cand && s < NS && key > lt3) {
          lt3 = key;
          uint64_t t;
          if (lt3 > lt2) { t = lt2; lt2 = lt3; lt3 = t; }
          if (lt2 > lt1) { t = lt1; lt1 = lt2; lt2 = t; }
          if (lt1 > lt0) { t = lt0; lt0 = lt1; lt1 = t; }
          ltf = lt3 != 0 ? unorderable_f32((uint32_t)(lt3 >> 32)) : -__builtin_huge_valf();
        }
      }
    } else {
      // Float prefilter (key >= thr implies score >= qtf for non-NaN scores; NaN
      // passes it and fails the exact test): a branch-free pass mask, and the
      // exact key path only when some lane of the wave has a candidate.
      uint32_t pm = 0;
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) pm |= (uint32_t)(!(fin[jj] < qtf)) << jj;
      // set bits only: one candidate per lane per round (rounds = the wave's
      // largest candidate count, usually 0 or 1)
      while (__ballot(pm != 0)) {
        const int b = pm != 0 ? __builtin_ctz(pm) : 0;
        const bool cand = pm != 0;
        pm &= pm - 1;
        float v = fin[0];
#pragma unroll
        for (int jj = 1; jj < JPW; ++jj) v = b == jj ? fin[jj] : v;
        const int j = b + joff;
        const int s = s0row + (j & 3) + 8 * (j >> 2) + 4 * h;
        const uint64_t key = make_key(v, idx_base + (uint32_t)s * (uint32_t)stride);
        const bool keep = cand && (q < Q) && (s < NS) && key >= qthr;
#ifdef IRC_SCAN_NO_STORE  // diagnostic build: survivors counted, never stored
        if (keep) ++nsurv;
#else
        push(keep, key);
#endif
      }
    }
    nst_hist = (nst_hist << 8) | (uint64_t)(nst < 255 ? nst : 255);
    // all reads of this buffer (and of xbuf) done before reuse; with the early issue
    // the slot was released above and the next iteration's two barriers precede any
    // xbuf write
    if (!IRC_SCAN_EARLY_ISSUE) wg_barrier();
  }

  if (MODE == LTOP) {
    // dense lists: keys[((q * G_total + worker) * NL + slice) * 4 + i], cap = lists
    // per query (G_total * NL); every list written, empty slots 0.  KS = 4: the two
    // half-lanes' lists of one (query, k-slice) are merged first (top 4 of 8; every
    // doc either list dropped is below the merged last key), so NL = 4 as for KS = 2
    // and each list covers tile rows [8 kh, 8 kh + 8).
    if constexpr (KS == 4) {
      const uint64_t p0 = __shfl_xor(lt0, 32, 64), p1 = __shfl_xor(lt1, 32, 64);
      const uint64_t p2 = __shfl_xor(lt2, 32, 64), p3 = __shfl_xor(lt3, 32, 64);
      const uint64_t pv[4] = {p0, p1, p2, p3};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t key = pv[i];
        if (key > lt3) {
          lt3 = key;
          uint64_t t;
          if (lt3 > lt2) { t = lt2; lt2 = lt3; lt3 = t; }
          if (lt2 > lt1) { t = lt1; lt1 = lt2; lt2 = t; }
          if (lt1 > lt0) { t = lt0; lt0 = lt1; lt1 = t; }
        }
      }
      if (q < Q && h == 0) {
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
        u64x2* dst = reinterpret_cast<u64x2*>(
            keys + (((int64_t)q * cap + (int64_t)worker * 4 + kh) * LT_M));
        dst[0] = (u64x2){lt0, lt1};
        dst[1] = (u64x2){lt2, lt3};
      }
    } else if (q < Q) {
      typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
      u64x2* dst = reinterpret_cast<u64x2*>(
          keys + (((int64_t)q * cap + (int64_t)worker * (2 * KS) + slice) * LT_M));
      dst[0] = (u64x2){lt0, lt1};
      dst[1] = (u64x2){lt2, lt3};
    }
    STAMP(3, 1);
    BLK_STAMP(1);
    return;
  }
  if (MODE != SCORES) {  // flush the shift buffer (newest first; order is irrelevant)
    if (sbn > 0) myreg[nsurv] = sb0;
    if (sbn > 1) myreg[nsurv + 1] = sb1;
    if (sbn > 2) myreg[nsurv + 2] = sb2;
    nsurv += (uint32_t)sbn;
  }
  if (MODE != SCORES && q < Qpad)
    counts[((int64_t)worker * Qpad + q) * (2 * KS) + slice] = nsurv;
  STAMP(thr == nullptr ? 2 : 3, 1);
  BLK_STAMP(1);
}

// ----------------------------------------------------------------- selection
// Key sources for the select kernel.
// NSL (slices per region group) is a power of two (1, 2 or 4) and the slice
// capacity is precomputed: region addressing is shifts and one multiply (a
// run-time integer division costs ~40 VALU instructions, 64-bit ~100, and the
// selects address every candidate this way).
struct RegionSource {  // scan workspace: G regions per query, NSL slices each
  const uint64_t* keys;
  const uint32_t* counts;
  int G;
  int Qpad;
  int64_t cap;
  int lnsl;           // log2(NSL)
  int64_t slice_cap;  // cap / NSL
  static constexpr bool kRegions = true;
  __device__ __forceinline__ int nregions() const { return G << lnsl; }
  __device__ __forceinline__ int64_t group(int q, int r) const {
    return (int64_t)(r >> lnsl) * Qpad + q;
  }
  __device__ __forceinline__ uint32_t count(int q, int r) const {
    return counts[(group(q, r) << lnsl) + (r & ((1 << lnsl) - 1))];
  }
  __device__ __forceinline__ const uint64_t* region(int q, int r) const {
    return keys + group(q, r) * cap + (r & ((1 << lnsl) - 1)) * slice_cap;
  }
  template <class F>
  __device__ __forceinline__ void for_each(int q, int tid, int nt, F&& f) const {
    for (int r = tid; r < nregions(); r += nt) {
      const uint32_t n = count(q, r);
      const uint64_t* p = region(q, r);
      for (uint32_t j = 0; j < n; ++j) f(p[j]);
    }
  }
};

static RegionSource region_source(const uint64_t* keys, const uint32_t* counts, int G, int Qpad,
                                  int64_t cap, int nsl) {
  int l = 0;
  while ((1 << l) < nsl) ++l;
  return RegionSource{keys, counts, G, Qpad, cap, l, cap >> l};
}

struct ListSource {  // merge input: [P][Q][kin] scores + global idx (-1 = empty)
  const float* score;
  const int64_t* idx;
  int P;
  int Q;
  int kin;
  static constexpr bool kRegions = false;
  __device__ __forceinline__ int nregions() const { return 0; }
  __device__ __forceinline__ uint32_t count(int, int) const { return 0; }
  __device__ __forceinline__ const uint64_t* region(int, int) const { return nullptr; }
  template <class F>
  __device__ __forceinline__ void for_each(int q, int tid, int nt, F&& f) const {
    // (p, j) stepped incrementally: no run-time division per element
    int p = tid / kin, j = tid - p * kin;
    const int dp = nt / kin, dj = nt - dp * kin;
    for (; p < P;) {
      const int64_t off = ((int64_t)p * Q + q) * kin + j;
      const int64_t id = idx[off];
      if (id >= 0) f(make_key(score[off], (uint32_t)id));
      p += dp;
      j += dj;
      if (j >= kin) {
        j -= kin;
        ++p;
      }
    }
  }
};

constexpr int SEL_NT = 256;
constexpr int SEL_NW = SEL_NT / 64;
constexpr int SEL_MAXK = 1024;
constexpr int SEL_STAGE = 4096;  // candidates staged in LDS when they fit (32 KB)
constexpr int SEL_MAXR = 4096;   // region table size for the parallel staging path

enum SelMode { SEL_THRESHOLD = 0, SEL_FINAL = 1 };

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

// Bitonic sort (descending) of the 64*E keys one wave holds in registers,
// blocked: lane l owns indices l*E .. l*E+E-1.  Strides below E swap inside a
// lane; wider ones exchange with lane ^ (stride / E) -- no LDS, no barrier.
template <int E>
__device__ __forceinline__ void wave_sort_desc(uint64_t (&v)[E], int lane) {
  constexpr int n = 64 * E;
#pragma unroll
  for (int size = 2; size <= n; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride < E) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int ep = e ^ stride;
          if (ep > e) {
            const bool desc = ((lane * E + e) & size) == 0;
            const uint64_t x = v[e], y = v[ep];
            if (desc ? (x < y) : (x > y)) {
              v[e] = y;
              v[ep] = x;
            }
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = lane * E + e;
          const uint64_t y = __shfl_xor(v[e], stride / E, 64);
          // the lower index of a descending pair keeps the larger key
          const bool keep_max = (((i & stride) == 0) == ((i & size) == 0));
          const uint64_t hi = v[e] > y ? v[e] : y, lo = v[e] > y ? y : v[e];
          v[e] = keep_max ? hi : lo;
        }
      }
    }
  }
}

// Wave 0 of the select: sort the npow (>= cnt) collected keys and write the k
// outputs of query q (slots past cnt are empty: -inf / -1).
template <int E>
__device__ __forceinline__ void sort_and_emit(const uint64_t* cand, int cnt, int k, int q,
                                              int lane, float smul, float* __restrict__ out_score,
                                              int64_t* __restrict__ out_idx) {
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    v[e] = i < cnt ? cand[i] : 0ull;
  }
  wave_sort_desc<E>(v, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane * E + e;
    if (i < k) {
      float sc = -__builtin_huge_valf();
      int64_t id = -1;
      if (i < cnt) {
        sc = unorderable_f32((uint32_t)(v[e] >> 32)) * smul;
        id = (int64_t)(uint32_t)(~(uint32_t)v[e]);
      }
      out_score[(int64_t)q * k + i] = sc;
      out_idx[(int64_t)q * k + i] = id;
    }
  }
  for (int i = 64 * E + lane; i < k; i += 64) {
    out_score[(int64_t)q * k + i] = -__builtin_huge_valf();
    out_idx[(int64_t)q * k + i] = -1;
  }
}

// Fast path of select_body for region sources whose candidates fit the stage
// (M <= SEL_STAGE: the scan's threshold and final selects on any input short of
// adversarial skew).  Round-1 phase stamps of select_body on MI355X (C2, k = 100,
// M ~ 1.8k): 12.5 us per final select, of which 3.4 us in two radix passes that
// re-read the staged keys from LDS, 1.2 us collecting, 2.3 us in wave 0's sort.
// Here thread t's keys (i = t + 256 u of the region-id map) stay in registers
// for every pass; the histogram is double-buffered (waves 1-3 clear the next
// pass's copy while wave 0 scans), so a pass costs two barriers; the winners are
// collected with one LDS atomic per wave and placed by rank (each counts the
// winners above it over broadcast LDS reads) -- no sort.  Same keys, same k-th
// key, same outputs as the general path.
template <class Src, bool BIGK>
__device__ __forceinline__ void select_fast(const Src& src, int q, int k, int mode, uint32_t M,
                                            const uint16_t* rid, const uint32_t* roff,
                                            uint32_t* hbuf, uint64_t* cand, uint64_t* s_mm,
                                            uint32_t* s_misc, uint32_t* s_coll,
                                            uint64_t* __restrict__ thr_out,
                                            float* __restrict__ out_score,
                                            int64_t* __restrict__ out_idx, float smul) {
  constexpr int U = SEL_STAGE / SEL_NT;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  uint64_t v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t i = tid + u * SEL_NT;
    v[u] = 0;
    if (i < M) {
      const int r = rid[i];
      v[u] = src.region(q, r)[i - roff[r]];
    }
  }
  uint32_t* h0 = hbuf;
  uint32_t* h1 = hbuf + SEL_NW * 256;
  for (int i = tid; i < SEL_NW * 256; i += SEL_NT) h0[i] = 0;
  uint64_t mn = ~0ull, mx = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (tid + u * SEL_NT < M) {
      mn = v[u] < mn ? v[u] : mn;
      mx = v[u] > mx ? v[u] : mx;
    }
  }
  // the smallest of the threads' own maxima: a lower bound of the k-th key once
  // min(M, SEL_NT) >= k threads hold a key (distinct keys) -- the radix window starts
  // there instead of at the minimum (as in dense_kth: fewer keys per first-pass bin)
  const uint64_t lbw = wave_min_u64((uint32_t)tid < M ? mx : ~0ull);
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if (lane == 0) {
    s_mm[wave] = mn;
    s_mm[SEL_NW + wave] = mx;
    s_mm[2 * SEL_NW + wave] = lbw;
  }
  __syncthreads();
  STAMP(mode, 2);
  if (IRC_SCAN_SEL_STOP == 2 && mode == SEL_FINAL) return;

  uint64_t kth = 0;  // 0 = keep everything
  if (M > (uint32_t)k) {
    mn = s_mm[0];
    mx = s_mm[SEL_NW];
    uint64_t lb = s_mm[2 * SEL_NW];
#pragma unroll
    for (int w = 1; w < SEL_NW; ++w) {
      mn = s_mm[w] < mn ? s_mm[w] : mn;
      mx = s_mm[SEL_NW + w] > mx ? s_mm[SEL_NW + w] : mx;
      lb = s_mm[2 * SEL_NW + w] < lb ? s_mm[2 * SEL_NW + w] : lb;
    }
    if ((M < (uint32_t)SEL_NT ? M : (uint32_t)SEL_NT) >= (uint32_t)k) mn = lb;
    const int top = 63 - __builtin_clzll((mn ^ mx) | 1ull);
    uint64_t pmask = top >= 63 ? 0ull : (~0ull << (top + 1));
    uint64_t prefix = mn & pmask;
    uint32_t kr = (uint32_t)k;
    int hi = top;
    for (int pass = 0;; ++pass) {
      uint32_t* h = (pass & 1) ? h1 : h0;
      uint32_t* hn = (pass & 1) ? h0 : h1;
      const int lo = hi >= 7 ? hi - 7 : 0;
      const uint32_t dm = (2u << (hi - lo)) - 1u;
      uint32_t* hw = h + wave * 256;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (tid + u * SEL_NT < M && (v[u] & pmask) == prefix)
          atomicAdd(&hw[(uint32_t)(v[u] >> lo) & dm], 1u);
      __syncthreads();
      if (wave == 0) {
        uint32_t bb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t t = 0;
#pragma unroll
          for (int w = 0; w < SEL_NW; ++w) t += h[w * 256 + 4 * lane + j];
          bb[j] = t;
        }
        const uint32_t cnt4 = bb[0] + bb[1] + bb[2] + bb[3];
        uint32_t suf = cnt4;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_down(suf, o, 64);
          if (lane + o < 64) suf += t;
        }
        const uint32_t above = suf - cnt4;
        if (suf >= kr && above < kr) {
          uint32_t acc = above;
          int sel = 4 * lane, selc = 0;
          for (int j = 3; j >= 0; --j) {
            if (acc + bb[j] >= kr) {
              sel = 4 * lane + j;
              selc = (int)bb[j];
              break;
            }
            acc += bb[j];
          }
          s_misc[2] = (uint32_t)sel;
          s_misc[1] = kr - acc;
          s_misc[3] = (uint32_t)selc == kr - acc;
        }
      } else {
        for (int i = tid - 64; i < SEL_NW * 256; i += SEL_NT - 64) hn[i] = 0;
      }
      __syncthreads();
      prefix |= (uint64_t)s_misc[2] << lo;
      pmask |= (uint64_t)dm << lo;
      kr = s_misc[1];
      STAMP(mode, 4 + pass);
      if (s_misc[3] || lo == 0 || (mode == SEL_THRESHOLD && pass == 1)) break;
      hi = lo - 1;  // s_misc is rewritten only after the next pass's first barrier
    }
    kth = prefix;
  }
  if (mode == SEL_THRESHOLD) {
    if (tid == 0) thr_out[q] = kth;
    return;
  }
  STAMP(mode, 12);
  if (IRC_SCAN_SEL_STOP == 3 && mode == SEL_FINAL) return;
  // collect the exactly min(M, k) keys >= kth: one LDS atomic per wave (its U
  // ballots counted first; a returning atomic per slot serialised U round trips)
  {
    uint64_t bal[U];
    uint32_t tot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bal[u] = __ballot(tid + u * SEL_NT < M && v[u] >= kth);
      tot += (uint32_t)__popcll(bal[u]);
    }
    if (tot != 0) {  // wave-uniform
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(s_coll, tot);
      base = __shfl(base, 0, 64);
      const uint64_t below = (1ull << lane) - 1;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if ((bal[u] >> lane) & 1ull) cand[base + __popcll(bal[u] & below)] = v[u];
        base += (uint32_t)__popcll(bal[u]);
      }
    }
  }
  __syncthreads();
  STAMP(mode, 13);
  if (IRC_SCAN_SEL_STOP == 4 && mode == SEL_FINAL) return;
  const int cnt = (int)(M < (uint32_t)k ? M : (uint32_t)k);
  if (cnt <= SEL_NT) {
    // winner tid goes to its rank (keys are distinct); slots past cnt are empty
    for (int i = tid; i < k; i += SEL_NT) {
      float sc = -__builtin_huge_valf();
      int64_t id = -1;
      int pos = i;
      if (i < cnt) {
        const uint64_t key = cand[i];
        int rank = 0;
        int j = 0;
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        for (; j + 8 <= cnt; j += 8) {  // 16-byte broadcast reads, 8 keys in flight
          u64x2 c[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) c[t] = *reinterpret_cast<const u64x2*>(&cand[j + 2 * t]);
#pragma unroll
          for (int t = 0; t < 4; ++t) rank += (int)(c[t][0] > key) + (int)(c[t][1] > key);
        }
        for (; j < cnt; ++j) rank += (int)(cand[j] > key);
        pos = rank;
        sc = unorderable_f32((uint32_t)(key >> 32)) * smul;
        id = (int64_t)(uint32_t)(~(uint32_t)key);
      }
      out_score[(int64_t)q * k + pos] = sc;
      out_idx[(int64_t)q * k + pos] = id;
    }
  } else if (wave == 0) {
    if (cnt <= 512 || !BIGK) sort_and_emit<8>(cand, cnt, k, q, lane, smul, out_score, out_idx);
    else sort_and_emit<16>(cand, cnt, k, q, lane, smul, out_score, out_idx);
  }
  STAMP(mode, 14);
}

// One workgroup per query: the exact k-th largest distinct key among the
// query's candidates by radix select, then the winners sorted.
//  * Region sources: all region counts are loaded at once (each thread owns up
//    to 16 consecutive regions), block-scanned, and turned into an LDS region-id
//    map, so every candidate load is independent; the keys are staged in LDS
//    (<= SEL_STAGE) and their min / max taken on the way.
//  * Digits are 8 bits wide and start right below the candidates' common
//    prefix (the highest bit where min and max differ), not at byte
//    boundaries: the first pass already spreads the keys over the buckets.
//    Early exit when the chosen bucket holds exactly the remaining rank.
//  * SEL_THRESHOLD only needs a LOWER BOUND of the k-th key (the filter keeps
//    key >= bound, so the FINAL pass still selects exactly): two passes, bound =
//    the common prefix + 16 selected bits, lower bits zero.
//  * The min(M, k) winners are sorted in registers by wave 0 (wave_sort_desc).
// smul: power-of-two factor applied to the returned scores (fp8 descale).
// BIGK: k > 512 (the register sort then holds 16 keys per lane); the common
// build sorts at most 512 and stays light enough for two workgroups per CU.
template <class Src, bool BIGK>
__device__ __forceinline__ void select_body(Src src, int k, int mode,
                                                         uint64_t* __restrict__ thr_out,
                                                         float* __restrict__ out_score,
                                                         int64_t* __restrict__ out_idx,
                                                         float smul) {
  __shared__ uint32_t hist[SEL_NW][256];
  __shared__ __attribute__((aligned(16))) uint64_t cand[SEL_MAXK];
  __shared__ uint64_t stage[SEL_STAGE];
  __shared__ uint16_t rid[SEL_STAGE];
  __shared__ uint32_t roff[SEL_MAXR];
  __shared__ uint64_t s_mm[3][SEL_NW];  // min, max, threads' lower bound (select_fast)
  __shared__ uint32_t s_wsum[SEL_NW];
  __shared__ uint32_t s_misc[4];  // 0: total count, 1: kr, 2: selected digit, 3: staging ctr
  __shared__ uint32_t s_coll;     // collect counter
  __shared__ bool s_exact;

  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
#define SEL_STOP(n)                                                     \
  do {                                                                  \
    if (IRC_SCAN_SEL_STOP == (n) && mode == SEL_FINAL) return;          \
  } while (0)

  STAMP(mode, 0);
  SEL_STOP(0);
  if (tid == 0) {
    s_misc[0] = 0;
    s_misc[3] = 0;
    s_coll = 0;
  }
  bool table = false;
  uint32_t M = 0;
  if constexpr (Src::kRegions) {
    const int R = src.nregions();
    table = R <= SEL_MAXR;
    if (table) {
      const int rpt = (R + SEL_NT - 1) / SEL_NT;  // <= 16
      uint32_t c[16];
      uint32_t mine = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = tid * rpt + u;
        c[u] = (u < rpt && r < R) ? src.count(q, r) : 0u;
        mine += c[u];
      }
      uint32_t incl = mine;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (lane == 63) s_wsum[wave] = incl;
      __syncthreads();
      uint32_t off = incl - mine;
#pragma unroll
      for (int w = 0; w < SEL_NW; ++w) {
        if (w < wave) off += s_wsum[w];
        M += s_wsum[w];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = tid * rpt + u;
        if (u < rpt && r < R) {
          roff[r] = off;
          if (M <= (uint32_t)SEL_STAGE)
            for (uint32_t j = 0; j < c[u]; ++j) rid[off + j] = (uint16_t)r;
          off += c[u];
        }
      }
    }
  }
  if (!table) {
    __syncthreads();
    uint32_t c = 0;
    src.for_each(q, tid, SEL_NT, [&](uint64_t) { ++c; });
    atomicAdd(&s_misc[0], c);
    __syncthreads();
    M = s_misc[0];
  }
  const bool staged = M <= (uint32_t)SEL_STAGE;
  __syncthreads();
  STAMP(mode, 1);
  SEL_STOP(1);
  if constexpr (Src::kRegions) {
    if (table && staged) {
      select_fast<Src, BIGK>(src, q, k, mode, M, rid, roff,
                             reinterpret_cast<uint32_t*>(stage), cand, &s_mm[0][0], s_misc,
                             &s_coll, thr_out, out_score, out_idx, smul);
      return;
    }
  }
  uint64_t mn = ~0ull, mx = 0;
  if (staged) {
    if (table) {
      constexpr int U = 8;  // independent loads in flight per thread
      for (uint32_t i0 = tid; i0 < M; i0 += SEL_NT * U) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = i0 + u * SEL_NT;
          if (i < M) {
            const int r = rid[i];
            v[u] = src.region(q, r)[i - roff[r]];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t i = i0 + u * SEL_NT;
          if (i < M) {
            stage[i] = v[u];
            mn = v[u] < mn ? v[u] : mn;
            mx = v[u] > mx ? v[u] : mx;
          }
        }
      }
    } else {
      src.for_each(q, tid, SEL_NT, [&](uint64_t key) {
        stage[atomicAdd(&s_misc[3], 1u)] = key;
        mn = key < mn ? key : mn;
        mx = key > mx ? key : mx;
      });
    }
  }
  auto visit = [&](auto&& f) {
    if (staged) {
      for (uint32_t i = tid; i < M; i += SEL_NT) f(stage[i]);
    } else {
      src.for_each(q, tid, SEL_NT, f);
    }
  };
  if (!staged && M > (uint32_t)k)
    visit([&](uint64_t key) {
      mn = key < mn ? key : mn;
      mx = key > mx ? key : mx;
    });
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if (lane == 0) {
    s_mm[0][wave] = mn;
    s_mm[1][wave] = mx;
  }
  __syncthreads();
  STAMP(mode, 2);
#ifdef IRC_SCAN_STAMPS
  if (blockIdx.x == 0 && tid == 0) *(volatile uint64_t*)&dbg_stamps[mode][21 + (tid & 0)] = M;
#endif

  uint64_t kth = 0;  // 0 = keep everything
  if (M > (uint32_t)k) {
    mn = s_mm[0][0];
    mx = s_mm[1][0];
#pragma unroll
    for (int w = 1; w < SEL_NW; ++w) {
      mn = s_mm[0][w] < mn ? s_mm[0][w] : mn;
      mx = s_mm[1][w] > mx ? s_mm[1][w] : mx;
    }
    const int top = 63 - __builtin_clzll((mn ^ mx) | 1ull);  // highest differing bit
    uint64_t pmask = top >= 63 ? 0ull : (~0ull << (top + 1));
    uint64_t prefix = mn & pmask;
    uint32_t kr = (uint32_t)k;
    int hi = top;
    for (int pass = 0;; ++pass) {
      const int lo = hi >= 7 ? hi - 7 : 0;
      const uint32_t dm = (2u << (hi - lo)) - 1u;  // digit = bits [lo, hi]
      for (int i = tid; i < SEL_NW * 256; i += SEL_NT) (&hist[0][0])[i] = 0;
      __syncthreads();
      visit([&](uint64_t key) {
        if ((key & pmask) == prefix) atomicAdd(&hist[wave][(uint32_t)(key >> lo) & dm], 1u);
      });
      __syncthreads();
      if (wave == 0) {
        // lane covers digits 4*lane .. 4*lane+3; suffix-scan from the top digit.
        uint32_t bb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t t = 0;
#pragma unroll
          for (int w = 0; w < SEL_NW; ++w) t += hist[w][4 * lane + j];
          bb[j] = t;
        }
        const uint32_t cnt4 = bb[0] + bb[1] + bb[2] + bb[3];
        uint32_t suf = cnt4;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = __shfl_down(suf, o, 64);
          if (lane + o < 64) suf += t;
        }
        const uint32_t above = suf - cnt4;  // count in digits of higher lanes
        if (suf >= kr && above < kr) {
          uint32_t acc = above;
          int sel = 4 * lane, selc = 0;
          for (int j = 3; j >= 0; --j) {
            if (acc + bb[j] >= kr) {
              sel = 4 * lane + j;
              selc = (int)bb[j];
              break;
            }
            acc += bb[j];
          }
          s_misc[2] = (uint32_t)sel;
          s_misc[1] = kr - acc;
          s_exact = (uint32_t)selc == kr - acc;  // the bucket holds exactly the rest
        }
      }
      __syncthreads();
      prefix |= (uint64_t)s_misc[2] << lo;
      pmask |= (uint64_t)dm << lo;
      kr = s_misc[1];
      STAMP(mode, 4 + pass);
      // Early exit: the chosen bucket holds exactly the remaining rank, so every
      // key with this prefix is selected and prefix (lower bits zero) admits
      // exactly k keys.  THRESHOLD stops after two digits (a lower bound).
      if (s_exact || lo == 0 || (mode == SEL_THRESHOLD && pass == 1)) break;
      hi = lo - 1;  // (wave 0 rewrites s_misc only two barriers later)
    }
    kth = prefix;
  }

  if (mode == SEL_THRESHOLD) {
    if (tid == 0) thr_out[q] = kth;
    return;
  }

  STAMP(mode, 12);
  // collect the (exactly min(M, k)) keys >= kth
  const int cnt = (int)(M < (uint32_t)k ? M : (uint32_t)k);
  visit([&](uint64_t key) {
    if (key >= kth) {
      const uint32_t slot = atomicAdd(&s_coll, 1u);
      if (slot < (uint32_t)SEL_MAXK) cand[slot] = key;
    }
  });
  __syncthreads();
  STAMP(mode, 13);
  if (wave == 0) {
    if (cnt <= 64) sort_and_emit<1>(cand, cnt, k, q, lane, smul, out_score, out_idx);
    else if (cnt <= 128) sort_and_emit<2>(cand, cnt, k, q, lane, smul, out_score, out_idx);
    else if (cnt <= 256) sort_and_emit<4>(cand, cnt, k, q, lane, smul, out_score, out_idx);
    else if (cnt <= 512 || !BIGK) sort_and_emit<8>(cand, cnt, k, q, lane, smul, out_score, out_idx);
    else sort_and_emit<16>(cand, cnt, k, q, lane, smul, out_score, out_idx);
  }
  STAMP(mode, 14);
}

template <class Src>
__global__ __launch_bounds__(SEL_NT) __attribute__((amdgpu_waves_per_eu(2)))
void select_kernel(Src src, int k, int mode, uint64_t* __restrict__ thr_out,
                   float* __restrict__ out_score, int64_t* __restrict__ out_idx, float smul) {
  select_body<Src, false>(src, k, mode, thr_out, out_score, out_idx, smul);
}

template <class Src>
__global__ __launch_bounds__(SEL_NT) void select_kernel_bigk(Src src, int k, int mode,
                                                             uint64_t* __restrict__ thr_out,
                                                             float* __restrict__ out_score,
                                                             int64_t* __restrict__ out_idx,
                                                             float smul) {
  select_body<Src, true>(src, k, mode, thr_out, out_score, out_idx, smul);
}

// ------------------------------------------------------------- select_dense
// Final select of the single-pass LTOP scan (no sample pass, no threshold
// select).  Per query: LS lists of LT_M keys (one per (worker, slice)), dense.
//  1. kth = the exact k-th largest nonzero key of all lists -- a LOWER bound of
//     the true k-th key (a subset's k-th key is never larger).
//  2. A list whose last slot holds a key >= kth may have dropped a winner: its
//     worker is rescanned -- every doc of the worker's tiles scored again with
//     the filter's own MFMA sequence (same operands, same k order, same two
//     k-slice partial sums added), so the keys are bit-identical -- and the
//     worker's lists are replaced by its keys >= the running bound.  The
//     rescanned keys are held in LDS; when the buffer fills, the union is cut to
//     its k-th key (a new, higher bound) and the scan goes on.
//  3. The exact top-k of the union, ranked as in select_fast.
// On random data a rescan is rare (each list holds ~0.1 winners on average at
// C2); a corpus sorted or clustered by score triggers it, at a cost, never a
// wrong result.
struct DenseArgs {
  const uint64_t* lists;          // [Q][LS][LT_M]
  const unsigned char* queries;   // [Q][D] elements of EB bytes
  const unsigned char* docs;      // [NS][D]
  int LS;                         // lists per query (workers * 2KS), LS * LT_M <= SEL_STAGE
  int NS;
  int tpw;                        // tiles (of TD docs) per worker
  uint32_t idx_base;
  int k;
  float smul;
  float* out_score;
  int64_t* out_idx;
};
constexpr int SD_XCAP = 2048;  // rescanned keys held at once (>= SEL_MAXK + 4 * TD)
// [queries whose select rescanned, workers rescanned] since the last reset
// (irc_scan_rescan_stats): one vector atomic pair per query that rescans.
__device__ unsigned long long g_dense_rescans[2];
constexpr int SD_DCAP = 2048;  // docs listed per rescan phase (64 tiles x 32 rows)

// Exact k-th largest nonzero key of v[] (registers, slot i = tid + 256 u) and
// xk[0, xn) (LDS); 0 when there are <= k of them.  Block-wide, every thread
// returns it.  *total = the number of nonzero keys.
template <int U>
__device__ uint64_t dense_kth(const uint64_t (&v)[U], const uint64_t* xk, uint32_t xn, int k,
                              uint32_t* hbuf, uint64_t* s_mm, uint32_t* s_cnt, uint32_t* s_misc,
                              uint32_t* total) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  uint32_t c = 0;
  uint64_t mn = ~0ull, mx = 0;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (v[u] != 0) {
      ++c;
      mn = v[u] < mn ? v[u] : mn;
      mx = v[u] > mx ? v[u] : mx;
    }
  for (uint32_t i = tid; i < xn; i += SEL_NT) {
    const uint64_t x = xk[i];
    ++c;
    mn = x < mn ? x : mn;
    mx = x > mx ? x : mx;
  }
  // Lower bound of the k-th key that is tighter than the minimum: the smallest of the
  // threads' own maxima.  Those are distinct keys, so once at least k threads hold a
  // key, k keys are >= it.  The radix passes then start at the top bit in which it and
  // the maximum differ -- on the global [min, max] the first digit put most keys in a
  // few bins, and their LDS atomics serialised (pass 0 4.3 us of the 12 us select at
  // Q = 1, profiles/r03_dense_t.txt; 1.6 us and one pass instead of two after it,
  // r03_dense_u.txt).  Keys below the window's prefix are below the k-th key and are
  // not counted: the same exact k-th key.
  const uint64_t tmax = c ? mx : ~0ull;
  const uint32_t nthr = (uint32_t)__popcll(__ballot(c != 0));
  uint32_t* h0 = hbuf;
  uint32_t* h1 = hbuf + SEL_NW * 256;
  for (int i = tid; i < SEL_NW * 256; i += SEL_NT) h0[i] = 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  const uint64_t lbw = wave_min_u64(tmax);
  if (lane == 0) {
    s_mm[wave] = mn;
    s_mm[SEL_NW + wave] = mx;
    s_mm[2 * SEL_NW + wave] = lbw;
    s_cnt[wave] = c;
    s_cnt[SEL_NW + wave] = nthr;
  }
  __syncthreads();
  uint32_t M = 0, nt = 0;
  mn = s_mm[0];
  mx = s_mm[SEL_NW];
  uint64_t lb = s_mm[2 * SEL_NW];
#pragma unroll
  for (int w = 0; w < SEL_NW; ++w) {
    M += s_cnt[w];
    nt += s_cnt[SEL_NW + w];
    mn = s_mm[w] < mn ? s_mm[w] : mn;
    mx = s_mm[SEL_NW + w] > mx ? s_mm[SEL_NW + w] : mx;
    lb = s_mm[2 * SEL_NW + w] < lb ? s_mm[2 * SEL_NW + w] : lb;
  }
  *total = M;
  STAMP(2, 25);
  if (M <= (uint32_t)k) return 0;
  if (nt >= (uint32_t)k) mn = lb;  // else the global minimum
  const int top = 63 - __builtin_clzll((mn ^ mx) | 1ull);
  uint64_t pmask = top >= 63 ? 0ull : (~0ull << (top + 1));
  uint64_t prefix = mn & pmask;
  uint32_t kr = (uint32_t)k;
  int hi = top;
  for (int pass = 0;; ++pass) {
    uint32_t* h = (pass & 1) ? h1 : h0;
    uint32_t* hn = (pass & 1) ? h0 : h1;
    const int lo = hi >= 7 ? hi - 7 : 0;
    const uint32_t dm = (2u << (hi - lo)) - 1u;
    uint32_t* hw = h + wave * 256;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (v[u] != 0 && (v[u] & pmask) == prefix) atomicAdd(&hw[(uint32_t)(v[u] >> lo) & dm], 1u);
    for (uint32_t i = tid; i < xn; i += SEL_NT) {
      const uint64_t x = xk[i];
      if ((x & pmask) == prefix) atomicAdd(&hw[(uint32_t)(x >> lo) & dm], 1u);
    }
    __syncthreads();
    if (wave == 0) {
      uint32_t bb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < SEL_NW; ++w) t += h[w * 256 + 4 * lane + j];
        bb[j] = t;
      }
      const uint32_t cnt4 = bb[0] + bb[1] + bb[2] + bb[3];
      uint32_t suf = cnt4;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += t;
      }
      const uint32_t above = suf - cnt4;
      if (suf >= kr && above < kr) {
        uint32_t acc = above;
        int sel = 4 * lane, selc = 0;
        for (int j = 3; j >= 0; --j) {
          if (acc + bb[j] >= kr) {
            sel = 4 * lane + j;
            selc = (int)bb[j];
            break;
          }
          acc += bb[j];
        }
        s_misc[2] = (uint32_t)sel;
        s_misc[1] = kr - acc;
        s_misc[3] = (uint32_t)selc == kr - acc;
      }
    } else {
      for (int i = tid - 64; i < SEL_NW * 256; i += SEL_NT - 64) hn[i] = 0;
    }
    __syncthreads();
    prefix |= (uint64_t)s_misc[2] << lo;
    pmask |= (uint64_t)dm << lo;
    kr = s_misc[1];
    const bool done = s_misc[3] || lo == 0;
    __syncthreads();  // s_misc is rewritten by the next pass (or the next call)
#ifdef IRC_SCAN_STAMPS  // diagnostic: radix passes of block 0's last dense_kth
    if (blockIdx.x == 0 && tid == 0) *(volatile uint64_t*)&dbg_stamps[2][24] = (uint64_t)pass + 1;
    if (pass < 2) STAMP(2, 26 + pass);
#endif
    if (done) break;
    hi = lo - 1;
  }
  return prefix;
}

// Scores of up to TD docs (ids dl[0, n)) against query q, as scan_tile_kernel
// computes them: the same MFMA sequence over the same operand bytes, the two
// k-slice partial sums added -- bit-identical (an MFMA row's result does not
// depend on the other rows).  Lane (r32, h) returns rows (j & 3) + 8 (j >> 2) + 4 h
// of column 0 in acc[j] (lanes 0 and 32 hold the query's column).
template <int D, int EB, int KS>
__device__ __forceinline__ f32x16 rescore_docs(const unsigned char* qlds,
                                               const unsigned char* __restrict__ docs,
                                               const uint32_t* dl, int n, int lane) {
  using G = Geo<D, EB, KS>;
  f32x16 part[KS == 4 ? 4 : 1];
  constexpr int NCW = (G::KK / KS) * EB / 2;
  const int r32 = lane & 31, h = lane >> 5;
  const bool live = r32 < n;
  const unsigned char* dr = docs + (int64_t)(live ? dl[r32] : 0u) * D * EB + 16 * h;
  const unsigned char* qr = qlds + 16 * h;
  f32x16 tot = (f32x16)0.0f;
#pragma unroll
  for (int kh = 0; kh < KS; ++kh) {
    f32x16 acc = (f32x16)0.0f;
    u16x8 af[NCW];  // the k-slice's A fragments, all in flight at once
#pragma unroll
    for (int c = 0; c < NCW; ++c)
      af[c] = live ? *reinterpret_cast<const u16x8*>(dr + kh * (D * EB / KS) + c * 32) : (u16x8)0;
#pragma unroll
    for (int c = 0; c < NCW; ++c) {
      const int off = kh * (D * EB / KS) + c * 32;
      const u16x8 av = af[c];
      u16x8 bv = *reinterpret_cast<const u16x8*>(qr + off);
      if (r32 != 0) bv = (u16x8)0;
      if constexpr (EB == 2) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av),
                                                      __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
      } else {
        typedef long l2 __attribute__((ext_vector_type(2)));
        const l2 a2 = __builtin_bit_cast(l2, av), b2 = __builtin_bit_cast(l2, bv);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a2[0], b2[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a2[1], b2[1], acc, 0, 0, 0);
      }
    }
    if constexpr (KS == 4) {
      part[kh] = acc;
    } else {
      if (kh == 0) tot = acc;
      else tot += acc;  // the filter's exchange: fl(half 0 + half 1), commutative
    }
  }
  if constexpr (KS == 4) tot = (part[0] + part[2]) + (part[1] + part[3]);  // the butterfly's order
  return tot;
}

// Score of doc dl[lane] (lanes 0-31, lane < n) against the query in qlds, as the GEMM
// filter (gemm_pp_kernel<EPI_SCAN>, the single-pass form at Q in (64, 256]) computes
// it: the same MFMA (v_mfma_f32_16x16x32_bf16; e4m3: v_mfma_scale_f32_16x16x128_f8f6f4
// with unit scales), the same per-lane k chunks and the same K-tile order from a zero
// accumulator -- bit-identical, since an output element depends only on its own row
// and column.  All 16 A rows carry the query; docs 0-15 / 16-31 are the B columns of
// two accumulators, and lane l reads element 0 (row 4 (l >> 4) of column l & 15) of
// the block that holds doc l.
template <int D, int EB>
__device__ __forceinline__ float rescore_docs_pp(const unsigned char* qlds,
                                                 const unsigned char* __restrict__ docs,
                                                 const uint32_t* dl, int n, int lane) {
  const int c = lane & 15, q4 = (lane >> 4) & 3;
  const bool l0 = c < n, l1 = 16 + c < n;
  const unsigned char* d0 = docs + (int64_t)(l0 ? dl[c] : 0u) * D * EB;
  const unsigned char* d1 = docs + (int64_t)(l1 ? dl[16 + c] : 0u) * D * EB;
  f32x4 acc0 = (f32x4)0.0f, acc1 = (f32x4)0.0f;
  if constexpr (EB == 2) {
#pragma unroll 4
    for (int kt = 0; kt < D / 64; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int off = (kt * 64 + 32 * s + 8 * q4) * 2;
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(qlds + off);
        const bf16x8 b0 = l0 ? *reinterpret_cast<const bf16x8*>(d0 + off) : (bf16x8)0;
        const bf16x8 b1 = l1 ? *reinterpret_cast<const bf16x8*>(d1 + off) : (bf16x8)0;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b1, acc1, 0, 0, 0);
      }
  } else {
    typedef int v8i32_t __attribute__((ext_vector_type(8)));
#pragma unroll 2
    for (int kt = 0; kt < D / 128; ++kt) {
      const int o0 = kt * 128 + 16 * q4, o1 = o0 + 64;
      const u16x8 a2[2] = {*reinterpret_cast<const u16x8*>(qlds + o0),
                           *reinterpret_cast<const u16x8*>(qlds + o1)};
      const u16x8 z = (u16x8)0;
      const u16x8 b02[2] = {l0 ? *reinterpret_cast<const u16x8*>(d0 + o0) : z,
                            l0 ? *reinterpret_cast<const u16x8*>(d0 + o1) : z};
      const u16x8 b12[2] = {l1 ? *reinterpret_cast<const u16x8*>(d1 + o0) : z,
                            l1 ? *reinterpret_cast<const u16x8*>(d1 + o1) : z};
      const v8i32_t av = __builtin_bit_cast(v8i32_t, a2);
      acc0 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
          av, __builtin_bit_cast(v8i32_t, b02), acc0, 0, 0, 0, 127, 0, 127);
      acc1 = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
          av, __builtin_bit_cast(v8i32_t, b12), acc1, 0, 0, 0, 127, 0, 127);
    }
  }
  return lane < 16 ? acc0[0] : acc1[0];
}

// Tile rows covered by list `sl` of a worker (slice kh * 2 + h for KS <= 2: rows
// (j & 3) + 8 (j >> 2) + 4 h, j in kh's share of the 16 registers; KS = 4: the merged
// half-lane lists, rows [8 sl, 8 sl + 8)).
template <int KS>
__device__ __forceinline__ uint32_t list_rows(int sl) {
  if constexpr (KS == 0) {  // GEMM-filter lists: one per 256-doc tile, every row
    return 0xFFFFFFFFu;
  } else if constexpr (KS == 4) {
    return 0xFFu << (8 * sl);
  } else {
    const int kh = sl >> 1, hh = sl & 1;
    constexpr int JPW = 16 / KS;
    uint32_t rows = 0;
    for (int j = kh * JPW; j < (kh + 1) * JPW; ++j) rows |= 1u << ((j & 3) + 8 * (j >> 2) + 4 * hh);
    return rows;
  }
}

// KS = 0: the lists of the GEMM filter's single-pass form (one list per 256-doc
// tile = worker of tpw = 8 TD-tiles; rescans with rescore_docs_pp).
template <int D, int EB, int KS>
__global__ __launch_bounds__(SEL_NT) void select_dense_kernel(DenseArgs a) {
  constexpr int NSL = KS == 0 ? 1 : (KS == 4 ? 4 : 2 * KS);  // lists per worker
  constexpr int U = SEL_STAGE / SEL_NT;
  constexpr int MAXW = SEL_STAGE / (LT_M * NSL);  // workers
  __shared__ uint32_t hbuf[2 * SEL_NW * 256];
  __shared__ __attribute__((aligned(16))) uint64_t cand[SEL_MAXK];
  __shared__ uint64_t xk[SD_XCAP];
  __shared__ uint64_t s_mm[3 * SEL_NW];
  __shared__ uint32_t s_cnt[2 * SEL_NW];
  __shared__ uint32_t s_misc[4];
  __shared__ uint32_t s_xn, s_coll, s_nv;
  __shared__ uint32_t vflag[MAXW];  // per worker: tile rows of its truncated lists
  __shared__ uint16_t vw[MAXW];
  __shared__ __attribute__((aligned(16))) unsigned char qlds[D * EB];
  __shared__ uint32_t dl[SD_DCAP];  // docs to rescore
  __shared__ uint32_t s_nd;
  const int q = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int M4 = a.LS * LT_M;
  const uint64_t* L = a.lists + (int64_t)q * M4;
  STAMP(2, 16);
  uint64_t v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = tid + u * SEL_NT;
    v[u] = i < M4 ? L[i] : 0ull;
  }
  const int nworkers = a.LS / NSL;
  for (int w = tid; w < nworkers; w += SEL_NT) vflag[w] = 0;
  if (tid == 0) {
    s_xn = 0;
    s_coll = 0;
    s_nv = 0;
  }
  uint32_t M = 0;
  uint64_t kth = dense_kth<U>(v, xk, 0, a.k, hbuf, s_mm, s_cnt, s_misc, &M);
  STAMP(2, 17);
  // lists whose last slot could have pushed out a winner -> the tile rows they
  // cover (slice kh * 2 + h: rows (j & 3) + 8 (j >> 2) + 4 h, j in kh's half)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = tid + u * SEL_NT;
    if ((i & (LT_M - 1)) == LT_M - 1 && i < M4 && v[u] != 0 && v[u] >= kth)
      atomicOr(&vflag[(i / LT_M) / NSL], list_rows<KS>((i / LT_M) % NSL));
  }
  __syncthreads();
  for (int w = tid; w < nworkers; w += SEL_NT)
    if (vflag[w]) vw[atomicAdd(&s_nv, 1u)] = (uint16_t)w;
  __syncthreads();
  const int nv = (int)s_nv;
  STAMP(2, 18);
  if (nv > 0 && tid == 0) {
    atomicAdd(&g_dense_rescans[0], 1ull);
    atomicAdd(&g_dense_rescans[1], (unsigned long long)nv);
  }
#ifdef IRC_SCAN_STAMPS  // diagnostic: rescanned workers, queries with a rescan
  if (tid == 0) {
    atomicAdd((unsigned long long*)&dbg_stamps[3][30], (unsigned long long)nv);
    atomicAdd((unsigned long long*)&dbg_stamps[3][31], (unsigned long long)(nv > 0));
  }
#endif
  if (nv > 0) {  // block-uniform
#pragma unroll
    for (int u = 0; u < U; ++u) {  // truncated lists: replaced by the rescan of their rows
      const int i = tid + u * SEL_NT;
      // the lists' row sets are disjoint: any overlap with the flags marks this one
      if (i < M4 && (vflag[(i / LT_M) / NSL] & list_rows<KS>((i / LT_M) % NSL)) != 0) v[u] = 0;
    }
    uint64_t thr = kth;
    const int ntiles = (a.NS + TD - 1) / TD;
    const int units = nv * a.tpw;  // (violated worker, tile) pairs
    {  // the query row, read by every rescan from LDS
      const unsigned char* qrow = a.queries + (int64_t)q * D * EB;
      for (int i = tid; i < D * EB / 16; i += SEL_NT)
        reinterpret_cast<u16x8*>(qlds)[i] = reinterpret_cast<const u16x8*>(qrow)[i];
    }
    // phases of <= SD_DCAP / TD units: list the docs of the truncated lists' rows,
    // then score them in dense 32-doc MFMA tiles, SEL_NW tiles per round
    for (int u0 = 0; u0 < units; u0 += SD_DCAP / TD) {
      if (tid == 0) s_nd = 0;
      __syncthreads();
      const int u1 = u0 + SD_DCAP / TD < units ? u0 + SD_DCAP / TD : units;
      for (int u = u0 + tid; u < u1; u += SEL_NT) {
        const int w = vw[u / a.tpw];
        const int tile = w * a.tpw + u % a.tpw;
        if (tile >= ntiles) continue;
        uint32_t rows = vflag[w];
        const int rem = a.NS - tile * TD;
        if (rem < TD) rows &= (1u << rem) - 1u;
        uint32_t o = atomicAdd(&s_nd, (uint32_t)__popc(rows));
        while (rows) {
          const int r = __builtin_ctz(rows);
          rows &= rows - 1u;
          dl[o++] = (uint32_t)(tile * TD + r);
        }
      }
      __syncthreads();
      const int nd = (int)s_nd;
      for (int c0 = 0; c0 < nd; c0 += SEL_NW * TD) {
        if (s_xn + SEL_NW * TD > (uint32_t)SD_XCAP) {
          // cut the union to its k-th key: a higher bound, at most k keys kept in xk
          uint32_t tot;
          const uint64_t kc = dense_kth<U>(v, xk, s_xn, a.k, hbuf, s_mm, s_cnt, s_misc, &tot);
          thr = kc > thr ? kc : thr;
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (v[u] < thr) v[u] = 0;
          const uint32_t xn0 = s_xn;
          for (uint32_t i = tid; i < xn0; i += SEL_NT)
            if (xk[i] >= thr) cand[atomicAdd(&s_coll, 1u)] = xk[i];
          __syncthreads();
          const uint32_t nk = s_coll;
          for (uint32_t i = tid; i < nk; i += SEL_NT) xk[i] = cand[i];
          __syncthreads();
          if (tid == 0) {
            s_xn = nk;
            s_coll = 0;
          }
          __syncthreads();
        }
        const int c = c0 + wave * TD;
        if constexpr (KS == 0) {
          if (c < nd) {  // wave-uniform
            const int n = nd - c < TD ? nd - c : TD;
            const float sc = rescore_docs_pp<D, EB>(qlds, a.docs, dl + c, n, lane);
            const uint64_t kk = lane < n ? make_key(sc, a.idx_base + dl[c + lane]) : 0ull;
            const bool keep = kk != 0 && kk >= thr;
            const uint64_t bal = __ballot(keep);
            uint32_t o = 0;
            if (lane == 0 && bal) o = atomicAdd(&s_xn, (uint32_t)__popcll(bal));
            o = __shfl(o, 0, 64);
            if (keep) xk[o + __popcll(bal & ((1ull << lane) - 1))] = kk;
          }
        } else if (c < nd) {
          const int n = nd - c < TD ? nd - c : TD;
          const f32x16 sc = rescore_docs<D, EB, KS>(qlds, a.docs, dl + c, n, lane);
          if ((lane & 31) == 0) {
            const int h = lane >> 5;
            uint64_t kk[16];
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const int r = (j & 3) + 8 * (j >> 2) + 4 * h;
              kk[j] = r < n ? make_key(sc[j], a.idx_base + dl[c + r]) : 0ull;
              cnt += (int)(kk[j] != 0 && kk[j] >= thr);
            }
            uint32_t o = cnt ? atomicAdd(&s_xn, (uint32_t)cnt) : 0u;
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if (kk[j] != 0 && kk[j] >= thr) xk[o++] = kk[j];
          }
        }
        __syncthreads();
      }
    }
    kth = dense_kth<U>(v, xk, s_xn, a.k, hbuf, s_mm, s_cnt, s_misc, &M);
  }
  STAMP(2, 19);
  // collect the exactly min(M, k) keys >= kth, then place them by rank.  The wave's
  // U ballots are counted first, so it takes its cand range with ONE LDS atomic (a
  // returning atomic per ballot serialised 16 round trips: ~1.3 us of the 12 us select
  // at Q = 1, profiles/r03_dense_s.txt); the order inside cand is irrelevant (ranked).
  const uint32_t xn = s_xn;
  {
    uint64_t bal[U];
    uint32_t tot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bal[u] = __ballot(v[u] != 0 && v[u] >= kth);
      tot += (uint32_t)__popcll(bal[u]);
    }
    if (tot != 0) {  // wave-uniform
      uint32_t b0 = 0;
      if (lane == 0) b0 = atomicAdd(&s_coll, tot);
      b0 = __shfl(b0, 0, 64);
      const uint64_t below = (1ull << lane) - 1;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if ((bal[u] >> lane) & 1ull) cand[b0 + __popcll(bal[u] & below)] = v[u];
        b0 += (uint32_t)__popcll(bal[u]);
      }
    }
  }
  for (uint32_t i = tid; i < xn; i += SEL_NT)
    if (xk[i] >= kth) cand[atomicAdd(&s_coll, 1u)] = xk[i];
  __syncthreads();
  const int k = a.k;  // <= SEL_NT (make_plan): one winner per thread at most
  const int cnt = (int)(M < (uint32_t)k ? M : (uint32_t)k);
  {
    for (int i = tid; i < k; i += SEL_NT) {
      float sc = -__builtin_huge_valf();
      int64_t id = -1;
      int pos = i;
      if (i < cnt) {
        const uint64_t key = cand[i];
        // rank = keys above this one: 16-byte broadcast reads, 8 keys per step in
        // flight (the one-key loop was LDS-latency bound, ~2 us at k = 100)
        int rank = 0, j = 0;
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        for (; j + 8 <= cnt; j += 8) {
          u64x2 c[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) c[t] = *reinterpret_cast<const u64x2*>(&cand[j + 2 * t]);
#pragma unroll
          for (int t = 0; t < 4; ++t) rank += (int)(c[t][0] > key) + (int)(c[t][1] > key);
        }
        for (; j < cnt; ++j) rank += (int)(cand[j] > key);
        pos = rank;
        sc = unorderable_f32((uint32_t)(key >> 32)) * a.smul;
        id = (int64_t)(uint32_t)(~(uint32_t)key);
      }
      a.out_score[(int64_t)q * k + pos] = sc;
      a.out_idx[(int64_t)q * k + pos] = id;
    }
  }
  STAMP(2, 20);
}

// One 256-thread workgroup per query (a wave-per-query variant made the whole call
// 40 us slower at Q = 1 and 35 us at Q = 256 on MI355X, 100k x 768, k = 100: one wave
// walked every region and every radix pass alone; removed in round 6).
static void launch_select(const RegionSource& src, int Q, int k, int mode, uint64_t* thr,
                          float* out_score, int64_t* out_idx, float smul, hipStream_t st) {
  if (k > 512)
      hipLaunchKernelGGL((select_kernel_bigk<RegionSource>), dim3((unsigned)Q), dim3(SEL_NT), 0,
                         st, src, k, mode, thr, out_score, out_idx, smul);
    else
      hipLaunchKernelGGL((select_kernel<RegionSource>), dim3((unsigned)Q), dim3(SEL_NT), 0, st,
                         src, k, mode, thr, out_score, out_idx, smul);
}

// Threshold of the sampled pipeline from the GEMM kernel's sample lists (the 4
// largest keys of every (256-doc sample tile, query)): thr[q] = the exact k-th largest
// nonzero key of the query's LS * 4 list keys -- real keys of k distinct docs, so a
// lower bound of the true k-th key -- or 0 (admit everything) when there are <= k.
__global__ __launch_bounds__(SEL_NT) void lists_kth_kernel(const uint64_t* __restrict__ lists,
                                                           int LS, int k, uint64_t* thr) {
  constexpr int U = SEL_STAGE / SEL_NT;
  __shared__ uint32_t hbuf[2 * SEL_NW * 256];
  __shared__ uint64_t s_mm[3 * SEL_NW];
  __shared__ uint32_t s_cnt[2 * SEL_NW];
  __shared__ uint32_t s_misc[4];
  const int q = blockIdx.x, tid = threadIdx.x;
  const int M4 = LS * LT_M;
  const uint64_t* L = lists + (int64_t)q * M4;
  uint64_t v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = tid + u * SEL_NT;
    v[u] = i < M4 ? L[i] : 0ull;
  }
  uint32_t M = 0;
  const uint64_t kth = dense_kth<U>(v, nullptr, 0, k, hbuf, s_mm, s_cnt, s_misc, &M);
  if (tid == 0) thr[q] = kth;
}

// ------------------------------------------------------------------ planning
struct Plan {
  int nw;  // waves = nq * ks
  int nq;  // 32-query groups per workgroup
  int ks;  // k-slices (D split across a wave pair)
  int qpad;
  int gy;
  bool two_phase;
  int64_t stride;  // sample stride
  int64_t S;       // sample size
  int g_s, tpw_s;
  int64_t cap_s;
  int g_f, tpw_f;
  int64_t cap_f;
  // single-pass LTOP scan + select_dense (no sample, no threshold select)
  bool ltop;
  int ls;  // lists per query
  // filter pass on the ping-pong GEMM (Q >= pp_min_q): regions = 256-doc tiles
  bool pp;
  // single pass on the ping-pong GEMM (Q in [ppl_min_q, 256]): lists of the 4 largest
  // keys per (256-doc tile, query), select_dense<KS = 0>; no sample, no threshold
  bool ppl;
  int pp_sG;  // 256-doc tiles of the threshold sample on the GEMM kernel (pp two-phase)
  int pp_G, pp_qpad;
  int64_t pp_cap;
  size_t off_thr, off_cnt, off_keys, bytes;
};

// IRC_SCAN_PP_MINQ sets the GEMM-kernel filter's Q floor (default 192; a value above
// every Q keeps the stationary-query kernel at every Q); IRC_SCAN_PP_MAX_GB caps its
// survivor workspace (256 slots per (256-doc tile,
// query) region: exact for any input, 8 KB x Q x N/256; default 24 GB of the
// 288 GB HBM, i.e. up to Q = 2048 over a 1.5M-doc shard).
static size_t pp_max_bytes() {
  static const size_t v = [] {
    const char* e = getenv("IRC_SCAN_PP_MAX_GB");
    return (size_t)((e ? atof(e) : 24.0) * (double)(1ull << 30));
  }();
  return v;
}

static int pp_min_q() {
  static const int v = [] {
    const char* m = getenv("IRC_SCAN_PP_MINQ");
    return m ? atoi(m) : 192;
  }();
  return v;
}

// LTOP up to IRC_SCAN_LTOP_MAXQ queries (default 64; 0 keeps the sampled-threshold
// pipeline, same results).  C2 corpus (100k x 768) on MI355X, whole call: Q = 1 / 16 /
// 32 / 64: 51.4 / 56.5 / 58.4 / 61.9 us against 60.0 / 64.9 / 67.3 / 71.5 with the sampled
// threshold; at Q = 96 / 128 the two pipelines are within each other's spread on the C3
// shard (145.7-149.9 vs 140.8-144.7 us / 146.1-149.0 vs 146.2-147.6 us), the single pass
// ahead at C2 Q = 128 (72.7-73.6 vs 87.3-89.0 us) and level at Q = 96, with a rescan
// (~15 us in select_dense) in some batches (profiles/r06_e_*).
static int ltop_max_q() {
  static const int v = [] {
    const char* e = getenv("IRC_SCAN_LTOP_MAXQ");
    return e ? atoi(e) : 64;
  }();
  return v;
}

// Smallest Q of the single-pass GEMM filter (its largest is 256, one query tile): off by
// default -- at C2 (Q = 256) the 4-key-list epilogue costs the filter 26 us (77.7 vs 51.8)
// and select_dense's rescans 32 us, against 36 us of sample pass + two selects
// (profiles/r04_d_scan_*_kernels.txt); irc_scan_set_ppl_min_q changes it at run time (the
// tests compare both pipelines).
static std::atomic<int>& ppl_min_q_ref() {
  static std::atomic<int> v{1 << 30};
  return v;
}
static int ppl_min_q() { return ppl_min_q_ref().load(std::memory_order_relaxed); }

static int pick_ks(int64_t D) { return D > 512 ? 2 : 1; }  // <= 128 fragment VGPRs/wave

static int pick_nq(int64_t D, int64_t Q) {
  const int nqmax = 8 / pick_ks(D);
  const int need = (int)((Q + 31) / 32);
  int p = 1;
  while (p < need && p < nqmax) p <<= 1;
  return p;
}

template <int D, int EB, int KS = (D > 512 ? 2 : 1)>
static size_t tile_lds_bytes() {
  using G = Geo<D, EB, KS>;
  return (size_t)G::NBUF * G::TILE_BYTES + G::XBUF_BYTES;
}

// Four k-slices in the single-pass scan for one 32-query group (Q <= 32) at D = 768 / 1024
// bf16: each wave gets half the DMA issue, MFMA chain and list insertions of a tile.  C3
// shard (250k x 768) filter at Q = 1 / 16 / 32: 78.5 / 85.0 / 86.0 -> 74.3 / 79.7 / 79.1 us;
// C2: 38.7 / 43.3 / 44.4 -> 34.5 / 37.8 / 38.0 us.  Two groups (8 waves): no gain (C3 Q =
// 33 / 64: 90.7 / 94.0 -> 90.2 / 95.6 us), so off there.
constexpr int LTOP_KS4_GROUPS = 1;

template <int EB>
static size_t lds_bytes_eb(int64_t D) {
  switch (D) {
    case 64: return tile_lds_bytes<64, EB>();
    case 128: return tile_lds_bytes<128, EB>();
    case 256: return tile_lds_bytes<256, EB>();
    case 384: return tile_lds_bytes<384, EB>();
    case 512: return tile_lds_bytes<512, EB>();
    case 768: return tile_lds_bytes<768, EB>();
    default: return tile_lds_bytes<1024, EB>();
  }
}
static size_t lds_bytes_for(int64_t D, int eb) {
  return eb == 1 ? lds_bytes_eb<1>(D) : lds_bytes_eb<2>(D);
}

// Workers own contiguous tile ranges; the worker count is a multiple of 8 so the
// XCD-aware block decode in scan_tile_kernel is a bijection.
static void plan_workers(int64_t ntiles, int gy, int64_t D, int eb, int nw, int* g, int* tpw) {
  int per_cu = (int)(IRC_LDS_BYTES / lds_bytes_for(D, eb));
  const int by_waves = 16 / nw > 0 ? 16 / nw : 1;  // keep <= 16 waves per CU
  if (per_cu > by_waves) per_cu = by_waves;
  if (per_cu < 1) per_cu = 1;
  const int64_t target = 256LL * per_cu;
  int64_t want = (target + gy - 1) / gy;
  if (want < 1) want = 1;
  if (want > ntiles) want = ntiles > 0 ? ntiles : 1;
  int64_t per = (ntiles + want - 1) / want;
  if (per < 1) per = 1;
  *tpw = (int)per;
  int64_t gg = (ntiles + per - 1) / per;
  gg = (gg + 7) / 8 * 8;
  *g = (int)gg;
}

// Threshold sample = N / SAMPLE_DIV docs (C2 whole call at Q = 64 / 256 / 1024 75.3 / 98.0 /
// 258 us against 75.8 / 101.6 / 274 at 8, and 98 / 115 / 296 at 32, tools/g4.sh).  Any
// value keeps the result exact (the threshold is the 2*KS-th group maximum of real
// scores); it trades the sample pass against the filter's survivor count.  Longer sample
// workers (more tiles each, fewer query-fragment loads) measured slower: C2 whole call
// at Q = 256 92.5 / 93.5 / 96.1 / 102.1 us for 1 / 3 / 5 / 8 tiles minimum (MI355X).
constexpr int64_t SAMPLE_DIV = 16;

static Plan make_plan(int64_t Q, int64_t N, int64_t D, int64_t k, int eb) {
  Plan p{};
  p.ks = pick_ks(D);
  p.nq = pick_nq(D, Q);
  p.nw = p.nq * p.ks;
  const int qb = p.nq * 32;
  p.gy = (int)((Q + qb - 1) / qb);
  if (p.gy < 1) p.gy = 1;
  p.qpad = p.gy * qb;
  // Sample of N/16 docs (>= 32k; GMAX leaves 2*KS keys per 32-doc tile, so >= 2k
  // group maxima per query for the threshold select, capped at its LDS stage).
  // The filter's survivors ~ k * N / S (~1.6k per query at k = 100, N / S = 16; at the cap, e.g. a 625k
  // shard, ~k * N / 32768).
  int64_t s_target = 32 * k;
  if (N / SAMPLE_DIV > s_target) s_target = N / SAMPLE_DIV;
  const int64_t s_cap = (int64_t)SEL_STAGE * TD / (2 * p.ks);
  if (s_target > s_cap) s_target = s_cap;
  p.stride = s_target > 0 ? N / s_target : 1;
  if (p.stride < 1) p.stride = 1;
  p.two_phase = p.stride > 1;
  p.S = p.two_phase ? (N + p.stride - 1) / p.stride : N;
  plan_workers((p.S + TD - 1) / TD, p.gy, D, eb, p.nw, &p.g_s, &p.tpw_s);
  p.cap_s = (int64_t)p.tpw_s * TD;
  plan_workers((N + TD - 1) / TD, p.gy, D, eb, p.nw, &p.g_f, &p.tpw_f);
  p.cap_f = (int64_t)p.tpw_f * TD;
  const int gmax = p.g_s > p.g_f ? p.g_s : p.g_f;
  int64_t kmax = (int64_t)p.g_f * p.cap_f;
  if (p.two_phase && (int64_t)p.g_s * p.cap_s > kmax) kmax = (int64_t)p.g_s * p.cap_s;
  size_t cnt_bytes = (size_t)gmax * p.qpad * 2 * p.ks * 4;
  size_t key_bytes = (size_t)kmax * p.qpad * 8;
  p.pp_G = (int)((N + 255) / 256);
  p.pp_qpad = (int)((Q + 255) / 256 * 256);
  p.pp_cap = 256;  // a 256-doc tile can never overflow its region
  const size_t pp_keys = (size_t)p.pp_G * p.pp_qpad * p.pp_cap * 8;
  // the GEMM-kernel filter: bf16, or fp8 with 128-byte K-tiles (D % 128 == 0)
  p.pp = (eb == 2 || D % 128 == 0) && Q >= pp_min_q() && N >= 256 &&
         pp_keys <= pp_max_bytes() && p.pp_G <= SEL_MAXR;
  p.pp_sG = (int)((p.S + 255) / 256);
  if (p.pp && p.two_phase) {  // the GEMM sample's lists share the survivor key buffer
    const size_t sb = (size_t)Q * p.pp_sG * LT_M * 8;
    if (sb > key_bytes) key_bytes = sb;
  }
  if (p.pp) {
    const size_t pc = (size_t)p.pp_G * p.pp_qpad * 4;
    if (pc > cnt_bytes) cnt_bytes = pc;
    if (pp_keys > key_bytes) key_bytes = pp_keys;
  }
  // the single-pass GEMM filter: one query tile, every tile's list in one select stage
  p.ppl = Q >= ppl_min_q() && Q <= 256 && N >= 256 && (eb == 2 || D % 128 == 0) &&
          (int64_t)p.pp_G * LT_M <= SEL_STAGE && k <= SEL_NT;
  if (p.ppl) {
    p.pp = false;
    p.two_phase = false;
    const size_t lb = (size_t)Q * p.pp_G * LT_M * 8;
    if (lb > key_bytes) key_bytes = lb;
  }
  // LTOP where the GEMM filter does not run and all lists fit one select stage
  p.ls = p.g_f * 2 * p.ks;
  p.ltop = !p.pp && !p.ppl && Q <= ltop_max_q() && (int64_t)p.ls * LT_M <= SEL_STAGE &&
           k <= SEL_NT;
  if (p.ltop) {
    p.two_phase = false;
    // four k-slices: same LDS (ring + a 16 KB exchange) and the same 4 lists per
    // worker and query (the half-lane lists are merged), so g_f / ls stand
    if (eb == 2 && (D == 768 || D == 1024) && p.nq <= LTOP_KS4_GROUPS) {
      p.ks = 4;
      p.nw = p.nq * 4;
    }
    const size_t lb = (size_t)p.qpad * p.ls * LT_M * 8;
    if (lb > key_bytes) key_bytes = lb;
  }
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const int qthr = p.pp && p.pp_qpad > p.qpad ? p.pp_qpad : p.qpad;
  p.off_thr = 0;
  p.off_cnt = al(p.off_thr + (size_t)qthr * 8);
  p.off_keys = al(p.off_cnt + cnt_bytes);
  p.bytes = al(p.off_keys + key_bytes);
  return p;
}

template <int D, int NQ, int MODE, int EB, int KS = (D > 512 ? 2 : 1)>
static void launch_tile(const Plan& p, int g, const unsigned char* qs, const unsigned char* docs,
                        int Q, int64_t NS, int64_t stride, int tpw, uint32_t idx_base,
                        const uint64_t* thr, uint64_t* keys, uint32_t* counts, int64_t cap,
                        float* scores, hipStream_t st) {
  const size_t lds = tile_lds_bytes<D, EB, KS>();
  static_assert(NQ * KS <= 8 || KS == 1, "wave budget");
  hipLaunchKernelGGL((scan_tile_kernel<D, NQ, KS, MODE, EB>), dim3(g * p.gy), dim3(NQ * KS * 64),
                     lds, st, qs, docs, Q, p.qpad, p.gy, (int)NS, (int)stride, tpw, idx_base, thr,
                     keys, counts, cap, scores);
}

template <int MODE, int EB>
static int dispatch_tile_eb(int64_t D, const Plan& p, int g, const unsigned char* qs,
                            const unsigned char* docs, int Q, int64_t NS, int64_t stride, int tpw,
                            uint32_t idx_base, const uint64_t* thr, uint64_t* keys,
                            uint32_t* counts, int64_t cap, float* scores, hipStream_t st) {
#define IRC_SCAN_ARGS p, g, qs, docs, Q, NS, stride, tpw, idx_base, thr, keys, counts, cap, scores, st
#define IRC_SCAN_CASE(DD)                                              \
  case DD:                                                             \
    if (p.ks == 4) {                                                   \
      if constexpr ((MODE == LTOP || MODE == SCORES) && EB == 2 &&     \
                    (DD == 768 || DD == 1024)) {                       \
        if (p.nq == 1) launch_tile<DD, 1, MODE, EB, 4>(IRC_SCAN_ARGS); \
        else launch_tile<DD, 2, MODE, EB, 4>(IRC_SCAN_ARGS);           \
      } else {                                                         \
        set_error("scan: four k-slices planned for an unsupported mode"); \
        return IRC_E_INVALID;                                          \
      }                                                                \
    } else if (p.nq == 1) launch_tile<DD, 1, MODE, EB>(IRC_SCAN_ARGS); \
    else if (p.nq == 2) launch_tile<DD, 2, MODE, EB>(IRC_SCAN_ARGS);   \
    else if (p.nq == 4) launch_tile<DD, 4, MODE, EB>(IRC_SCAN_ARGS);   \
    else launch_tile<DD, (DD > 512 ? 4 : 8), MODE, EB>(IRC_SCAN_ARGS); \
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
#undef IRC_SCAN_ARGS
  return check_launch("scan_tile_kernel");
}

template <int MODE>
static int dispatch_tile(int eb, int64_t D, const Plan& p, int g, const void* qs, const void* docs,
                         int Q, int64_t NS, int64_t stride, int tpw, uint32_t idx_base,
                         const uint64_t* thr, uint64_t* keys, uint32_t* counts, int64_t cap,
                         float* scores, hipStream_t st) {
  const unsigned char* q8 = static_cast<const unsigned char*>(qs);
  const unsigned char* d8 = static_cast<const unsigned char*>(docs);
  if (eb == 1)
    return dispatch_tile_eb<MODE, 1>(D, p, g, q8, d8, Q, NS, stride, tpw, idx_base, thr, keys,
                                     counts, cap, scores, st);
  return dispatch_tile_eb<MODE, 2>(D, p, g, q8, d8, Q, NS, stride, tpw, idx_base, thr, keys,
                                   counts, cap, scores, st);
}

template <int EB>
static void launch_dense_eb(int64_t D, int ks, int Q, const DenseArgs& a, hipStream_t st) {
#define IRC_DENSE_CASE(DD)                                                                 \
  case DD:                                                                                 \
    if (ks == 0) {                                                                         \
      if constexpr (EB == 2 || DD % 128 == 0)                                              \
        hipLaunchKernelGGL((select_dense_kernel<DD, EB, 0>), dim3((unsigned)Q), dim3(SEL_NT), 0, st, a); \
      break;                                                                               \
    }                                                                                      \
    if constexpr (EB == 2 && (DD == 768 || DD == 1024)) {                                  \
      if (ks == 4) {                                                                       \
        hipLaunchKernelGGL((select_dense_kernel<DD, EB, 4>), dim3((unsigned)Q), dim3(SEL_NT), 0, st, a); \
        break;                                                                             \
      }                                                                                    \
    }                                                                                      \
    hipLaunchKernelGGL((select_dense_kernel<DD, EB, (DD > 512 ? 2 : 1)>), dim3((unsigned)Q), \
                       dim3(SEL_NT), 0, st, a);                                            \
    break;
  switch (D) {
    IRC_DENSE_CASE(64)
    IRC_DENSE_CASE(128)
    IRC_DENSE_CASE(256)
    IRC_DENSE_CASE(384)
    IRC_DENSE_CASE(512)
    IRC_DENSE_CASE(768)
    default: IRC_DENSE_CASE(1024)
  }
#undef IRC_DENSE_CASE
}
static void launch_dense(int eb, int64_t D, int ks, int Q, const DenseArgs& a, hipStream_t st) {
  if (eb == 1) launch_dense_eb<1>(D, ks, Q, a, st);
  else launch_dense_eb<2>(D, ks, Q, a, st);
}

static bool supported_d(int64_t D) {
  return D == 64 || D == 128 || D == 256 || D == 384 || D == 512 || D == 768 || D == 1024;
}

static void launch_select(const RegionSource& src, int Q, int k, int mode, uint64_t* thr,
                          float* out_score, int64_t* out_idx, float smul, hipStream_t st);

// Shards too large for the GEMM filter's plan (its survivor workspace, 2 KB per (256-doc
// tile, query), over pp_max_bytes, or more tiles than the select's region table) are
// scanned as doc chunks that fit it, and the chunks' exact top-k lists merged by the same
// (score desc, index asc) rule -- the result is identical to one pass.  Without this a
// 5M-doc shard at Q = 2048 (config C4 on one GPU) would fall back to the stationary-query
// kernel, which re-reads the corpus once per 128 queries.  Returns N (no chunking) or the
// chunk size (a multiple of 256; the chunks are equal but for the last).
static int64_t chunk_docs(int64_t Q, int64_t N, int64_t D, int64_t k, int eb) {
  if (Q < pp_min_q() || N < 256 || !(eb == 2 || D % 128 == 0)) return N;
  const int64_t qpad = (Q + 255) / 256 * 256;
  int64_t tiles = (int64_t)(pp_max_bytes() / ((size_t)qpad * 256 * 8));
  if (tiles > SEL_MAXR) tiles = SEL_MAXR;
  if (tiles < 1) return N;
  const int64_t ntiles = (N + 255) / 256;
  if (ntiles <= tiles) return N;
  const int64_t nch = (ntiles + tiles - 1) / tiles;
  return (ntiles + nch - 1) / nch * 256;  // balanced chunks of whole 256-doc tiles
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Workspace of a chunked scan: the per-chunk lists [nch][Q][k] (fp32 scores, int64 ids)
// ahead of one chunk's own plan.
static size_t workspace_bytes_for(int64_t Q, int64_t N, int64_t D, int64_t k, int eb) {
  const int64_t nc = chunk_docs(Q, N, D, k, eb);
  if (nc >= N) return make_plan(Q, N, D, k, eb).bytes;
  const int64_t nch = (N + nc - 1) / nc;
  return align256((size_t)nch * Q * k * 12) + make_plan(Q, nc, D, k, eb).bytes;
}

static int scan_topk_impl(int eb, float smul, const void* queries, const void* docs, int64_t Q,
                          int64_t N, int64_t D, int64_t k, int64_t doc_offset, void* workspace,
                          int64_t workspace_bytes, float* out_score, int64_t* out_idx,
                          hipStream_t st);

static int scan_topk_chunked(int eb, float smul, const void* queries, const void* docs, int64_t Q,
                             int64_t N, int64_t D, int64_t k, int64_t doc_offset, int64_t nc,
                             void* workspace, int64_t workspace_bytes, float* out_score,
                             int64_t* out_idx, hipStream_t st) {
  const int64_t nch = (N + nc - 1) / nc;
  const size_t lists = align256((size_t)nch * Q * k * 12);
  IRC_REQUIRE(workspace != nullptr && workspace_bytes >= (int64_t)workspace_bytes_for(Q, N, D, k, eb),
              "scan_topk: workspace %lld < required %lld bytes", (long long)workspace_bytes,
              (long long)workspace_bytes_for(Q, N, D, k, eb));
  char* ws = static_cast<char*>(workspace);
  float* cs = reinterpret_cast<float*>(ws);
  int64_t* ci = reinterpret_cast<int64_t*>(ws + (size_t)nch * Q * k * 4);
  for (int64_t c = 0; c < nch; ++c) {
    const int64_t c0 = c * nc, n = (N - c0 < nc) ? N - c0 : nc;
    const int rc = scan_topk_impl(eb, smul, queries, static_cast<const char*>(docs) + c0 * D * eb,
                                  Q, n, D, k, doc_offset + c0, ws + lists,
                                  workspace_bytes - (int64_t)lists, cs + c * Q * k, ci + c * Q * k,
                                  st);
    if (rc) return rc;
  }
  ListSource src{cs, ci, (int)nch, (int)Q, (int)k};
  if (k > 512)
    hipLaunchKernelGGL((select_kernel_bigk<ListSource>), dim3(Q), dim3(SEL_NT), 0, st, src, (int)k,
                       (int)SEL_FINAL, nullptr, out_score, out_idx, 1.0f);
  else
    hipLaunchKernelGGL((select_kernel<ListSource>), dim3(Q), dim3(SEL_NT), 0, st, src, (int)k,
                       (int)SEL_FINAL, nullptr, out_score, out_idx, 1.0f);
  return check_launch("select_kernel(chunk merge)");
}

// The scan for both element widths (eb = 2: bf16, 1: e4m3; smul scales the
// returned scores, 1 for bf16).
static int scan_topk_impl(int eb, float smul, const void* queries, const void* docs, int64_t Q,
                          int64_t N, int64_t D, int64_t k, int64_t doc_offset, void* workspace,
                          int64_t workspace_bytes, float* out_score, int64_t* out_idx,
                          hipStream_t st) {
  IRC_REQUIRE(Q >= 0 && N >= 0, "scan_topk: negative size");
  IRC_REQUIRE(k >= 1 && k <= SEL_MAXK, "scan_topk: k=%lld outside [1, %d]", (long long)k,
              SEL_MAXK);
  IRC_REQUIRE(supported_d(D), "scan_topk: unsupported D=%lld", (long long)D);
  IRC_REQUIRE(doc_offset >= 0 && doc_offset + N <= (int64_t)0xFFFFFFFFll,
              "scan_topk: global doc index must fit 32 bits");
  IRC_REQUIRE(Q < (1 << 24), "scan_topk: Q too large");
  IRC_REQUIRE(N < (1ll << 31) - 64, "scan_topk: shard too large (N < 2^31)");
  IRC_REQUIRE(((uintptr_t)queries % 16) == 0 && ((uintptr_t)docs % 16) == 0,
              "scan_topk: queries and docs must be 16-byte aligned");
  if (Q == 0) return IRC_OK;
  if (N == 0) {
    // nothing to rank: every slot empty
    ListSource src{out_score, out_idx, 0, (int)Q, 1};
    hipLaunchKernelGGL((select_kernel<ListSource>), dim3(Q), dim3(SEL_NT), 0, st, src, (int)k,
                       (int)SEL_FINAL, nullptr, out_score, out_idx, 1.0f);
    return check_launch("select_kernel(empty)");
  }
  const int64_t nc = chunk_docs(Q, N, D, k, eb);
  if (nc < N)
    return scan_topk_chunked(eb, smul, queries, docs, Q, N, D, k, doc_offset, nc, workspace,
                             workspace_bytes, out_score, out_idx, st);
  const Plan p = make_plan(Q, N, D, k, eb);
  IRC_REQUIRE(workspace != nullptr && workspace_bytes >= (int64_t)p.bytes,
              "scan_topk: workspace %lld < required %lld bytes", (long long)workspace_bytes,
              (long long)p.bytes);
  char* ws = static_cast<char*>(workspace);
  uint64_t* thr = reinterpret_cast<uint64_t*>(ws + p.off_thr);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ws + p.off_cnt);
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + p.off_keys);
  const uint32_t base = (uint32_t)doc_offset;
  const double alg_bytes = (double)N * D * eb + (double)Q * D * eb;
  int rc;
  if (p.ltop) {
    prof_begin(st);
    rc = dispatch_tile<LTOP>(eb, D, p, p.g_f, queries, docs, (int)Q, N, 1, p.tpw_f, base, nullptr,
                             keys, cnt, p.ls, nullptr, st);
    prof_end("scan_filter", st, alg_bytes);
    if (rc) return rc;
    DenseArgs da{keys, static_cast<const unsigned char*>(queries),
                 static_cast<const unsigned char*>(docs), p.ls, (int)N, p.tpw_f, base, (int)k, smul,
                 out_score, out_idx};
    launch_dense(eb, D, p.ks, (int)Q, da, st);
    return check_launch("select_dense_kernel");
  }
  if (p.ppl) {
    // single pass: the GEMM filter keeps the 4 largest keys of every (256-doc tile,
    // query); select_dense takes the k-th of all lists and rescans the tiles whose
    // 4th key reaches it
    gpp::PArgs a{};
    a.A = static_cast<const unsigned short*>(queries);
    a.B = static_cast<const unsigned short*>(docs);
    a.M = (int)Q;
    a.N = (int)N;
    a.K = (int)(D * eb / 2);  // 2-byte units
    a.kchunk = a.K;
    a.lda = a.K;
    a.ldb = a.K;
    a.alpha = 1.f;
    a.qpad = p.pp_qpad;
    a.stride = 1;
    a.idx_base = base;
    a.lists = keys;
    a.ls = p.pp_G;
    prof_begin(st);
    gpp::run_scan(a, st, eb == 1);
    prof_end("scan_filter", st, alg_bytes);
    if ((rc = check_launch("gemm_pp_kernel(scan lists)"))) return rc;
    DenseArgs da{keys, static_cast<const unsigned char*>(queries),
                 static_cast<const unsigned char*>(docs), p.pp_G, (int)N, 256 / TD, base, (int)k,
                 smul, out_score, out_idx};
    launch_dense(eb, D, 0, (int)Q, da, st);
    return check_launch("select_dense_kernel(gemm lists)");
  }
  if (p.two_phase && p.pp && p.pp_sG * LT_M <= SEL_STAGE &&
      p.pp_sG * LT_M >= 4 * k) {
    // threshold sample on the GEMM kernel: the sample docs (every stride-th row) as B
    // with row stride ldb = stride * D, the 4 largest keys per (256-doc sample tile,
    // query) kept, thr[q] = their k-th.  Only where the lists hold >= 4 k keys (C2's
    // 6,250-doc sample has 25 tiles = 100 keys: no threshold at k = 100, every doc
    // survives -- 640 us a call, profiles/r04_b_ppl_ab.txt; the tile kernel's GMAX
    // pass keeps 4 keys per 32 docs).  (The tile kernel's GMAX pass ran at ~0.05 of
    // the MFMA peak at Q = 2048: 699 us of a 3.3 ms C4 call, profiles/r03_scan_p_kernels.txt.)
    gpp::PArgs a{};
    a.A = static_cast<const unsigned short*>(queries);
    a.B = static_cast<const unsigned short*>(docs);
    a.M = (int)Q;
    a.N = (int)p.S;
    a.K = (int)(D * eb / 2);  // 2-byte units
    a.kchunk = a.K;
    a.lda = a.K;
    a.ldb = (int64_t)a.K * p.stride;
    a.alpha = 1.f;
    a.qpad = p.pp_qpad;
    a.stride = (int)p.stride;
    a.idx_base = base;
    a.lists = keys;
    a.ls = p.pp_sG;
    gpp::run_scan(a, st, eb == 1);
    if ((rc = check_launch("gemm_pp_kernel(scan sample)"))) return rc;
    hipLaunchKernelGGL(lists_kth_kernel, dim3((unsigned)Q), dim3(SEL_NT), 0, st, keys, p.pp_sG,
                       (int)k, thr);
    if ((rc = check_launch("lists_kth_kernel"))) return rc;
  } else if (p.two_phase) {
    rc = dispatch_tile<GMAX>(eb, D, p, p.g_s, queries, docs, (int)Q, p.S, p.stride, p.tpw_s,
                             base, nullptr, keys, cnt, p.cap_s, nullptr, st);
    if (rc) return rc;
    const RegionSource s1 = region_source(keys, cnt, p.g_s, p.qpad, p.cap_s, 2 * p.ks);
    launch_select(s1, (int)Q, (int)k, SEL_THRESHOLD, thr, nullptr, nullptr, 1.0f, st);
    if ((rc = check_launch("select_kernel(threshold)"))) return rc;
  }
  if (p.pp) {
    // filter = NT GEMM C[q][doc] = Q . Docs^T on the ping-pong kernel with a
    // threshold epilogue; regions are (256-doc tile, query) with cap 256.
    gpp::PArgs a{};
    a.A = static_cast<const unsigned short*>(queries);
    a.B = static_cast<const unsigned short*>(docs);
    a.M = (int)Q;
    a.N = (int)N;
    a.K = (int)(D * eb / 2);  // 2-byte units
    a.kchunk = a.K;
    a.lda = a.K;
    a.ldb = a.K;
    a.alpha = 1.f;
    a.thr = p.two_phase ? thr : nullptr;
    a.keys = keys;
    a.counts = cnt;
    a.cap = p.pp_cap;
    a.qpad = p.pp_qpad;
    a.stride = 1;
    a.idx_base = base;
    prof_begin(st);
    gpp::run_scan(a, st, eb == 1);
    prof_end("scan_filter", st, alg_bytes);
    if ((rc = check_launch("gemm_pp_kernel(scan)"))) return rc;
    const RegionSource s2 = region_source(keys, cnt, p.pp_G, p.pp_qpad, p.pp_cap, 1);
    launch_select(s2, (int)Q, (int)k, SEL_FINAL, nullptr, out_score, out_idx, smul, st);
    return check_launch("select_kernel(final)");
  }
  prof_begin(st);
  rc = dispatch_tile<KEYS>(eb, D, p, p.g_f, queries, docs, (int)Q, N, 1, p.tpw_f, base,
                           p.two_phase ? thr : nullptr, keys, cnt, p.cap_f, nullptr, st);
  prof_end("scan_filter", st, alg_bytes);  // algorithmic bytes
  if (rc) return rc;
  const RegionSource s2 = region_source(keys, cnt, p.g_f, p.qpad, p.cap_f, 2 * p.ks);
  launch_select(s2, (int)Q, (int)k, SEL_FINAL, nullptr, out_score, out_idx, smul, st);
  return check_launch("select_kernel(final)");
}

}  // namespace scan
}  // namespace irc

using namespace irc;
using namespace irc::scan;

// Diagnostic builds only (-DIRC_SCAN_STAMPS): copy the phase stamps out.
extern "C" int irc_scan_dbg_stamps(uint64_t* out /* [4][32] */) {
#ifdef IRC_SCAN_STAMPS
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dbg_stamps), sizeof(dbg_stamps)) == hipSuccess ? 0 : -1;
#else
  (void)out;
  return -1;
#endif
}

// Diagnostic builds only: per-block start / end stamps of the last filter launch
// (out: 2 * 8192 uint64, s_memrealtime ticks at 100 MHz; zeroed after the copy).
extern "C" int irc_scan_dbg_blocks(uint64_t* out) {
#ifdef IRC_SCAN_STAMPS
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(dbg_blk), sizeof(dbg_blk)) != hipSuccess) return -1;
  static uint64_t zero[2 * 8192];
  return hipMemcpyToSymbol(HIP_SYMBOL(dbg_blk), zero, sizeof(dbg_blk)) == hipSuccess ? 0 : -1;
#else
  (void)out;
  return -1;
#endif
}

// Rescan statistics of the single-pass scan's select (host pointer, synchronises
// the device): out[0] = queries whose select rescanned, out[1] = workers rescanned.
extern "C" int irc_scan_rescan_stats(uint64_t* out, int reset) {
  IRC_REQUIRE(out != nullptr, "scan_rescan_stats: null out");
  if (hipDeviceSynchronize() != hipSuccess) return check_launch("scan_rescan_stats");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dense_rescans), 2 * sizeof(uint64_t)) != hipSuccess)
    return check_launch("scan_rescan_stats");
  if (reset) {
    const unsigned long long z[2] = {0ull, 0ull};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dense_rescans), z, sizeof(z)) != hipSuccess)
      return check_launch("scan_rescan_stats");
  }
  return IRC_OK;
}

// Smallest query batch of the single-pass GEMM filter (Q in [q, 256]); > 256 turns it
// off (the sampled-threshold pipeline then runs).  Returns the previous value.
extern "C" int irc_scan_set_ppl_min_q(int q) { return ppl_min_q_ref().exchange(q); }

extern "C" int64_t irc_scan_topk_workspace(int64_t Q, int64_t N, int64_t D, int64_t k) {
  if (Q <= 0 || N <= 0 || k <= 0) return 256;
  return (int64_t)workspace_bytes_for(Q, N, D, k, 2);
}

extern "C" int64_t irc_scan_topk_fp8_workspace(int64_t Q, int64_t N, int64_t D, int64_t k) {
  if (Q <= 0 || N <= 0 || k <= 0) return 256;
  return (int64_t)workspace_bytes_for(Q, N, D, k, 1);
}

extern "C" int irc_scan_topk(const void* queries, const void* docs, int64_t Q, int64_t N,
                             int64_t D, int64_t k, int64_t doc_offset, void* workspace,
                             int64_t workspace_bytes, float* out_score, int64_t* out_idx,
                             irc_stream_t stream) {
  return scan_topk_impl(2, 1.0f, queries, docs, Q, N, D, k, doc_offset, workspace,
                        workspace_bytes, out_score, out_idx, as_stream(stream));
}

// `batches` query batches of one shape against one shard with `depth` of them in flight:
// the host loop of ShardedDenseIndex.search_many (irc_amd/retrieval.py) in one call, so a
// C2 batch (~70 us of GPU work) is not paced by the Python side of one search() per batch.
// Every stream first waits for the work queued on `origin`; batch b runs irc_scan_topk on
// streams[b % depth] with workspaces[b % depth] into rows [b Q, (b + 1) Q) of the outputs;
// `origin` then waits for every stream (also after an error, for what was queued).
extern "C" int irc_scan_topk_many(const void* const* queries, int64_t batches, const void* docs,
                                  int64_t Q, int64_t N, int64_t D, int64_t k, int64_t doc_offset,
                                  void* const* workspaces, int64_t workspace_bytes, int64_t depth,
                                  float* out_score, int64_t* out_idx,
                                  const irc_stream_t* streams, irc_stream_t origin) {
  IRC_REQUIRE(batches >= 0 && depth >= 1 && depth <= 16, "scan_topk_many: bad batches / depth");
  IRC_REQUIRE(batches == 0 || (queries && workspaces && streams && out_score && out_idx),
              "scan_topk_many: null array");
  if (batches == 0) return IRC_OK;
  const hipStream_t org = as_stream(origin);
  const int nd = (int)std::min<int64_t>(depth, batches);
  hipEvent_t ev[17];
  for (int s = 0; s <= nd; ++s)
    if (hipEventCreateWithFlags(&ev[s], hipEventDisableTiming) != hipSuccess) {
      for (int t = 0; t < s; ++t) hipEventDestroy(ev[t]);
      return check_launch("scan_topk_many: event");
    }
  hipEventRecord(ev[nd], org);
  for (int s = 0; s < nd; ++s) hipStreamWaitEvent(as_stream(streams[s]), ev[nd], 0);
  int rc = IRC_OK;
  for (int64_t b = 0; b < batches && rc == IRC_OK; ++b) {
    const int s = (int)(b % nd);
    rc = scan_topk_impl(2, 1.0f, queries[b], docs, Q, N, D, k, doc_offset, workspaces[s],
                        workspace_bytes, out_score + b * Q * k, out_idx + b * Q * k,
                        as_stream(streams[s]));
  }
  for (int s = 0; s < nd; ++s) {
    hipEventRecord(ev[s], as_stream(streams[s]));
    hipStreamWaitEvent(org, ev[s], 0);
  }
  for (int s = 0; s <= nd; ++s) hipEventDestroy(ev[s]);
  return rc;
}

static bool pow2_scale(float s) {
  int e;
  return s > 0.f && std::isfinite(s) && std::frexp(s, &e) == 0.5f;
}

extern "C" int irc_scan_topk_fp8(const void* queries, const void* docs, int64_t Q, int64_t N,
                                 int64_t D, int64_t k, int64_t doc_offset, float score_scale,
                                 void* workspace, int64_t workspace_bytes, float* out_score,
                                 int64_t* out_idx, irc_stream_t stream) {
  IRC_REQUIRE(pow2_scale(score_scale), "scan_topk_fp8: score_scale must be a power of two");
  return scan_topk_impl(1, score_scale, queries, docs, Q, N, D, k, doc_offset, workspace,
                        workspace_bytes, out_score, out_idx, as_stream(stream));
}

// ------------------------------------------------------------ fp8 corpus
namespace irc {
namespace scan {
// out[i] = e4m3fn(RNE(x[i] * scale)), saturated to +-448 (OCP e4m3fn, the gfx950
// v_cvt_pk_fp8_f32 encoding).  8 elements per thread, 8-byte stores.
template <typename T>
__global__ __launch_bounds__(256) void quantize_fp8_kernel(const T* __restrict__ x, int64_t n,
                                                           float scale,
                                                           unsigned char* __restrict__ out) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i0 >= n) return;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float f = 0.f;
    if (i0 + j < n) {
      if constexpr (sizeof(T) == 2)
        f = bf16_to_f32(reinterpret_cast<const unsigned short*>(x)[i0 + j]);
      else
        f = reinterpret_cast<const float*>(x)[i0 + j];
    }
    f *= scale;
    v[j] = f != f ? f : fminf(fmaxf(f, -448.f), 448.f);
  }
  uint32_t w0 = 0, w1 = 0;
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], w0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], w0, true);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], w1, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], w1, true);
  if (i0 + 8 <= n && (((uintptr_t)(out + i0)) & 7) == 0) {
    *reinterpret_cast<uint2*>(out + i0) = make_uint2(w0, w1);
  } else {
    for (int j = 0; j < 8 && i0 + j < n; ++j)
      out[i0 + j] = (unsigned char)(((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xff);
  }
}
}  // namespace scan
}  // namespace irc

extern "C" int irc_quantize_fp8(int in_dtype, const void* x, int64_t n, float scale, void* out,
                                irc_stream_t stream) {
  IRC_REQUIRE(n >= 0, "quantize_fp8: negative size");
  IRC_REQUIRE(in_dtype == 0 || in_dtype == 1, "quantize_fp8: in_dtype must be 0 (bf16) or 1 (fp32)");
  if (n == 0) return IRC_OK;
  const unsigned blocks = (unsigned)((n + 2047) / 2048);
  hipStream_t st = as_stream(stream);
  if (in_dtype == 0)
    hipLaunchKernelGGL((quantize_fp8_kernel<unsigned short>), dim3(blocks), dim3(256), 0, st,
                       static_cast<const unsigned short*>(x), n, scale,
                       static_cast<unsigned char*>(out));
  else
    hipLaunchKernelGGL((quantize_fp8_kernel<float>), dim3(blocks), dim3(256), 0, st,
                       static_cast<const float*>(x), n, scale, static_cast<unsigned char*>(out));
  return check_launch("quantize_fp8_kernel");
}

extern "C" int irc_topk_merge(const float* in_score, const int64_t* in_idx, int64_t P, int64_t Q,
                              int64_t kin, int64_t kout, float* out_score, int64_t* out_idx,
                              irc_stream_t stream) {
  IRC_REQUIRE(P >= 1 && Q >= 0 && kin >= 1, "topk_merge: bad sizes");
  IRC_REQUIRE(kout >= 1 && kout <= SEL_MAXK, "topk_merge: kout outside [1, %d]", SEL_MAXK);
  if (Q == 0) return IRC_OK;
  ListSource src{in_score, in_idx, (int)P, (int)Q, (int)kin};
  if (kout > 512)
    hipLaunchKernelGGL((select_kernel_bigk<ListSource>), dim3(Q), dim3(SEL_NT), 0,
                       as_stream(stream), src, (int)kout, (int)SEL_FINAL, nullptr, out_score,
                       out_idx, 1.0f);
  else
    hipLaunchKernelGGL((select_kernel<ListSource>), dim3(Q), dim3(SEL_NT), 0, as_stream(stream),
                       src, (int)kout, (int)SEL_FINAL, nullptr, out_score, out_idx, 1.0f);
  return check_launch("select_kernel(merge)");
}

extern "C" int irc_scan_scores(const void* queries, const void* docs, int64_t Q, int64_t N,
                               int64_t D, float* out, irc_stream_t stream) {
  IRC_REQUIRE(Q >= 0 && N >= 0, "scan_scores: negative size");
  IRC_REQUIRE(supported_d(D), "scan_scores: unsupported D=%lld", (long long)D);
  IRC_REQUIRE(((uintptr_t)queries % 16) == 0 && ((uintptr_t)docs % 16) == 0,
              "scan_scores: queries and docs must be 16-byte aligned");
  if (Q == 0 || N == 0) return IRC_OK;
  Plan p = make_plan(Q, N, D, 1, 2);
  if (p.pp || p.ppl) {
    // same MFMA arithmetic as irc_scan_topk's filter on this path
    gpp::PArgs a{};
    a.A = static_cast<const unsigned short*>(queries);
    a.B = static_cast<const unsigned short*>(docs);
    a.C = out;
    a.M = (int)Q;
    a.N = (int)N;
    a.K = (int)D;
    a.kchunk = (int)D;
    a.lda = D;
    a.ldb = D;
    a.ldc = N;
    a.alpha = 1.f;
    a.vec_c = (N % 8 == 0) && ((uintptr_t)out % 16) == 0;
    gpp::run(1, 0, 0, 0, a, 1, 1, as_stream(stream));
    return check_launch("gemm_pp_kernel(scores)");
  }
  return dispatch_tile<SCORES>(2, D, p, p.g_f, queries, docs, (int)Q, N, 1, p.tpw_f, 0, nullptr,
                               nullptr, nullptr, 0, out, as_stream(stream));
}

// Raw (unscaled) dot products of e4m3 queries and docs, fp32 accumulation: the
// arithmetic of irc_scan_topk_fp8's filter.
extern "C" int irc_scan_scores_fp8(const void* queries, const void* docs, int64_t Q, int64_t N,
                                   int64_t D, float* out, irc_stream_t stream) {
  IRC_REQUIRE(Q >= 0 && N >= 0, "scan_scores_fp8: negative size");
  IRC_REQUIRE(supported_d(D), "scan_scores_fp8: unsupported D=%lld", (long long)D);
  IRC_REQUIRE(((uintptr_t)queries % 16) == 0 && ((uintptr_t)docs % 16) == 0,
              "scan_scores_fp8: queries and docs must be 16-byte aligned");
  if (Q == 0 || N == 0) return IRC_OK;
  Plan p = make_plan(Q, N, D, 1, 1);
  if (p.pp || p.ppl) {
    // same MFMA arithmetic as irc_scan_topk_fp8's filter on this path
    gpp::PArgs a{};
    a.A = static_cast<const unsigned short*>(queries);
    a.B = static_cast<const unsigned short*>(docs);
    a.C = out;
    a.M = (int)Q;
    a.N = (int)N;
    a.K = (int)(D / 2);
    a.kchunk = a.K;
    a.lda = a.K;
    a.ldb = a.K;
    a.ldc = N;
    a.alpha = 1.f;
    a.vec_c = (N % 8 == 0) && ((uintptr_t)out % 16) == 0;
    gpp::run_scores_fp8(a, as_stream(stream));
    return check_launch("gemm_pp_kernel(scores fp8)");
  }
  return dispatch_tile<SCORES>(1, D, p, p.g_f, queries, docs, (int)Q, N, 1, p.tpw_f, 0, nullptr,
                               nullptr, nullptr, 0, out, as_stream(stream));
}
