// Ping-pong 256x256x64 bf16 GEMM for gfx950 (the large-shape path of irc_gemm).
//
//   C[M, N] (=|+=) alpha * op(A) . op(B) (+ bias) (-> GELU / GELU' / residual)
//
// Used for every big bf16 GEMM of the path: the BERT forward projections
// (contrastive_module.py:39 -> HF modeling_bert), the trainable encoder's dX and
// dW products, the LSTM input projections (src/model.py:16-26) -- all four operand
// layouts: A [M][K] or [K][M], B [N][K] or [K][N].
//
// Structure (cdna_hip_programming.md §5, "ping-pong" of two wave groups):
//  * 8 waves = 2 groups of 4.  Group g owns output rows 128g..128g+127 of the
//    block tile; wave (g, wn) a 128 x 64 sub-tile = 8 x 4 accumulators of
//    v_mfma_f32_16x16x32_bf16 (128 VGPRs).
//  * The K loop alternates two sections per 64-deep K-tile: L (read the tile's
//    fragments from LDS into registers, issue the LDS-DMA of the NEXT tile's
//    halves this group owns) and M (64 MFMAs from registers).  Group 1 starts one
//    section late (an extra barrier), so at every moment one group runs MFMAs
//    while the other reads LDS / issues DMA: each SIMD hosts one wave of each
//    group and its matrix pipe alternates between them.
//  * LDS: 2 K-tile buffers x {A rows 0-127, A rows 128-255, B cols 0-127,
//    B cols 128-255} x 16-17 KB = 128-136 KB, filled by global_load_lds_dwordx4 (no
//    VGPR staging).  Group g DMAs A half g and B half g.  Waits are per-group
//    vmcnt(0) placed where that group's DMA has had a full section to land; all
//    barriers are raw s_barrier (no vmcnt drain).
//  * K-major tiles ([rows][64 k], 128-B rows) use the 16-B chunk XOR (row & 7),
//    applied on the DMA SOURCE address (the DMA destination is lane-linear), and
//    are read with ds_read_b128; K-outer tiles are stored column-chunk-major
//    (8 columns x 64 k per 1-KB chunk, padded) and read with ds_read_b64_tr_b16
//    (hardware transpose) at base + immediate addresses.
//  * Epilogue through LDS (per wave, 32-row passes) -> 16-byte coalesced stores,
//    fused bias / GELU / GELU' / residual / pre-activation save / fp32 accumulate,
//    or raw fp32 split-K slabs reduced afterwards in a fixed order.
#include "gemm_pp.h"
#include "mx.h"

#include <atomic>
#include <cstdlib>
#include <mutex>

namespace irc {
namespace gemm {
// shared with gemm.hip
enum Epi {
  EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RESID = 3, EPI_RESID = 4,
  EPI_DGELU = 5, EPI_BIAS_GELU_SAVE = 6
};
}  // namespace gemm

namespace gpp {
using namespace irc::gemm;

#ifdef IRC_SCAN_STAMPS  // diagnostic build: EPI_SCAN phase stamps of block 0 (s_memrealtime)
__device__ uint64_t pp_stamps[16];
#define PSTAMP(i)                                                              \
  do {                                                                         \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                   \
      *(volatile uint64_t*)&pp_stamps[(i) + (int)(threadIdx.x & 0)] =          \
          __builtin_amdgcn_s_memrealtime();                                    \
  } while (0)
#else
#define PSTAMP(i) \
  do {            \
  } while (0)
#endif

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
// K-outer half-tile image: 16 blocks of 4 k-rows, each block = [4 k-rows][16
// column-chunk slots][16 B] (1 KB) + a 64-B pad (BPITCH); slot c of k-row a holds
// chunk c ^ 2a.  One DMA wave-instruction fills one block from 4 whole 256-B
// k-rows of global memory, 16 consecutive lanes per k-row (coalesced); a 16-lane
// group's transposed reads (4 k-rows x 2 chunks) cover one aligned 128-B window,
// and the two groups of a 32-lane half (k-rows 8 apart = 2 blocks apart) land on
// disjoint bank halves thanks to the pad.  K-major images are 128 rows x 128 B.
constexpr int BPITCH = 1024 + 64;
// half-tile slot bytes of a K-major / K-outer operand; one K-tile = A0 A1 B0 B1
constexpr int slot_bytes(bool kmajor) { return kmajor ? 16384 : 16 * BPITCH; }
constexpr int buf_bytes(bool ak, bool bk) { return 2 * slot_bytes(ak) + 2 * slot_bytes(bk); }
constexpr int LDS_BYTES = 2 * buf_bytes(false, false);  // 136 KB (allocation for all variants)
constexpr int EP_PITCH = 68;          // epilogue staging row pitch (floats)

__device__ __forceinline__ float gelu_f(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
  float p = 1.061405429f;
  p = p * t - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const float e = 1.0f - p * t * __expf(-az * az);
  return 0.5f * x * (1.0f + copysignf(e, z));
}
// Two lanes' worth of gelu_f / gelu_grad_f on <2 x float>: the polynomial, scale and
// blend steps issue as v_pk_fma_f32 / v_pk_mul_f32 (2 results per lane per op), only
// rcp / exp / copysign stay scalar. Same operations in the same order as the scalar
// forms, so the results are the same bits. The epilogue of the 256x256 tile is
// VALU-bound (one workgroup per CU, nothing to overlap it with), so this is the
// FFN1 + GELU launch's tail.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void erf_as_parts(f32x2 x, f32x2& z, f32x2& t, f32x2& ez) {
  z = x * 0.70710678118654752f;
  f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 d = 1.0f + 0.3275911f * az;
  t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const f32x2 n = -az * az;
  ez = f32x2{__expf(n.x), __expf(n.y)};
}
__device__ __forceinline__ f32x2 erf_as_poly(f32x2 t) {
  f32x2 p = 1.061405429f * t - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  return p;
}
__device__ __forceinline__ f32x2 gelu_f2(f32x2 x) {
  f32x2 z, t, ez;
  erf_as_parts(x, z, t, ez);
  const f32x2 e = 1.0f - erf_as_poly(t) * t * ez;
  const f32x2 s = {copysignf(e.x, z.x), copysignf(e.y, z.y)};
  return 0.5f * x * (1.0f + s);
}
__device__ __forceinline__ f32x2 gelu_grad_f2(f32x2 x) {
  f32x2 z, t, ez;
  erf_as_parts(x, z, t, ez);
  const f32x2 e = 1.0f - erf_as_poly(t) * t * ez;
  const f32x2 s = {copysignf(e.x, z.x), copysignf(e.y, z.y)};
  return 0.5f * (1.0f + s) + x * 0.3989422804014327f * ez;
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * az);
  float p = 1.061405429f;
  p = p * t - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  const float ez = __expf(-az * az);
  const float e = 1.0f - p * t * ez;
  return 0.5f * (1.0f + copysignf(e, z)) + x * 0.3989422804014327f * ez;
}

__device__ __forceinline__ bool has_bias(int e) {
  return e == EPI_BIAS || e == EPI_BIAS_GELU || e == EPI_BIAS_RESID || e == EPI_BIAS_GELU_SAVE;
}

// DMA one half-tile (128 rows/cols x 64 k) of operand X into `img`, by the 256
// threads (4 waves, wave index wq) of one group: 4 wave-instructions each.
//  KMAJOR: X[r][k] (row stride ld) rows r0..r0+127 (clamped to < nrows), k0..k0+63.
//  else:   X[k][c] (row stride ld) k-rows k0..k0+63, columns c0..c0+127 in 16-B
//          chunks, 4 whole k-rows per wave-instruction (chunks past ncols clamped
//          to the last whole chunk; never stored).
template <bool KMAJOR>
__device__ __forceinline__ void stage_half(const unsigned short* __restrict__ X, int64_t ld,
                                           int r0, int nrows, int k0, char* img, int wq,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = (i * 4 + wq) * 64 + lane;  // 16-B LDS chunk index (lane-linear)
    if constexpr (KMAJOR) {
      const int row = p >> 3;
      const int c = (p & 7) ^ (row & 7);
      int gr = r0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      glds16(X + (int64_t)gr * ld + k0 + c * 8, img + (i * 4 + wq) * 1024);
    } else {
      // 4 k-rows per block; lane -> (k-row a = lane >> 4, LDS slot lane & 15), and
      // the slot holds column chunk (slot ^ 2a): 16 consecutive lanes read one
      // k-row's 256 contiguous bytes (coalesced), and the transposed reads of the
      // 4 k-rows (256 B apart) land on distinct banks.
      const int blk = i * 4 + wq;
      const int a = lane >> 4;
      int gc = r0 + ((lane & 15) ^ (2 * a)) * 8;
      gc = gc + 8 <= nrows ? gc : nrows - 8;
      glds16(X + (int64_t)(k0 + 4 * blk + a) * ld + gc, img + blk * BPITCH);
    }
  }
}

typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4s ds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// 16x16x32 operand fragment: lane l gets X[row0 + (l & 15)][32 s + 8 (l >> 4) + j], j < 8.
template <bool KMAJOR>
__device__ __forceinline__ bf16x8 frag(const char* img, int row0, int s, int lane) {
  if constexpr (KMAJOR) {
    const int row = row0 + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * (c ^ (row & 7)));
  } else {
    // 16-lane group q reads k-rows 32s+8q+{0..3} then +{4..7}; lane 4a+b of the
    // group addresses row a, columns row0 + 4b .. +3 (chunk col >> 3 sits in slot
    // (col >> 3) ^ 2a of the block's k-row a, see stage_half)
    const int q = lane >> 4, a = (lane >> 2) & 3, b = lane & 3;
    const int col = row0 + 4 * b;
    const char* p =
        img + (8 * s + 2 * q) * BPITCH + a * 256 + (((col >> 3) ^ (2 * a)) * 16) + (col & 7) * 2;
    const v4s lo = ds_tr16(p);            // k-rows 32s + 8q + a
    const v4s hi = ds_tr16(p + BPITCH);   // k-rows 32s + 8q + 4 + a
    const v4s both[2] = {lo, hi};
    return __builtin_bit_cast(bf16x8, both);
  }
}

// F8: both operands are e4m3 bytes (the fp8 corpus scan, BASELINE config C5),
// passed as 2-byte units (K, ld in units of 2 fp8 values): the DMA and LDS
// images are byte-identical to bf16, and each 128-byte K-tile row feeds one
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales) per accumulator instead
// of two 16x16x32 bf16 MFMAs -- twice the bf16 rate per element.  A and B
// fragments take the same bytes of the row, so the k order is consistent.
typedef int v8i32 __attribute__((ext_vector_type(8)));

// MX MFMA with the A / B scale bytes chosen by op_sel (immediates: the callers'
// unrolled loop indices fold the switch to one instruction).
template <int OA, int OB>
__device__ __forceinline__ f32x4 mfma_mx(v8i32 a, v8i32 b, f32x4 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OA, sa, OB, sb);
}
__device__ __forceinline__ f32x4 mfma_mx_sel(int oa, int ob, v8i32 a, v8i32 b, f32x4 c, int sa,
                                             int sb) {
  switch (oa * 4 + ob) {
#define IRC_MXS(OA, OB) \
  case OA * 4 + OB:     \
    return mfma_mx<OA, OB>(a, b, c, sa, sb);
    IRC_MXS(0, 0) IRC_MXS(0, 1) IRC_MXS(0, 2) IRC_MXS(0, 3)
    IRC_MXS(1, 0) IRC_MXS(1, 1) IRC_MXS(1, 2) IRC_MXS(1, 3)
    IRC_MXS(2, 0) IRC_MXS(2, 1) IRC_MXS(2, 2) IRC_MXS(2, 3)
    IRC_MXS(3, 0) IRC_MXS(3, 1) IRC_MXS(3, 2)
#undef IRC_MXS
    default:
      return mfma_mx<3, 3>(a, b, c, sa, sb);
  }
}

// MX-fp8 (F8 == 2, the encoder's fp8 linear layers): e4m3 operands with one
// power-of-two (E8M0) scale per 32 consecutive k of a row, applied by the MFMA
// itself (v_mfma_scale_f32_16x16x128_f8f6f4's per-lane block scales).  Scale
// layout in HBM ("MX layout"): [K8 / 128][rows padded to 256][4] bytes, so one
// 256-row K-tile's scales are 1 KB contiguous; they ride the tile's DMA into LDS
// at MX_SC_OFF + buffer * 2 KB as [A half 0 | B half 0 | A half 1 | B half 1].
constexpr int MX_SC_OFF = 2 * buf_bytes(true, true);  // 128 KB: past both K-major buffers
static_assert(MX_SC_OFF + 2 * 2048 <= LDS_BYTES, "MX scale slots");

// The scales of K-tile `kt` (64 two-byte units = 128 e4m3) for group g's A and B
// halves (512 contiguous bytes each, mx_scale_index): wave 0 of the group, lanes
// 0-31 the A half, 32-63 the B half.
__device__ __forceinline__ void stage_scales(const PArgs& g, int m0, int n0, int kt, char* sc,
                                             int grp, int wq, int lane) {
  if (wq != 0) return;
  // re-derived per call: hoisted out of the K loop, the per-lane pointer would hold
  // two more VGPRs through it (the MX loop sits at the 256-register limit)
  int ln = lane;
  asm volatile("" : "+v"(ln));
  const bool isb = ln >= 32;
  const unsigned char* src = isb ? g.sbx + (int64_t)kt * g.npad * 4 + (n0 >> 8) * 1024
                                 : g.sax + (int64_t)kt * g.mpad * 4 + (m0 >> 8) * 1024;
  glds16(src + grp * 512 + 16 * (ln & 31), sc + grp * 1024);
}

// One 64-deep K-tile of both operands into the LDS image at `base`: group g stages
// A rows/cols [128g, +128) and B rows/cols [128g, +128).
template <bool AK, bool BK_, bool REDERIVE = false>
__device__ __forceinline__ void stage_tile(const PArgs& g, const unsigned short* A,
                                           const unsigned short* B, int m0, int n0, int k0,
                                           char* base, int grp, int wq, int lane) {
  constexpr int SA = slot_bytes(AK), SB = slot_bytes(BK_);
  if constexpr (REDERIVE) {  // per-lane DMA addresses recomputed per call, not kept live
    asm volatile("" : "+v"(lane));
  }
  stage_half<AK>(A, g.lda, m0 + 128 * grp, g.M, k0, base + grp * SA, wq, lane);
  stage_half<BK_>(B, g.ldb, n0 + 128 * grp, g.N, k0, base + 2 * SA + grp * SB, wq, lane);
}

// 1: group 1 issues its half of K-tile kt + 1 at the start of its M section of
// K-tile kt - 1 instead of its L section of K-tile kt (the buffer is free from the
// barrier between them), so its DMA, like group 0's, has a whole K-tile of sections
// to land before group 0 reads it; 0: the round-2 order (one section); 1: the MX
// kernel only (default); 2: every kernel.  The per-lane DMA addresses are then
// re-derived per call (kept live across the M section they spill 12-28 VGPRs).
// Measured on MI355X (profiles/r03_gemm_j_*): MX qkv / FFN1 (MX out) / FFN2 101 /
// 184 / 119 us against 110 / 194 / 135; the bf16 forms gain nothing on qkv / FFN2
// and lose on FFN1 + GELU (237 vs 200 us) and 4096^3 (127 vs 108 us).
#define IRC_PP_G1_EARLY 1

// The ping-pong K loop of one 256x256 output tile over nk K-tiles from kbeg.
// K-tile kt lives in LDS buffer (kt + par) & 1, the buffers `pitch` bytes apart.
// staged: K-tile 0's DMA was already issued by the caller.  pub != null: thread 0
// stores pub_val there before its last barrier, so every wave reads it after the
// loop.  On return every wave of the CALLER's group is past its last MFMA and every
// wave of both groups past its last fragment read; group 1 may still be in its last
// MFMAs when group 0 returns (registers only: LDS is free for the epilogue).
template <bool AK, bool BK_, int F8>
__device__ __forceinline__ void mainloop(const PArgs& g, const unsigned short* A,
                                         const unsigned short* B, int m0, int n0, int kbeg,
                                         int nk, char* lds, int pitch, int par, bool staged,
                                         f32x4 (&acc)[8][4], int grp, int wq, int lane, int* pub,
                                         int pub_val) {
  constexpr int SA = slot_bytes(AK), SB = slot_bytes(BK_);
  constexpr bool G1E = IRC_PP_G1_EARLY != 0 && (F8 == 2 || IRC_PP_G1_EARLY == 2);
  constexpr bool RD = F8 == 2 || G1E;  // DMA addresses re-derived per call (register budget)
  const int wn = wq;  // 64-column slab of the tile
  const int bh = wn >> 1, bcol = 64 * (wn & 1);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)0.0f;

  if (nk > 0) {
    if (!staged) stage_tile<AK, BK_>(g, A, B, m0, n0, kbeg, lds + par * pitch, grp, wq, lane);
    if constexpr (F8 == 2) stage_scales(g, m0, n0, kbeg / BK, lds + MX_SC_OFF + par * 2048, grp, wq, lane);
    wait_vmcnt<0>();
    wg_barrier();
    if (grp == 1) {  // group 1 runs one section behind
      if (G1E && nk > 1) {
        // its half of K-tile 1 now: group 1 issues K-tile kt + 1 in its M section of
        // kt - 1 (below), so its DMA has two sections to land, as group 0's has
        stage_tile<AK, BK_, RD>(g, A, B, m0, n0, kbeg + BK, lds + (par ^ 1) * pitch, grp, wq, lane);
        if constexpr (F8 == 2)
          stage_scales(g, m0, n0, kbeg / BK + 1, lds + MX_SC_OFF + (par ^ 1) * 2048, grp, wq, lane);
      }
      wg_barrier();
    }
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = (kt + par) & 1;
      // ---- L section: next tile's DMA (group 0; group 1 too when not G1E),
      // this tile's fragments
#ifdef IRC_PP_DIAG_NODMA  // diagnostic build: only K-tile 0 is loaded (MFMA + LDS-read rate)
      if (kt + 1 < nk && kt < 0) {
#else
      if (kt + 1 < nk && (grp == 0 || !G1E)) {
#endif
        stage_tile<AK, BK_, RD>(g, A, B, m0, n0, kbeg + (kt + 1) * BK, lds + (cur ^ 1) * pitch,
                                grp, wq, lane);
        if constexpr (F8 == 2)
          stage_scales(g, m0, n0, kbeg / BK + kt + 1, lds + MX_SC_OFF + (cur ^ 1) * 2048, grp, wq,
                       lane);
      }
      const char* la = lds + cur * pitch + grp * SA;
      const char* lb = lds + cur * pitch + 2 * SA + bh * SB;
      bf16x8 fa[8][2], fb[4][2];
      uint2 xa;     // MX: the lane's E8M0 block scales of its A rows 16 i + r (byte i)
      uint32_t xb;  // ... and of its B cols (byte j)
      if constexpr (F8 == 2) {
        // The 16x16x128 f8 MFMA's operand map (probed on MI355X, tools/probe/mx_probe.hip):
        // lane l holds k [16q, 16q + 16) and [64 + 16q, 64 + 16q + 16) of row / col
        // l & 15, q = l >> 4 -- the same two 16-byte chunks q, q + 4 as the
        // unit-scale path -- and the scale of row i, 32-k block b comes from lane
        // i + 16 b.  So the fragments keep the natural k order and lane l supplies
        // the E8M0 byte of block q = l >> 4.
        const int q = lane >> 4;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j][c] = frag<BK_>(lb, bcol + 16 * j, c, lane);
#pragma unroll
          for (int i = 0; i < 8; ++i) fa[i][c] = frag<AK>(la, 16 * i, c, lane);
        }
        const char* sc = lds + MX_SC_OFF + cur * 2048;
        const int rq = (q * 16 + (lane & 15)) * 8;
        xa = *reinterpret_cast<const uint2*>(sc + grp * 1024 + rq);
        xb = *reinterpret_cast<const uint32_t*>(sc + bh * 1024 + 512 + rq + 4 * (wn & 1));
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[j][s] = frag<BK_>(lb, bcol + 16 * j, s, lane);
#pragma unroll
          for (int i = 0; i < 8; ++i) fa[i][s] = frag<AK>(la, 16 * i, s, lane);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (grp == 1) wait_vmcnt<0>();  // group 0 reads this DMA in the next section
      wg_barrier();
      // ---- M section
#ifndef IRC_PP_DIAG_NODMA
      // group 1: its half of K-tile kt + 2 into this tile's buffer, which both groups
      // finished reading at the barrier above
      if (G1E && grp == 1 && kt + 2 < nk) {
        stage_tile<AK, BK_, RD>(g, A, B, m0, n0, kbeg + (kt + 2) * BK, lds + cur * pitch, grp, wq,
                                lane);
        if constexpr (F8 == 2)
          stage_scales(g, m0, n0, kbeg / BK + kt + 2, lds + MX_SC_OFF + cur * 2048, grp, wq, lane);
      }
#endif
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8 == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x8 a2[2] = {fa[i][0], fa[i][1]};
            const bf16x8 b2[2] = {fb[j][0], fb[j][1]};
            acc[i][j] = mfma_mx_sel(i & 3, j, __builtin_bit_cast(v8i32, a2),
                                    __builtin_bit_cast(v8i32, b2), acc[i][j],
                                    (int)(i < 4 ? xa.x : xa.y), (int)xb);
          }
      } else if constexpr (F8) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x8 a2[2] = {fa[i][0], fa[i][1]};
            const bf16x8 b2[2] = {fb[j][0], fb[j][1]};
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                __builtin_bit_cast(v8i32, a2), __builtin_bit_cast(v8i32, b2), acc[i][j], 0, 0, 0,
                127, 0, 127);
          }
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], fb[j][s], acc[i][j],
                                                                  0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if (grp == 0) {
        wait_vmcnt<0>();
        if (kt == nk - 1 && pub != nullptr && threadIdx.x == 0) {
          *pub = pub_val;
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
      }
      // Group 1's last M section ends without a barrier, and group 0 does not wait
      // for it after the loop: group 0's last barrier above already follows group
      // 1's last fragment reads, so group 0 starts its epilogue while group 1's last
      // 64 MFMAs run (one barrier fewer for each group keeps the counts matched).
      if (!(grp == 1 && kt == nk - 1)) wg_barrier();
    }
  }
}

// Vectorised epilogue of one 256x256 tile (16-byte aligned C / R rows, or raw fp32
// split-K slabs): per wave, four 32-row passes through its LDS staging rows (the
// first 8 * 32 * EP_PITCH floats of LDS), fused bias / GELU / GELU' / residual /
// pre-activation save / fp32 accumulate, then coalesced 16-byte stores.
// LN: the LayerNorm-fold instantiation (irc_gemm_ln; see LnArgs) -- a template flag so the
// other instantiations keep their register allocation.
template <typename TO, int EPI, int F8, bool LN = false>
__device__ __forceinline__ void epilogue_vec(const PArgs& g, const f32x4 (&acc)[8][4], char* lds,
                                             int m0, int n0, int batch, int grp, int wn, int wave,
                                             int lane, int split = 0) {
  const int rbase0 = m0 + 128 * grp;
  const int cbase = n0 + 64 * wn;
  float* st = reinterpret_cast<float*>(lds) + wave * (32 * EP_PITCH);
  const bool slab = g.P != nullptr;
  if (slab || g.vec_c) {
    const float* bias = g.bias ? g.bias + batch * g.sBias : nullptr;
    float bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cbase + 16 * j + (lane & 15);
      bv[j] = (!slab && has_bias(EPI) && col < g.N) ? bias[col] : 0.f;
    }
    const float alpha = slab ? 1.f : g.alpha;
    // LayerNorm fold (bf16 C only; uniform): the staged values are raw acc, the fold,
    // bias and GELU are applied per 8-column chunk below
    constexpr bool LNOK = LN && sizeof(TO) == 2 && F8 == 0;
    const bool lnfold = LNOK && !slab && g.ln.fold_s != nullptr;
    const bool lnres = LNOK && !slab && g.ln.gamma != nullptr;
    const bool lnout = LNOK && !slab && g.ln.st_out != nullptr;
    float* lst = reinterpret_cast<float*>(lds) + 8 * 32 * EP_PITCH;  // [256 rows][2] partials
    if (lnout) {
      lst[threadIdx.x] = 0.f;  // 512 threads, 512 floats
      __syncthreads();
    }
    // fp8 linear layers: per-row (A) and per-column (B) dequantisation scales
    float sbv[4] = {1.f, 1.f, 1.f, 1.f};
    float sav[8][4];
    if constexpr (F8 == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = cbase + 16 * j + (lane & 15);
        sbv[j] = (g.sb != nullptr && col < g.N) ? g.sb[col] : 1.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase0 + 16 * i + 4 * (lane >> 4) + e;
          sav[i][e] = (g.sa != nullptr && row < g.M) ? g.sa[row] : 1.f;
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {  // 32-row passes
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x2 v[2];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (F8 == 1)
              v[e >> 1][e & 1] = acc[2 * p + ii][j][e] * (alpha * sav[2 * p + ii][e] * sbv[j]) +
                                 bv[j];
            else
              v[e >> 1][e & 1] = acc[2 * p + ii][j][e] * alpha + (lnfold ? 0.f : bv[j]);
          }
          if (!slab && EPI == EPI_BIAS_GELU && !lnfold) {
            if constexpr (sizeof(TO) == 2 || F8 == 2) {  // bf16 / MX output
              v[0] = gelu_lite2(v[0]);
              v[1] = gelu_lite2(v[1]);
            } else {
              v[0] = gelu_f2(v[0]);
              v[1] = gelu_f2(v[1]);
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rl = 16 * ii + 4 * (lane >> 4) + e;
            st[rl * EP_PITCH + 16 * j + (lane & 15)] = v[e >> 1][e & 1];
          }
        }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int rbase = rbase0 + 32 * p;
      if (slab) {
        float* P = g.P + ((int64_t)batch * gridDim.z + split) * g.M * g.N;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int c = it * 64 + lane;
          const int rl = c >> 4, c4 = (c & 15) * 4;
          const int row = rbase + rl, col = cbase + c4;
          if (row >= g.M || col >= g.N) continue;
          const f32x4 v = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c4]);
          if (col + 4 <= g.N && (g.N & 3) == 0) {
            *reinterpret_cast<f32x4*>(P + (int64_t)row * g.N + col) = v;
          } else {
            for (int t = 0; t < 4 && col + t < g.N; ++t) P[(int64_t)row * g.N + col + t] = v[t];
          }
        }
      } else if constexpr (sizeof(TO) == 2) {
        const unsigned short* R = reinterpret_cast<const unsigned short*>(g.R) + batch * g.sR;
        unsigned short* C = reinterpret_cast<unsigned short*>(g.C) + batch * g.sC;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int c = it * 64 + lane;
          const int rl = c >> 3, c8 = (c & 7) * 8;
          const int row = rbase + rl, col = cbase + c8;
          if (row >= g.M || col >= g.N) continue;
          const f32x4 v0 = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c8]);
          const f32x4 v1 = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c8 + 4]);
          float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          if constexpr (LNOK && (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU)) {
            if (lnfold) {  // y = r acc + (-r mu) s + t, then GELU
              float mu, rs;
              ln_row_stats(g.ln, row, mu, rs);
              const float nrm = -rs * mu;
              const float* sc = g.ln.fold_s + col;
              const float* tc = g.bias + batch * g.sBias + col;
              const f32x4 s0 = *reinterpret_cast<const f32x4*>(sc), s1 = *reinterpret_cast<const f32x4*>(sc + 4);
              const f32x4 t0 = *reinterpret_cast<const f32x4*>(tc), t1 = *reinterpret_cast<const f32x4*>(tc + 4);
              const float ss[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
              const float tt[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
              for (int t = 0; t < 8; ++t) v[t] = __builtin_fmaf(rs, v[t], __builtin_fmaf(nrm, ss[t], tt[t]));
              if (EPI == EPI_BIAS_GELU) {
#pragma unroll
                for (int t = 0; t < 8; t += 2) {
                  const f32x2 gg = gelu_lite2(f32x2{v[t], v[t + 1]});
                  v[t] = gg.x;
                  v[t + 1] = gg.y;
                }
              }
            }
          }
          if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
            const u16x8 rr = *reinterpret_cast<const u16x8*>(R + (int64_t)row * g.ldr + col);
            if (EPI == EPI_BIAS_RESID && lnres) {  // residual = LN(R) as the LN kernel writes it
              float mu, rs;
              ln_row_stats(g.ln, row, mu, rs);
              const f32x4 g0 = *reinterpret_cast<const f32x4*>(g.ln.gamma + col);
              const f32x4 g1 = *reinterpret_cast<const f32x4*>(g.ln.gamma + col + 4);
              const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.ln.beta + col);
              const f32x4 b1 = *reinterpret_cast<const f32x4*>(g.ln.beta + col + 4);
              const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
              const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
              for (int t = 0; t < 8; ++t)
                v[t] += bf16_to_f32(f32_to_bf16(__builtin_fmaf((bf16_to_f32(rr[t]) - mu) * rs, gg[t], bb[t])));
            } else if constexpr (EPI == EPI_DGELU) {
#pragma unroll
              for (int t = 0; t < 8; t += 2) {
                const f32x2 g2 = gelu_grad_f2(f32x2{bf16_to_f32(rr[t]), bf16_to_f32(rr[t + 1])});
                v[t] *= g2.x;
                v[t + 1] *= g2.y;
              }
            } else {
#pragma unroll
              for (int t = 0; t < 8; ++t) v[t] += bf16_to_f32(rr[t]);
            }
          }
          if (EPI == EPI_BIAS_GELU_SAVE) {
            u16x8 pre;
#pragma unroll
            for (int t = 0; t < 8; t += 2) {
              pre[t] = f32_to_bf16(v[t]);
              pre[t + 1] = f32_to_bf16(v[t + 1]);
              const f32x2 g2 = gelu_f2(f32x2{v[t], v[t + 1]});
              v[t] = g2.x;
              v[t + 1] = g2.y;
            }
            *reinterpret_cast<u16x8*>(const_cast<unsigned short*>(R) + (int64_t)row * g.ldr + col) =
                pre;
          }
          if (F8 == 2 && g.cx != nullptr) {
            // MX-fp8 output (the next GEMM's A operand): 4 lanes = one 32-col block;
            // rows / cols past the tile edge are never stored (N, M multiples of 32
            // and 8 for this path, checked by the host)
            uint2 q8;
#pragma unroll
            for (int t = 0; t < 8; ++t) v[t] = bf16_to_f32(f32_to_bf16(v[t]));  // as the bf16 output
            const unsigned e8 = mx_quant8(v, q8);
            unsigned char* C8 = reinterpret_cast<unsigned char*>(g.C);
            *reinterpret_cast<uint2*>(C8 + (int64_t)row * g.ldc + col) = q8;
            if ((lane & 3) == 0) g.cx[mx_scale_index(row, col, g.mpad)] = (unsigned char)e8;
            continue;
          }
          u16x8 o;
#pragma unroll
          for (int t = 0; t < 8; ++t) o[t] = f32_to_bf16(v[t]);
          if (lnout) {  // row partials of the bf16 output (this tile's columns)
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              const float x = bf16_to_f32(o[t]);
              s1 += x;
              s2 = __builtin_fmaf(x, x, s2);
            }
            const int lr = row - m0;
            atomicAdd(&lst[2 * lr], s1);
            atomicAdd(&lst[2 * lr + 1], s2);
          }
#ifdef IRC_PP_DIAG_NOSTORE  // diagnostic build: the epilogue without its C stores
          if (o[0] == 0x7fc1 && o[7] == 0x7fc3)
#endif
          *reinterpret_cast<u16x8*>(C + (int64_t)row * g.ldc + col) = o;
        }
      } else {
        const float* R = reinterpret_cast<const float*>(g.R) + batch * g.sR;
        float* C = reinterpret_cast<float*>(g.C) + batch * g.sC;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int c = it * 64 + lane;
          const int rl = c >> 4, c4 = (c & 15) * 4;
          const int row = rbase + rl, col = cbase + c4;
          if (row >= g.M || col >= g.N) continue;
          f32x4 v = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c4]);
          if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
            const f32x4 r = *reinterpret_cast<const f32x4*>(R + (int64_t)row * g.ldr + col);
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = EPI == EPI_DGELU ? v[t] * gelu_grad_f(r[t]) : v[t] + r[t];
          }
          if (EPI == EPI_BIAS_GELU_SAVE) {
            *reinterpret_cast<f32x4*>(const_cast<float*>(R) + (int64_t)row * g.ldr + col) = v;
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] = gelu_f(v[t]);
          }
          float* dst = C + (int64_t)row * g.ldc + col;
          if (g.accumulate) v += *reinterpret_cast<const f32x4*>(dst);
          *reinterpret_cast<f32x4*>(dst) = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (lnout) {  // this tile's (sum, sum of squares) of every row, one pair per tile column
      lds_barrier();
      const int lr = threadIdx.x >> 1, row = m0 + lr;
      if (row < g.M)
        g.ln.st_out[((int64_t)row * g.ln.nt_out + n0 / BN) * 2 + (threadIdx.x & 1)] = lst[threadIdx.x];
    }
    return;
  }
}

// Threshold epilogue of the scan filter (EPI_SCAN) for one 256-query x 256-doc
// tile: rows = queries, cols = docs.  Needs LDS [0, 4096 + 512 * 128) = [0, PBUF)
// only, so a persistent caller can DMA into buffer 1 meanwhile; `after_init` runs
// right after the first barrier (once the threshold loads are consumed, so the
// compiler's waits for them do not also wait for DMA issued there).
template <typename Fn>
__device__ __forceinline__ void epilogue_scan(const PArgs& g, const f32x4 (&acc)[8][4], char* lds,
                                              int m0, int n0, int tn, int grp, int wn, int lane,
                                              Fn after_init) {
  const int cbase = n0 + 64 * wn;
  // per-query survivor counters + thresholds (key and its float prefilter: key >=
  // thr implies score >= float(thr >> 32) for non-NaN scores).
  PSTAMP(1);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(lds);
  uint64_t* thk = reinterpret_cast<uint64_t*>(lds + 1024);
  float* thf = reinterpret_cast<float*>(lds + 3072);
  if (threadIdx.x < 256) {
    const int q = m0 + threadIdx.x;
    const uint64_t t = (g.thr != nullptr && q < g.M) ? g.thr[q] : 0ull;
    cnt[threadIdx.x] = 0;
    thk[threadIdx.x] = t;
    const uint32_t hi = (uint32_t)(t >> 32);
    // padded query rows never pass; no threshold (hi == 0) admits everything
    thf[threadIdx.x] = q >= g.M ? __builtin_huge_valf()
                                : (hi == 0 ? -__builtin_huge_valf() : unorderable_f32(hi));
  }
  lds_barrier();
  after_init();
#ifdef IRC_PP_SCAN_NOEPI  // diagnostic build: main loop + counters only
  if (threadIdx.x < 256 && m0 + (int)threadIdx.x < g.qpad)
    g.counts[(int64_t)tn * g.qpad + m0 + threadIdx.x] = acc[0][0][0] == 12345.f ? 1u : 0u;
  return;
#endif
  // Pass test of the lane's 128 scores (bit 16 i + 4 j + e) as a branch-free
  // mask; then per quarter (i = 2 qq, 2 qq + 1) the lane's 32 accumulators are
  // staged in its private 128-B LDS slot (8 x 16-byte writes, unconditional) and
  // only the set bits (a few per lane: the threshold admits ~16k of N per query)
  // read their score back by a dynamic LDS index for the exact-key / slot / store
  // path.  The slot's 16-byte chunk c sits at position c ^ ((lane >> 1) & 7): the
  // 16 lanes of one ds_write_b128 group then cover all 64 banks (slots 128 B apart).
  float* slotv = reinterpret_cast<float*>(lds + 4096) + threadIdx.x * 32;
  const int sw = (lane >> 1) & 7;
  uint64_t pm[2] = {0, 0};
  const float* thq = thf + 128 * grp + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f32x4 tf = *reinterpret_cast<const f32x4*>(&thq[16 * i]);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int bit = 16 * i + 4 * j + e;
        pm[bit >> 6] |= (uint64_t)(!(acc[i][j][e] < tf[e])) << (bit & 63);
      }
  }
  PSTAMP(2);
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    uint32_t bits = (uint32_t)(pm[qq >> 1] >> (32 * (qq & 1)));
    if (__ballot(bits != 0) == 0) continue;  // wave-uniform
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(slotv + 4 * ((4 * i + j) ^ sw)) = acc[2 * qq + i][j];
    while (__ballot(bits != 0) != 0) {
      if (bits != 0) {
        const int b = __builtin_ctz(bits);
        bits &= bits - 1;
        const float v = slotv[4 * ((b >> 2) ^ sw) + (b & 3)];
        const int bit = 32 * qq + b;
        const int ql = 128 * grp + 16 * (bit >> 4) + 4 * (lane >> 4) + (bit & 3);
        const int q = m0 + ql;
        const int d = cbase + 16 * ((bit >> 2) & 3) + (lane & 15);
        if (q < g.M && d < g.N) {
          const uint64_t key = make_key(v, g.idx_base + (uint32_t)d * (uint32_t)g.stride);
          if (key >= thk[ql]) {
            const uint32_t slot = atomicAdd(&cnt[ql], 1u);
            g.keys[((int64_t)tn * g.qpad + q) * g.cap + slot] = key;
          }
        }
      }
    }
  }
  PSTAMP(3);
  lds_barrier();
  PSTAMP(4);
  if (threadIdx.x < 256 && m0 + (int)threadIdx.x < g.qpad)
    g.counts[(int64_t)tn * g.qpad + m0 + threadIdx.x] = cnt[threadIdx.x];
}

// Single-pass filter epilogue (g.lists != null, no threshold): the 4 largest keys of
// every (query, 256-doc tile), exact, for select_dense (scan_topk.hip), which rescans
// a tile whose 4th key reaches the k-th key of all lists (the tile may hold more
// winners).  Four passes of 64 queries: the owning group stages its 64 x 256 fp32
// scores in LDS (row-major, 1 KB rows; column c of row r at c ^ 32 (r & 1), so the
// readers' ds_read_b128 lane groups -- 4 rows, 4 chunks each -- cover 64 distinct
// banks), then thread t takes query t >> 3 and the 32 docs {4 (t & 7) + 32 c + e}:
// the top 4 of its docs by insertion in increasing doc order (strict >, so a tie keeps
// the lower index), then three xor-shuffle rounds with its 7 neighbours (bitonic
// 4 + 4 -> 4 under (score desc, doc asc)).  Ragged docs (>= N) never enter; padded
// query rows (>= M) are not stored.  Doc d's global index is idx_base + d * stride
// (stride > 1: the threshold sample of the sampled pipeline, B rows ldb apart).  LDS [0, 64 KB) < PBUF, so a persistent caller's
// prestage into buffer 1 may run meanwhile.
__device__ __forceinline__ bool top_better(float va, int ia, float vb, int ib) {
  return va > vb || (va == vb && ia < ib);
}
__device__ __forceinline__ void top_cswap(float& va, int& ia, float& vb, int& ib) {
  const bool sw = top_better(vb, ib, va, ia);
  const float tv = sw ? vb : va, uv = sw ? va : vb;
  const int ti = sw ? ib : ia, ui = sw ? ia : ib;
  va = tv; ia = ti; vb = uv; ib = ui;
}
template <typename Fn>
__device__ __forceinline__ void epilogue_scan_lists(const PArgs& g, const f32x4 (&acc)[8][4],
                                                    char* lds, int m0, int n0, int tn, int grp,
                                                    int wn, int lane, Fn after_init) {
  float* S = reinterpret_cast<float*>(lds);
  after_init();
  const int tid = threadIdx.x;
  const int rq = tid >> 3, seg = tid & 7, flip = rq & 1;
  const int nval = g.N - n0;  // docs of this tile
  const float NEG = -__builtin_huge_valf();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (grp == (p >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 16 * ii + 4 * (lane >> 4) + e;
            const int c = (64 * wn + 16 * j + (lane & 15)) ^ ((e & 1) << 5);
            S[r * 256 + c] = acc[4 * (p & 1) + ii][j][e];
          }
    }
    lds_barrier();
    float tv[4] = {NEG, NEG, NEG, NEG};
    int ti[4] = {0x7fffffff, 0x7fffffff, 0x7fffffff, 0x7fffffff};
    const float* row = S + rq * 256 + 4 * seg;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(row + 32 * (c ^ flip));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int pos = 4 * seg + 32 * c + e;
        const float x = pos < nval ? v[e] : NEG;
        if (x > tv[3]) {
          const bool c0 = x > tv[0], c1 = x > tv[1], c2 = x > tv[2];
          tv[3] = c2 ? tv[2] : x;
          ti[3] = c2 ? ti[2] : pos;
          tv[2] = c1 ? tv[1] : (c2 ? x : tv[2]);
          ti[2] = c1 ? ti[1] : (c2 ? pos : ti[2]);
          tv[1] = c0 ? tv[0] : (c1 ? x : tv[1]);
          ti[1] = c0 ? ti[0] : (c1 ? pos : ti[1]);
          tv[0] = c0 ? x : tv[0];
          ti[0] = c0 ? pos : ti[0];
        }
      }
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      float bv[4];
      int bi[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bv[r] = __shfl_xor(tv[r], m, 64);
        bi[r] = __shfl_xor(ti[r], m, 64);
      }
      // max of own (desc) and partner reversed (asc): a bitonic sequence holding the top 4
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (top_better(bv[3 - r], bi[3 - r], tv[r], ti[r])) {
          tv[r] = bv[3 - r];
          ti[r] = bi[3 - r];
        }
      }
      top_cswap(tv[0], ti[0], tv[2], ti[2]);
      top_cswap(tv[1], ti[1], tv[3], ti[3]);
      top_cswap(tv[0], ti[0], tv[1], ti[1]);
      top_cswap(tv[2], ti[2], tv[3], ti[3]);
    }
    const int q = m0 + 64 * p + rq;
    if (seg == 0 && q < g.M) {
      uint64_t kk[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        kk[r] = tv[r] == NEG ? 0ull
                             : make_key(tv[r], g.idx_base + (uint32_t)(n0 + ti[r]) * (uint32_t)g.stride);
      uint64_t* dst = g.lists + ((int64_t)q * g.ls + tn) * 4;
      reinterpret_cast<ulonglong2*>(dst)[0] = make_ulonglong2(kk[0], kk[1]);
      reinterpret_cast<ulonglong2*>(dst)[1] = make_ulonglong2(kk[2], kk[3]);
    }
    lds_barrier();  // every reader is done with S before the next pass writes it
  }
}

template <bool AK, bool BK_, typename TO, int EPI, int F8 = 0, bool LN = false>
__global__ __launch_bounds__(NT, 1) void gemm_pp_kernel(PArgs g) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const int tiles_m = (g.M + BM - 1) / BM;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  // XCD-aware bijective remap over the whole grid: workgroups go to the 8 XCDs round
  // robin in dispatch order (x fastest), so XCD x gets the contiguous run x of the work
  // list (batch, split, tile), tile fastest -- the tiles of one K-slice / batch entry
  // share their A and B K-tiles through one XCD's L2 (the K-outer dW GEMMs of the
  // trainable encoder read 3.4-5x their operand bytes from HBM when the slices of a run
  // spread over every XCD, profiles/r04_h_pmc_shapes_bert.txt)
  int bid, batch, split;
  {
    const int nz = gridDim.y * gridDim.z;
    const int total = ntiles * nz;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int q = total / 8, r = total % 8, x = lin % 8;
    const int w = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lin / 8;
    bid = w % ntiles;
    const int rest = w / ntiles;
    split = rest % gridDim.z;
    batch = rest / gridDim.z;
  }
  // EPI_SCAN: query tiles fastest, so the blocks of one doc tile run back to back
  // on one XCD and read it from that XCD's L2 (C4: 2048 queries = 8 query tiles)
  int tm, tn;
  if (EPI == EPI_SCAN) {
    tm = bid % tiles_m;
    tn = bid / tiles_m;
  } else {
    grouped_tile(bid, tiles_m, tiles_n, g.group_m, tm, tn);
  }
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int nk = (kend - kbeg) / BK;
  const unsigned short* A = g.A + batch * g.sA;
  const unsigned short* B = g.B + batch * g.sB;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wq = wave & 3;  // group = row half; wq = wave within group
  const int wn = wq;                          // 64-column slab of the tile

  if (EPI == EPI_SCAN) PSTAMP(0);
  f32x4 acc[8][4];
  mainloop<AK, BK_, F8>(g, A, B, m0, n0, kbeg, nk, lds, buf_bytes(AK, BK_), 0, false, acc, grp,
                        wq, lane, nullptr, 0);

  // ---------------------------------------------------------------- epilogue
  // acc[i][j] element e -> row 128 grp + 16 i + 4 (lane >> 4) + e, col 64 wn + 16 j + (lane & 15)
  const int rbase0 = m0 + 128 * grp;
  const int cbase = n0 + 64 * wn;
  if constexpr (EPI == EPI_SCAN) {
    if (g.lists != nullptr)
      epilogue_scan_lists(g, acc, lds, m0, n0, tn, grp, wn, lane, [] {});
    else
      epilogue_scan(g, acc, lds, m0, n0, tn, grp, wn, lane, [] {});
    return;
  }
#ifdef IRC_PP_DIAG_NOEPI  // diagnostic build: main loop only (a guarded store of the sum of
  {                        // every accumulator keeps all the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) reinterpret_cast<float*>(g.C)[threadIdx.x] = t;
    return;
  }
#endif
  if (g.P != nullptr || g.vec_c) {
    epilogue_vec<TO, EPI, F8, LN>(g, acc, lds, m0, n0, batch, grp, wn, wave, lane, split);
    return;
  }
  // scalar epilogue (unaligned C / R)
  const float* bias = g.bias ? g.bias + batch * g.sBias : nullptr;
  const TO* R = reinterpret_cast<const TO*>(g.R) + (g.R ? batch * g.sR : 0);
  TO* C = reinterpret_cast<TO*>(g.C) + batch * g.sC;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = cbase + 16 * j + (lane & 15);
    if (col >= g.N) continue;
    const float bvv = has_bias(EPI) ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase0 + 16 * i + 4 * (lane >> 4) + e;
        if (row >= g.M) continue;
        float v = acc[i][j][e] * g.alpha + bvv;
        if (EPI == EPI_BIAS_GELU) v = sizeof(TO) == 2 ? gelu_lite(v) : gelu_f(v);
        if (EPI == EPI_BIAS_GELU_SAVE) {
          TO* pre = const_cast<TO*>(R) + (int64_t)row * g.ldr + col;
          if constexpr (sizeof(TO) == 2)
            *reinterpret_cast<unsigned short*>(pre) = f32_to_bf16(v);
          else
            *reinterpret_cast<float*>(pre) = v;
          v = gelu_f(v);
        }
        if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU) {
          float r;
          if constexpr (sizeof(TO) == 2)
            r = bf16_to_f32(reinterpret_cast<const unsigned short*>(R)[(int64_t)row * g.ldr + col]);
          else
            r = reinterpret_cast<const float*>(R)[(int64_t)row * g.ldr + col];
          v = EPI == EPI_DGELU ? v * gelu_grad_f(r) : v + r;
        }
        TO* dst = C + (int64_t)row * g.ldc + col;
        if constexpr (sizeof(TO) == 2) {
          *reinterpret_cast<unsigned short*>(dst) = f32_to_bf16(v);
        } else {
          if (g.accumulate)
            *reinterpret_cast<float*>(dst) += v;
          else
            *reinterpret_cast<float*>(dst) = v;
        }
      }
  }
}

// Persistent form of the same tile (batch 1, no split-K, vectorised epilogue), for
// launches of more tiles than CUs.  Each workgroup runs tiles until none is left:
// its first tile by the XCD-aware map of blockIdx over the first G tiles, every
// later one fetched from a per-launch tile counter (dynamic, so workgroups that
// start late -- CUs held by kernels of other streams, e.g. the heads' cluster
// recurrences beside the BERT prefetch -- take fewer tiles instead of stretching the
// launch).  Between two tiles, the next tile's first K-tile is DMA'd into LDS
// buffer 1 while this tile's epilogue stages through buffer 0 (buffers PBUF apart,
// PBUF = the 8 waves' staging rows), and the counter fetch for the tile after
// that is in flight meanwhile, so neither the prologue DMA nor the fetch is exposed.
// ctr[0] = tiles handed out past G, ctr[1] = finished workgroups; the last one to
// finish zeroes both for the next launch that uses this counter slot.
constexpr int PBUF = 8 * 32 * EP_PITCH * 4;  // 69,632 B
static_assert(PBUF >= buf_bytes(false, false) && 2 * PBUF <= LDS_BYTES, "persistent LDS plan");

template <bool AK, bool BK_, typename TO, int EPI, int F8 = 0>
__global__ __launch_bounds__(NT, 1) void gemm_pp_pers_kernel(PArgs g, uint32_t* ctr, int mode) {
  // mode 1: dynamic tiles + prestage; 2: static waves of G tiles + prestage;
  // 3: static, no prestage (A/B of what each part buys)
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  __shared__ int s_next;
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  // tile -> (row tile, col tile) as gemm_pp_kernel: EPI_SCAN walks query tiles fastest
  auto tile_m = [&](int t) {
    int tm, tn;
    grouped_tile(t, tiles_m, tiles_n, g.group_m, tm, tn);
    return EPI == EPI_SCAN ? t % tiles_m : tm;
  };
  auto tile_n = [&](int t) {
    int tm, tn;
    grouped_tile(t, tiles_m, tiles_n, g.group_m, tm, tn);
    return EPI == EPI_SCAN ? t / tiles_m : tn;
  };
  const int G = gridDim.x;  // <= ntiles
  int slot;
  {
    const int q = G / 8, r = G % 8, x = blockIdx.x % 8;
    slot = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blockIdx.x / 8;
  }
  int tile = slot;
  const bool dyn = mode == 1, pre = mode != 3;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wq = wave & 3;
  const int nk = g.K / BK;
  int pending = G + slot;  // the tile after the next one (thread 0 when dynamic)
  if (dyn && threadIdx.x == 0) pending = G + (int)atomicAdd(ctr, 1u);
  if (pre)
    stage_tile<AK, BK_>(g, g.A, g.B, tile_m(tile) * BM, tile_n(tile) * BN, 0, lds + PBUF, grp, wq,
                        lane);
  f32x4 acc[8][4];
  while (true) {
    // a lane index the compiler must re-derive per tile: otherwise it hoists the
    // epilogue's and the DMA's per-lane addresses out of this loop, keeps them live
    // through the K loop and spills
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int tn = tile_n(tile);
    const int m0 = tile_m(tile) * BM, n0 = tn * BN;
    mainloop<AK, BK_, F8>(g, g.A, g.B, m0, n0, 0, nk, lds, PBUF, 1, pre, acc, grp, wq, ln,
                          dyn ? &s_next : nullptr, pending);
    int next;
    if (dyn) {
      // published before the loop's last barrier (uniform: keep it in an SGPR)
      next = __builtin_amdgcn_readfirstlane(s_next);
      if (next < ntiles && threadIdx.x == 0) pending = G + (int)atomicAdd(ctr, 1u);
    } else {
      next = tile + G;
    }
    auto prestage = [&] {
      if (pre && next < ntiles)
        stage_tile<AK, BK_>(g, g.A, g.B, tile_m(next) * BM, tile_n(next) * BN, 0, lds + PBUF, grp,
                            wq, ln);
    };
    if constexpr (EPI == EPI_SCAN) {
      if (g.lists != nullptr)
        epilogue_scan_lists(g, acc, lds, m0, n0, tn, grp, wq, ln, prestage);
      else
        epilogue_scan(g, acc, lds, m0, n0, tn, grp, wq, ln, prestage);
    } else {
      prestage();
      epilogue_vec<TO, EPI, F8>(g, acc, lds, m0, n0, 0, grp, wq, wave, ln);
    }
    if (next >= ntiles) break;
    tile = next;
    if (!pre) wg_barrier();  // every wave's epilogue is done with buffer 0
  }
  if (dyn && threadIdx.x == 0 && atomicAdd(ctr + 1, 1u) == (uint32_t)G - 1) {
    atomicExch(ctr, 0u);
    atomicExch(ctr + 1, 0u);
  }
}

}  // namespace gpp

// ------------------------------------------------------------------ host side
// Called from irc_gemm (gemm.hip) for bf16 inputs.  Returns -1 when the shape /
// alignment does not qualify (the caller then uses the general 128x128 kernel).
// la/lb: 0 = K-major (A [M][K] / B [N][K]), 1 = K-outer (A [K][M] / B [K][N]).
namespace gpp {

template <bool AK, bool BKM, typename TO>
static void launch_epi(int epi, const PArgs& a, dim3 grid, hipStream_t st) {
  switch (epi) {
#define IRC_PP(E)                                                                           \
  case E:                                                                                   \
    hipLaunchKernelGGL((gemm_pp_kernel<AK, BKM, TO, E>), grid, dim3(NT), 0, st, a); \
    break;
    IRC_PP(0) IRC_PP(1) IRC_PP(2) IRC_PP(3) IRC_PP(4) IRC_PP(5) IRC_PP(6)
#undef IRC_PP
  }
}

template <typename TO>
static void launch_layout(int la, int lb, int epi, const PArgs& a, dim3 grid, hipStream_t st);

extern "C" int irc_pp_dbg_stamps(uint64_t* out /* [16] */) {
#ifdef IRC_SCAN_STAMPS
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pp_stamps), sizeof(pp_stamps)) == hipSuccess ? 0 : -1;
#else
  (void)out;
  return -1;
#endif
}

// The persistent form is off by default (BERT shapes within +-2%, the GEMM scan filter
// +3% at C2, profiles/r02_gemm_ab_f_*); irc_gemm_set_persistent switches it at run time
// (the tests compare every mode bit for bit).
static std::atomic<int>& pers_mode() {
  static std::atomic<int> on{0};
  return on;
}
static bool pers_enabled() { return pers_mode().load(std::memory_order_relaxed) != 0; }

int cu_count() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = -1;
    cus[dev] = n;
  }
  return cus[dev];
}

// Tile-counter slots of the persistent launches, one 64-byte slot per launch in
// rotation (so launches on concurrent streams never share one); zeroed once, and
// each launch leaves its slot zeroed again.  A launch being captured into a HIP
// graph gets no slot (nullptr: the caller takes the one-tile-per-workgroup
// kernel): a replay would keep its slot forever while the rotation hands the
// same slot to a later eager launch that may run beside that replay.
constexpr int PERS_SLOTS = 1024;
static uint32_t* pers_counter(hipStream_t st) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone)
    return nullptr;
  static std::mutex mu;
  static uint32_t* base[64] = {};
  static std::atomic<uint32_t> next{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (base[dev] == nullptr) {
      void* p = nullptr;
      if (hipMalloc(&p, PERS_SLOTS * 64) != hipSuccess) return nullptr;
      if (hipMemset(p, 0, PERS_SLOTS * 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(p);
        return nullptr;
      }
      base[dev] = static_cast<uint32_t*>(p);
    }
  }
  return base[dev] + (next.fetch_add(1) % PERS_SLOTS) * 16;
}

void run_scan(const PArgs& a, hipStream_t st, bool fp8) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  if (pers_enabled()) {
    const int ncu = cu_count();
    uint32_t* ctr = (ncu > 0 && tiles > ncu) ? pers_counter(st) : nullptr;
    if (ctr != nullptr) {
      const int mode = pers_mode().load(std::memory_order_relaxed);
      if (fp8)
        hipLaunchKernelGGL((gemm_pp_pers_kernel<true, true, float, EPI_SCAN, true>), dim3(ncu),
                           dim3(NT), 0, st, a, ctr, mode);
      else
        hipLaunchKernelGGL((gemm_pp_pers_kernel<true, true, float, EPI_SCAN>), dim3(ncu), dim3(NT),
                           0, st, a, ctr, mode);
      return;
    }
  }
  if (fp8)
    hipLaunchKernelGGL((gemm_pp_kernel<true, true, float, EPI_SCAN, true>), dim3((unsigned)tiles),
                       dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_pp_kernel<true, true, float, EPI_SCAN>), dim3((unsigned)tiles),
                       dim3(NT), 0, st, a);
}

void run_scores_fp8(const PArgs& a, hipStream_t st) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  hipLaunchKernelGGL((gemm_pp_kernel<true, true, float, EPI_NONE, true>), dim3((unsigned)tiles),
                     dim3(NT), 0, st, a);
}

void run_mx(int epi, const PArgs& a, hipStream_t st) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  const dim3 grid((unsigned)tiles);
  switch (epi) {
#define IRC_PPX(E)                                                                        \
  case E:                                                                                 \
    hipLaunchKernelGGL((gemm_pp_kernel<true, true, unsigned short, E, 2>), grid, dim3(NT), 0, \
                       st, a);                                                            \
    break;
    IRC_PPX(0) IRC_PPX(1) IRC_PPX(2) IRC_PPX(3)
#undef IRC_PPX
  }
}

void run_fp8(int epi, const PArgs& a, hipStream_t st) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  const dim3 grid((unsigned)tiles);
  switch (epi) {
#define IRC_PP8(E)                                                                          \
  case E:                                                                                   \
    hipLaunchKernelGGL((gemm_pp_kernel<true, true, unsigned short, E, true>), grid, dim3(NT), \
                       0, st, a);                                                           \
    break;
    IRC_PP8(0) IRC_PP8(1) IRC_PP8(2) IRC_PP8(3)
#undef IRC_PP8
  }
}

// LayerNorm-fold GEMM (irc_gemm_ln): bf16 A / B K-major, bf16 C, epilogues 1-3
void run_ln(int epi, const PArgs& a, hipStream_t st) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  const dim3 grid((unsigned)tiles);
  switch (epi) {
#define IRC_PPL(E)                                                                             \
  case E:                                                                                      \
    hipLaunchKernelGGL((gemm_pp_kernel<true, true, unsigned short, E, 0, true>), grid, dim3(NT), \
                       0, st, a);                                                              \
    break;
    IRC_PPL(1) IRC_PPL(2) IRC_PPL(3)
#undef IRC_PPL
  }
}

template <typename TO>
static void launch_layout(int la, int lb, int epi, const PArgs& a, dim3 grid, hipStream_t st) {
  if (la == 0 && lb == 0) launch_epi<true, true, TO>(epi, a, grid, st);
  else if (la == 0) launch_epi<true, false, TO>(epi, a, grid, st);
  else if (lb == 0) launch_epi<false, true, TO>(epi, a, grid, st);
  else launch_epi<false, false, TO>(epi, a, grid, st);
}

}  // namespace gpp
}  // namespace irc

namespace irc {
namespace gpp {

int device_cu_count() {
  const int n = cu_count();
  return n > 0 ? n : 256;
}

// Split count: fill (at most) one wave of 256 blocks when the output tile grid
// alone cannot (fp32 C, no fused epilogue), each K slice >= 1024 deep.
int splits_for(int out_f32, int epi, int64_t M, int64_t N, int64_t K, int64_t batch,
               int64_t budget) {
  if (!out_f32 || epi != 0) return 1;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256) * batch;
  if (tiles >= 160) return 1;
  int64_t s = budget / tiles;        // at most `budget` blocks (256: one wave on 256 CUs)
  const int64_t smax = K / 1024;     // >= 16 K-tiles per slice
  if (s > smax) s = smax;
  if (s > 32) s = 32;
  if (s < 2) return 1;
  const int64_t chunk = ((K + s - 1) / s + 63) / 64 * 64;
  return (int)((K + chunk - 1) / chunk);
}

// Does the ping-pong kernel take this bf16 GEMM?  la/lb: 0 = K-major, 1 = K-outer.
bool qualifies(int la, int lb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
               int64_t sA, const void* B, int64_t ldb, int64_t sB, int64_t batch, int splits) {
  if (K % 64 != 0 || K == 0) return false;
  // both operands K-outer with a small output (split-K slab traffic dominates):
  // the 128x128 kernel's smaller slabs are faster
  if (la == 1 && lb == 1 && ((M + 255) / 256) * ((N + 255) / 256) * batch < 16) return false;
  // Wave quantisation on the CUs: the 256x384 big-tile kernel wins where its waves
  // cost less than the 256x256 tiles' -- one big tile is 1.5 of them (N = 768 / 2304
  // at M = 512 L: 252 big tiles in one wave against 378 in two at L = 63; a batch's
  // joint padding rarely lands on L = 64, and requiring whole waves of big tiles sent
  // every other L to 1.5 waves of 256x256 tiles: 9.29 vs 8.18 ms per C2 step).  Ties
  // go to the big-tile kernel too (FFN1 + GELU, N = 3072: 4 waves of 256x384 against 6 of
  // 256x256): alone the two are within a few us either way from box to box, but in the
  // overlapped C2 step the big tiles gain 4%: 30.9-31.0k vs 29.6-29.7k pairs/s, three
  // interleaved pairs (profiles/r05_y_ties_ab.txt, r05_w_ffn1_pp_vs_big.txt).
  if (la == 0 && lb == 0 && N % 384 == 0) {
    const int64_t t384 = ((M + 255) / 256) * (N / 384) * batch;
    const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256) * batch;
    int64_t ncu = cu_count();
    if (ncu <= 0) ncu = 256;
    if (3 * ((t384 + ncu - 1) / ncu) <= 2 * ((t256 + ncu - 1) / ncu)) return false;
  }
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16) return false;
  if (lda % 8 || ldb % 8 || sA % 8 || sB % 8) return false;
  if (la == 1 && M % 8) return false;
  if (lb == 1 && N % 8) return false;
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  return tiles * batch * splits >= 32;
}

template <bool AK, bool BKM, typename TO>
static void launch_pers(int epi, const PArgs& a, unsigned grid, uint32_t* ctr, hipStream_t st) {
  const int mode = pers_mode().load(std::memory_order_relaxed);
  switch (epi) {
#define IRC_PPP(E)                                                                       \
  case E:                                                                                \
    hipLaunchKernelGGL((gemm_pp_pers_kernel<AK, BKM, TO, E>), dim3(grid), dim3(NT), 0, st, a, \
                       ctr, mode);                                                           \
    break;
    IRC_PPP(0) IRC_PPP(1) IRC_PPP(2) IRC_PPP(3) IRC_PPP(4) IRC_PPP(5) IRC_PPP(6)
#undef IRC_PPP
  }
}

void run(int out_f32, int la, int lb, int epi, const PArgs& a, int64_t batch, int splits,
         hipStream_t st, int64_t max_grid) {
  const int64_t tiles = ((int64_t)(a.M + 255) / 256) * ((a.N + 255) / 256);
  // persistent form: one launch-wide pass over more tiles than CUs (or than the caller's
  // grid cap), A K-major
  const bool pers_ok = splits == 1 && batch == 1 && a.vec_c && la == 0;
  const int ncu = pers_ok ? cu_count() : 0;
  int64_t pgrid = 0;
  uint32_t* ctr = nullptr;
  if (pers_ok && max_grid > 0 && tiles > max_grid && (ncu <= 0 || max_grid < ncu)) {
    // the caller's cap: static waves of max_grid tiles (the dynamic mode takes its
    // counter slot as usual; without one, the static form needs none)
    pgrid = max_grid;
    if (pers_mode().load(std::memory_order_relaxed) == 1) ctr = pers_counter(st);
    if (pers_mode().load(std::memory_order_relaxed) == 1 && ctr == nullptr) pgrid = 0;
  } else if (pers_ok && pers_enabled() && ncu > 0 && tiles > ncu) {
    ctr = pers_counter(st);
    pgrid = ctr != nullptr ? ncu : 0;
  }
  if (pgrid > 0) {
    if (out_f32) {
      if (lb == 0) launch_pers<true, true, float>(epi, a, (unsigned)pgrid, ctr, st);
      else launch_pers<true, false, float>(epi, a, (unsigned)pgrid, ctr, st);
    } else {
      if (lb == 0) launch_pers<true, true, unsigned short>(epi, a, (unsigned)pgrid, ctr, st);
      else launch_pers<true, false, unsigned short>(epi, a, (unsigned)pgrid, ctr, st);
    }
    return;
  }
  const dim3 grid((unsigned)tiles, (unsigned)batch, (unsigned)splits);
  if (splits > 1)  // raw fp32 slabs, no epilogue (reduced afterwards)
    launch_layout<float>(la, lb, 0, a, grid, st);
  else if (out_f32)
    launch_layout<float>(la, lb, epi, a, grid, st);
  else
    launch_layout<unsigned short>(la, lb, epi, a, grid, st);
}

}  // namespace gpp
}  // namespace irc

// Persistent tile loop mode of the 256x256 GEMM (0 off, 1-3 see irc.h); returns the previous one.
extern "C" int irc_gemm_set_persistent(int mode) {
  return irc::gpp::pers_mode().exchange(mode < 0 ? 0 : mode > 3 ? 1 : mode);
}
