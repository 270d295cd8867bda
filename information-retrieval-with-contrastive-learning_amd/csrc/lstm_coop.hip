// Multi-CU MFMA BiLSTM recurrences for the production head width H = 256
// (reference: nn.LSTM in src/model.py:16-22, 39 -- gate order i, f, g, o, zero
// initial state, the padded sequence processed as is).
//
// Why: a single-CU recurrence must stream all of W_hh (512 KB bf16 per
// direction) through one CU every step; the per-CU L2 path bounds that at
// ~3.4 us/step.  Here each (group of 32 sequences, direction) is a CLUSTER of
// P = 4 workgroups, one per CU, each holding a quarter of W_hh (128 KB) resident
// for the whole sequence -- in VGPRs since round 5 (each wave's MFMA B fragments,
// 128 VGPRs of its 406 / 360; re-read from LDS every step they set the MFMA phase:
// forward 287 -> 267 us, backward 357 -> 304 us per layer at C2,
// profiles/r05_p_coop.txt; with the v_rcp_f32 gates below 221 / 291 us,
// profiles/r05_q_coop.txt) -- so the per-step traffic is only the hidden state
// exchange.  One workgroup per CU by VGPRs (4 waves at > 256 each).
//
// Forward: member m owns hidden units [64m, 64m+64) and all four gates of them;
//   per step gates[32 x 256] = xp_t + h_{t-1}[32 x 256] . W_slice with
//   v_mfma_f32_16x16x32_bf16 (wave w: 16 units x 4 gates, 2 row blocks); the
//   cell update is lane-local (c in registers); the member's 4 KB slice of h_t
//   is published and the other three slices gathered into LDS.
// Backward (K-split): member m holds dgates of its own units (32 x 256: the A
//   operand, local) and W_hh rows of those gate columns; it computes a PARTIAL
//   dh over all 256 units, publishes it (fp32), and sums the four partials of
//   its own units in member order 0..3 (deterministic).
//
// Inter-workgroup hand-off (cdna_hip_programming.md Guideline 16, form R2: the
// data IS the flag): every 32-bit payload word travels in an 8-byte granule
// {tag = epoch, value} stored write-through (relaxed agent-scope atomic store =
// global_store_dwordx2 sc1) and read with relaxed agent-scope atomic loads
// (global_load_dwordx2 sc1); a consumer wave re-reads its granules until every
// tag equals the step's epoch (bounded spins).  No flag, drain or fence.  Buffers
// are double-buffered by step parity (a member can be at most one step ahead of
// any other) and zeroed by hipMemsetAsync every call (tag 0 is never an epoch).
// Co-residency: <= 16 groups per launch (<= 128 workgroups per direction pair,
// one per CU), so two concurrent launches (query and key encoders) fit
// the 256 CUs; spins are bounded and set a timeout word instead of hanging.
#include <cstdlib>

#include "irc_common.h"

namespace irc {
namespace lstmc {

constexpr int H = 256;
constexpr int P = 4;            // workgroups per cluster
constexpr int BG = 32;          // sequences per group
constexpr int NW = 4;           // waves per workgroup
constexpr int NTH = NW * 64;
constexpr int UPW = H / P;      // 64 units per member
constexpr int UPV = UPW / NW;   // 16 units per wave (forward)
constexpr int KKF = H / 32;     // forward k-steps (K = 256)
constexpr int HP = H + 8;       // LDS row pitch (bf16) of h / dgates
constexpr int WSLICE = 4 * UPW * H;          // bf16 elements of one member's W slice (64K)
constexpr int GSTEP = BG * 4 * H;            // floats of gates per (dir, group, t)
constexpr int CSTEP = BG * H;                // floats of c per (dir, group, t)
constexpr int MAX_GROUPS = 16;               // per launch (co-residency bound)
constexpr unsigned SPIN_MAX = 1u << 24;      // default spin bound (IRC_LSTM_COOP_SPIN_MAX)
constexpr int NFLAG = P * NW;                // backward flag words per (dir, group)

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// v_rcp_f32 (1 ulp) instead of the correctly rounded division (~12 instructions with its
// scale / fixup and denormal-mode switches): 40 of them per lane per step were most of
// the recurrence's cell update (profiles/r05_p_coop_stamps.txt)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f;
}

__device__ __forceinline__ void st_sc1(void* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_sc1(const void* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long granule(unsigned epoch, unsigned v) {
  return ((unsigned long long)epoch << 32) | v;
}

// Two adjacent granules in ONE 16-byte write-through store (global_store_dwordx4
// sc1: ~2.7x cheaper per byte than two dwordx2 sc1 stores; each 8-byte half is
// observed untorn on gfx950).  Inline asm: the compiler does not count it in
// vmcnt, which only makes its in-order waits for later loads stricter (safe);
// nothing waits on this store's completion (form R2).  The trailing s_nop: a
// store of more than 8 bytes reads its data VGPRs late, so the next VALU op must
// not overwrite them for 2 wait states -- a hazard the compiler pads for its own
// stores but cannot see inside inline asm (without it the next v_accvgpr_read /
// v_mov into the data registers corrupts the stored value).
__device__ __forceinline__ void st_sc1_pair(void* p, unsigned long long a, unsigned long long b) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

// One wave sweeps its N granules (addresses from addr(k)) until every tag ==
// epoch; values out.  Wave-uniform loop; on timeout sets tmo + the LDS abort word.
template <int N, typename F>
__device__ __forceinline__ void sweep(F addr, unsigned epoch, unsigned (&v)[N], unsigned* tmo,
                                      int* abort_lds, unsigned spin_max) {
  for (unsigned spins = 0;;) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const unsigned long long x = ld_sc1(addr(k));
      v[k] = (unsigned)x;
      ok &= (unsigned)(x >> 32) == epoch;
    }
    if (__all(ok) && spin_max) return;  // spin_max 0: forced timeout (debug)
    if (++spins > spin_max) {
      if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *abort_lds = 1;
      }
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte write-through store / load (global_*_dwordx4 sc1) for the flag-based
// hand-off (form R1); the store pads the data-VGPR hazard as st_sc1_pair does.  The asm store is drained by the explicit vmcnt(0) before
// the flag; the asm loads are completed by wait_loaded(), which takes the
// loaded registers as in/out operands so no use can be scheduled before it.
__device__ __forceinline__ void st_sc1_x4(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u32x4 ld_sc1_x4(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// R1 publish: every storing wave drains its stores, barrier, one lane sets the flag.
__device__ __forceinline__ void publish_flag(unsigned* flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store((gu32*)flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// R1 consume: wave 0 polls the P member flags (word NW*member; relaxed, >= epoch),
// then a barrier.
__device__ __forceinline__ void poll_flags(unsigned* flags, unsigned epoch, unsigned* tmo,
                                           int* abort_lds, unsigned spin_max) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    for (unsigned spins = 0;;) {
      bool ok = true;
      if (lane < P)
        ok = __hip_atomic_load((gu32*)(flags + lane * NW), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok) && spin_max) break;
      if (++spins > spin_max) {
        if (lane == 0) {
          __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *abort_lds = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// Wave 0 polls one sentinel granule per producer (lanes 0..P-1; cheap, while the
// producers may still be computing) until every tag == epoch, then a barrier; the
// full sweep that follows then normally needs a single pass.
__device__ __forceinline__ void poll_sentinels(const unsigned long long* const* sent,
                                               unsigned epoch, unsigned* tmo, int* abort_lds,
                                               unsigned spin_max) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    for (unsigned spins = 0;;) {
      bool ok = true;
      if (lane < P) ok = (unsigned)(ld_sc1(sent[lane]) >> 32) == epoch;
      if (__all(ok) && spin_max) break;
      if (++spins > spin_max) {
        if (lane == 0) {
          __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *abort_lds = 1;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

// Cluster decode: blocks b, b+8, b+16, b+24 of each 32-block chunk are the 4
// members of group (chunk*8 + b%8) -- same XCD (speed only, never correctness).
struct Member {
  int m, grp, dir;
};
__device__ __forceinline__ Member decode() {
  const int bx = blockIdx.x;
  const int rest = bx >> 3;
  return Member{rest & 3, (rest >> 2) * 8 + (bx & 7), (int)blockIdx.y};
}

#ifdef IRC_COOP_STAMPS  // diagnostic build: per-step phase stamps of block 0 (member 0 of
// cluster 0, direction 0), wave 0 of the forward -- 0 step top, 1 MFMAs issued, 2 first
// barrier passed, 3 cell update + publish issued, 4 gather complete, 5 gathered h in LDS
// + saves / hout issued, 6 last barrier passed.  s_memtime (shader clock) and
// s_memrealtime (100 MHz); read by irc_coop_dbg_stamps (this build only).
__device__ uint64_t coop_stamps[64][7][2];
#define CSTAMP(s, i)                                                                       \
  do {                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && (s) < 64) {              \
      uint64_t c_, r_;                                                                     \
      asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"            \
                   : "=s"(c_), "=s"(r_)::"memory");                                        \
      *(volatile uint64_t*)&coop_stamps[(s)][(i)][0] = c_;                                 \
      *(volatile uint64_t*)&coop_stamps[(s)][(i)][1] = r_;                                 \
    }                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                     \
  } while (0)
#else
#define CSTAMP(s, i) \
  do {               \
  } while (0)
#endif

// ---------------------------------------------------------------- forward
// xp [B*L][ndir*4H] fp32 with per-unit interleaved gates (column 4u+g, plus
// b_ih + b_hh), wpk [ndir][P][NW][4][KKF][64][8] bf16 (forward fragments),
// hout [B*L][ndir*H] bf16; gsave/csave (may be null) in the member-fragment
// order read back by lstm_bwd_coop; xch [ndir][ngrp][2][BG][H] bf16 granules, tmo [1].
// The member's W slice lives in VGPRs (each wave's 4 gates x 8 k-steps of B fragments,
// 128 VGPRs), not in LDS: re-reading it from LDS every step (32 KB per wave, 128 KB
// per CU) set the step's MFMA phase (~1.9 us of a stamped 7.8 us step at 72 cycles
// per MFMA, profiles/r05_o_coop_stamps_bg32.txt).
__global__ __launch_bounds__(NTH, 1) void lstm_fwd_coop(
    const float* __restrict__ xp, const unsigned short* __restrict__ wpk,
    unsigned short* __restrict__ hout, float* __restrict__ gsave, float* __restrict__ csave,
    unsigned short* __restrict__ hprev, unsigned short* xch, unsigned* flags, unsigned* tmo, int B,
    int L, int ndir, int grp0, int ngrp_launch, int ngrp_total, unsigned spin_max, int sentinels,
    int wpub) {
  constexpr int RB = 2, BGT = BG;  // 16-row blocks per wave, sequences per cluster
  __shared__ __attribute__((aligned(16))) unsigned short hb[BGT][HP];
  __shared__ int abort_lds;
  const Member mb = decode();
  if (mb.grp >= ngrp_launch) return;  // the whole cluster is absent
  const int m = mb.m, dir = mb.dir, grp = grp0 + mb.grp;
  if (grp >= ngrp_total) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, q4 = lane >> 4;
  const int b0 = grp * BGT;
  const int64_t xld = (int64_t)ndir * 4 * H, hld = (int64_t)ndir * H;

  bf16x8 wr[4][KKF];  // this wave's W fragments: gate g, k-step kk
  {  // resident W slice + zero h_{-1}
    const u16x8* src = reinterpret_cast<const u16x8*>(wpk + (int64_t)(dir * P + m) * WSLICE);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int kk = 0; kk < KKF; ++kk)
        wr[g][kk] = *reinterpret_cast<const bf16x8*>(&src[((w * 4 + g) * KKF + kk) * 64 + lane]);
    for (int i = threadIdx.x; i < BGT * HP; i += NTH) (&hb[0][0])[i] = 0;
    if (threadIdx.x == 0) abort_lds = 0;
  }
  if (hprev) {  // h_{-1} = 0: the first step's row of hprev (own slice)
    const int t0 = dir == 0 ? 0 : L - 1;
    for (int p = threadIdx.x; p < BGT * UPW / 8; p += NTH) {
      const int row = p / (UPW / 8), col = m * UPW + (p % (UPW / 8)) * 8;
      if (b0 + row < B)
        *reinterpret_cast<u16x8*>(hprev + (((int64_t)dir * B + b0 + row) * L + t0) * H + col) =
            u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const int u = m * UPW + w * UPV + r16;  // this lane's hidden unit
  float c[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[rb][i] = 0.f;
  auto load_xp = [&](int t, f32x4 (&dst)[RB][4]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int b = b0 + rb * 16 + 4 * q4 + i;
        b = b < B ? b : B - 1;
        dst[rb][i] = *reinterpret_cast<const f32x4*>(xp + ((int64_t)b * L + t) * xld +
                                                     (int64_t)dir * 4 * H + 4 * u);
      }
  };
  f32x4 xr[RB][4];
  load_xp(dir == 0 ? 0 : L - 1, xr);
  // granules [2 parity][BGT][H/2]: {epoch, two bf16 of units 2c, 2c+1}
  unsigned long long* X =
      reinterpret_cast<unsigned long long*>(xch) + (int64_t)(dir * ngrp_total + grp) * 2 * BGT * (H / 2);
  (void)flags;
  __syncthreads();

  for (int s = 0; s < L; ++s) {
    CSTAMP(s, 0);
    const int t = dir == 0 ? s : L - 1 - s;
    f32x4 acc[RB][4];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[rb][g][i] = xr[rb][i][g];
    if (s + 1 < L) load_xp(dir == 0 ? t + 1 : t - 1, xr);
    if (s > 0) {
#pragma unroll
      for (int kk = 0; kk < KKF; ++kk) {
        bf16x8 a[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          a[rb] = *reinterpret_cast<const bf16x8*>(&hb[rb * 16 + r16][kk * 32 + 8 * q4]);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
            acc[rb][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], wr[g][kk], acc[rb][g], 0, 0, 0);
      }
    }
    CSTAMP(s, 1);
    __syncthreads();  // every read of h_{t-1} done
    CSTAMP(s, 2);
    f32x4 gv[RB][4], cv[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ig = sigm(acc[rb][0][i]);
        const float fg = sigm(acc[rb][1][i]);
        const float g2 = tanh_f(acc[rb][2][i]);
        const float og = sigm(acc[rb][3][i]);
        const float cn = fg * c[rb][i] + ig * g2;
        c[rb][i] = cn;
        hb[rb * 16 + 4 * q4 + i][u] = f32_to_bf16(og * tanh_f(cn));
        gv[rb][i] = f32x4{ig, fg, g2, og};
        cv[rb][i] = cn;
      }
    if (wpub) {
      // per-wave publish: this wave's 16 units x BGT rows go out as soon as the wave
      // has written them (LDS ops of one wave complete in order: no barrier), as RB
      // granule pairs per lane, and its hout / hprev rows as 16-byte stores per lane
      if (s + 1 < L) {
        unsigned long long* Xp = X + (s & 1) * BGT * (H / 2);
#pragma unroll
        for (int k = 0; k < RB; ++k) {
          const int idx = k * 64 + lane, pr = idx >> 2, pc = m * UPW + w * UPV + 4 * (idx & 3);
          const uint2 hv = *reinterpret_cast<const uint2*>(&hb[pr][pc]);
          st_sc1_pair(Xp + pr * (H / 2) + pc / 2, granule((unsigned)(s + 1), hv.x),
                      granule((unsigned)(s + 1), hv.y));
        }
      }
#pragma unroll
      for (int h2 = 0; h2 < RB / 2; ++h2) {
        const int row = 32 * h2 + (lane >> 1), col = m * UPW + w * UPV + 8 * (lane & 1);
        if (b0 + row < B) {
          const u16x8 hv = *reinterpret_cast<const u16x8*>(&hb[row][col]);
          *reinterpret_cast<u16x8*>(hout + ((int64_t)(b0 + row) * L + t) * hld + dir * H + col) = hv;
          const int tn = dir == 0 ? t + 1 : t - 1;
          if (hprev && tn >= 0 && tn < L)
            *reinterpret_cast<u16x8*>(hprev + (((int64_t)dir * B + b0 + row) * L + tn) * H + col) =
                hv;
        }
      }
    } else {
      __syncthreads();  // own slice of h_t complete in LDS
    }
    CSTAMP(s, 3);
    if (s + 1 < L) {
      // publish the own BGT x 64 slice as granules (2 per store) ...
      const unsigned ep = (unsigned)(s + 1);
      unsigned long long* Xp = X + (s & 1) * BGT * (H / 2);
#pragma unroll
      for (int k = 0; k < BGT * UPW / 4 / NTH; ++k) {
        if (wpub) break;
        const int p = k * NTH + threadIdx.x;
        const int row = p / (UPW / 4), c2 = m * (UPW / 2) + (p % (UPW / 4)) * 2;
        const uint2 hv = *reinterpret_cast<const uint2*>(&hb[row][2 * c2]);
        st_sc1_pair(Xp + row * (H / 2) + c2, granule(ep, hv.x), granule(ep, hv.y));
      }
      // ... and gather the other three
      if (sentinels) {  // sentinel: each producer's first granule (own slot: already ours)
        const unsigned long long* sent[P];
#pragma unroll
        for (int q = 0; q < P; ++q) sent[q] = Xp + q * (UPW / 2);
        poll_sentinels(sent, ep, tmo, &abort_lds, spin_max);
      }
      constexpr int NG = 3 * BGT * UPW / 2 / NTH;
      unsigned v[NG];
      auto addr = [&](int k) {
        const int idx = k * NTH + threadIdx.x;
        const int mm = (m + 1 + idx / (BGT * UPW / 2)) & 3, loc = idx % (BGT * UPW / 2);
        return Xp + (loc / (UPW / 2)) * (H / 2) + mm * (UPW / 2) + loc % (UPW / 2);
      };
      sweep<NG>(addr, ep, v, tmo, &abort_lds, spin_max);
      CSTAMP(s, 4);
#pragma unroll
      for (int k = 0; k < NG; ++k) {
        const int idx = k * NTH + threadIdx.x;
        const int mm = (m + 1 + idx / (BGT * UPW / 2)) & 3, loc = idx % (BGT * UPW / 2);
        *reinterpret_cast<unsigned*>(&hb[loc / (UPW / 2)][2 * (mm * (UPW / 2) + loc % (UPW / 2))]) =
            v[k];
      }
    }
    // saves + h_t rows (own slice) after the hand-off: they drain under the next MFMAs.
    if (gsave) {
      float* gs = gsave + ((int64_t)(dir * ngrp_total + grp) * L + t) * GSTEP;
      float* cs = csave + ((int64_t)(dir * ngrp_total + grp) * L + t) * CSTEP;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<f32x4*>(gs + ((((m * NW + w) * 2 + rb) * 4 + i) * 64 + lane) * 4) =
              gv[rb][i];
        *reinterpret_cast<f32x4*>(cs + (((m * NW + w) * 2 + rb) * 64 + lane) * 4) = cv[rb];
      }
    }
    for (int p = threadIdx.x; p < BGT * UPW / 8 && !wpub; p += NTH) {  // h_t -> hout (own slice)
      const int row = p / (UPW / 8), col = m * UPW + (p % (UPW / 8)) * 8;
      if (b0 + row < B) {
        const u16x8 hv = *reinterpret_cast<const u16x8*>(&hb[row][col]);
        *reinterpret_cast<u16x8*>(hout + ((int64_t)(b0 + row) * L + t) * hld + dir * H + col) = hv;
        // ... and into hprev at the next step's row (the dW_hh operand: no separate pass)
        const int tn = dir == 0 ? t + 1 : t - 1;
        if (hprev && tn >= 0 && tn < L)
          *reinterpret_cast<u16x8*>(hprev + (((int64_t)dir * B + b0 + row) * L + tn) * H + col) =
              hv;
      }
    }
    CSTAMP(s, 5);
    __syncthreads();  // h_t complete for the next step (and the abort word)
    CSTAMP(s, 6);
    if (abort_lds) return;
  }
}

// ---------------------------------------------------------------- backward
// dy [B*L][ndir*H] fp32; wtpk [ndir][P][NW][4 cb][KKB][64][8] bf16: member m's
// rows of W_hh (its 256 gate columns, k order g*64 + local unit) as B fragments
// for all 256 output units (wave w: units 64w + 16cb + lane&15); gsave/csave from
// lstm_fwd_coop; dg out [B*L][ndir*4H] bf16 (original gate order); xch fp32
// [ndir][ngrp][2][P][64 units/wave-block ... fragment order] partials, flags, tmo.
constexpr int KKB = 4 * UPW / 32;  // 8 k-steps over the member's 256 gate columns
constexpr int PART = BG * H;       // floats of one member's partial dh

__global__ __launch_bounds__(NTH, 1) void lstm_bwd_coop(
    const float* __restrict__ dy, const unsigned short* __restrict__ wtpk,
    const float* __restrict__ gsave, const float* __restrict__ csave,
    unsigned short* __restrict__ dg, float* xch, unsigned* flags, unsigned* tmo, int B, int L,
    int ndir, int grp0, int ngrp_launch, int ngrp_total, unsigned spin_max, int tagged) {
  __shared__ __attribute__((aligned(16))) unsigned short dgl[BG][HP];  // own dgates, k = g*64+lu
  __shared__ int abort_lds;
  const Member mb = decode();
  if (mb.grp >= ngrp_launch) return;
  const int m = mb.m, dir = mb.dir, grp = grp0 + mb.grp;
  if (grp >= ngrp_total) return;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, q4 = lane >> 4;
  const int b0 = grp * BG;
  const int64_t hld = (int64_t)ndir * H, gld = (int64_t)ndir * 4 * H;
  bf16x8 wr[4][KKB];  // this wave's W^T fragments (VGPRs, as the forward's): block cb, k-step kk
  {
    const u16x8* src = reinterpret_cast<const u16x8*>(wtpk + (int64_t)(dir * P + m) * WSLICE);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int kk = 0; kk < KKB; ++kk)
        wr[cb][kk] = *reinterpret_cast<const bf16x8*>(&src[((w * 4 + cb) * KKB + kk) * 64 + lane]);
    if (threadIdx.x == 0) abort_lds = 0;
  }
  // cell ownership as in the forward: lane -> unit u (own), rows rb*16 + 4*q4 + i
  const int lu = w * UPV + r16;  // local unit 0..63
  const int u = m * UPW + lu;
  float dc[2][4];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int i = 0; i < 4; ++i) dc[rb][i] = 0.f;
  // partials [2 parity][P member][block = (w*4 + cb)*2 + rb][64 lanes][4] fp32
  float* X = reinterpret_cast<float*>(xch) + (int64_t)(dir * ngrp_total + grp) * 2 * P * PART;
  auto store_dg = [&](int tt) {  // own dgates rows (LDS) -> dg at time tt
    for (int p = threadIdx.x; p < BG * 4 * UPW / 8; p += NTH) {
      const int row = p / (4 * UPW / 8), r = p % (4 * UPW / 8);
      const int g = r / (UPW / 8), c8 = (r % (UPW / 8)) * 8;
      if (b0 + row < B)
        *reinterpret_cast<u16x8*>(dg + ((int64_t)(b0 + row) * L + tt) * gld + dir * 4 * H +
                                  g * H + m * UPW + c8) =
            *reinterpret_cast<const u16x8*>(&dgl[row][g * UPW + c8]);
    }
  };
  unsigned* fl = flags + (dir * ngrp_total + grp) * NFLAG;
  __syncthreads();

  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? L - 1 - s : s;   // reverse of the forward order
    const int tp = dir == 0 ? t - 1 : t + 1;  // previous forward step
    const bool has_prev = tp >= 0 && tp < L;
    // this step's saved gates / c / c_prev / dy: issued now, consumed after the
    // MFMAs and the exchange (their latency hides behind both)
    f32x4 pgv[2][4], pcv[2], pcp[2];
    float pdy[2][4];
    {
      const float* gs = gsave + ((int64_t)(dir * ngrp_total + grp) * L + t) * GSTEP;
      const float* cs = csave + ((int64_t)(dir * ngrp_total + grp) * L + t) * CSTEP;
      const float* csp =
          has_prev ? csave + ((int64_t)(dir * ngrp_total + grp) * L + tp) * CSTEP : nullptr;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int64_t co = (((m * NW + w) * 2 + rb) * 64 + lane) * 4;
        pcv[rb] = *reinterpret_cast<const f32x4*>(cs + co);
        pcp[rb] = csp ? *reinterpret_cast<const f32x4*>(csp + co) : (f32x4)0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pgv[rb][i] = *reinterpret_cast<const f32x4*>(
              gs + ((((m * NW + w) * 2 + rb) * 4 + i) * 64 + lane) * 4);
          const int b = b0 + rb * 16 + 4 * q4 + i;
          pdy[rb][i] = b < B ? dy[((int64_t)b * L + t) * hld + dir * H + u] : 0.f;
        }
      }
    }
    // dh from dgates of the step after (K-split partial over own gate columns)
    f32x4 dh[2];  // own cells' summed recurrent gradient
    dh[0] = dh[1] = (f32x4)0.f;
    if (s > 0) {
      f32x4 acc[2][4];  // partial for units 64w + 16cb + r16
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = (f32x4)0.f;
#pragma unroll
      for (int kk = 0; kk < KKB; ++kk) {
        bf16x8 a[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          a[rb] = *reinterpret_cast<const bf16x8*>(&dgl[rb * 16 + r16][kk * 32 + 8 * q4]);
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], wr[cb][kk], acc[rb][cb], 0, 0, 0);
      }
      const unsigned ep = (unsigned)s;
      if (tagged == 1) {
        // R2 (the data is the flag): each partial float travels as a granule
        // {value, epoch}, two per 16-byte write-through store; block (wave w = unit
        // block 64w = destination member w, cb, rb), lane, 4 rows -> 4 granules
        unsigned long long* G = reinterpret_cast<unsigned long long*>(xch) +
                                (int64_t)(dir * ngrp_total + grp) * 2 * P * PART;
        unsigned long long* Gs = G + (int64_t)(s & 1) * P * PART;
        unsigned long long* Gp = Gs + (int64_t)m * PART;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            unsigned long long* q = Gp + ((((w * 4 + cb) * 2 + rb) * 64 + lane) * 4);
            st_sc1_pair(q, granule(ep, __float_as_uint(acc[rb][cb][0])),
                        granule(ep, __float_as_uint(acc[rb][cb][1])));
            st_sc1_pair(q + 2, granule(ep, __float_as_uint(acc[rb][cb][2])),
                        granule(ep, __float_as_uint(acc[rb][cb][3])));
          }
        // own units (block m, cb = w) from every member; sweep until every tag is ep
        u32x4 v[P][2][2];
        for (unsigned spins = 0;;) {
#pragma unroll
          for (int mm = 0; mm < P; ++mm)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                v[mm][rb][j] =
                    ld_sc1_x4(Gs + (int64_t)mm * PART + ((((m * 4 + w) * 2 + rb) * 64 + lane) * 4) + 2 * j);
          asm volatile("s_waitcnt vmcnt(0)"
                       : "+v"(v[0][0][0]), "+v"(v[0][0][1]), "+v"(v[0][1][0]), "+v"(v[0][1][1]),
                         "+v"(v[1][0][0]), "+v"(v[1][0][1]), "+v"(v[1][1][0]), "+v"(v[1][1][1]),
                         "+v"(v[2][0][0]), "+v"(v[2][0][1]), "+v"(v[2][1][0]), "+v"(v[2][1][1]),
                         "+v"(v[3][0][0]), "+v"(v[3][0][1]), "+v"(v[3][1][0]), "+v"(v[3][1][1])
                       :
                       : "memory");
          bool ok = true;
#pragma unroll
          for (int mm = 0; mm < P; ++mm)
#pragma unroll
            for (int rb = 0; rb < 2; ++rb)
#pragma unroll
              for (int j = 0; j < 2; ++j) ok &= v[mm][rb][j][1] == ep && v[mm][rb][j][3] == ep;
          if (__all(ok) && spin_max) break;
          if (++spins > spin_max) {
            if (lane == 0) {
              __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              abort_lds = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        // sum in member order 0..3, as the flag form does
#pragma unroll
        for (int mm = 0; mm < P; ++mm)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int i = 0; i < 4; ++i) dh[rb][i] += __uint_as_float(v[mm][rb][i >> 1][(i & 1) * 2]);
      } else {
      // publish the partial (R1): block (wave w = unit block 64w, cb, rb), each
      // lane's 4 rows as one 16-byte write-through store
      float* Xs = X + (int64_t)(s & 1) * P * PART;
      float* Xp = Xs + (int64_t)m * PART;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          st_sc1_x4(Xp + ((((w * 4 + cb) * 2 + rb) * 64 + lane) * 4),
                    __builtin_bit_cast(u32x4, acc[rb][cb]));
      if (tagged == 2) {
        // per-wave flags: wave w's partial is member w's alone, so each wave drains its
        // own stores and raises its own flag, and reader wave w of member m waits only
        // for wave m of every member -- no workgroup barrier on either side
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store((gu32*)(fl + m * NW + w), ep, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        for (unsigned spins = 0;;) {
          bool ok = true;
          if (lane < P)
            ok = __hip_atomic_load((gu32*)(fl + lane * NW + m), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) >= ep;
          if (__all(ok) && spin_max) break;
          if (++spins > spin_max) {
            if (lane == 0) {
              __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              abort_lds = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
        publish_flag(fl + m * NW, ep);
        poll_flags(fl, ep, tmo, &abort_lds, spin_max);
        if (abort_lds) return;
      }
      // own units live in every member's block m, cb = w: sum in member order
      u32x4 v[P][2];
#pragma unroll
      for (int mm = 0; mm < P; ++mm)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
          v[mm][rb] = ld_sc1_x4(Xs + (int64_t)mm * PART + ((((m * 4 + w) * 2 + rb) * 64 + lane) * 4));
      asm volatile("s_waitcnt vmcnt(0)"
                   : "+v"(v[0][0]), "+v"(v[0][1]), "+v"(v[1][0]), "+v"(v[1][1]), "+v"(v[2][0]),
                     "+v"(v[2][1]), "+v"(v[3][0]), "+v"(v[3][1])
                   :
                   : "memory");
#pragma unroll
      for (int mm = 0; mm < P; ++mm)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int i = 0; i < 4; ++i) dh[rb][i] += __uint_as_float(v[mm][rb][i]);
      }
    }
    __syncthreads();  // all reads of dgl (MFMA) done before it is overwritten
    if (abort_lds) return;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const f32x4 cv = pcv[rb], cp = pcp[rb];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = rb * 16 + 4 * q4 + i;
        const float ig = pgv[rb][i][0], fg = pgv[rb][i][1], gg = pgv[rb][i][2], og = pgv[rb][i][3];
        const float dht = pdy[rb][i] + dh[rb][i];
        const float tc = tanh_f(cv[i]);
        const float dct = dht * og * (1.f - tc * tc) + dc[rb][i];
        dc[rb][i] = dct * fg;
        dgl[row][0 * UPW + lu] = f32_to_bf16(dct * gg * ig * (1.f - ig));
        dgl[row][1 * UPW + lu] = f32_to_bf16(dct * cp[i] * fg * (1.f - fg));
        dgl[row][2 * UPW + lu] = f32_to_bf16(dct * ig * (1.f - gg * gg));
        dgl[row][3 * UPW + lu] = f32_to_bf16(dht * tc * og * (1.f - og));
      }
    }
    __syncthreads();  // own dgates complete: next step's A operand, and the dg rows
    store_dg(t);
  }
}

// W_hh [ndir][4H][H] fp32 -> the resident slices of both recurrences (bf16).
//  fwd: [dir][m][w][g][kk][lane][8] = W[g*H + 64m + 16w + (lane&15)][kk*32 + 8(lane>>4) + j]
//  bwd: [dir][m][w][cb][kk][lane][8] = W[g*H + 64m + lu][64w + 16cb + (lane&15)] with
//       k = kk*32 + 8(lane>>4) + j = g*64 + lu  (the member's gate columns)
__global__ void pack_coop_kernel(const float* __restrict__ whh, unsigned short* __restrict__ wf,
                                 unsigned short* __restrict__ wb, int ndir) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)P * WSLICE;  // = 4H*H
  if (e >= per * ndir) return;
  const int dir = (int)(e / per);
  int64_t r = e % per;
  const int j = (int)(r & 7), lane = (int)((r >> 3) & 63);
  const int kk = (int)((r >> 9) % KKF);
  const int x = (int)((r >> 9) / KKF);  // ((m*NW + w)*4 + g|cb)
  const int gc = x & 3, w = (x >> 2) % NW, m = (x >> 2) / NW;
  const float* W = whh + dir * per;
  {
    const int u = m * UPW + w * UPV + (lane & 15);
    const int k = kk * 32 + 8 * (lane >> 4) + j;
    wf[e] = f32_to_bf16(W[(int64_t)(gc * H + u) * H + k]);
  }
  {
    const int n = w * 64 + gc * 16 + (lane & 15);       // output unit
    const int k = kk * 32 + 8 * (lane >> 4) + j;        // member-local gate column
    const int g = k / UPW, lu = k % UPW;
    wb[e] = f32_to_bf16(W[(int64_t)(g * H + m * UPW + lu) * H + n]);
  }
}

// After a launch whose clusters timed out (tmo != 0), the output is overwritten
// with bf16 NaN on the device, so a timeout can never pass for a result: the
// NaN reaches the embeddings / gradients and the loss, whoever the caller is.
// Every block reads the one word and leaves at once in the normal case.
__global__ void poison_on_timeout_kernel(const unsigned* __restrict__ tmo,
                                         unsigned short* __restrict__ out, int64_t n,
                                         unsigned short* __restrict__ out2, int64_t n2) {
  if (__hip_atomic_load((const gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = 0x7FC0;  // bf16 quiet NaN
  if (out2)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
         i += (int64_t)gridDim.x * blockDim.x)
      out2[i] = 0x7FC0;
}

// Sticky fault word: *fault |= timeout word (device side, no host sync).
__global__ void fault_or_kernel(const unsigned* __restrict__ tmo, unsigned* fault) {
  const unsigned t = __hip_atomic_load((const gu32*)tmo, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  if (t) atomicOr(fault, t);
}

}  // namespace lstmc
}  // namespace irc

using namespace irc;

extern "C" int irc_lstm_coop_supported(int64_t H) { return H == lstmc::H; }

extern "C" int64_t irc_lstm_coop_sizes(int64_t B, int64_t L, int64_t H, int64_t ndir, int which) {
  // 0: gates floats, 1: c floats, 2: fwd exchange bytes, 3: bwd exchange bytes, 4: flag bytes
  const int64_t ngrp = (B + lstmc::BG - 1) / lstmc::BG;
  switch (which) {
    case 0: return ndir * ngrp * L * lstmc::GSTEP;
    case 1: return ndir * ngrp * L * lstmc::CSTEP;
    case 2: return ndir * ngrp * 2 * lstmc::BG * (H / 2) * 8;   // granules
    case 3: return ndir * ngrp * 2 * lstmc::P * lstmc::PART * 8;  // fp32 partials as granules
    case 4: return ((ndir * ngrp * lstmc::NFLAG + 1) * 4 + 15) / 16 * 16;
  }
  return -1;
}

extern "C" int irc_lstm_coop_pack(const float* whh, int64_t H, int64_t ndir, void* wf, void* wb,
                                  irc_stream_t stream) {
  IRC_REQUIRE(H == lstmc::H, "lstm_coop_pack: H=%lld", (long long)H);
  const int64_t n = ndir * 4 * H * H;
  hipLaunchKernelGGL(lstmc::pack_coop_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), whh, (unsigned short*)wf, (unsigned short*)wb, (int)ndir);
  return check_launch("lstm_coop_pack");
}

// Spin bound of the cross-CU hand-off (IRC_LSTM_COOP_SPIN_MAX overrides; a
// debug knob: 0 makes the first cross-CU wait of every workgroup time out, ready
// or not, which the fault-path tests use).  ~1.6e9 cycles by default -- a true deadlock only.
static unsigned coop_spin_max() {
  const char* e = getenv("IRC_LSTM_COOP_SPIN_MAX");
  return e ? (unsigned)strtoul(e, nullptr, 10) : lstmc::SPIN_MAX;
}

// Clusters per launch such that every workgroup of the q- and k-encoder launches
// (which may run concurrently on two streams) is co-resident: one workgroup per
// CU (by VGPRs), so 2 * groups * P * ndir <= CUs.  The CU count comes
// from the device, not a constant; on MI355X (256 CUs, ndir 2) this is 16.
static int coop_groups_per_launch(int64_t ndir) {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  int g = cus / (2 * lstmc::P * (int)ndir);
  g = g < lstmc::MAX_GROUPS ? g : lstmc::MAX_GROUPS;
  return g < 1 ? 1 : g;
}

static void coop_poison(const unsigned* tmo, void* out, int64_t n, hipStream_t st,
                        void* out2 = nullptr, int64_t n2 = 0) {
  hipLaunchKernelGGL(lstmc::poison_on_timeout_kernel, dim3(256), dim3(256), 0, st, tmo,
                     (unsigned short*)out, n, (unsigned short*)out2, n2);
}

// sync: flags (ndir*ngrp*P words) followed by the timeout word; zeroed here.
extern "C" int irc_lstm_fwd_coop(const float* xp_packed, const void* wf, void* hout, float* gsave,
                                 float* csave, void* hprev, void* xch, void* sync, int64_t B,
                                 int64_t L, int64_t H, int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(H == lstmc::H, "lstm_fwd_coop: H=%lld", (long long)H);
  IRC_REQUIRE((gsave == nullptr) == (csave == nullptr), "lstm_fwd_coop: gsave/csave together");
  if (B == 0 || L == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const int ngrp = (int)((B + lstmc::BG - 1) / lstmc::BG);
  const int gpl = coop_groups_per_launch(ndir);
  const unsigned spin_max = coop_spin_max();
  // The granule sweep polls by itself: 287 vs 316 us per layer at C2 with the wave-0
  // sentinel pass + barrier in front of it (IRC_LSTM_COOP_SENTINELS=1 restores that)
  const char* se = getenv("IRC_LSTM_COOP_SENTINELS");
  const int sentinels = se ? atoi(se) : 0;
  // Each wave publishes its own units right after its cell update (no workgroup barrier
  // between the cell update and the hand-off): 287 vs 297 us per layer at C2,
  // bit-identical; IRC_LSTM_COOP_WAVE_PUBLISH=0 restores the workgroup publish
  const char* we = getenv("IRC_LSTM_COOP_WAVE_PUBLISH");
  const int wpub = we ? atoi(we) : 1;
  unsigned* flags = static_cast<unsigned*>(sync);
  unsigned* tmo = flags + ndir * ngrp * lstmc::NFLAG;
  hipMemsetAsync(sync, 0, irc_lstm_coop_sizes(B, L, H, ndir, 4), st);
  hipMemsetAsync(xch, 0, irc_lstm_coop_sizes(B, L, H, ndir, 2), st);
  prof_begin(st);
  for (int g0 = 0; g0 < ngrp; g0 += gpl) {
    const int n = ngrp - g0 < gpl ? ngrp - g0 : gpl;
    const dim3 grid((unsigned)((n + 7) / 8 * 32), (unsigned)ndir);
    hipLaunchKernelGGL(lstmc::lstm_fwd_coop, grid, dim3(lstmc::NTH), 0, st, xp_packed,
                       (const unsigned short*)wf, (unsigned short*)hout, gsave, csave,
                       (unsigned short*)hprev, (unsigned short*)xch, flags, tmo, (int)B, (int)L,
                       (int)ndir, g0, n, ngrp, spin_max, sentinels, wpub);
  }
  prof_end("lstm_fwd", st, 2.0 * B * L * ndir * 4.0 * H * H);
  coop_poison(tmo, hout, B * L * ndir * H, st, hprev, hprev ? B * L * ndir * H : 0);
  return check_launch("lstm_fwd_coop");
}

extern "C" int irc_lstm_bwd_coop(const float* dy, const void* wb, const float* gsave,
                                 const float* csave, void* dg, void* xch, void* sync, int64_t B,
                                 int64_t L, int64_t H, int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(H == lstmc::H, "lstm_bwd_coop: H=%lld", (long long)H);
  if (B == 0 || L == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  const int ngrp = (int)((B + lstmc::BG - 1) / lstmc::BG);
  const int gpl = coop_groups_per_launch(ndir);
  const unsigned spin_max = coop_spin_max();
  unsigned* flags = static_cast<unsigned*>(sync);
  unsigned* tmo = flags + ndir * ngrp * lstmc::NFLAG;
  // IRC_LSTM_COOP_BWD_TAGGED=2: per-wave flags (no workgroup barrier in the hand-off);
  // IRC_LSTM_COOP_BWD_TAGGED=1: tagged granules (R2) instead of the flag hand-off (R1);
  // bit-identical, but 505 vs 350 us per layer at C2 (16 granule loads per lane per
  // sweep pass against 8 plain loads after one flag poll)
  const char* te = getenv("IRC_LSTM_COOP_BWD_TAGGED");
  const int tagged = te ? atoi(te) : 0;
  hipMemsetAsync(sync, 0, irc_lstm_coop_sizes(B, L, H, ndir, 4), st);
  if (tagged == 1) hipMemsetAsync(xch, 0, irc_lstm_coop_sizes(B, L, H, ndir, 3), st);
  prof_begin(st);
  for (int g0 = 0; g0 < ngrp; g0 += gpl) {
    const int n = ngrp - g0 < gpl ? ngrp - g0 : gpl;
    const dim3 grid((unsigned)((n + 7) / 8 * 32), (unsigned)ndir);
    hipLaunchKernelGGL(lstmc::lstm_bwd_coop, grid, dim3(lstmc::NTH), 0, st, dy,
                       (const unsigned short*)wb, gsave, csave, (unsigned short*)dg, (float*)xch,
                       flags, tmo, (int)B, (int)L, (int)ndir, g0, n, ngrp, spin_max, tagged);
  }
  prof_end("lstm_bwd", st, 2.0 * B * L * ndir * 4.0 * H * H);
  coop_poison(tmo, dg, B * L * ndir * 4 * H, st);
  return check_launch("lstm_bwd_coop");
}

extern "C" int irc_lstm_coop_fault(const void* sync, int64_t B, int64_t ndir, void* fault,
                                   irc_stream_t stream) {
  IRC_REQUIRE(sync != nullptr && fault != nullptr, "lstm_coop_fault: null pointer");
  const int64_t ngrp = (B + lstmc::BG - 1) / lstmc::BG;
  const unsigned* tmo = static_cast<const unsigned*>(sync) + ndir * ngrp * lstmc::NFLAG;
  hipLaunchKernelGGL(lstmc::fault_or_kernel, dim3(1), dim3(64), 0, as_stream(stream), tmo,
                     static_cast<unsigned*>(fault));
  return check_launch("lstm_coop_fault");
}

#ifdef IRC_COOP_STAMPS
extern "C" int irc_coop_dbg_stamps(uint64_t* out /* [64][7][2] */) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(irc::lstmc::coop_stamps),
                             sizeof(irc::lstmc::coop_stamps)) == hipSuccess ? 0 : -1;
}
#endif
