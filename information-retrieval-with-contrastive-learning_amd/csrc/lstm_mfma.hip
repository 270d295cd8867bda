// MFMA BiLSTM recurrences for the production head shape (H = 256, bf16 operands,
// fp32 state).  Reference: nn.LSTM in src/model.py:16-22, 39 (gate order i, f, g,
// o; zero initial state; the padded sequence is processed as is).
//
// Forward, per (batch group of 32 sequences, direction) workgroup of 4 waves:
//   gates[32 x 4H] = xp_t + h_{t-1}[32 x H] . W_hh^T   (v_mfma_f32_32x32x16_bf16)
// * h_{t-1} lives in LDS (bf16, padded rows) and is the A operand;
// * W_hh (bf16, 512 KB per direction, shared by every group) streams from L2
//   each step, pre-packed fragment-native so every wave load is 1 KB contiguous
//   (no partial-line over-fetch);
// * wave w (of 8, two per SIMD) owns hidden units [w*H/8, (w+1)*H/8) and ALL FOUR
//   gates of them (4 accumulator blocks of 32 columns at H = 256), so the cell
//   update is lane-local and c stays in registers for the whole sequence;
// * xp arrives with its gate columns interleaved per unit (4u + g, lstm_pack_wih)
//   so each lane reads the 4 gate pre-activations of one (row, unit) as one
//   float4, prefetched one step ahead in registers;
// * the activated gates and c are saved in a fragment-native layout (16-byte
//   coalesced stores, read back the same way by the backward kernel); h_t is
//   copied LDS -> hout in whole 16-byte rows.
// Backward: the mirror image -- dh_{t+1} = dgates . W_hh with W_hh^T streamed as
// B fragments, dgates (bf16) in LDS as the A operand and written out in rows for
// the weight-gradient GEMMs, dc in registers.
#include "irc_common.h"

namespace irc {
namespace lstmm {

constexpr int BG = 32;   // sequences per workgroup (M of the MFMA)
constexpr int NW = 8;    // waves per workgroup (2 per SIMD)
constexpr int NTH = NW * 64;

// v_rcp_f32 (1 ulp) instead of the correctly rounded division (~12 instructions with its
// scale / fixup and denormal-mode switches): 40 of them per lane per step were most of
// the recurrence's cell update (profiles/r05_p_coop_stamps.txt)
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f;
}

template <int H>
struct Geo {
  static constexpr int NU = H / NW;      // units per wave
  static constexpr int NH = NU / 32;     // 32-unit halves per wave
  static constexpr int NB = 4 * NH;      // accumulator blocks per wave (forward)
  static constexpr int HP = H + 8;       // padded LDS row (bf16 elems)
  static constexpr int GP = 4 * H + 8;   // padded dgates row (bf16 elems)
  static constexpr int KKF = H / 16;     // forward k-steps
  static constexpr int KKB = 4 * H / 16; // backward k-steps
  // fragment-native save strides (floats) per (dir, group, t)
  static constexpr int GSTEP = NTH * NB * 16;
  static constexpr int CSTEP = NTH * NH * 16;
};

// row (within the group) of accumulator register e for lane half h
__device__ __forceinline__ int rowb(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

template <int H>
__global__ __launch_bounds__(NTH, 1) void lstm_fwd_mfma(
    const float* __restrict__ xp, const unsigned short* __restrict__ whh,
    unsigned short* __restrict__ hout, float* __restrict__ gsave, float* __restrict__ csave,
    int B, int L, int ndir) {
  using G = Geo<H>;
  __shared__ __attribute__((aligned(16))) unsigned short hb[2][BG][G::HP];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, r32 = lane & 31;
  const int grp = blockIdx.x, dir = blockIdx.y;
  const int ngrp = gridDim.x;
  const int b0 = grp * BG;
  const int64_t xld = (int64_t)ndir * 4 * H;
  const int64_t hld = (int64_t)ndir * H;
  const unsigned short* W = whh + (int64_t)dir * 4 * H * H;

  for (int i = threadIdx.x; i < 2 * BG * G::HP; i += NTH) (&hb[0][0][0])[i] = 0;

  float c[G::NH][16];
#pragma unroll
  for (int hf = 0; hf < G::NH; ++hf)
#pragma unroll
    for (int e = 0; e < 16; ++e) c[hf][e] = 0.f;

  // xp of (row b, permuted unit column) -> float4 of the 4 gates
  auto load_xp = [&](int t, f32x4 (&dst)[G::NH][16]) {
#pragma unroll
    for (int hf = 0; hf < G::NH; ++hf)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        int b = b0 + rowb(e, h);
        if (b >= B) b = B - 1;
        const int pc = (w * G::NU + hf * 32 + r32) * 4;  // interleaved gates of unit u
        dst[hf][e] = *reinterpret_cast<const f32x4*>(xp + ((int64_t)b * L + t) * xld +
                                                     (int64_t)dir * 4 * H + pc);
      }
  };
  f32x4 xr[G::NH][16];
  load_xp(dir == 0 ? 0 : L - 1, xr);
  __syncthreads();

  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? s : L - 1 - s;
    const int cur = s & 1, nxt = cur ^ 1;
    f32x16 acc[G::NB];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int hf = 0; hf < G::NH; ++hf)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g * G::NH + hf][e] = xr[hf][e][g];
    if (s + 1 < L) load_xp(dir == 0 ? t + 1 : t - 1, xr);  // prefetch next step
    if (s > 0) {
      const unsigned short* arow = &hb[cur][r32][0];
#pragma unroll 4
      for (int kk = 0; kk < G::KKF; ++kk) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(arow + kk * 16 + 8 * h);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int hf = 0; hf < G::NH; ++hf) {
            // fragment-native: one contiguous 1 KB per wave per (block, kk)
            const bf16x8 bw = *reinterpret_cast<const bf16x8*>(
                W + ((int64_t)((w * G::NB + g * G::NH + hf) * G::KKF + kk) * 64 + lane) * 8);
            acc[g * G::NH + hf] =
                __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bw, acc[g * G::NH + hf], 0, 0, 0);
          }
      }
    }
    // cell update: lane owns units u = w*NU + hf*32 + r32 for rows rowb(e, h)
    float* gs = gsave ? gsave + ((int64_t)(dir * ngrp + grp) * L + t) * G::GSTEP : nullptr;
    float* cs = csave ? csave + ((int64_t)(dir * ngrp + grp) * L + t) * G::CSTEP : nullptr;
#pragma unroll
    for (int hf = 0; hf < G::NH; ++hf) {
      const int u = w * G::NU + hf * 32 + r32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f32x4 gi, gf, gg, go, cv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 4 * q + r;
          const float ig = sigm(acc[0 * G::NH + hf][e]);
          const float fg = sigm(acc[1 * G::NH + hf][e]);
          const float g2 = tanh_f(acc[2 * G::NH + hf][e]);
          const float og = sigm(acc[3 * G::NH + hf][e]);
          const float cn = fg * c[hf][e] + ig * g2;
          c[hf][e] = cn;
          const float hv = og * tanh_f(cn);
          hb[nxt][rowb(e, h)][u] = f32_to_bf16(hv);
          gi[r] = ig;
          gf[r] = fg;
          gg[r] = g2;
          go[r] = og;
          cv[r] = cn;
        }
        if (gs) {
          // fragment-native: [wave][block j][q][lane][4]
          float* base = gs + (int64_t)w * (G::NB * 16 * 64) + q * 256 + lane * 4;
          *reinterpret_cast<f32x4*>(base + (0 * G::NH + hf) * 1024) = gi;
          *reinterpret_cast<f32x4*>(base + (1 * G::NH + hf) * 1024) = gf;
          *reinterpret_cast<f32x4*>(base + (2 * G::NH + hf) * 1024) = gg;
          *reinterpret_cast<f32x4*>(base + (3 * G::NH + hf) * 1024) = go;
        }
        if (cs)
          *reinterpret_cast<f32x4*>(cs + (int64_t)w * (G::NH * 1024) + hf * 1024 + q * 256 +
                                    lane * 4) = cv;
      }
    }
    __syncthreads();
    // h_t rows -> hout[(b0+b)*L + t][dir*H ...] in 16-byte pieces
    constexpr int PIECES = BG * H / 8;
    for (int p = threadIdx.x; p < PIECES; p += NTH) {
      const int b = p / (H / 8), c8 = (p % (H / 8)) * 8;
      if (b0 + b < B)
        *reinterpret_cast<u16x8*>(hout + ((int64_t)(b0 + b) * L + t) * hld + dir * H + c8) =
            *reinterpret_cast<const u16x8*>(&hb[nxt][b][c8]);
    }
  }
}

// Backward.  dy [B*L][ndir*H] fp32 (dL/dh_t from above), whhT [ndir][H][4H] bf16,
// gsave/csave from lstm_fwd_mfma; dg out [B*L][ndir*4H] bf16 (original gate order per
// direction), so the layer's dx is ONE GEMM with K = ndir*4H.
template <int H>
__global__ __launch_bounds__(NTH, 1) void lstm_bwd_mfma(
    const float* __restrict__ dy, const unsigned short* __restrict__ whhT,
    const float* __restrict__ gsave, const float* __restrict__ csave,
    unsigned short* __restrict__ dg, int B, int L, int ndir) {
  using G = Geo<H>;
  __shared__ __attribute__((aligned(16))) unsigned short dgl[BG][G::GP];
  __shared__ __attribute__((aligned(16))) float dyl[BG][H];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, r32 = lane & 31;
  const int grp = blockIdx.x, dir = blockIdx.y;
  const int ngrp = gridDim.x;
  const int b0 = grp * BG;
  const int64_t hld = (int64_t)ndir * H;
  const unsigned short* WT = whhT + (int64_t)dir * H * 4 * H;

  float dc[G::NH][16];
#pragma unroll
  for (int hf = 0; hf < G::NH; ++hf)
#pragma unroll
    for (int e = 0; e < 16; ++e) dc[hf][e] = 0.f;

  for (int s = 0; s < L; ++s) {
    const int t = dir == 0 ? L - 1 - s : s;       // reverse of the forward order
    const int tp = dir == 0 ? t - 1 : t + 1;      // previous forward step
    const bool has_prev = tp >= 0 && tp < L;
    // stage dy_t [BG][H] (fp32) into LDS with 16-byte loads
    constexpr int DP = BG * H / 4;
    for (int p = threadIdx.x; p < DP; p += NTH) {
      const int b = p / (H / 4), c4 = (p % (H / 4)) * 4;
      f32x4 v = (f32x4)0.f;
      if (b0 + b < B)
        v = *reinterpret_cast<const f32x4*>(dy + ((int64_t)(b0 + b) * L + t) * hld + dir * H + c4);
      *reinterpret_cast<f32x4*>(&dyl[b][c4]) = v;
    }
    // dh_next = dgates_{prev step} . W_hh  (K = 4H), lane units u = w*NU + hf*32 + r32
    f32x16 acc[G::NH];
#pragma unroll
    for (int hf = 0; hf < G::NH; ++hf) acc[hf] = (f32x16)0.f;
    if (s > 0) {
      const unsigned short* arow = &dgl[r32][0];
#pragma unroll 4
      for (int kk = 0; kk < G::KKB; ++kk) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(arow + kk * 16 + 8 * h);
#pragma unroll
        for (int hf = 0; hf < G::NH; ++hf) {
          const bf16x8 bw = *reinterpret_cast<const bf16x8*>(
              WT + ((int64_t)((w * G::NH + hf) * G::KKB + kk) * 64 + lane) * 8);
          acc[hf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bw, acc[hf], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // dgl reads done; dyl visible
    const float* gs = gsave + ((int64_t)(dir * ngrp + grp) * L + t) * G::GSTEP;
    const float* cs = csave + ((int64_t)(dir * ngrp + grp) * L + t) * G::CSTEP;
    const float* csp = has_prev ? csave + ((int64_t)(dir * ngrp + grp) * L + tp) * G::CSTEP
                                : nullptr;
#pragma unroll
    for (int hf = 0; hf < G::NH; ++hf) {
      const int u = w * G::NU + hf * 32 + r32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float* base = gs + (int64_t)w * (G::NB * 16 * 64) + q * 256 + lane * 4;
        const f32x4 gi = *reinterpret_cast<const f32x4*>(base + (0 * G::NH + hf) * 1024);
        const f32x4 gf = *reinterpret_cast<const f32x4*>(base + (1 * G::NH + hf) * 1024);
        const f32x4 gg = *reinterpret_cast<const f32x4*>(base + (2 * G::NH + hf) * 1024);
        const f32x4 go = *reinterpret_cast<const f32x4*>(base + (3 * G::NH + hf) * 1024);
        const int64_t co = (int64_t)w * (G::NH * 1024) + hf * 1024 + q * 256 + lane * 4;
        const f32x4 cv = *reinterpret_cast<const f32x4*>(cs + co);
        const f32x4 cp = csp ? *reinterpret_cast<const f32x4*>(csp + co) : (f32x4)0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = 4 * q + r;
          const int b = rowb(e, h);
          const float dht = dyl[b][u] + acc[hf][e];
          const float tc = tanh_f(cv[r]);
          const float dot = dht * tc;
          const float dct = dht * go[r] * (1.f - tc * tc) + dc[hf][e];
          dc[hf][e] = dct * gf[r];
          const float di = dct * gg[r] * gi[r] * (1.f - gi[r]);
          const float df = dct * cp[r] * gf[r] * (1.f - gf[r]);
          const float dgg = dct * gi[r] * (1.f - gg[r] * gg[r]);
          const float dox = dot * go[r] * (1.f - go[r]);
          dgl[b][u] = f32_to_bf16(di);
          dgl[b][H + u] = f32_to_bf16(df);
          dgl[b][2 * H + u] = f32_to_bf16(dgg);
          dgl[b][3 * H + u] = f32_to_bf16(dox);
        }
      }
    }
    __syncthreads();  // dgl complete (next step's A operand)
    constexpr int PIECES = BG * 4 * H / 8;
    const int64_t gld = (int64_t)ndir * 4 * H;
    unsigned short* dgd = dg + (int64_t)dir * 4 * H;
    for (int p = threadIdx.x; p < PIECES; p += NTH) {
      const int b = p / (4 * H / 8), c8 = (p % (4 * H / 8)) * 8;
      if (b0 + b < B)
        *reinterpret_cast<u16x8*>(dgd + ((int64_t)(b0 + b) * L + t) * gld + c8) =
            *reinterpret_cast<const u16x8*>(&dgl[b][c8]);
    }
  }
}

// W_ih rows + bias permuted into the (wave, half, lane, gate) column order the
// forward kernel reads as float4, cast to bf16.  src [ndir*4H][In] fp32.
template <int H>
__global__ void pack_wih_kernel(const float* __restrict__ wih, const float* __restrict__ bih,
                                const float* __restrict__ bhh, unsigned short* __restrict__ dst,
                                float* __restrict__ bias_dst, int In, int ndir) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rows = (int64_t)ndir * 4 * H;
  if (e >= rows * In) return;
  const int r = (int)(e / In), k = (int)(e % In);
  const int dir = r / (4 * H), pc = r % (4 * H);
  const int g = pc & 3, u = pc >> 2;  // packed column 4u + g  <-  original g*H + u
  const int orig = dir * 4 * H + g * H + u;
  dst[e] = f32_to_bf16(wih[(int64_t)orig * In + k]);
  if (k == 0) bias_dst[r] = bih[orig] + bhh[orig];
}

// W_hh [ndir][4H][H] fp32 -> bf16 B fragments in the order the recurrences read
// them (each wave's 64 x 16-byte fragment of one (block, kk) is 1 KB contiguous):
//   w  [dir][wave][block g*NH+hf][kk < H/16][lane][8]:  W[g*H + u][kk*16 + 8h + j]
//   wT [dir][wave][hf][kk < 4H/16][lane][8]:            W[kk*16 + 8h + j][u]
// with u = wave*NU + hf*32 + (lane & 31), h = lane >> 5.
template <int H>
__global__ void pack_whh_kernel(const float* __restrict__ whh, unsigned short* __restrict__ w,
                                unsigned short* __restrict__ wT, int ndir) {
  using G = Geo<H>;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)4 * H * H;
  if (e >= per * ndir) return;
  const int dir = (int)(e / per);
  const int64_t r = e % per;
  const int j = (int)(r & 7), lane = (int)((r >> 3) & 63);
  const int h = lane >> 5, r32 = lane & 31;
  const float* W = whh + dir * per;
  {  // forward fragments: r = ((wv*NB + blk)*KKF + kk)*512 + lane*8 + j
    const int kk = (int)((r >> 9) % G::KKF);
    const int blk = (int)((r >> 9) / G::KKF % G::NB), wv = (int)((r >> 9) / G::KKF / G::NB);
    const int g = blk / G::NH, hf = blk % G::NH;
    const int u = wv * G::NU + hf * 32 + r32;
    w[e] = f32_to_bf16(W[(int64_t)(g * H + u) * H + kk * 16 + 8 * h + j]);
  }
  {  // backward fragments: r = ((wv*NH + hf)*KKB + kk)*512 + lane*8 + j
    const int kk = (int)((r >> 9) % G::KKB);
    const int hf = (int)((r >> 9) / G::KKB % G::NH), wv = (int)((r >> 9) / G::KKB / G::NH);
    const int u = wv * G::NU + hf * 32 + r32;
    wT[e] = f32_to_bf16(W[(int64_t)(kk * 16 + 8 * h + j) * H + u]);
  }
}

// hprev[dir][b*L + t] = h_{t-1} (forward order) of direction dir, 0 at the start.
__global__ void hprev_kernel(const unsigned short* __restrict__ hout,
                             unsigned short* __restrict__ hprev, int B, int L, int H, int ndir) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)B * L * H;
  if (e >= per * ndir) return;
  const int dir = (int)(e / per);
  const int64_t r = e % per;
  const int u = (int)(r % H);
  const int64_t row = r / H;
  const int t = (int)(row % L);
  const int tp = dir == 0 ? t - 1 : t + 1;
  unsigned short v = 0;
  if (tp >= 0 && tp < L) v = hout[(row - t + tp) * ((int64_t)ndir * H) + dir * H + u];
  hprev[e] = v;
}

}  // namespace lstmm
}  // namespace irc

using namespace irc;

static inline unsigned nb256(int64_t n) { return (unsigned)((n + 255) / 256); }

extern "C" int irc_lstm_mfma_supported(int64_t H) { return H == 256; }

extern "C" int64_t irc_lstm_mfma_save_floats(int64_t B, int64_t L, int64_t H, int64_t ndir,
                                             int which) {
  // per (dir, group, t): gates 32 rows x 4H, c 32 rows x H (fragment-native order)
  const int64_t ngrp = (B + lstmm::BG - 1) / lstmm::BG;
  const int64_t gstep = (int64_t)lstmm::BG * 4 * H;
  const int64_t cstep = (int64_t)lstmm::BG * H;
  return ndir * ngrp * L * (which == 0 ? gstep : cstep);
}

extern "C" int irc_lstm_pack(const float* wih, const float* bih, const float* bhh,
                             const float* whh, int64_t In, int64_t H, int64_t ndir,
                             void* wih_packed, float* bias_packed, void* whh_bf16,
                             void* whhT_bf16, irc_stream_t stream) {
  IRC_REQUIRE(H == 256, "lstm_pack: H=%lld has no MFMA path", (long long)H);
  hipStream_t st = as_stream(stream);
  const int64_t n1 = ndir * 4 * H * In;
    hipLaunchKernelGGL(lstmm::pack_wih_kernel<256>, dim3(nb256(n1)), dim3(256), 0, st, wih, bih,
                       bhh, (unsigned short*)wih_packed, bias_packed, (int)In, (int)ndir);
  IRC_REQUIRE((whh_bf16 == nullptr) == (whhT_bf16 == nullptr), "lstm_pack: whh outputs together");
  if (whh_bf16 == nullptr) return check_launch("lstm_pack");  // the cluster path packs W_hh itself
  const int64_t n2 = ndir * 4 * H * H;
  hipLaunchKernelGGL(lstmm::pack_whh_kernel<256>, dim3(nb256(n2)), dim3(256), 0, st, whh,
                     (unsigned short*)whh_bf16, (unsigned short*)whhT_bf16, (int)ndir);
  return check_launch("lstm_pack");
}

extern "C" int irc_lstm_fwd_mfma(const float* xp_packed, const void* whh_bf16, void* hout,
                                 float* gsave, float* csave, void* hprev, int64_t B, int64_t L,
                                 int64_t H, int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(H == 256, "lstm_fwd_mfma: H=%lld", (long long)H);
  IRC_REQUIRE((gsave == nullptr) == (csave == nullptr), "lstm_fwd_mfma: gsave/csave together");
  if (B == 0 || L == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((B + lstmm::BG - 1) / lstmm::BG), (unsigned)ndir);
  prof_begin(st);
    hipLaunchKernelGGL(lstmm::lstm_fwd_mfma<256>, grid, dim3(lstmm::NTH), 0, st, xp_packed,
                       (const unsigned short*)whh_bf16, (unsigned short*)hout, gsave, csave,
                       (int)B, (int)L, (int)ndir);
  prof_end("lstm_fwd", st, 2.0 * B * L * ndir * 4.0 * H * H);
  int rc = check_launch("lstm_fwd_mfma");
  if (rc || hprev == nullptr) return rc;
  hipLaunchKernelGGL(lstmm::hprev_kernel, dim3(nb256(ndir * B * L * H)), dim3(256), 0, st,
                     (const unsigned short*)hout, (unsigned short*)hprev, (int)B, (int)L, (int)H,
                     (int)ndir);
  return check_launch("hprev_kernel");
}

extern "C" int irc_lstm_hprev(const void* hout, void* hprev, int64_t B, int64_t L, int64_t H,
                              int64_t ndir, irc_stream_t stream) {
  if (B == 0 || L == 0) return IRC_OK;
  hipLaunchKernelGGL(lstmm::hprev_kernel, dim3(nb256(ndir * B * L * H)), dim3(256), 0,
                     as_stream(stream), (const unsigned short*)hout, (unsigned short*)hprev, (int)B,
                     (int)L, (int)H, (int)ndir);
  return check_launch("hprev_kernel");
}

extern "C" int irc_lstm_bwd_mfma(const float* dy, const void* whhT_bf16, const float* gsave,
                                 const float* csave, void* dg, int64_t B, int64_t L, int64_t H,
                                 int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(H == 256, "lstm_bwd_mfma: H=%lld", (long long)H);
  if (B == 0 || L == 0) return IRC_OK;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((B + lstmm::BG - 1) / lstmm::BG), (unsigned)ndir);
  prof_begin(st);
    hipLaunchKernelGGL(lstmm::lstm_bwd_mfma<256>, grid, dim3(lstmm::NTH), 0, st, dy,
                       (const unsigned short*)whhT_bf16, gsave, csave, (unsigned short*)dg,
                       (int)B, (int)L, (int)ndir);
  prof_end("lstm_bwd", st, 2.0 * B * L * ndir * 4.0 * H * H);
  return check_launch("lstm_bwd_mfma");
}
