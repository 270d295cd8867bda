// BiLSTM recurrences for the encoder head (src/model.py:16-22, 39: nn.LSTM,
// batch_first, bidirectional, gate order i, f, g, o; zero initial state; the
// padded sequence is processed as is, so the reverse direction starts on PAD).
//
// The input projections xp = x W_ih^T + b_ih + b_hh of both directions are one
// GEMM (gemm.hip) issued by the host; these kernels run the sequential part:
//   forward : gates_t = xp_t + h_{t-1} W_hh^T ; c_t = f c_{t-1} + i g ; h_t = o tanh(c_t)
//   backward: BPTT producing d(gate pre-activations) for every t (the weight
//             gradients are then GEMMs over all (b, t) issued by the host).
// Layouts: xp [B, L, ndir*4H] fp32; h out [B, L, ndir*H]; saved gates
// [ndir, B, L, 4H] (activated i, f, g, o) and c [ndir, B, L, H] fp32;
// h_prev [ndir, B, L, H] (the h_{t-1} each step consumed: the dW_hh operand).
//
// lstm_*_valu: any H, fp32 math, W_hh streamed from L2 per step.  One
// workgroup per (batch group, direction); state lives in LDS.
#include "irc_common.h"

namespace irc {
namespace lstm {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2)
    return bf16_to_f32(reinterpret_cast<const unsigned short*>(p)[i]);
  else
    return reinterpret_cast<const float*>(p)[i];
}
template <typename T>
__device__ __forceinline__ void stf(T* p, int64_t i, float v) {
  if constexpr (sizeof(T) == 2)
    reinterpret_cast<unsigned short*>(p)[i] = f32_to_bf16(v);
  else
    reinterpret_cast<float*>(p)[i] = v;
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

struct FwdArgs {
  const float* xp;      // [B, L, ndir*4H]
  const void* whh;      // [ndir, 4H, H]
  void* hout;           // [B, L, ndir*H]
  float* gsave;         // [ndir, B, L, 4H] or null
  float* csave;         // [ndir, B, L, H] or null
  void* hprev;          // [ndir, B, L, H] or null
  int B, L, H, ndir, bg;
};

template <typename T>
__global__ __launch_bounds__(256) void lstm_fwd_valu(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, G4 = 4 * H, bg = a.bg;
  float* hs = sm;                 // [bg][H]
  float* cs = hs + bg * H;        // [bg][H]
  float* gs = cs + bg * H;        // [bg][4H]
  const int dir = blockIdx.y;
  const int b0 = blockIdx.x * bg;
  const int nb = min(bg, a.B - b0);
  const T* W = reinterpret_cast<const T*>(a.whh) + (int64_t)dir * G4 * H;
  for (int i = threadIdx.x; i < bg * H; i += blockDim.x) hs[i] = cs[i] = 0.f;
  __syncthreads();
  const int64_t xld = (int64_t)a.ndir * G4;
  const int64_t hld = (int64_t)a.ndir * H;
  for (int step = 0; step < a.L; ++step) {
    const int t = dir == 0 ? step : a.L - 1 - step;
    for (int e = threadIdx.x; e < nb * G4; e += blockDim.x) {
      const int b = e / G4, gcol = e % G4;
      float acc = a.xp[((int64_t)(b0 + b) * a.L + t) * xld + dir * G4 + gcol];
      const float* hb = hs + b * H;
      const int64_t wr = (int64_t)gcol * H;
      for (int k = 0; k < H; ++k) acc += hb[k] * ldf(W, wr + k);
      gs[b * G4 + gcol] = acc;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * H; e += blockDim.x) {
      const int b = e / H, u = e % H;
      const float ig = sigm(gs[b * G4 + u]);
      const float fg = sigm(gs[b * G4 + H + u]);
      const float gg = tanhf(gs[b * G4 + 2 * H + u]);
      const float og = sigm(gs[b * G4 + 3 * H + u]);
      const float hp = hs[b * H + u];
      const float c = fg * cs[b * H + u] + ig * gg;
      const float h = og * tanhf(c);
      const int64_t row = (int64_t)(b0 + b) * a.L + t;
      if (a.gsave) {
        float* gp = a.gsave + ((int64_t)dir * a.B * a.L + row) * G4;
        gp[u] = ig;
        gp[H + u] = fg;
        gp[2 * H + u] = gg;
        gp[3 * H + u] = og;
      }
      if (a.csave) a.csave[((int64_t)dir * a.B * a.L + row) * H + u] = c;
      if (a.hprev) stf(reinterpret_cast<T*>(a.hprev), ((int64_t)dir * a.B * a.L + row) * H + u, hp);
      stf(reinterpret_cast<T*>(a.hout), row * hld + dir * H + u, h);
      cs[b * H + u] = c;
      gs[b * G4 + u] = h;  // stash new h; gate i slot no longer needed
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * H; e += blockDim.x) {
      const int b = e / H, u = e % H;
      hs[b * H + u] = gs[b * G4 + u];
    }
    __syncthreads();
  }
}

struct BwdArgs {
  const float* dy;     // [B, L, ndir*H] gradient wrt the layer output
  const void* whh;     // [ndir, 4H, H]
  const float* gsave;  // [ndir, B, L, 4H]
  const float* csave;  // [ndir, B, L, H]
  float* dgates;       // [ndir, B, L, 4H] d(pre-activation)
  int B, L, H, ndir, bg;
};

template <typename T>
__global__ __launch_bounds__(256) void lstm_bwd_valu(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, G4 = 4 * H, bg = a.bg;
  float* dh = sm;                 // [bg][H]  dh_next
  float* dc = dh + bg * H;        // [bg][H]  dc_next
  float* dg = dc + bg * H;        // [bg][4H]
  const int dir = blockIdx.y;
  const int b0 = blockIdx.x * bg;
  const int nb = min(bg, a.B - b0);
  const T* W = reinterpret_cast<const T*>(a.whh) + (int64_t)dir * G4 * H;
  for (int i = threadIdx.x; i < bg * H; i += blockDim.x) dh[i] = dc[i] = 0.f;
  __syncthreads();
  const int64_t hld = (int64_t)a.ndir * H;
  const int64_t dbase = (int64_t)dir * a.B * a.L;
  for (int step = 0; step < a.L; ++step) {
    // reverse of the forward processing order
    const int t = dir == 0 ? a.L - 1 - step : step;
    const int tp = dir == 0 ? t - 1 : t + 1;  // previous step in forward order
    const bool has_prev = tp >= 0 && tp < a.L;
    for (int e = threadIdx.x; e < nb * H; e += blockDim.x) {
      const int b = e / H, u = e % H;
      const int64_t row = (int64_t)(b0 + b) * a.L + t;
      const float* gp = a.gsave + (dbase + row) * G4;
      const float ig = gp[u], fg = gp[H + u], gg = gp[2 * H + u], og = gp[3 * H + u];
      const float c = a.csave[(dbase + row) * H + u];
      const float cprev =
          has_prev ? a.csave[(dbase + (int64_t)(b0 + b) * a.L + tp) * H + u] : 0.f;
      const float dht = a.dy[row * hld + dir * H + u] + dh[b * H + u];
      const float tc = tanhf(c);
      const float dot = dht * tc;
      const float dct = dht * og * (1.f - tc * tc) + dc[b * H + u];
      const float di = dct * gg, dgg = dct * ig, df = dct * cprev;
      dc[b * H + u] = dct * fg;
      float* out = a.dgates + (dbase + row) * G4;
      const float p0 = di * ig * (1.f - ig), p1 = df * fg * (1.f - fg);
      const float p2 = dgg * (1.f - gg * gg), p3 = dot * og * (1.f - og);
      out[u] = p0;
      out[H + u] = p1;
      out[2 * H + u] = p2;
      out[3 * H + u] = p3;
      dg[b * G4 + u] = p0;
      dg[b * G4 + H + u] = p1;
      dg[b * G4 + 2 * H + u] = p2;
      dg[b * G4 + 3 * H + u] = p3;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nb * H; e += blockDim.x) {
      const int b = e / H, k = e % H;
      float acc = 0.f;
      const float* d = dg + b * G4;
      for (int gcol = 0; gcol < G4; ++gcol) acc += d[gcol] * ldf(W, (int64_t)gcol * H + k);
      dh[b * H + k] = acc;
    }
    __syncthreads();
  }
}

}  // namespace lstm
}  // namespace irc

using namespace irc;

extern "C" int irc_lstm_fwd(int dtype, const float* xp, const void* whh, void* hout, float* gsave,
                            float* csave, void* hprev, int64_t B, int64_t L, int64_t H,
                            int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(B >= 0 && L >= 0 && H >= 1 && (ndir == 1 || ndir == 2), "lstm_fwd: bad sizes");
  if (B == 0 || L == 0) return IRC_OK;
  int bg = (int)((32 * 1024) / (6 * H * 4));  // LDS: 6*bg*H floats <= 32 KB
  if (bg < 1) bg = 1;
  if (bg > 8) bg = 8;
  const size_t lds = (size_t)6 * bg * H * 4;
  IRC_REQUIRE(lds <= (size_t)IRC_LDS_BYTES, "lstm_fwd: H too large");
  lstm::FwdArgs a{xp, whh, hout, gsave, csave, hprev, (int)B, (int)L, (int)H, (int)ndir, bg};
  dim3 grid((unsigned)((B + bg - 1) / bg), (unsigned)ndir);
  if (dtype == 0)
    hipLaunchKernelGGL((lstm::lstm_fwd_valu<unsigned short>), grid, dim3(256), lds,
                       as_stream(stream), a);
  else
    hipLaunchKernelGGL((lstm::lstm_fwd_valu<float>), grid, dim3(256), lds, as_stream(stream), a);
  return check_launch("lstm_fwd_valu");
}

extern "C" int irc_lstm_bwd(int dtype, const float* dy, const void* whh, const float* gsave,
                            const float* csave, float* dgates, int64_t B, int64_t L, int64_t H,
                            int64_t ndir, irc_stream_t stream) {
  IRC_REQUIRE(B >= 0 && L >= 0 && H >= 1 && (ndir == 1 || ndir == 2), "lstm_bwd: bad sizes");
  if (B == 0 || L == 0) return IRC_OK;
  int bg = (int)((32 * 1024) / (6 * H * 4));
  if (bg < 1) bg = 1;
  if (bg > 8) bg = 8;
  const size_t lds = (size_t)6 * bg * H * 4;
  IRC_REQUIRE(lds <= (size_t)IRC_LDS_BYTES, "lstm_bwd: H too large");
  lstm::BwdArgs a{dy, whh, gsave, csave, dgates, (int)B, (int)L, (int)H, (int)ndir, bg};
  dim3 grid((unsigned)((B + bg - 1) / bg), (unsigned)ndir);
  if (dtype == 0)
    hipLaunchKernelGGL((lstm::lstm_bwd_valu<unsigned short>), grid, dim3(256), lds,
                       as_stream(stream), a);
  else
    hipLaunchKernelGGL((lstm::lstm_bwd_valu<float>), grid, dim3(256), lds, as_stream(stream), a);
  return check_launch("lstm_bwd_valu");
}
