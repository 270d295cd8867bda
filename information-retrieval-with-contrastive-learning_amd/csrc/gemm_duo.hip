// Two-workgroups-per-CU bf16 GEMM for gfx950 (experimental path of irc_gemm, off by
// default: irc_gemm_set_duo / IRC_GEMM_DUO).
//
//   C[M, N] = alpha * A[M][K] . B[N][K]^T (+ bias) (-> GELU) (+ residual), bf16 out
//
// Why ("Where the GEMM time goes"): on the BERT shapes the 256 x 256 /
// 256 x 384 one-workgroup-per-CU kernels leave the matrix pipe idle during every tile's
// epilogue (FFN1 + GELU: 82 of 207 us; the bias epilogue alone 29 us), and every CU
// reaches its epilogue at the same time, so the C stores arrive as one HBM burst.  Here
// a workgroup is 4 waves on a 128 x 256 tile with 72 KB of LDS and <= 256 VGPRs, so two
// workgroups share each CU (one wave of each per SIMD): while one runs its epilogue
// (VALU + stores) the other's MFMAs keep the matrix pipe busy.  The two first
// workgroups on a CU are staggered (the second sleeps ~half a tile, found by a per-CU
// arrival counter), so their epilogues stay apart.  Price: each 128 x 256 tile DMAs
// 1.5x the operand bytes per flop of a 256 x 256 tile.
//
//  * Wave w of a workgroup owns all 128 rows x columns [64 w, 64 w + 64): 8 x 4
//    accumulators of v_mfma_f32_16x16x32_bf16 (128 VGPRs), as one ping-pong group of
//    gemm_pp_kernel.
//  * K in 32-deep stages (64-byte LDS rows) through a 3-slot ring filled by
//    global_load_lds_dwordx4 with counted vmcnt: stage kt + 2 is issued right after the
//    barrier of stage kt.  The 16-byte chunk c of row r sits in slot c ^ key(r),
//    key(r) = (-(r >> 2)) & 3: a 16x16x32 fragment read (lane l: row l & 15, chunk
//    l >> 4) puts the 16 lanes of each ds_read_b128 group on 16 distinct bank slots.
//  * Epilogue through LDS (32-row passes per wave, the ring is free by then), fused
//    bias / GELU (gelu_lite2: bf16 output) / residual, 16-byte stores.
#include "gemm_pp.h"

#include <atomic>
#include <cstdlib>

namespace irc {
namespace duo {

constexpr int BM = 128, BN = 256, BK = 32, NT = 256, NSTG = 3;
constexpr int ROWB = BK * 2;  // 64-byte LDS rows
constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STG = A_BYTES + B_BYTES;  // 8 / 16 / 24 KB
constexpr int LDS_BYTES = NSTG * STG;                                           // 72 KB
constexpr int PER_STAGE = (BM + BN) * 4 / NT;  // DMA wave-instructions per stage per wave: 6
constexpr int EP_PITCH = 68;                   // epilogue staging pitch (floats)
static_assert(4 * 32 * EP_PITCH * 4 <= LDS_BYTES, "epilogue staging fits the ring");

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RESID = 3, EPI_RESID = 4 };

struct DArgs {
  const unsigned short* A;
  const unsigned short* B;
  unsigned short* C;
  const float* bias;
  const unsigned short* R;
  int M, N, K;
  int64_t lda, ldb, ldc, ldr;
  float alpha;
  int first_wave;  // blocks of the first dispatch round (2 per CU)
  int sleeps;      // stagger: s_sleep 127 rounds of the second workgroup on a CU
  uint32_t* cu_ctr;
};

__device__ __forceinline__ int key(int r) { return (-(r >> 2)) & 3; }

// rows [r0, r0 + ROWS) x k [k0, k0 + 32) of X into a lane-linear image: chunk p = row
// 4 r + slot s holds logical chunk s ^ key(r); 64 chunks (16 rows) per wave-instruction
template <int ROWS>
__device__ __forceinline__ void stage(const unsigned short* __restrict__ X, int64_t ld, int r0,
                                      int nrows, int k0, char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < ROWS * 4 / NT; ++i) {
    const int p = (i * 4 + wave) * 64 + lane;
    const int row = p >> 2;
    const int c = (p & 3) ^ key(row);
    int gr = r0 + row;
    gr = gr < nrows ? gr : nrows - 1;
    glds16(X + (int64_t)gr * ld + k0 + c * 8, img + (i * 4 + wave) * 1024);
  }
}

__device__ __forceinline__ bf16x8 frag(const char* img, int row0, int lane) {
  const int row = row0 + (lane & 15);
  const int c = lane >> 4;
  return *reinterpret_cast<const bf16x8*>(img + row * ROWB + 16 * (c ^ key(row)));
}

template <int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_duo_kernel(DArgs g) {
  // one LDS object (a second __shared__ variable can make hipcc wait vmcnt(0) before
  // the fragment reads, cdna_hip_programming.md §5 item 4(a)); the stagger flag sits
  // past the ring
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES + 16];
  const int tiles_m = (g.M + BM - 1) / BM;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap: blocks sharing an XCD walk consecutive tiles
    const int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  // consecutive tiles share the weight (B) column tile: rows fastest
  const int tm = bid % tiles_m, tn = bid / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  if (g.sleeps > 0 && (int)blockIdx.x < g.first_wave) {
    // stagger the two first workgroups of a CU by ~half a tile (speed only)
    int* s_late = reinterpret_cast<int*>(lds + LDS_BYTES);
    if (threadIdx.x == 0) *s_late = (int)(atomicAdd(&g.cu_ctr[__smid() & 1023], 1u) & 1u);
    __syncthreads();
    if (*s_late)
      for (int i = 0; i < g.sleeps; ++i) __builtin_amdgcn_s_sleep(127);
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)0.0f;

  const int nk = g.K / BK;
  stage<BM>(g.A, g.lda, m0, g.M, 0, lds, wave, lane);
  stage<BN>(g.B, g.ldb, n0, g.N, 0, lds + A_BYTES, wave, lane);
  if (nk > 1) {
    stage<BM>(g.A, g.lda, m0, g.M, BK, lds + STG, wave, lane);
    stage<BN>(g.B, g.ldb, n0, g.N, BK, lds + STG + A_BYTES, wave, lane);
  }
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (stage kt + 1 may still be in flight); every wave is past its
    // fragment reads of stage kt - 1, whose slot receives stage kt + 2 below
    if (kt + 1 < nk) wait_vmcnt<PER_STAGE>();
    else wait_vmcnt<0>();
    wg_barrier();
    if (kt + 2 < nk) {
      const int s2 = slot == 0 ? 2 : slot - 1;  // (kt + 2) % 3
      char* img = lds + s2 * STG;
      stage<BM>(g.A, g.lda, m0, g.M, (kt + 2) * BK, img, wave, lane);
      stage<BN>(g.B, g.ldb, n0, g.N, (kt + 2) * BK, img + A_BYTES, wave, lane);
    }
    const char* la = lds + slot * STG;
    const char* lb = la + A_BYTES;
    bf16x8 fa[8], fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag(lb, 64 * wave + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = frag(la, 16 * i, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    slot = slot == 2 ? 0 : slot + 1;
  }
  // ---- epilogue: acc[i][j] element e -> row 16 i + 4 (lane >> 4) + e, col 64 wave + 16 j + (lane & 15)
  lds_barrier();  // every wave is past its last fragment reads: the ring becomes staging
  float* st = reinterpret_cast<float*>(lds) + wave * (32 * EP_PITCH);
  const int cbase = n0 + 64 * wave;
  float bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = cbase + 16 * j + (lane & 15);
    bv[j] = (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESID) && col < g.N
                ? g.bias[col] : 0.f;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // 32-row passes
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x2_t v[2];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e >> 1][e & 1] = acc[2 * p + ii][j][e] * g.alpha + bv[j];
        if (EPI == EPI_BIAS_GELU) {
          v[0] = gelu_lite2(v[0]);
          v[1] = gelu_lite2(v[1]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          st[(16 * ii + 4 * (lane >> 4) + e) * EP_PITCH + 16 * j + (lane & 15)] = v[e >> 1][e & 1];
      }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int rbase = m0 + 32 * p;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int c = it * 64 + lane;
      const int rl = c >> 3, c8 = (c & 7) * 8;
      const int row = rbase + rl, col = cbase + c8;
      if (row >= g.M || col >= g.N) continue;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c8]);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(&st[rl * EP_PITCH + c8 + 4]);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      if (EPI == EPI_BIAS_RESID || EPI == EPI_RESID) {
        const u16x8 rr = *reinterpret_cast<const u16x8*>(g.R + (int64_t)row * g.ldr + col);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] += bf16_to_f32(rr[t]);
      }
      u16x8 o;
#pragma unroll
      for (int t = 0; t < 8; ++t) o[t] = f32_to_bf16(v[t]);
      *reinterpret_cast<u16x8*>(g.C + (int64_t)row * g.ldc + col) = o;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

__device__ uint32_t g_duo_cu_ctr[1024];

static int cu_count() {
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

// IRC_DUO_SLEEPS: s_sleep 127 rounds (~3.4 us each) of the staggered workgroup; default
// ~half a 128 x 256 tile at 0.5 of the shared CU's MFMA rate: K / 256 rounds.
static int sleeps_for(int K) {
  static const int env = [] {
    const char* e = getenv("IRC_DUO_SLEEPS");
    return e ? atoi(e) : -1;
  }();
  if (env >= 0) return env;
  const int s = (K + 128) / 256;
  return s < 1 ? 1 : s;
}

}  // namespace duo

namespace gpp {
// the duo path: bf16 NT (A [M][K], B [N][K]), bf16 C, one batch, epilogues 0-4, 16-byte
// aligned rows, K % 32 == 0, and enough tiles for two rounds of two per CU
bool duo_qualifies(int la, int lb, int epi, int out_f32, int accumulate, int64_t M, int64_t N,
                   int64_t K, const void* A, int64_t lda, const void* B, int64_t ldb,
                   const void* C, int64_t ldc, const void* R, int64_t ldr, int64_t batch) {
  if (la != 0 || lb != 0 || out_f32 || accumulate || batch != 1 || epi < 0 || epi > 4) return false;
  if (K % duo::BK != 0 || K == 0 || N % 8 != 0) return false;
  if (lda % 8 || ldb % 8 || ldc % 8 || (R && ldr % 8)) return false;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)R) % 16) return false;
  const int64_t tiles = ((M + duo::BM - 1) / duo::BM) * ((N + duo::BN - 1) / duo::BN);
  const int ncu = duo::cu_count();
  return ncu > 0 && tiles >= 4 * ncu;
}

void duo_run(int epi, const unsigned short* A, int64_t lda, const unsigned short* B, int64_t ldb,
             unsigned short* C, int64_t ldc, const float* bias, const unsigned short* R,
             int64_t ldr, int M, int N, int K, float alpha, hipStream_t st) {
  uint32_t* ctr = nullptr;
  (void)hipGetSymbolAddress(reinterpret_cast<void**>(&ctr), HIP_SYMBOL(duo::g_duo_cu_ctr));
  duo::DArgs g{A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha,
               2 * duo::cu_count(), ctr ? duo::sleeps_for(K) : 0, ctr};
  const int tiles = ((M + duo::BM - 1) / duo::BM) * ((N + duo::BN - 1) / duo::BN);
  switch (epi) {
#define IRC_DUO(E)                                                                       \
  case E:                                                                                \
    hipLaunchKernelGGL((duo::gemm_duo_kernel<E>), dim3(tiles), dim3(duo::NT), 0, st, g); \
    break;
    IRC_DUO(0) IRC_DUO(1) IRC_DUO(2) IRC_DUO(3) IRC_DUO(4)
#undef IRC_DUO
  }
}
}  // namespace gpp
}  // namespace irc
