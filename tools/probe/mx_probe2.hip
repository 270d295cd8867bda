// Probe 2 of v_mfma_scale_f32_16x16x128_f8f6f4: which scale lane governs which
// bytes of which data lane.  Block (l, T): e4m3 1.0 in all 32 bytes of data lane
// l only (A in mode 0, B in mode 1; the other operand all ones), every scale 2^0
// except scale lane T's = 2^10.  out[l][T] = C at lane l's row (A) / column (B):
// 32 + 1023 * (number of lane-l bytes whose block scale comes from lane T).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe2(float* out, int mode) {
  const int l = blockIdx.x, T = blockIdx.y, lane = threadIdx.x;
  v8i32 ones, zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) ones[i] = 0x38383838;
  const bool me = lane == l;
  const v8i32 a = mode == 0 ? (me ? ones : zero) : ones;
  const v8i32 b = mode == 1 ? (me ? ones : zero) : ones;
  const int s = lane == T ? 127 + 10 : 127;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, mode == 0 ? s : 127, 0,
                                                        mode == 1 ? s : 127);
  // C: col = lane & 15, row = 4 (lane >> 4) + e.  Mode 0 wants row l & 15, col 0;
  // mode 1 wants row 0, col l & 15.
  const int want_row = mode == 0 ? (l & 15) : 0, want_col = mode == 0 ? 0 : (l & 15);
  if ((lane & 15) == want_col && (lane >> 4) == (want_row >> 2))
    out[l * 64 + T] = c[want_row & 3];
}

extern "C" int mx_probe2(float* out, int mode) {
  hipLaunchKernelGGL(probe2, dim3(64, 64), dim3(64), 0, 0, out, mode);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
