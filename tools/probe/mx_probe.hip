// Probe of v_mfma_scale_f32_16x16x128_f8f6f4's operand and scale lane maps
// (diagnostic, not part of the library).  Wave w (64 of them) puts e4m3 1.0 into
// the A operand of lane (w & 63) only -- bytes [0, 32) -- with B = all ones, unit
// B scales, and A scale bytes 127 + lane (distinct per lane) in byte OPSEL of the
// scale VGPR.  out[w][16x16] = C; the host reads which row got the data and which
// lane's scale multiplied it.  mode 1: the same for B (A ones, B one lane).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef int v8i32 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int OPSEL>
__global__ void probe(float* out, int mode) {
  const int w = blockIdx.x, lane = threadIdx.x;
  v8i32 ones, zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) ones[i] = 0x38383838;  // e4m3 1.0
  const bool me = lane == w;
  v8i32 a = mode == 0 ? (me ? ones : zero) : ones;
  v8i32 b = mode == 1 ? (me ? ones : zero) : ones;
  const int sdist = (127 + (lane & 63) - 32) << (8 * OPSEL);  // 2^(lane - 32)
  const int sunit = 127 << (8 * OPSEL);
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OPSEL,
                                                        mode == 0 ? sdist : sunit, OPSEL,
                                                        mode == 1 ? sdist : sunit);
  // C layout: col = lane & 15, row = 4 (lane >> 4) + e
  for (int e = 0; e < 4; ++e) out[(w * 16 + 4 * (lane >> 4) + e) * 16 + (lane & 15)] = c[e];
}

extern "C" int mx_probe(float* out, int mode, int opsel) {
  if (opsel == 0) hipLaunchKernelGGL(probe<0>, dim3(64), dim3(64), 0, 0, out, mode);
  else if (opsel == 1) hipLaunchKernelGGL(probe<1>, dim3(64), dim3(64), 0, 0, out, mode);
  else if (opsel == 2) hipLaunchKernelGGL(probe<2>, dim3(64), dim3(64), 0, 0, out, mode);
  else hipLaunchKernelGGL(probe<3>, dim3(64), dim3(64), 0, 0, out, mode);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
