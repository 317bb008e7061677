// Byte output of v_cvt_pk_fp8_f32 (word_sel 0 then 1) for known floats: which e4m3 encoding
// (OCP e4m3fn vs fnuz) and which byte order the fp8 attention kernel's pack_fp8x4 produces.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* x, int* y) {
  const int l = threadIdx.x;
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * l], x[4 * l + 1], 0, false);
  y[l] = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * l + 2], x[4 * l + 3], w, true);
}
int main() {
  float h[16] = {1.0f, 0.1f, 3.0f, -2.5f, 448.f, 0.001953125f, 300.f, 17.f, 0.5f, 2.f, 256.f, 1.0625f, 1.125f, 0.015625f, -1.f, 100.f};
  float* d; int* o; int r[4];
  (void)hipMalloc(&d, 64); (void)hipMalloc(&o, 16);
  (void)hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(4), 0, 0, d, o);
  (void)hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i)
    for (int b = 0; b < 4; ++b) printf("%g -> 0x%02x\n", h[4 * i + b], (r[i] >> (8 * b)) & 255);
  return 0;
}
