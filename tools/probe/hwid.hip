// Diagnostic: which SIMD does each wave of a 512-thread workgroup land on?
#include <hip/hip_runtime.h>
extern "C" __global__ void hwid_kernel(unsigned* out) {
  unsigned v = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);  // HW_REG_HW_ID
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = v;
}
extern "C" int run_hwid(unsigned* host, int blocks, int threads) {
  unsigned* d;
  int n = blocks * threads / 64;
  if (hipMalloc(&d, n * 4)) return 1;
  hipLaunchKernelGGL(hwid_kernel, dim3(blocks), dim3(threads), 0, 0, d);
  if (hipMemcpy(host, d, n * 4, hipMemcpyDeviceToHost)) return 2;
  hipFree(d);
  return 0;
}
