// Which workgroups share a CU?  512 workgroups of 256 threads with 72 KiB of dynamic LDS each
// (two fit a CU, as the V6/V7 GEMM configurations) record (XCC, SE, SH, CU) and spin long enough
// that the whole first round stays resident together.
#include <hip/hip_runtime.h>
extern "C" __global__ void placement_kernel(unsigned* out, unsigned long long spin) {
  extern __shared__ char lds[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    lds[0] = 1;
    out[blockIdx.x * 2] = hw;
    out[blockIdx.x * 2 + 1] = xcc;
  }
  while (__builtin_amdgcn_s_memtime() - t0 < spin) __builtin_amdgcn_s_sleep(8);
}
extern "C" int run_placement(unsigned* host, int blocks, int lds_bytes, unsigned long long spin) {
  unsigned* d;
  if (hipMalloc(&d, blocks * 8)) return 1;
  if (hipFuncSetAttribute((const void*)placement_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes)) return 3;
  hipLaunchKernelGGL(placement_kernel, dim3(blocks), dim3(256), lds_bytes, 0, d, spin);
  if (hipMemcpy(host, d, blocks * 8, hipMemcpyDeviceToHost)) return 2;
  hipFree(d);
  return 0;
}
