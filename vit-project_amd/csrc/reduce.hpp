// Column reduction of an [S][N] f32 partial-sum matrix: out[j] (+)= sum_z part[z][j].
// Block = 64 columns x 16 row-slices (1024 threads), 4 independent accumulators
// per thread, LDS tree over the slices.  Used for the second stage of bias /
// LayerNorm-affine gradients (S = a few hundred partial rows).
#pragma once
#include "common.hpp"

namespace {
// block (x, y): columns x*64 .. x*64+63, partial rows [y*rows_per, min(S, (y+1)*rows_per))
__global__ __launch_bounds__(1024) void colreduce_kernel(const float* __restrict__ part, int S, int N, int rows_per,
                                                         float* __restrict__ out, int64_t ldo, int accumulate) {
  __shared__ float red[16][65];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  const int z0 = blockIdx.y * rows_per, z1 = min(S, z0 + rows_per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (j < N) {
    int z = z0 + sl;
    for (; z + 48 < z1; z += 64) {
      a0 += part[(int64_t)z * N + j];
      a1 += part[(int64_t)(z + 16) * N + j];
      a2 += part[(int64_t)(z + 32) * N + j];
      a3 += part[(int64_t)(z + 48) * N + j];
    }
    for (; z < z1; z += 16) a0 += part[(int64_t)z * N + j];
  }
  red[sl][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && j < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][c];
    float* o = out + (int64_t)blockIdx.y * ldo + j;
    *o = accumulate ? *o + s : s;
  }
}

// out[j] (+)= sum_z part[z][j].  With `scratch` (>= ceil(S/64)*N floats) and S > 64
// the rows are first reduced in 64-row groups by ceil(S/64) x ceil(N/64) blocks
// (enough workgroups to hide load latency), then the group sums in a second pass.
inline void launch_colreduce(const float* part, int S, int N, float* out, int accumulate, hipStream_t s,
                             float* scratch = nullptr) {
  const int nb = (N + 63) / 64;
  if (scratch != nullptr && S > 64) {
    const int G = (S + 63) / 64;
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, G), dim3(1024), 0, s, part, S, N, 64, scratch, (int64_t)N, 0);
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, 1), dim3(1024), 0, s, (const float*)scratch, G, N, G, out,
                       (int64_t)0, accumulate);
  } else {
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, 1), dim3(1024), 0, s, part, S, N, S, out, (int64_t)0, accumulate);
  }
}
inline int64_t colreduce_scratch_floats(int S, int N) { return S > 64 ? (int64_t)((S + 63) / 64) * N : 0; }
}  // namespace
