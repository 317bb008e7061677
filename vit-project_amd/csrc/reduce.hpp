// Column reduction of an [S][N] f32 partial-sum matrix: out[j] (+)= sum_z part[z][j].
// Block = 64 columns x 16 row-slices (1024 threads), 4 independent accumulators
// per thread, LDS tree over the slices.  Used for the second stage of bias /
// LayerNorm-affine gradients (S = a few hundred partial rows).
#pragma once
#include "common.hpp"

namespace {
__global__ __launch_bounds__(1024) void colreduce_kernel(const float* __restrict__ part, int S, int N,
                                                         float* __restrict__ out, int accumulate) {
  __shared__ float red[16][65];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (j < N) {
    int z = sl;
    for (; z + 48 < S; z += 64) {
      a0 += part[(int64_t)z * N + j];
      a1 += part[(int64_t)(z + 16) * N + j];
      a2 += part[(int64_t)(z + 32) * N + j];
      a3 += part[(int64_t)(z + 48) * N + j];
    }
    for (; z < S; z += 16) a0 += part[(int64_t)z * N + j];
  }
  red[sl][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && j < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][c];
    out[j] = accumulate ? out[j] + s : s;
  }
}

inline void launch_colreduce(const float* part, int S, int N, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(colreduce_kernel, dim3((N + 63) / 64), dim3(1024), 0, s, part, S, N, out, accumulate);
}
}  // namespace
