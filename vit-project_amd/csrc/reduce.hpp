// Column reduction of an [S][N] f32 partial-sum matrix: out[j] (+)= sum_z part[z][j].
// Block = 64 columns x 16 row-slices (1024 threads), 4 independent accumulators
// per thread, LDS tree over the slices.  Used for the second stage of bias /
// LayerNorm-affine gradients (S = a few hundred partial rows).
#pragma once
#include "common.hpp"

namespace {
struct ColOut {
  float* p[3];
};

// block (x, y, z): columns x*64 .. x*64+63 of partial matrix z (part + z*zin), partial rows
// [y*rows_per, min(S, (y+1)*rows_per)) -> out.p[z][y*ldo + column]
__global__ __launch_bounds__(1024) void colreduce_kernel(const float* __restrict__ part, int64_t zin, int S, int N,
                                                         int rows_per, ColOut out, int64_t ldo, int accumulate) {
  __shared__ float red[16][65];
  part += blockIdx.z * zin;
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
    float* o = out.p[blockIdx.z] + (int64_t)blockIdx.y * ldo + j;
    *o = accumulate ? *o + s : s;
  }
}

inline int64_t colreduce_scratch_floats(int S, int N) { return S > 64 ? (int64_t)((S + 63) / 64) * N : 0; }

// out[q][j] (+)= sum_z part[q][z][j] for nq (<= 3) stacked [S][N] partial matrices, in one
// launch per stage.  With `scratch` (>= nq * colreduce_scratch_floats(S, N) floats) and
// S > 64 the rows are first reduced in 64-row groups by ceil(S/64) x ceil(N/64) blocks per
// matrix (enough workgroups to hide load latency), then the group sums in a second pass.
inline void launch_colreduce_multi(const float* part, int nq, int S, int N, float* const* outs, int accumulate,
                                   hipStream_t s, float* scratch = nullptr) {
  if (part == nullptr || nq < 1 || S <= 0 || N <= 0) return;
  for (int q = 0; q < nq; ++q)
    if (outs[q] == nullptr) return;
  const int nb = (N + 63) / 64;
  ColOut o{};
  for (int q = 0; q < nq; ++q) o.p[q] = outs[q];
  if (scratch != nullptr && S > 64) {
    const int G = (S + 63) / 64;
    ColOut sc{};
    for (int q = 0; q < nq; ++q) sc.p[q] = scratch + (int64_t)q * G * N;
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, G, nq), dim3(1024), 0, s, part, (int64_t)S * N, S, N, 64, sc,
                       (int64_t)N, 0);
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, 1, nq), dim3(1024), 0, s, (const float*)scratch, (int64_t)G * N, G,
                       N, G, o, (int64_t)0, accumulate);
  } else {
    hipLaunchKernelGGL(colreduce_kernel, dim3(nb, 1, nq), dim3(1024), 0, s, part, (int64_t)S * N, S, N, S, o,
                       (int64_t)0, accumulate);
  }
}

// out[j] (+)= sum_z part[z][j] (scratch: >= colreduce_scratch_floats(S, N) floats).
inline void launch_colreduce(const float* part, int S, int N, float* out, int accumulate, hipStream_t s,
                             float* scratch = nullptr) {
  launch_colreduce_multi(part, 1, S, N, &out, accumulate, s, scratch);
}
}  // namespace
