// Kernels around the CLIP-HBA forward/loss (NEWP:287-304, 994):
// token embedding + positional add for the text tower, row gather/scatter (EOT
// pooling of the text tower, CLS rows of the visual tower), the L2 row
// normalisation with the exp(logit_scale) factor of CLIP.forward, and nn.MSELoss.
// The GEMMs, LayerNorms and attention of both towers run through gemm.hip,
// norm.hip and attention.hip.  All HBM-bound and small (66 x 77 tokens, 64 x 768
// features): one wave per row, 16-B loads where the rows allow it.
#include "common.hpp"

// x[s*L + t][:] = table[tokens[s*L + t]][:] + pos[t][:]   (nn.Embedding + positional_embedding)
__global__ __launch_bounds__(256) void token_embed_kernel(const int64_t* __restrict__ tok, const float* __restrict__ table,
                                                          const float* __restrict__ pos, float* __restrict__ x, int rows,
                                                          int L, int D, int vocab) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  int64_t id = tok[row];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // clamp: never read outside the table
  const float* e = table + id * D;
  const float* p = pos + (int64_t)(row % L) * D;
  float* o = x + (int64_t)row * D;
  for (int d = lane * 4; d < D; d += 256) {
    f32x4 a = *reinterpret_cast<const f32x4*>(e + d), b = *reinterpret_cast<const f32x4*>(p + d);
    *reinterpret_cast<f32x4*>(o + d) = a + b;
  }
}

// dst[i][:] = src[idx[i]][:]  (SCATTER = 0)   or   dst[idx[i]][:] = src[i][:]  (SCATTER = 1)
template <int SCATTER>
__global__ __launch_bounds__(256) void rows_kernel(const float* __restrict__ src, int64_t ld_src,
                                                   const int64_t* __restrict__ idx, float* __restrict__ dst,
                                                   int64_t ld_dst, int n, int D) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t r = idx[i];
  const float* s = src + (SCATTER ? (int64_t)i : r) * ld_src;
  float* o = dst + (SCATTER ? r : (int64_t)i) * ld_dst;
  for (int d = lane; d < D; d += 64) o[d] = s[d];
}

// y = exp(log_scale) * x / ||x||, rnorm = 1 / ||x||   (CLIP.forward feature normalisation)
__global__ __launch_bounds__(256) void rownorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ log_scale,
                                                          float* __restrict__ y, float* __restrict__ rnorm, int n, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  const float* xr = x + (int64_t)row * D;
  float ss = 0.f;
  for (int d = lane; d < D; d += 64) ss = fmaf(xr[d], xr[d], ss);
  ss = wave_sum(ss);
  const float rn = 1.0f / sqrtf(ss);
  const float sc = (log_scale ? expf(*log_scale) : 1.0f) * rn;
  float* yr = y + (int64_t)row * D;
  for (int d = lane; d < D; d += 64) yr[d] = xr[d] * sc;
  if (lane == 0) rnorm[row] = rn;
}

// dx = s * rnorm * (dy - xhat * <xhat, dy>),  xhat = x * rnorm
__global__ __launch_bounds__(256) void rownorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const float* __restrict__ rnorm,
                                                          const float* __restrict__ log_scale, float* __restrict__ dx,
                                                          int n, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= n) return;
  const float* xr = x + (int64_t)row * D;
  const float* gr = dy + (int64_t)row * D;
  const float rn = rnorm[row];
  float dot = 0.f;
  for (int d = lane; d < D; d += 64) dot = fmaf(xr[d] * rn, gr[d], dot);
  dot = wave_sum(dot);
  const float sc = (log_scale ? expf(*log_scale) : 1.0f) * rn;
  float* o = dx + (int64_t)row * D;
  for (int d = lane; d < D; d += 64) o[d] = sc * (gr[d] - xr[d] * rn * dot);
}

// nn.MSELoss() (mean): loss = sum((p - t)^2) / n, one workgroup
__global__ __launch_bounds__(1024) void mse_fwd_kernel(const float* __restrict__ p, const float* __restrict__ t, int n,
                                                       float* __restrict__ loss) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float d = p[i] - t[i];
    s = fmaf(d, d, s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int w = 0; w < 16; ++w) a += red[w];
    *loss = a / (float)n;
  }
}

// dp = 2 (p - t) / n * g
__global__ __launch_bounds__(256) void mse_bwd_kernel(const float* __restrict__ p, const float* __restrict__ t,
                                                      const float* __restrict__ g, int n, float* __restrict__ dp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float gs = g ? *g : 1.0f;
  dp[i] = 2.0f * (p[i] - t[i]) / (float)n * gs;
}

extern "C" {

int vit_token_embed(int rows, int L, int D, int vocab, const int64_t* tokens, const float* table, const float* pos,
                    float* x, void* stream) {
  if (rows <= 0) return 0;
  if (D % 4 || L <= 0 || vocab <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(token_embed_kernel, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, tokens, table, pos, x,
                     rows, L, D, vocab);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_gather_rows(int n, int D, const float* src, int64_t ld_src, const int64_t* idx, float* dst, int64_t ld_dst,
                    void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rows_kernel<0>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src, ld_src, idx, dst, ld_dst,
                     n, D);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_scatter_rows(int n, int D, const float* src, int64_t ld_src, const int64_t* idx, float* dst, int64_t ld_dst,
                     void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rows_kernel<1>, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, src, ld_src, idx, dst, ld_dst,
                     n, D);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_rownorm_fwd(int n, int D, const float* x, const float* log_scale, float* y, float* rnorm, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rownorm_fwd_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, log_scale, y, rnorm, n,
                     D);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_rownorm_bwd(int n, int D, const float* x, const float* dy, const float* rnorm, const float* log_scale,
                    float* dx, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(rownorm_bwd_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, x, dy, rnorm, log_scale,
                     dx, n, D);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_mse_fwd(int n, const float* pred, const float* target, float* loss, void* stream) {
  if (n <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mse_fwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, pred, target, n, loss);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_mse_bwd(int n, const float* pred, const float* target, const float* grad_loss, float* dpred, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mse_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, pred, target, grad_loss, n,
                     dpred);
  VIT_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
