// Byte/element-wise kernels around the ViT step: patch unfold (Conv2d 16/16 as
// GEMM operand), cls/pos fill and their grads, fused softmax-cross-entropy,
// multi-tensor SGD (torch.optim.SGD semantics) with a bf16 shadow write, casts.
#include "common.hpp"
#include <type_traits>

// ---------------------------------------------------------------------------
// patch unfold: img f32 [B, C, Himg, Wimg] -> U [B*gh*gw, C*ps*ps] (T),
// column = c*ps*ps + ky*ps + kx (Conv2d weight [D, C, ps, ps] flattening).
// One thread per (b, c, py, ky, px) image-row segment of ps pixels.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void patch_unfold_kernel(const float* __restrict__ img, T* __restrict__ U, int B, int C, int Hi, int Wi,
                                    int ps, int ldu) {
  const int gh = Hi / ps, gw = Wi / ps;
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)B * C * gh * ps * gw;
  if (idx >= total) return;
  int px = idx % gw; int64_t t = idx / gw;
  int ky = t % ps; t /= ps;
  int py = t % gh; t /= gh;
  int c = t % C; int b = (int)(t / C);
  const float* src = img + (((int64_t)b * C + c) * Hi + py * ps + ky) * Wi + px * ps;
  const int K = C * ps * ps;
  T* urow = U + ((int64_t)b * gh * gw + py * gw + px) * ldu;
  T* dst = urow + c * ps * ps + ky * ps;
  if (c == 0 && ky == 0)  // the row's padding columns [K, ldu) (a GEMM reduction padded to its tile depth)
    for (int k = K; k < ldu; ++k) urow[k] = (T)0.f;
  if constexpr (std::is_same<T, bf16>::value) {
    if (ps == 16 && (ldu % 8) == 0 && ((uintptr_t)U & 15) == 0 && (Wi % 4) == 0 && ((uintptr_t)img & 15) == 0) {
      // one 64-B row segment in, two 16-B stores out (consecutive threads: consecutive patches)
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4*>(src + 4 * u);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = v[2 * h], b = v[2 * h + 1];
        *reinterpret_cast<bf16x8*>(dst + 8 * h) =
            bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
      }
      return;
    }
  }
  if (ps % 4 == 0) {
    for (int kx = 0; kx < ps; kx += 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(src + kx);
      for (int u = 0; u < 4; ++u) dst[kx + u] = (T)v[u];
    }
  } else {
    for (int kx = 0; kx < ps; ++kx) dst[kx] = (T)src[kx];
  }
}

template <typename T>
__global__ void copy_rows_pad_kernel(const T* __restrict__ src, int64_t lds, T* __restrict__ dst, int64_t ldd,
                                     int cols, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t r = i / ldd, c = i - r * ldd;
  dst[i] = c < cols ? src[r * lds + c] : (T)0.f;
}

// x[b*S + 0][j] = cls[j] + pos[0][j]
__global__ void cls_pos_fill_kernel(float* __restrict__ x, const float* __restrict__ cls, const float* __restrict__ pos,
                                    int B, int S, int D) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * D) return;
  int b = idx / D, j = idx - b * D;
  x[(int64_t)b * S * D + j] = cls[j] + pos[j];
}

// dpos[t][j] = sum_b dx[b*S + t][j]; dcls[j] = dpos[0][j]
// Vector path (S*D % 4 == 0): a workgroup owns 256 consecutive floats of the flattened
// [S*D] (one f32x4 per lane); its POS_WAVES waves take interleaved images with four
// independent accumulators each and combine through LDS in a fixed order (deterministic).
constexpr int POS_WAVES = 8;
__global__ __launch_bounds__(64 * POS_WAVES) void pos_grad_vec_kernel(const float* __restrict__ dx, int B, int64_t n,
                                                                      float* __restrict__ dpos,
                                                                      float* __restrict__ dcls, int D) {
  __shared__ f32x4 red[POS_WAVES][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const bool ok = c < n;
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (ok) {
    int b = wv;
    for (; b + 3 * POS_WAVES < B; b += 4 * POS_WAVES) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += *reinterpret_cast<const f32x4*>(dx + (int64_t)(b + u * POS_WAVES) * n + c);
    }
    for (; b < B; b += POS_WAVES) acc[0] += *reinterpret_cast<const f32x4*>(dx + (int64_t)b * n + c);
  }
  red[wv][lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (wv == 0 && ok) {
    f32x4 s = red[0][lane];
#pragma unroll
    for (int w = 1; w < POS_WAVES; ++w) s += red[w][lane];
    *reinterpret_cast<f32x4*>(dpos + c) = s;
    if (dcls && c < D) *reinterpret_cast<f32x4*>(dcls + c) = s;
  }
}
__global__ void pos_grad_kernel(const float* __restrict__ dx, int B, int S, int D, float* __restrict__ dpos,
                                float* __restrict__ dcls) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)S * D) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += dx[(int64_t)b * S * D + idx];
  dpos[idx] = s;
  if (idx < D && dcls) dcls[idx] = s;
}

// ---------------------------------------------------------------------------
// cross entropy (F.cross_entropy, mean reduction; VIT:140)
// ---------------------------------------------------------------------------
__global__ void ce_fwd_kernel(const float* __restrict__ logits, int64_t ld, const int64_t* __restrict__ target,
                              int B, int C, float* __restrict__ row_lse, float* __restrict__ row_loss) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const float* x = logits + (int64_t)row * ld;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, x[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(x[c] - m);
  s = wave_sum(s);
  if (lane == 0) {
    float l = m + logf(s);
    row_lse[row] = l;
    row_loss[row] = l - x[target[row]];
  }
}

__global__ void mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = ((red[0] + red[1]) + (red[2] + red[3])) / (float)n;
}

template <typename TO>
__global__ void ce_bwd_kernel(const float* __restrict__ logits, int64_t ld, const int64_t* __restrict__ target,
                              const float* __restrict__ row_lse, const float* __restrict__ gscale, int B, int C,
                              TO* __restrict__ dlogits, int64_t ldd) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * C) return;
  int row = idx / C, c = idx - (int64_t)row * C;
  float g = (gscale ? *gscale : 1.0f) / (float)B;
  float p = __expf(logits[(int64_t)row * ld + c] - row_lse[row]);
  if (c == target[row]) p -= 1.0f;
  dlogits[(int64_t)row * ldd + c] = (TO)(p * g);
}

// ---------------------------------------------------------------------------
// multi-tensor SGD: torch.optim.SGD(lr, momentum, weight_decay), dampening 0,
// nesterov off (VIT:294-299).  Momentum buffers start at zero, which makes
// buf = m*0 + d identical to torch's first-step clone.  Writes the bf16 shadow
// copy used by the GEMMs in the same pass.
// ---------------------------------------------------------------------------
struct SgdTensor { float* p; const float* g; float* buf; bf16* shadow; int64_t n; };
struct SgdChunk { int tensor; int pad; int64_t start; };
constexpr int SGD_CHUNK = 4096;

__global__ __launch_bounds__(256) void sgd_kernel(const SgdTensor* __restrict__ ts, const SgdChunk* __restrict__ chunks,
                                                  const float* __restrict__ lr_ptr, float momentum, float wd) {
  const SgdChunk ch = chunks[blockIdx.x];
  const SgdTensor t = ts[ch.tensor];
  const float lr = *lr_ptr;
  const int64_t end = min(t.n, ch.start + SGD_CHUNK);
  const bool vec = ((((uintptr_t)t.p) | ((uintptr_t)t.g) | ((uintptr_t)t.buf)) & 15) == 0 &&
                   (!t.shadow || (((uintptr_t)t.shadow) & 7) == 0) && (ch.start % 4 == 0);
  if (vec) {
    for (int64_t i = ch.start + threadIdx.x * 4; i + 4 <= end; i += 256 * 4) {
      f32x4 p = *reinterpret_cast<const f32x4*>(t.p + i);
      f32x4 g = *reinterpret_cast<const f32x4*>(t.g + i);
      f32x4 b = *reinterpret_cast<const f32x4*>(t.buf + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float d = __fadd_rn(g[u], __fmul_rn(wd, p[u]));
        b[u] = __fadd_rn(__fmul_rn(b[u], momentum), d);
        p[u] = __fsub_rn(p[u], __fmul_rn(lr, b[u]));
      }
      *reinterpret_cast<f32x4*>(t.p + i) = p;
      *reinterpret_cast<f32x4*>(t.buf + i) = b;
      if (t.shadow) *reinterpret_cast<bf16x4*>(t.shadow + i) = bf16x4{(bf16)p[0], (bf16)p[1], (bf16)p[2], (bf16)p[3]};
    }
    // tail (n not multiple of 4)
    int64_t tail = ch.start + ((end - ch.start) / 4) * 4;
    for (int64_t i = tail + threadIdx.x; i < end; i += 256) {
      float d = __fadd_rn(t.g[i], __fmul_rn(wd, t.p[i]));
      float b = __fadd_rn(__fmul_rn(t.buf[i], momentum), d);
      float p = __fsub_rn(t.p[i], __fmul_rn(lr, b));
      t.buf[i] = b; t.p[i] = p;
      if (t.shadow) t.shadow[i] = (bf16)p;
    }
  } else {
    for (int64_t i = ch.start + threadIdx.x; i < end; i += 256) {
      float d = __fadd_rn(t.g[i], __fmul_rn(wd, t.p[i]));
      float b = __fadd_rn(__fmul_rn(t.buf[i], momentum), d);
      float p = __fsub_rn(t.p[i], __fmul_rn(lr, b));
      t.buf[i] = b; t.p[i] = p;
      if (t.shadow) t.shadow[i] = (bf16)p;
    }
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, int64_t n) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
    *reinterpret_cast<bf16x4*>(y + i) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  } else {
    for (; i < n; ++i) y[i] = (bf16)x[i];
  }
}

extern "C" {

int vit_patch_unfold_ld(int dtype, int B, int C, int Hi, int Wi, int ps, int ldu, const float* img, void* U,
                        void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (Hi % ps || Wi % ps || ldu < C * ps * ps) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)B * C * (Hi / ps) * ps * (Wi / ps);
  dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == VIT_BF16)
    hipLaunchKernelGGL(patch_unfold_kernel<bf16>, grid, dim3(256), 0, s, img, (bf16*)U, B, C, Hi, Wi, ps, ldu);
  else
    hipLaunchKernelGGL(patch_unfold_kernel<float>, grid, dim3(256), 0, s, img, (float*)U, B, C, Hi, Wi, ps, ldu);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_patch_unfold(int dtype, int B, int C, int Hi, int Wi, int ps, const float* img, void* U, void* stream) {
  return vit_patch_unfold_ld(dtype, B, C, Hi, Wi, ps, C * ps * ps, img, U, stream);
}

// dst[r][c] = src[r][c] for c < cols, 0 for cols <= c < ld_dst (a weight matrix padded along its
// reduction dimension to the GEMM tile depth)
int vit_copy_rows_padded(int dtype, int rows, int cols, const void* src, int64_t ld_src, void* dst, int64_t ld_dst,
                         void* stream) {
  if (rows < 0 || cols < 0 || ld_src < cols || ld_dst < cols) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)rows * ld_dst;
  if (total == 0) return 0;
  dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VIT_BF16)
    hipLaunchKernelGGL(copy_rows_pad_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)src, ld_src, (bf16*)dst, ld_dst,
                       cols, total);
  else
    hipLaunchKernelGGL(copy_rows_pad_kernel<float>, grid, dim3(256), 0, s, (const float*)src, ld_src, (float*)dst,
                       ld_dst, cols, total);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_cls_pos_fill(int B, int S, int D, float* x, const float* cls, const float* pos, void* stream) {
  hipLaunchKernelGGL(cls_pos_fill_kernel, dim3((B * D + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, cls, pos, B, S, D);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_pos_grad(int B, int S, int D, const float* dx, float* dpos, float* dcls, void* stream) {
  int64_t n = (int64_t)S * D;
  if (n % 4 == 0 && D % 4 == 0 && ((uintptr_t)dx & 15) == 0 && ((uintptr_t)dpos & 15) == 0 &&
      ((uintptr_t)dcls & 15) == 0) {
    hipLaunchKernelGGL(pos_grad_vec_kernel, dim3((unsigned)((n + 255) / 256)), dim3(64 * POS_WAVES), 0,
                       (hipStream_t)stream, dx, B, n, dpos, dcls, D);
    VIT_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(pos_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dx, B, S, D, dpos, dcls);
  VIT_CHECK_LAUNCH();
  return 0;
}

// loss (1 float) = mean_i CE(logits_i, target_i); row_lse/row_loss: scratch [B] each.
int vit_cross_entropy_fwd(int B, int C, const float* logits, int64_t ld, const int64_t* target, float* row_lse,
                          float* row_loss, float* loss, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, s, logits, ld, target, B, C, row_lse, row_loss);
  VIT_CHECK_LAUNCH();
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(256), 0, s, row_loss, B, loss);
  VIT_CHECK_LAUNCH();
  return 0;
}

// dlogits = (softmax(logits) - onehot(target)) * (*grad_loss) / B
int vit_cross_entropy_bwd(int dtype_out, int B, int C, const float* logits, int64_t ld, const int64_t* target,
                          const float* row_lse, const float* grad_loss, void* dlogits, int64_t ldd, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int64_t n = (int64_t)B * C;
  dim3 grid((unsigned)((n + 255) / 256));
  if (dtype_out == VIT_BF16)
    hipLaunchKernelGGL(ce_bwd_kernel<bf16>, grid, dim3(256), 0, s, logits, ld, target, row_lse, grad_loss, B, C, (bf16*)dlogits, ldd);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<float>, grid, dim3(256), 0, s, logits, ld, target, row_lse, grad_loss, B, C, (float*)dlogits, ldd);
  VIT_CHECK_LAUNCH();
  return 0;
}

// One fused SGD step over a table of tensors.  `tensors` / `chunks` are device
// arrays of SgdTensor {p, g, buf, shadow, n} / SgdChunk {tensor, pad, start}
// (chunk = 4096 elements), built once by the host; `lr` is a device scalar so a
// captured graph follows the schedule.
int vit_sgd_step(const void* tensors, const void* chunks, int nchunks, const float* lr, float momentum,
                 float weight_decay, void* stream) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(sgd_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, (const SgdTensor*)tensors,
                     (const SgdChunk*)chunks, lr, momentum, weight_decay);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_sgd_chunk_size(void) { return SGD_CHUNK; }
int vit_sgd_tensor_bytes(void) { return (int)sizeof(SgdTensor); }
int vit_sgd_chunk_bytes(void) { return (int)sizeof(SgdChunk); }

int vit_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
  int64_t threads = (n + 3) / 4;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, (bf16*)y, n);
  VIT_CHECK_LAUNCH();
  return 0;
}

int vit_zero(void* p, int64_t bytes, void* stream) {
  return (int)hipMemsetAsync(p, 0, (size_t)bytes, (hipStream_t)stream);
}

int vit_abi_version(void) { return 10; }

}  // extern "C"
