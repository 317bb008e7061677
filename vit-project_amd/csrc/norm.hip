// LayerNorm over the last dim (timm norm1/norm2/norm, eps 1e-6; CLIP eps 1e-5).
// One wave per row.  Forward: biased variance, two-pass in registers, saves
// mean/rstd.  Backward: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma,
// plus a fused residual-gradient add and an optional typed copy of dx (the next
// GEMM operand, optionally with the CLS rows dropped); dgamma/dbeta via
// per-block partials + a final reduce.
//
// NV = float4 groups per lane (D = 256*NV: 3 for ViT-B's 768, 4 for 1024); a
// scalar kernel (NV = 0) covers any other D (test configs).
#include "common.hpp"
#include "reduce.hpp"
#include <stdlib.h>
#include <type_traits>

constexpr int LN_WAVES = 4;   // rows per block in the forward (one per wave)
constexpr int LN_SMAX = 32;   // scalar path: D <= 64*32
// rows per backward block (one partial row each); VIT_LN_BWD_ROWS overrides (tuning)
static int ln_bwd_rows() {
  static int r = 0;
  if (r <= 0) {
    const char* s = getenv("VIT_LN_BWD_ROWS");
    r = s ? atoi(s) : 32;
    if (r < 4) r = 32;
  }
  return r;
}

template <typename T> __device__ __forceinline__ f32x4 ld4(const T* p);
template <> __device__ __forceinline__ f32x4 ld4<float>(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
template <> __device__ __forceinline__ f32x4 ld4<bf16>(const bf16* p) {
  bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
}
template <typename T> __device__ __forceinline__ void st4(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
template <> __device__ __forceinline__ void st4<bf16>(bf16* p, f32x4 v) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// first column of float4 group k of this lane
__device__ __forceinline__ int col4(int lane, int k) { return (k * 64 + lane) * 4; }

template <int NV, typename TX, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const TX* __restrict__ x, int64_t ldx, TY* __restrict__ y,
                                                     int64_t ldy, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TX* xr = x + (int64_t)row * ldx;
  TY* yr = y + (int64_t)row * ldy;
  if constexpr (NV > 0) {
    f32x4 v[NV];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) { v[k] = ld4<TX>(xr + col4(lane, k)); s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]); }
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int t = 0; t < 4; ++t) { float d = v[k][t] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int c = col4(lane, k);
      f32x4 g = *reinterpret_cast<const f32x4*>(w + c), bb = *reinterpret_cast<const f32x4*>(b + c), o;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (v[k][t] - mu) * rs * g[t] + bb[t];
      st4<TY>(yr + c, o);
    }
    if (lane == 0) { if (mean) mean[row] = mu; if (rstd) rstd[row] = rs; }
  } else {
    float s = 0.f;
    for (int c = lane; c < D; c += 64) s += (float)xr[c];
    const float mu = wave_sum(s) / D;
    float q = 0.f;
    for (int c = lane; c < D; c += 64) { float d = (float)xr[c] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
    for (int c = lane; c < D; c += 64) yr[c] = (TY)(((float)xr[c] - mu) * rs * w[c] + b[c]);
    if (lane == 0) { if (mean) mean[row] = mu; if (rstd) rstd[row] = rs; }
  }
}

// Residual add + LayerNorm forward (bf16 step): s = x + r with x the f32 residual
// stream and r a Linear's bf16 output (bias included) -- the Linear's f32 output under autocast
// rounded to bf16, then added in f32 as timm's `x + attn(...)` / `x + mlp(...)` does -- written to
// xs (f32, may alias x), and y = LN(s) (bf16, optional: y == null writes only the sum).  One wave per
// row; the Linear's epilogue then stores 2 bytes per element instead of reading and writing the
// f32 stream (4 + 4), and that traffic moves into this streaming kernel.
template <int NV, typename TR, typename TY>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const TR* __restrict__ r, int64_t ldr,
                                                         float* __restrict__ xs, int64_t ldxs, TY* __restrict__ y,
                                                         int64_t ldy, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ mean,
                                                         float* __restrict__ rstd, int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ldx;
  const TR* rr = r + (int64_t)row * ldr;
  float* sr = xs + (int64_t)row * ldxs;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = col4(lane, k);
    v[k] = ld4<float>(xr + c) + ld4<TR>(rr + c);
    s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) st4<float>(sr + col4(lane, k), v[k]);
  if (y == nullptr) return;
  const float mu = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int t = 0; t < 4; ++t) { float d = v[k][t] - mu; q += d * d; }
  const float rs = rsqrtf(wave_sum(q) / D + eps);
  TY* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = col4(lane, k);
    f32x4 g = *reinterpret_cast<const f32x4*>(w + c), bb = *reinterpret_cast<const f32x4*>(b + c), o;
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (v[k][t] - mu) * rs * g[t] + bb[t];
    st4<TY>(yr + c, o);
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

__device__ __forceinline__ bool copy_row(int row, int compact_np, int64_t& orow) {
  orow = row;
  if (compact_np > 0) {
    int bb = row / (compact_np + 1), p = row - bb * (compact_np + 1);
    orow = (int64_t)bb * compact_np + p - 1;
    return p != 0;
  }
  return true;
}

// Backward: block = 4 waves over rows [blk*rows_per, ...), wave-strided.
template <int NV, typename TX, typename TD, typename TC>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const TX* __restrict__ x, int64_t ldx, const TD* __restrict__ dy, int64_t lddy,
    const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ dres, int64_t ldres, float* __restrict__ dx, int64_t lddx,
    TC* __restrict__ dxc, int64_t ldc, int compact_np, float* __restrict__ part_g,
    float* __restrict__ part_b, float* __restrict__ part_s, int rows, int D, int rows_per) {
  constexpr int NP = NV > 0 ? NV * 4 : LN_SMAX;  // partial slots per lane
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pg[NP], pb[NP], ps[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t) { pg[t] = 0.f; pb[t] = 0.f; ps[t] = 0.f; }
  __shared__ float red[LN_WAVES][192];
  const int r0 = blockIdx.x * rows_per, r1 = min(rows, r0 + rows_per);
  for (int row = r0 + wv; row < r1; row += LN_WAVES) {
    const TX* xr = x + (int64_t)row * ldx;
    const TD* dyr = dy + (int64_t)row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float* dxr = dx + (int64_t)row * lddx;
    int64_t orow = row;
    const bool keep = (dxc != nullptr) && copy_row(row, compact_np, orow);
    if constexpr (NV > 0) {
      f32x4 xh[NV], g[NV], rv[NV];
      float s1 = 0.f, s2 = 0.f;
      // the residual gradient is loaded with x and dy, so a row costs one memory round trip
      if (dres) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
          rv[k] = *reinterpret_cast<const f32x4*>(dres + (int64_t)row * ldres + col4(lane, k));
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        int c = col4(lane, k);
        f32x4 xv = ld4<TX>(xr + c), dv = ld4<TD>(dyr + c), wv4 = *reinterpret_cast<const f32x4*>(w + c);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          xh[k][t] = (xv[t] - mu) * rs;
          g[k][t] = dv[t] * wv4[t];
          s1 += g[k][t];
          s2 += g[k][t] * xh[k][t];
          pg[k * 4 + t] += dv[t] * xh[k][t];
          pb[k * 4 + t] += dv[t];
        }
      }
      s1 = wave_sum(s1) / D;
      s2 = wave_sum(s2) / D;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        int c = col4(lane, k);
        f32x4 o;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] = rs * (g[k][t] - s1 - xh[k][t] * s2);
        if (dres) o += rv[k];
#pragma unroll
        for (int t = 0; t < 4; ++t) ps[k * 4 + t] += o[t];
        *reinterpret_cast<f32x4*>(dxr + c) = o;
        if (keep) st4<TC>(dxc + orow * ldc + c, o);
      }
    } else {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < LN_SMAX; ++k) {
        int c = lane + 64 * k;
        if (c < D) {
          float xh = ((float)xr[c] - mu) * rs, dv = (float)dyr[c], g = dv * w[c];
          s1 += g; s2 += g * xh;
          pg[k] += dv * xh; pb[k] += dv;
        }
      }
      s1 = wave_sum(s1) / D;
      s2 = wave_sum(s2) / D;
#pragma unroll
      for (int k = 0; k < LN_SMAX; ++k) {
        const int c = lane + 64 * k;
        if (c >= D) break;
        float xh = ((float)xr[c] - mu) * rs, g = (float)dyr[c] * w[c];
        float o = rs * (g - s1 - xh * s2);
        if (dres) o += dres[(int64_t)row * ldres + c];
        ps[k] += o;
        dxr[c] = o;
        if (keep) dxc[orow * ldc + c] = (TC)o;
      }
    }
  }
  if (!part_g && !part_s) return;
  if constexpr (NV > 0) {
    // per-block partials of dgamma / dbeta / dsum: one LDS round (one barrier pair) per
    // quantity, the four waves each summing a quarter of the slots
    __shared__ float redv[LN_WAVES][NP][64];
    auto flush = [&](const float (&p)[NP], float* out) {
#pragma unroll
      for (int k = 0; k < NP; ++k) redv[wv][k][lane] = p[k];
      __syncthreads();
#pragma unroll
      for (int k = wv; k < NP; k += LN_WAVES) {
        const float v = (redv[0][k][lane] + redv[1][k][lane]) + (redv[2][k][lane] + redv[3][k][lane]);
        out[(int64_t)blockIdx.x * D + col4(lane, k >> 2) + (k & 3)] = v;
      }
      __syncthreads();
    };
    if (part_g) {
      flush(pg, part_g);
      flush(pb, part_b);
    }
    if (part_s) flush(ps, part_s);
    return;
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int c = NV > 0 ? col4(lane, k >> 2) + (k & 3) : k * 64 + lane;
    if (NV == 0 && k * 64 >= D) break;  // uniform across the block
    red[wv][lane] = pg[k];
    red[wv][64 + lane] = pb[k];
    red[wv][128 + lane] = ps[k];
    __syncthreads();
    if (wv == 0 && c < D) {
      const int64_t o = (int64_t)blockIdx.x * D + c;
      if (part_g) {
        part_g[o] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        part_b[o] = (red[0][64 + lane] + red[1][64 + lane]) + (red[2][64 + lane] + red[3][64 + lane]);
      }
      if (part_s) part_s[o] = (red[0][128 + lane] + red[1][128 + lane]) + (red[2][128 + lane] + red[3][128 + lane]);
    }
    __syncthreads();
  }
}


// Backward, vector form (D = 256 * NV), software-pipelined: a wave issues row r+4's loads (x, dy,
// the residual gradient, mean / rstd) before row r's arithmetic and stores, so the loads overlap
// the previous row's stores instead of queueing behind them (vmcnt counts loads and stores in
// order: the plain loop paid a load and a store latency per row, 8 us per row at the step shape,
// 4.5 TB/s).  gamma is loaded once per wave.  Same arithmetic, in the same order, as
// ln_bwd_kernel (the compiler's FMA contraction may differ: equal to rounding).
template <int NV, typename TX, typename TD> struct LnRow {
  f32x4 x[NV], r[NV];
  typename std::conditional<std::is_same<TD, float>::value, f32x4, bf16x4>::type d[NV];
  float mu, rs;
};

template <int NV, typename TX, typename TD, typename TC>
__global__ __launch_bounds__(256) void ln_bwd_pipe_kernel(
    const TX* __restrict__ x, int64_t ldx, const TD* __restrict__ dy, int64_t lddy,
    const float* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ dres, int64_t ldres, float* __restrict__ dx, int64_t lddx,
    TC* __restrict__ dxc, int64_t ldc, int compact_np, float* __restrict__ part_g,
    float* __restrict__ part_b, float* __restrict__ part_s, int rows, int D, int rows_per) {
  constexpr int NP = NV * 4;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float pg[NP], pb[NP], ps[NP];
#pragma unroll
  for (int t = 0; t < NP; ++t) { pg[t] = 0.f; pb[t] = 0.f; ps[t] = 0.f; }
  f32x4 wg[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) wg[k] = *reinterpret_cast<const f32x4*>(w + col4(lane, k));
  const int r0 = blockIdx.x * rows_per, r1 = min(rows, r0 + rows_per);
  using Row = LnRow<NV, TX, TD>;
  auto load = [&](int row, Row& R) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = col4(lane, k);
      R.x[k] = ld4<TX>(x + (int64_t)row * ldx + c);
      if constexpr (std::is_same<TD, float>::value) R.d[k] = *reinterpret_cast<const f32x4*>(dy + (int64_t)row * lddy + c);
      else R.d[k] = *reinterpret_cast<const bf16x4*>(dy + (int64_t)row * lddy + c);
      R.r[k] = dres ? *reinterpret_cast<const f32x4*>(dres + (int64_t)row * ldres + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    R.mu = mean[row];
    R.rs = rstd[row];
  };
  auto process = [&](int row, const Row& R) {
    const float mu = R.mu, rs = R.rs;
    f32x4 xh[NV], g[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      f32x4 dv;
      if constexpr (std::is_same<TD, float>::value) dv = R.d[k];
      else dv = f32x4{(float)R.d[k][0], (float)R.d[k][1], (float)R.d[k][2], (float)R.d[k][3]};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xh[k][t] = (R.x[k][t] - mu) * rs;
        g[k][t] = dv[t] * wg[k][t];
        s1 += g[k][t];
        s2 += g[k][t] * xh[k][t];
        pg[k * 4 + t] += dv[t] * xh[k][t];
        pb[k * 4 + t] += dv[t];
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
    int64_t orow = row;
    const bool keep = (dxc != nullptr) && copy_row(row, compact_np, orow);
    float* dxr = dx + (int64_t)row * lddx;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = col4(lane, k);
      f32x4 o;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = rs * (g[k][t] - s1 - xh[k][t] * s2);
      if (dres) o += R.r[k];
#pragma unroll
      for (int t = 0; t < 4; ++t) ps[k * 4 + t] += o[t];
      *reinterpret_cast<f32x4*>(dxr + c) = o;
      if (keep) st4<TC>(dxc + orow * ldc + c, o);
    }
  };
  // two row buffers, alternated by a 2x unrolled loop (no register copies)
  Row A, B;
  int row = r0 + wv;
  if (row < r1) load(row, A);
  while (row < r1) {
    if (row + LN_WAVES < r1) load(row + LN_WAVES, B);
    process(row, A);
    row += LN_WAVES;
    if (row >= r1) break;
    if (row + LN_WAVES < r1) load(row + LN_WAVES, A);
    process(row, B);
    row += LN_WAVES;
  }
  if (!part_g && !part_s) return;
  __shared__ float redv[LN_WAVES][NP][64];
  auto flush = [&](const float (&p)[NP], float* out) {
#pragma unroll
    for (int k = 0; k < NP; ++k) redv[wv][k][lane] = p[k];
    __syncthreads();
#pragma unroll
    for (int k = wv; k < NP; k += LN_WAVES) {
      const float v = (redv[0][k][lane] + redv[1][k][lane]) + (redv[2][k][lane] + redv[3][k][lane]);
      out[(int64_t)blockIdx.x * D + col4(lane, k >> 2) + (k & 3)] = v;
    }
    __syncthreads();
  };
  if (part_g) {
    flush(pg, part_g);
    flush(pb, part_b);
  }
  if (part_s) flush(ps, part_s);
}


template <typename TX, typename TY>
static void launch_fwd(int nv, dim3 grid, hipStream_t s, const void* x, int64_t ldx, void* y, int64_t ldy,
                       const float* w, const float* b, float* mean, float* rstd, int rows, int D, float eps) {
#define F(NV) hipLaunchKernelGGL((ln_fwd_kernel<NV, TX, TY>), grid, dim3(64 * LN_WAVES), 0, s, (const TX*)x, ldx, (TY*)y, ldy, w, b, mean, rstd, rows, D, eps)
  switch (nv) {
    case 1: F(1); break;
    case 2: F(2); break;
    case 3: F(3); break;
    case 4: F(4); break;
    case 6: F(6); break;
    case 8: F(8); break;
    default: F(0); break;
  }
#undef F
}

static int g_ln_pipe = -1;  // VIT_LN_BWD_PIPE / vit_layer_norm_bwd_variant: 1 pipelined (default), 0 plain loop

template <typename TX, typename TD, typename TC>
static void launch_bwd(int nv, int nblk, hipStream_t s, const void* x, int64_t ldx, const void* dy, int64_t lddy,
                       const float* w, const float* mean, const float* rstd, const float* dres, int64_t ldres,
                       float* dx, int64_t lddx, void* dxc, int64_t ldc, int compact_np, float* pg, float* pb,
                       float* ps, int rows, int D, int rows_per) {
#define B(K, NV) hipLaunchKernelGGL((K<NV, TX, TD, TC>), dim3(nblk), dim3(64 * LN_WAVES), 0, s, (const TX*)x, ldx, \
                                 (const TD*)dy, lddy, w, mean, rstd, dres, ldres, dx, lddx, (TC*)dxc, ldc, compact_np, pg, pb, ps, rows, D, rows_per)
  if (g_ln_pipe < 0) { const char* v = getenv("VIT_LN_BWD_PIPE"); g_ln_pipe = v ? atoi(v) : 1; }
  const int pipe = g_ln_pipe;
  switch (nv) {
    case 3: if (pipe) B(ln_bwd_pipe_kernel, 3); else B(ln_bwd_kernel, 3); break;
    case 4: if (pipe) B(ln_bwd_pipe_kernel, 4); else B(ln_bwd_kernel, 4); break;
    default: B(ln_bwd_kernel, 0); break;
  }
#undef B
}

extern "C" {

// F.layer_norm forward over rows of x (row stride ldx; f32 or bf16 in) -> y (dtype_y).
int vit_layer_norm_fwd(int dtype_x, int dtype_y, int rows, int D, const void* x, int64_t ldx, void* y,
                       int64_t ldy, const float* w, const float* b, float* mean, float* rstd, float eps,
                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (rows <= 0) return 0;
  if (D > 64 * LN_SMAX) return (int)hipErrorInvalidValue;
  dim3 grid((rows + LN_WAVES - 1) / LN_WAVES);
  bool vec = (D % 256 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0);
  int nv = vec ? D / 256 : 0;
  if (dtype_x == VIT_F32 && dtype_y == VIT_F32) launch_fwd<float, float>(nv, grid, s, x, ldx, y, ldy, w, b, mean, rstd, rows, D, eps);
  else if (dtype_x == VIT_F32) launch_fwd<float, bf16>(nv, grid, s, x, ldx, y, ldy, w, b, mean, rstd, rows, D, eps);
  else if (dtype_y == VIT_BF16) launch_fwd<bf16, bf16>(nv, grid, s, x, ldx, y, ldy, w, b, mean, rstd, rows, D, eps);
  else launch_fwd<bf16, float>(nv, grid, s, x, ldx, y, ldy, w, b, mean, rstd, rows, D, eps);
  VIT_CHECK_LAUNCH();
  return 0;
}

// xs = x + r (f32 + bf16 / f32 -> f32; xs may alias x) and, when y is non-null, y = LayerNorm(xs) (bf16 / f32)
// with its mean / rstd: the residual add of a Linear's bf16 output fused into the LayerNorm that
// follows it.  D must be a multiple of 256 (ViT-B 768, ViT-L 1024) and every stride of 4 elements.
int vit_add_layer_norm_fwd(int dtype_r, int dtype_y, int rows, int D, const float* x, int64_t ldx, const void* r,
                           int64_t ldr, float* xs, int64_t ldxs, void* y, int64_t ldy, const float* w, const float* b,
                           float* mean, float* rstd, float eps, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (rows <= 0) return 0;
  if (D % 256 || D > 2048 || (ldx | ldr | ldxs | ldy) % 4) return (int)hipErrorInvalidValue;
  if (y && (!w || !b || !mean || !rstd)) return (int)hipErrorInvalidValue;
  dim3 grid((rows + LN_WAVES - 1) / LN_WAVES);
  if ((dtype_r != VIT_BF16 && dtype_r != VIT_F32) || (dtype_y != VIT_BF16 && dtype_y != VIT_F32))
    return (int)hipErrorInvalidValue;
#define A(NV, TR, TY)                                                                                          \
  hipLaunchKernelGGL((add_ln_fwd_kernel<NV, TR, TY>), grid, dim3(64 * LN_WAVES), 0, s, x, ldx, (const TR*)r, ldr, xs, \
                     ldxs, (TY*)y, ldy, w, b, mean, rstd, rows, D, eps)
#define AD(NV)                                                         \
  if (dtype_r == VIT_BF16 && dtype_y == VIT_BF16) A(NV, bf16, bf16);   \
  else if (dtype_r == VIT_BF16) A(NV, bf16, float);                    \
  else if (dtype_y == VIT_BF16) A(NV, float, bf16);                    \
  else A(NV, float, float);
  switch (D / 256) {
    case 1: AD(1) break;
    case 2: AD(2) break;
    case 3: AD(3) break;
    case 4: AD(4) break;
    case 5: AD(5) break;
    case 6: AD(6) break;
    case 7: AD(7) break;
    case 8: AD(8) break;
    default: return (int)hipErrorInvalidValue;
  }
#undef AD
#undef A
  VIT_CHECK_LAUNCH();
  return 0;
}

// LayerNorm backward.  dx (f32) = dres + LN'(dy).  dx_copy (optional, dtype_copy,
// row stride ld_copy) is the GEMM-operand copy of dx; compact_np > 0 drops the
// CLS row of every (compact_np+1)-row image (patch-embed wgrad operand).
// dgamma/dbeta and dsum = column sums of dx (the bias gradient of the Linear that
// produced the LayerNorm's residual input) may each be null; `partial` must hold
// vit_layer_norm_bwd_partial_floats(rows, D) floats when any of them is requested.
// Tuning hook: 1 = the software-pipelined vector backward (default), 0 = the plain row loop.
int vit_layer_norm_bwd_variant(int v) { g_ln_pipe = v; return 0; }

int vit_layer_norm_bwd_blocks(int rows) { return (rows + ln_bwd_rows() - 1) / ln_bwd_rows(); }

int vit_layer_norm_bwd_partial_floats(int rows, int D) {
  const int nblk = vit_layer_norm_bwd_blocks(rows);
  return (int)(3 * (int64_t)nblk * D + 3 * colreduce_scratch_floats(nblk, D));
}

int vit_layer_norm_bwd(int dtype_x, int dtype_dy, int rows, int D, const void* x, int64_t ldx,
                       const void* dy, int64_t lddy, const float* w, const float* mean, const float* rstd,
                       const float* dres, int64_t ldres, float* dx, int64_t lddx, void* dx_copy, int64_t ld_copy,
                       int dtype_copy, int compact_np, float* dgamma, float* dbeta, float* dsum, float* partial,
                       int64_t partial_floats, int defer_reduce, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (rows <= 0) return 0;
  if (D > 64 * LN_SMAX) return (int)hipErrorInvalidValue;
  const int rows_per = ln_bwd_rows();
  const int nblk = vit_layer_norm_bwd_blocks(rows);
  const bool want = dgamma != nullptr || dsum != nullptr;
  if (want && (partial == nullptr || partial_floats < vit_layer_norm_bwd_partial_floats(rows, D)))
    return (int)hipErrorInvalidValue;
  float* pg = dgamma ? partial : nullptr;
  float* pb = dgamma ? partial + (int64_t)nblk * D : nullptr;
  float* ps = dsum ? partial + 2 * (int64_t)nblk * D : nullptr;
  float* scratch = want ? partial + 3 * (int64_t)nblk * D : nullptr;
  bool vec = (D % 256 == 0) && (ldx % 4 == 0) && (lddy % 4 == 0) && (lddx % 4 == 0) && (ldres % 4 == 0) &&
             (ld_copy % 4 == 0);
  int nv = vec ? D / 256 : 0;
#define LB(TX, TD) \
  if (dtype_copy == VIT_BF16) launch_bwd<TX, TD, bf16>(nv, nblk, s, x, ldx, dy, lddy, w, mean, rstd, dres, ldres, dx, lddx, dx_copy, ld_copy, compact_np, pg, pb, ps, rows, D, rows_per); \
  else launch_bwd<TX, TD, float>(nv, nblk, s, x, ldx, dy, lddy, w, mean, rstd, dres, ldres, dx, lddx, dx_copy, ld_copy, compact_np, pg, pb, ps, rows, D, rows_per);
  if (dtype_x == VIT_F32 && dtype_dy == VIT_F32) { LB(float, float) }
  else if (dtype_x == VIT_F32) { LB(float, bf16) }
  else if (dtype_dy == VIT_BF16) { LB(bf16, bf16) }
  else { LB(bf16, float) }
#undef LB
  VIT_CHECK_LAUNCH();
  if (defer_reduce) return 0;  // the caller reduces the partials (vit_colreduce)
  {
    // the [pg | pb | ps] partial matrices are stacked: one two-stage reduction for all
    float* outs[3] = {dgamma, dbeta, dsum};
    if (dgamma) launch_colreduce_multi(pg, dsum ? 3 : 2, nblk, D, outs, 0, s, scratch);
    else if (dsum) launch_colreduce_multi(ps, 1, nblk, D, outs + 2, 0, s, scratch);
  }
  VIT_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
