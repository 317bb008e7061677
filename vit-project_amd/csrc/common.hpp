// Shared device helpers for the gfx950 (CDNA4, MI355X) ViT hot-path kernels.
// Wave = 64 lanes; MFMA = v_mfma_f32_16x16x32_bf16 (bf16 path) and
// v_mfma_f32_16x16x4_f32 (exact-f32 parity path).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

enum { VIT_F32 = 0, VIT_BF16 = 1 };

static constexpr int WAVE = 64;

template <typename T> __device__ __forceinline__ float to_f32(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x) { return (T)x; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p passes the LDS byte
// address of (row q, cols 4p..4p+3) of a 4x16 block; lane i receives column i
// of the 4 rows (row q in element q).
__device__ __forceinline__ bf16x4 lds_read_tr(const void* lds_byte_ptr) {
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds_byte_ptr));
  return __builtin_bit_cast(bf16x4, r);
}

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  // d/dx [0.5 x (1 + erf(x/sqrt2))] = 0.5 (1 + erf(x/sqrt2)) + x * exp(-x^2/2)/sqrt(2 pi)
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) +
         x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
// erf via Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, below bf16 and fp16
// resolution): one v_rcp, one v_exp, five FMAs -- used by the bf16 GEMM
// epilogues, where ocml's erff made the GELU epilogue as long as the MFMA loop.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-ax * ax);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_fast(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_fast_grad(float x) {
  return 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
// GELU and its derivative from one erf evaluation (the forward epilogue stores both:
// the activation for fc2 and GELU'(pre) for the backward's dgrad epilogue).
__device__ __forceinline__ void gelu_fast_both(float x, float& g, float& gp) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __expf(-az * az);  // exp(-x^2 / 2)
  const float cdf = 0.5f + 0.5f * copysignf(1.0f - p * t * e, z);
  g = x * cdf;
  gp = fmaf(x * 0.39894228040143268f, e, cdf);
}
// The same on two elements at once, op for op (so bit for bit: the compiled gelu_fast_both is the sequence
// below, `__expf(v)` being exp2(v * -log2(e)) here with v = |z|^2): the FMAs and multiplies become
// v_pk_fma_f32 / v_pk_mul_f32, which do two lanes' worth each; rcp / exp / copysign stay per element.
// 21 instructions per pair instead of 34 -- the GELU pair epilogues' VALU time.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_fast_both2(f32x2 x, f32x2& g, f32x2& gp) {
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 az = __builtin_elementwise_abs(z);
  const f32x2 den = __builtin_elementwise_fma(az, f32x2(0.3275911f), f32x2(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  const f32x2 q = (az * az) * -1.44269504088896341f;
  const f32x2 e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  f32x2 p = __builtin_elementwise_fma(f32x2(1.061405429f), t, f32x2(-1.453152027f));
  p = __builtin_elementwise_fma(p, t, f32x2(1.421413741f));
  p = __builtin_elementwise_fma(p, t, f32x2(-0.284496736f));
  p = __builtin_elementwise_fma(p, t, f32x2(0.254829592f));
  const f32x2 y = __builtin_elementwise_fma(-e, t * p, f32x2(1.0f));
  const f32x2 cs = {copysignf(y.x, z.x), copysignf(y.y, z.y)};
  const f32x2 cdf = __builtin_elementwise_fma(cs, f32x2(0.5f), f32x2(0.5f));
  g = x * cdf;
  gp = __builtin_elementwise_fma(x * 0.39894228040143268f, e, cdf);
}
__device__ __forceinline__ void gelu_erf_both(float x, float& g, float& gp) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  g = x * cdf;
  gp = cdf + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ float quick_gelu(float x) { return x / (1.0f + __expf(-1.702f * x)); }
__device__ __forceinline__ void quick_gelu_both(float x, float& g, float& gp) {
  const float s = 1.0f / (1.0f + __expf(-1.702f * x));
  g = x * s;
  gp = s + 1.702f * x * s * (1.0f - s);
}
__device__ __forceinline__ float quick_gelu_grad(float x) {
  float s = 1.0f / (1.0f + __expf(-1.702f * x));
  return s + 1.702f * x * s * (1.0f - s);
}

#define VIT_CHECK_LAUNCH() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
