// ImageNet input transforms on the GPU: the reference's
// RandomResizedCrop(224) + RandomHorizontalFlip + ToTensor + Normalize (VIT:32-38,
// MEAS:152-158) and Resize(256) + CenterCrop(224) + ToTensor + Normalize (VIT:41-46),
// applied to a ragged batch of decoded RGB uint8 images resident in HBM.
//
// torchvision hands PIL images to Pillow's Image.resize(BILINEAR), so the resampling is
// Pillow's 8-bit two-pass convolution (libImaging/Resample.c), restated exactly:
// float64 coefficients per output pixel (precompute_coeffs) quantised to 22-bit fixed
// point (normalize_coeffs_8bpc), a horizontal pass into an 8-bit intermediate, then a
// vertical pass, each rounding with clip8((2^21 + sum w*p) >> 22).  Results are
// bit-identical to Pillow (oracle/image_ref.py pins the restatement against it); the
// float outputs are then ((v / 255) - mean) / std in IEEE float32 like ToTensor+Normalize.
//
// Byte work, HBM/latency bound: no MFMA.  Per image and direction one coefficient row per
// output pixel; the horizontal pass reads each needed source row once and writes
// rows x 224 x 3 bytes; the vertical pass writes the f32 NCHW tensor the patch
// embedding consumes.
#include "common.hpp"

#pragma clang fp contract(off)

namespace {

constexpr int IMG_PARAMS = 12;  // per-image int64 fields, see vit_image_transform
constexpr int PREC = 22;        // Pillow PRECISION_BITS for 8-bit images

struct Norm3 {
  float mean[3], stdv[3];
};

// coefficient table of one image, one direction: [S][2 + kmax] int32 = (start, count, w...)
__device__ __forceinline__ int* coeff_row(int* ws, int b, int dir, int S, int kmax, int o) {
  return ws + (((int64_t)b * 2 + dir) * S + o) * (2 + kmax);
}

__global__ __launch_bounds__(256) void img_coeff_kernel(const int64_t* __restrict__ params, int S, int kmax,
                                                        int* __restrict__ ws) {
  const int b = blockIdx.x, dir = blockIdx.y;
  const int64_t* p = params + (int64_t)b * IMG_PARAMS;
  const int in_size = (int)(dir == 0 ? p[5] : p[4]);
  const int out_size = (int)(dir == 0 ? p[7] : p[6]);
  const int start = (int)(dir == 0 ? p[9] : p[8]);
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double ss = 1.0 / filterscale;
  for (int o = threadIdx.x; o < S; o += blockDim.x) {
    const int xx = start + o;
    const double center = (xx + 0.5) * scale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int* row = coeff_row(ws, b, dir, S, kmax, o);
    if (xmax > kmax) {  // host sized kmax from the same formula: cannot happen
      row[0] = 0;
      row[1] = 0;
      continue;
    }
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      ww += t < 1.0 ? 1.0 - t : 0.0;
    }
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      double w = t < 1.0 ? 1.0 - t : 0.0;
      if (ww != 0.0) w /= ww;
      const double v = w * (double)(1 << PREC);
      row[2 + x] = w < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
    }
    row[0] = xmin;
    row[1] = xmax;
  }
}

__device__ __forceinline__ int clip8(int s) {
  s >>= PREC;
  return s < 0 ? 0 : (s > 255 ? 255 : s);
}

// horizontal pass: intermediate rows [0, h) of the source region x S window columns x 3
__global__ __launch_bounds__(256) void img_hpass_kernel(const uint8_t* __restrict__ src,
                                                        const int64_t* __restrict__ params, int S, int kmax,
                                                        const int* __restrict__ ws, uint8_t* __restrict__ tmp,
                                                        int rows_per_block) {
  const int b = blockIdx.y;
  const int64_t* p = params + (int64_t)b * IMG_PARAMS;
  const int64_t src_off = p[0], stride = p[1] * 3, top = p[2], left = p[3];
  const int h = (int)p[4];
  const int y0 = blockIdx.x * rows_per_block, y1 = min(h, y0 + rows_per_block);
  if (y0 >= h) return;
  uint8_t* t = tmp + p[11];
  for (int x = threadIdx.x; x < S; x += blockDim.x) {
    const int* row = coeff_row(const_cast<int*>(ws), b, 0, S, kmax, x);
    const int xmin = row[0], n = row[1];
    for (int y = y0; y < y1; ++y) {
      const uint8_t* s = src + src_off + (top + y) * stride + (left + xmin) * 3;
      int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
      for (int k = 0; k < n; ++k) {
        const int w = row[2 + k];
        a0 += (int)s[3 * k] * w;
        a1 += (int)s[3 * k + 1] * w;
        a2 += (int)s[3 * k + 2] * w;
      }
      uint8_t* o = t + ((int64_t)y * S + x) * 3;
      o[0] = (uint8_t)clip8(a0);
      o[1] = (uint8_t)clip8(a1);
      o[2] = (uint8_t)clip8(a2);
    }
  }
}

// vertical pass + flip + ToTensor + Normalize: output row y of image b -> out [B][3][S][S] f32
__global__ __launch_bounds__(256) void img_vpass_kernel(const int64_t* __restrict__ params, int S, int kmax,
                                                        const int* __restrict__ ws, const uint8_t* __restrict__ tmp,
                                                        float* __restrict__ out, Norm3 nm) {
  const int y = blockIdx.x, b = blockIdx.y;
  const int64_t* p = params + (int64_t)b * IMG_PARAMS;
  const bool flip = p[10] != 0;
  const uint8_t* t = tmp + p[11];
  const int* row = coeff_row(const_cast<int*>(ws), b, 1, S, kmax, y);
  const int ymin = row[0], n = row[1];
  for (int x = threadIdx.x; x < S; x += blockDim.x) {
    int a[3] = {1 << (PREC - 1), 1 << (PREC - 1), 1 << (PREC - 1)};
    for (int k = 0; k < n; ++k) {
      const int w = row[2 + k];
      const uint8_t* s = t + ((int64_t)(ymin + k) * S + x) * 3;
      a[0] += (int)s[0] * w;
      a[1] += (int)s[1] * w;
      a[2] += (int)s[2] * w;
    }
    const int xo = flip ? S - 1 - x : x;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = (float)clip8(a[c]) / 255.0f;
      out[(((int64_t)b * 3 + c) * S + y) * S + xo] = (v - nm.mean[c]) / nm.stdv[c];
    }
  }
}

}  // namespace

extern "C" {

// Bytes of the coefficient workspace for B images at output size S with at most kmax taps.
int vit_image_coeff_bytes(int B, int S, int kmax) { return (int)((int64_t)B * 2 * S * (2 + kmax) * 4); }

// params: device int64 [B][12] per image = {src byte offset, image width (row stride / 3),
// region top, region left, region rows h, region cols w, resized rows RH, resized cols RW,
// window top oy0, window left ox0, flip (0/1), intermediate byte offset (>= h*S*3 bytes
// each)}.  The region is resampled as an image of its own (torchvision's crop-then-resize:
// Pillow clamps taps to the region) to RH x RW, and the S x S window at (oy0, ox0) of the
// result is written, mirrored when flip, normalised: out[b][c][y][x] = (v/255 - mean[c]) /
// std[c].  kmax >= ceil(max(region/resized, 1)) * 2 + 1 over every image and direction;
// max_rows >= every region's h.  norm6 (host) = mean[3], std[3].
int vit_image_transform(int B, int S, const uint8_t* src, const int64_t* params, int kmax, int max_rows,
                        int* coeff_ws, uint8_t* tmp_ws, float* out, const float* norm6, void* stream) {
  if (B <= 0) return 0;
  if (S <= 0 || kmax <= 0 || max_rows <= 0 || !src || !params || !coeff_ws || !tmp_ws || !out || !norm6)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  Norm3 nm;
  for (int c = 0; c < 3; ++c) {
    nm.mean[c] = norm6[c];
    nm.stdv[c] = norm6[3 + c];
  }
  hipLaunchKernelGGL(img_coeff_kernel, dim3(B, 2), dim3(256), 0, s, params, S, kmax, coeff_ws);
  const int rpb = 4;
  hipLaunchKernelGGL(img_hpass_kernel, dim3((max_rows + rpb - 1) / rpb, B), dim3(256), 0, s, src, params, S, kmax,
                     (const int*)coeff_ws, tmp_ws, rpb);
  hipLaunchKernelGGL(img_vpass_kernel, dim3(S, B), dim3(256), 0, s, params, S, kmax, (const int*)coeff_ws,
                     (const uint8_t*)tmp_ws, out, nm);
  VIT_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
