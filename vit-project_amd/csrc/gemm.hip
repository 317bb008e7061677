// MFMA GEMMs for the ViT step: every nn.Linear / patch-embed Conv2d of timm
// vit_base_patch16_224 (forward, dgrad, wgrad) runs through here.
//
//   C[i][j] = epi( sum_r P(i,r) * Q(j,r) )
//
//   P layout RC: P[i*ldp + r]   (r contiguous)      CR: P[r*ldp + i]   (i contiguous)
//   Q layout RC: Q[j*ldq + r]                       CR: Q[r*ldq + j]
//
//   forward  Y = X W^T + b   : P = X  (RC), Q = W (RC)         (F.linear)
//   dgrad    dX = dY W       : P = dY (RC), Q = W (CR)
//   wgrad    dW = dY^T X     : P = dY (CR), Q = X (CR), split over r (rows of X)
//
// Fast path (bf16, i%128==0, j%128==0, r%64==0): 128x128x64 tile, 4 waves (2x2,
// 64x64 each), v_mfma_f32_16x16x32_bf16, global_load_lds (16 B/lane) into a
// double-buffered XOR-swizzled LDS image, ds_read_b128 for r-contiguous operands
// and ds_read_b64_tr_b16 for r-strided ones.  The MFMA computes C^T (Q is the
// A-operand) so each lane owns 4 consecutive output columns -> vector epilogue.
// Generic path (any shape/stride, f32 or bf16 in, fp32 FMA): parity mode and
// odd shapes (classifier head N=1000).
#include "common.hpp"
#include <string.h>

enum { LAY_RC = 0, LAY_CR = 1 };
enum { EPI_STORE = 0, EPI_BIAS_GELU = 1, EPI_RESID = 2, EPI_GELU_BWD = 3, EPI_PATCH = 4,
       EPI_BIAS_QGELU = 5, EPI_QGELU_BWD = 6 };

struct Epi {
  void* C; int64_t ldc;
  const float* bias;        // [N] or null
  const void* aux; int64_t ld_aux;  // EPI_RESID: f32 residual;  *_BWD: pre-activation (T)
  void* aux_out;            // BIAS_GELU: activation output (T, ld = ldc)
  const float* pos;         // EPI_PATCH: pos_embed [seq, N]
  int n_patch;              // EPI_PATCH: patches per image (seq = n_patch + 1)
  int64_t slab;             // split-r: element offset of slab z
};

template <typename T> __device__ __forceinline__ void store4(T* p, f32x4 v);
template <> __device__ __forceinline__ void store4<float>(float* p, f32x4 v) {
  *reinterpret_cast<f32x4*>(p) = v;
}
template <> __device__ __forceinline__ void store4<bf16>(bf16* p, f32x4 v) {
  bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *reinterpret_cast<bf16x4*>(p) = o;
}
template <typename T> __device__ __forceinline__ f32x4 load4(const T* p);
template <> __device__ __forceinline__ f32x4 load4<float>(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}
template <> __device__ __forceinline__ f32x4 load4<bf16>(const bf16* p) {
  bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
}

// Apply the epilogue to 4 consecutive output columns j..j+3 of row i.
template <int EPI, typename TO, typename TA>
__device__ __forceinline__ void epi4(const Epi& e, int i, int j, f32x4 v) {
  if (e.bias) {
    f32x4 b = *reinterpret_cast<const f32x4*>(e.bias + j);
    v += b;
  }
  if constexpr (EPI == EPI_STORE) {
    store4<TO>((TO*)e.C + e.slab * blockIdx.z + (int64_t)i * e.ldc + j, v);
  } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
    f32x4 pre_r;
    // the activation is computed from the rounded pre-activation that backward sees
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, v);
    pre_r = load4<TO>((const TO*)e.C + (int64_t)i * e.ldc + j);
    f32x4 a;
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = (EPI == EPI_BIAS_GELU) ? gelu_erf(pre_r[t]) : quick_gelu(pre_r[t]);
    store4<TO>((TO*)e.aux_out + (int64_t)i * e.ldc + j, a);
  } else if constexpr (EPI == EPI_RESID) {
    f32x4 r = load4<float>((const float*)e.aux + (int64_t)i * e.ld_aux + j);
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, v + r);
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    f32x4 pre = load4<TA>((const TA*)e.aux + (int64_t)i * e.ld_aux + j);
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] *= (EPI == EPI_GELU_BWD) ? gelu_erf_grad(pre[t]) : quick_gelu_grad(pre[t]);
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, v);
  } else if constexpr (EPI == EPI_PATCH) {
    int b = i / e.n_patch, p = i - b * e.n_patch;
    int64_t row = (int64_t)b * (e.n_patch + 1) + 1 + p;
    f32x4 ps = *reinterpret_cast<const f32x4*>(e.pos + (int64_t)(1 + p) * e.ldc + j);
    store4<TO>((TO*)e.C + row * e.ldc + j, v + ps);
  }
}

// Scalar form for the generic kernel (ragged edges).
template <int EPI, typename TO, typename TA>
__device__ __forceinline__ void epi1(const Epi& e, int i, int j, float v) {
  if (e.bias) v += e.bias[j];
  if constexpr (EPI == EPI_STORE) {
    ((TO*)e.C)[e.slab * blockIdx.z + (int64_t)i * e.ldc + j] = (TO)v;
  } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
    TO pr = (TO)v;
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = pr;
    float pf = (float)pr;
    ((TO*)e.aux_out)[(int64_t)i * e.ldc + j] = (TO)((EPI == EPI_BIAS_GELU) ? gelu_erf(pf) : quick_gelu(pf));
  } else if constexpr (EPI == EPI_RESID) {
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = (TO)(v + ((const float*)e.aux)[(int64_t)i * e.ld_aux + j]);
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    float pre = (float)((const TA*)e.aux)[(int64_t)i * e.ld_aux + j];
    v *= (EPI == EPI_GELU_BWD) ? gelu_erf_grad(pre) : quick_gelu_grad(pre);
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = (TO)v;
  } else if constexpr (EPI == EPI_PATCH) {
    int b = i / e.n_patch, p = i - b * e.n_patch;
    int64_t row = (int64_t)b * (e.n_patch + 1) + 1 + p;
    ((TO*)e.C)[row * e.ldc + j] = (TO)(v + e.pos[(int64_t)(1 + p) * e.ldc + j]);
  }
}

// ----------------------------------------------------------------------------
// Fast bf16 kernel
// ----------------------------------------------------------------------------
namespace fast {
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int IMG = 128 * 64 * 2;       // bytes of one operand image (16 KiB)
constexpr int STAGE = 2 * IMG;           // P + Q
constexpr int LDS_BYTES = 2 * STAGE;     // double buffer: 64 KiB

// r-contiguous image: 128 rows x 64 r (128 B rows); chunk c (16 B) of row at
// row*128 + ((c ^ ((row>>1)&7)) << 4).  Conflict-free for the 16x16x32 fragment
// ds_read_b128 pattern (16 consecutive rows, chunks g+4kk).
__device__ __forceinline__ int rc_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }
// r-strided image: 64 r-rows x 128 cols (256 B rows); chunk c in 0..15 at
// r*256 + ((c ^ f(r)) << 4), f(r) = ((r&3)<<2)|((r>>2)&3).  Conflict-free for the
// two ds_read_b64_tr_b16 of a 16x16x32 fragment (rows 8g+q and 8g+4+q).
__device__ __forceinline__ int cr_f(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int cr_off(int r, int c) { return r * 256 + ((c ^ cr_f(r)) << 4); }

// Stage one 128x64 operand tile into an LDS image with global_load_lds.
// RC: 16 wave-instructions of 8 rows; CR: 16 of 4 r-rows.  Each wave issues 4.
template <int LAY>
__device__ __forceinline__ void stage(char* img, const bf16* base, int64_t ld, int row0, int r0, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int t = wave * 4 + u;
    const bf16* src;
    if constexpr (LAY == LAY_RC) {
      int row = t * 8 + (lane >> 3);
      int c = (lane & 7) ^ ((row >> 1) & 7);
      src = base + (int64_t)(row0 + row) * ld + r0 + c * 8;
    } else {
      int r = t * 4 + (lane >> 4);
      int c = (lane & 15) ^ cr_f(r);
      src = base + (int64_t)(r0 + r) * ld + row0 + c * 8;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(img + t * 1024), 16, 0, 0);
  }
}

// Fragment for rows s*16..s*16+15 of the tile, r-substep kk (32 wide).
template <int LAY>
__device__ __forceinline__ bf16x8 frag(const char* img, int s, int kk, int lane) {
  if constexpr (LAY == LAY_RC) {
    int row = s * 16 + (lane & 15);
    int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + rc_off(row, c));
  } else {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int c = 2 * s + (p >> 1);
    int r0 = kk * 32 + 8 * g + q;
    int r1 = r0 + 4;
    bf16x4 lo = lds_read_tr(img + cr_off(r0, c) + (p & 1) * 8);
    bf16x4 hi = lds_read_tr(img + cr_off(r1, c) + (p & 1) * 8);
    return cat4(lo, hi);
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks that share an XCD (bid % 8) get a contiguous range of tiles
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7, k = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <int PL, int QL, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const bf16* __restrict__ P, int64_t ldp,
                                                      const bf16* __restrict__ Q, int64_t ldq,
                                                      int M, int N, int R, int r_chunk, Epi e) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_j = N / BN;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int ti = t / tiles_j, tj = t - ti * tiles_j;
  const int i0 = ti * BM, j0 = tj * BN;
  const int rb = blockIdx.z * r_chunk;
  const int re = min(R, rb + r_chunk);
  const int nk = (re - rb) / BK;
  const int wi = wave >> 1, wj = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    stage<PL>(smem, P, ldp, i0, rb, wave, lane);
    stage<QL>(smem + IMG, Q, ldq, j0, rb, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * STAGE;
      stage<PL>(nxt, P, ldp, i0, rb + (kt + 1) * BK, wave, lane);
      stage<QL>(nxt + IMG, Q, ldq, j0, rb + (kt + 1) * BK, wave, lane);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 pf[4], qf[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) pf[a] = frag<PL>(cur, wi * 4 + a, kk, lane);
#pragma unroll
      for (int b = 0; b < 4; ++b) qf[b] = frag<QL>(cur + IMG, wj * 4 + b, kk, lane);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(qf[b], pf[a], acc[a][b]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue: acc[a][b] holds C[i][j..j+3] with i = lane&15, j = 4*(lane>>4)
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    int i = i0 + wi * 64 + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int j = j0 + wj * 64 + b * 16 + 4 * (lane >> 4);
      epi4<EPI, TO, TA>(e, i, j, acc[a][b]);
    }
  }
}
}  // namespace fast

// ----------------------------------------------------------------------------
// Generic strided kernel: any M, N, R; f32 or bf16 inputs; fp32 FMA.
//   P(i,r) = P[i*sPi + r*sPr], Q(j,r) = Q[j*sQj + r*sQr]
// ----------------------------------------------------------------------------
namespace gen {
constexpr int TM = 64, TN = 64, TK = 16;
template <typename T, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ P, int64_t sPi, int64_t sPr,
                                                   const T* __restrict__ Q, int64_t sQj, int64_t sQr,
                                                   int M, int N, int R, int r_chunk, Epi e) {
  __shared__ float Ps[TK][TM + 4];
  __shared__ float Qs[TK][TN + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  const int rb = blockIdx.z * r_chunk, re = min(R, rb + r_chunk);
  float acc[4][4] = {};
  for (int k0 = rb; k0 < re; k0 += TK) {
    for (int idx = tid; idx < TK * TM; idx += 256) {
      int kk = idx / TM, ii = idx % TM;
      int i = i0 + ii, r = k0 + kk;
      Ps[kk][ii] = (i < M && r < re) ? (float)P[(int64_t)i * sPi + (int64_t)r * sPr] : 0.f;
    }
    for (int idx = tid; idx < TK * TN; idx += 256) {
      int kk = idx / TN, jj = idx % TN;
      int j = j0 + jj, r = k0 + kk;
      Qs[kk][jj] = (j < N && r < re) ? (float)Q[(int64_t)j * sQj + (int64_t)r * sQr] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      float pv[4], qv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) pv[a] = Ps[kk][ty + 16 * a];
#pragma unroll
      for (int b = 0; b < 4; ++b) qv[b] = Qs[kk][tx * 4 + b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(pv[a], qv[b], acc[a][b]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    int i = i0 + ty + 16 * a;
    if (i >= M) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      int j = j0 + tx * 4 + b;
      if (j < N) epi1<EPI, TO, TA>(e, i, j, acc[a][b]);
    }
  }
}
}  // namespace gen

// ----------------------------------------------------------------------------
// reductions used by the wgrad / bias-grad path
// ----------------------------------------------------------------------------
__global__ void splitk_reduce_kernel(const float* __restrict__ slabs, int nslab, int64_t n,
                                     float* __restrict__ out) {
  int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n) {
    f32x4 s = *reinterpret_cast<const f32x4*>(slabs + i4);
    for (int z = 1; z < nslab; ++z) s += *reinterpret_cast<const f32x4*>(slabs + z * n + i4);
    *reinterpret_cast<f32x4*>(out + i4) = s;
  } else {
    for (int64_t k = i4; k < n; ++k) {
      float s = 0.f;
      for (int z = 0; z < nslab; ++z) s += slabs[z * n + k];
      out[k] = s;
    }
  }
}

// Column sums out[j] = sum_i X[i*ld + j] (bias gradients, dpos).  Stage 1: grid
// (ceil(N/256), S) partial sums over row chunks; stage 2 sums the S partials.
template <typename T>
__global__ void colsum_partial_kernel(const T* __restrict__ X, int64_t ld, int M, int N, int rows_per,
                                      float* __restrict__ part) {
  int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= N) return;
  int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = r0;
  for (; i + 4 <= r1; i += 4) {
    s0 += (float)X[(int64_t)i * ld + j];
    s1 += (float)X[(int64_t)(i + 1) * ld + j];
    s2 += (float)X[(int64_t)(i + 2) * ld + j];
    s3 += (float)X[(int64_t)(i + 3) * ld + j];
  }
  for (; i < r1; ++i) s0 += (float)X[(int64_t)i * ld + j];
  part[(int64_t)blockIdx.y * N + j] = (s0 + s1) + (s2 + s3);
}

__global__ void colsum_final_kernel(const float* __restrict__ part, int S, int N, float* __restrict__ out,
                                    int accumulate) {
  int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= N) return;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += part[(int64_t)z * N + j];
  out[j] = accumulate ? out[j] + s : s;
}

// ----------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------
static bool fast_ok(int dtype, int M, int N, int R, const void* P, const void* Q, int64_t ldp, int64_t ldq) {
  if (dtype != VIT_BF16) return false;
  if (M % fast::BM || N % fast::BN || R % fast::BK) return false;
  if ((ldp % 8) || (ldq % 8)) return false;
  if (((uintptr_t)P & 15) || ((uintptr_t)Q & 15)) return false;
  return true;
}

template <int PL, int QL, int EPI, typename TO, typename TA>
static int launch_fast(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R,
                       int split, const Epi& e, hipStream_t s) {
  int r_chunk = ((R / split + fast::BK - 1) / fast::BK) * fast::BK;
  int nz = (R + r_chunk - 1) / r_chunk;
  dim3 grid((M / fast::BM) * (N / fast::BN), 1, nz);
  hipLaunchKernelGGL((fast::gemm_kernel<PL, QL, EPI, TO, TA>), grid, dim3(256), 0, s,
                     (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

template <typename T, int EPI, typename TO, typename TA>
static int launch_gen(const void* P, int64_t sPi, int64_t sPr, const void* Q, int64_t sQj, int64_t sQr,
                      int M, int N, int R, int split, const Epi& e, hipStream_t s) {
  int r_chunk = ((R / split + gen::TK - 1) / gen::TK) * gen::TK;
  if (r_chunk <= 0) r_chunk = gen::TK;
  int nz = (R + r_chunk - 1) / r_chunk;
  if (nz == 0) nz = 1;
  dim3 grid((N + gen::TN - 1) / gen::TN, (M + gen::TM - 1) / gen::TM, nz);
  hipLaunchKernelGGL((gen::gemm_kernel<T, EPI, TO, TA>), grid, dim3(256), 0, s,
                     (const T*)P, sPi, sPr, (const T*)Q, sQj, sQr, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

// One dispatcher for all layouts/epilogues.  out_dtype selects TO; for the
// *_BWD epilogues the pre-activation has the input dtype.
template <int EPI>
static int gemm_dispatch(int dtype, int out_dtype, int pl, int ql, int M, int N, int R,
                         const void* P, int64_t ldp, const void* Q, int64_t ldq, int split,
                         const Epi& e, hipStream_t s, bool allow_fast) {
  if (M <= 0 || N <= 0) return 0;
  if (allow_fast && fast_ok(dtype, M, N, R, P, Q, ldp, ldq) && (e.ldc % 4 == 0)) {
#define FAST(PLx, QLx)                                                                                  \
    if (out_dtype == VIT_F32) return launch_fast<PLx, QLx, EPI, float, bf16>(P, ldp, Q, ldq, M, N, R, split, e, s); \
    else return launch_fast<PLx, QLx, EPI, bf16, bf16>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (pl == LAY_RC && ql == LAY_RC) { FAST(LAY_RC, LAY_RC) }
    if (pl == LAY_RC && ql == LAY_CR) { FAST(LAY_RC, LAY_CR) }
    if (pl == LAY_CR && ql == LAY_CR) { FAST(LAY_CR, LAY_CR) }
    if (pl == LAY_CR && ql == LAY_RC) { FAST(LAY_CR, LAY_RC) }
#undef FAST
  }
  int64_t sPi = pl == LAY_RC ? ldp : 1, sPr = pl == LAY_RC ? 1 : ldp;
  int64_t sQj = ql == LAY_RC ? ldq : 1, sQr = ql == LAY_RC ? 1 : ldq;
  if (dtype == VIT_BF16) {
    if (out_dtype == VIT_F32) return launch_gen<bf16, EPI, float, bf16>(P, sPi, sPr, Q, sQj, sQr, M, N, R, split, e, s);
    return launch_gen<bf16, EPI, bf16, bf16>(P, sPi, sPr, Q, sQj, sQr, M, N, R, split, e, s);
  }
  if (out_dtype == VIT_F32) return launch_gen<float, EPI, float, float>(P, sPi, sPr, Q, sQj, sQr, M, N, R, split, e, s);
  return launch_gen<float, EPI, bf16, float>(P, sPi, sPr, Q, sQj, sQr, M, N, R, split, e, s);
}

static int gemm_any(int epi, int dtype, int out_dtype, int pl, int ql, int M, int N, int R,
                    const void* P, int64_t ldp, const void* Q, int64_t ldq, int split, const Epi& e,
                    hipStream_t s, bool allow_fast = true) {
  switch (epi) {
    case EPI_STORE: return gemm_dispatch<EPI_STORE>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_BIAS_GELU: return gemm_dispatch<EPI_BIAS_GELU>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_BIAS_QGELU: return gemm_dispatch<EPI_BIAS_QGELU>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_RESID: return gemm_dispatch<EPI_RESID>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_GELU_BWD: return gemm_dispatch<EPI_GELU_BWD>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_QGELU_BWD: return gemm_dispatch<EPI_QGELU_BWD>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_PATCH: return gemm_dispatch<EPI_PATCH>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
  }
  return (int)hipErrorInvalidValue;
}

static Epi make_epi() { Epi e; memset(&e, 0, sizeof(e)); return e; }

extern "C" {

// Raw dispatcher (exported for tests/benchmarks of individual layouts).
int vit_gemm(int dtype, int out_dtype, int p_layout, int q_layout, int epi, int M, int N, int R,
             const void* P, int64_t ldp, const void* Q, int64_t ldq, void* C, int64_t ldc,
             const float* bias, const void* aux, int64_t ld_aux, void* aux_out, int allow_fast,
             void* stream) {
  Epi e = make_epi();
  e.C = C; e.ldc = ldc; e.bias = bias; e.aux = aux; e.ld_aux = ld_aux; e.aux_out = aux_out;
  return gemm_any(epi, dtype, out_dtype, p_layout, q_layout, M, N, R, P, ldp, Q, ldq, 1, e,
                  (hipStream_t)stream, allow_fast != 0);
}

// F.linear forward: Y[M,N] = X[M,K] W[N,K]^T + b with a fused epilogue
//   epi = EPI_STORE (Y out_dtype), EPI_BIAS_GELU / EPI_BIAS_QGELU (Y = pre, act_out = act),
//   EPI_RESID (Y f32 = resid + X W^T + b; Y may alias resid).
int vit_linear_fwd(int dtype, int out_dtype, int epi, int M, int N, int K, const void* X, int64_t ldx,
                   const void* W, const float* bias, void* Y, int64_t ldy, const void* resid,
                   void* act_out, void* stream) {
  Epi e = make_epi();
  e.C = Y; e.ldc = ldy; e.bias = bias; e.aux = resid; e.ld_aux = ldy; e.aux_out = act_out;
  return gemm_any(epi, dtype, out_dtype, LAY_RC, LAY_RC, M, N, K, X, ldx, W, K, 1, e, (hipStream_t)stream);
}

// Linear input gradient: dX[M,K] = dY[M,N] W[N,K]  (epi EPI_STORE or *_GELU_BWD with pre [M,K])
int vit_linear_dgrad(int dtype, int out_dtype, int epi, int M, int N, int K, const void* dY, int64_t lddy,
                     const void* W, void* dX, int64_t lddx, const void* pre, void* stream) {
  Epi e = make_epi();
  e.C = dX; e.ldc = lddx; e.aux = pre; e.ld_aux = lddx;
  return gemm_any(epi, dtype, out_dtype, LAY_RC, LAY_CR, M, K, N, dY, lddy, W, K, 1, e, (hipStream_t)stream);
}

// Linear weight gradient: dW[N,K] (f32) = dY[M,N]^T X[M,K], split over M into
// `split` fp32 slabs in `workspace` (>= split*N*K*4 bytes) then reduced.
int vit_linear_wgrad(int dtype, int M, int N, int K, const void* dY, int64_t lddy, const void* X,
                     int64_t ldx, float* dW, int split, void* workspace, int64_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (split < 1) split = 1;
  if (split > 1 && (workspace == nullptr || ws_bytes < (int64_t)split * N * K * 4)) return (int)hipErrorInvalidValue;
  Epi e = make_epi();
  if (split == 1) {
    e.C = dW; e.ldc = K;
    return gemm_any(EPI_STORE, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, M, dY, lddy, X, ldx, 1, e, s);
  }
  e.C = workspace; e.ldc = K; e.slab = (int64_t)N * K;
  // the launchers round the chunk to the tile depth; count the real slabs
  bool fast = fast_ok(dtype, N, K, M, dY, X, lddy, ldx);
  int tk = fast ? fast::BK : gen::TK;
  int r_chunk = ((M / split + tk - 1) / tk) * tk;
  int nz = (M + r_chunk - 1) / r_chunk;
  int rc = gemm_any(EPI_STORE, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, M, dY, lddy, X, ldx, split, e, s);
  if (rc) return rc;
  int64_t n = (int64_t)N * K;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n / 4 + 255) / 256 + 1)), dim3(256), 0, s,
                     (const float*)workspace, nz, n, dW);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Column sum (bias grads): out[N] (f32) = sum_i X[i*ld + j]; partial buffer >= S*N floats
// with S = ceil(M / rows_per); `accumulate` adds into out.
int vit_colsum(int dtype, int M, int N, const void* X, int64_t ld, float* out, float* partial,
               int64_t partial_floats, int accumulate, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int S = (int)(partial_floats / (N > 0 ? N : 1));
  if (S > 256) S = 256;
  if (S > M) S = M > 0 ? M : 1;
  if (S < 1) return (int)hipErrorInvalidValue;
  int rows_per = (M + S - 1) / S;
  S = (M + rows_per - 1) / rows_per;
  if (S < 1) S = 1;
  dim3 g1((N + 255) / 256, S);
  if (dtype == VIT_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, g1, dim3(256), 0, s, (const bf16*)X, ld, M, N, rows_per, partial);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, g1, dim3(256), 0, s, (const float*)X, ld, M, N, rows_per, partial);
  VIT_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 255) / 256), dim3(256), 0, s, partial, S, N, out, accumulate);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Patch embedding forward (timm PatchEmbed Conv2d 16/16 + _pos_embed):
//   x[b*(np+1) + 1 + p][n] = U[b*np + p] . Wpe[n] + bpe[n] + pos[1+p][n]   (f32 out)
// U = unfolded patches [B*np, K] (vit_patch_unfold).  CLS rows: vit_cls_pos_fill.
int vit_patch_embed_fwd(int dtype, int B, int np, int D, int K, const void* U, const void* W,
                        const float* bias, const float* pos, float* x, void* stream) {
  Epi e = make_epi();
  e.C = x; e.ldc = D; e.bias = bias; e.pos = pos; e.n_patch = np;
  return gemm_any(EPI_PATCH, dtype, VIT_F32, LAY_RC, LAY_RC, B * np, D, K, U, K, W, K, 1, e, (hipStream_t)stream);
}

}  // extern "C"
