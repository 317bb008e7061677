// Scaled-dot-product attention for timm Attention: per (batch, head)
// softmax(q k^T * hd^-0.5) v, N <= 288 tokens (197 for ViT-B/16, 257 for CLIP
// ViT-L/14, 77 for the CLIP text tower), head_dim 64; unmasked or causal (the
// text tower's build_attention_mask: key > query gets -inf).
//
// q/k/v are read in place from the fused qkv GEMM output [B*N, 3*D] (row stride
// ld_qkv), the output o is written as [B*N, D] (the proj GEMM operand), and the
// backward writes dq/dk/dv into a [B*N, 3*D] buffer laid out like qkv so the
// qkv dgrad/wgrad GEMMs consume it directly.
//
// bf16 path: one workgroup (4 waves) per (b, h); the whole K and V of the head
// live in LDS (<= 2 x 36 KiB); S^T = K Q^T with v_mfma_f32_16x16x32_bf16 so each
// lane owns one query column and the softmax row-max/row-sum are in-lane plus two
// cross-lane shuffles; P stays in registers and feeds the PV MFMA as its
// B-operand (k-slot permutation pi), V^T comes from ds_read_b64_tr_b16.
// f32 path (parity mode): scalar-FMA online softmax.
#include "common.hpp"
#include "reduce.hpp"

extern "C" int vit_colsum(int dtype, int M, int N, const void* X, int64_t ld, float* out, float* partial,
                          int64_t partial_floats, int accumulate, void* stream);

// 128-B row image with XOR swizzle (row & 6) on 16-B chunks: conflict-free for
// the 16x16x32 ds_read_b128 fragment reads and for the ds_read_b64_tr_b16 reads
// of 8 consecutive rows (LDS images).
__device__ __forceinline__ int at_off(int row, int c) { return row * 128 + ((c ^ (row & 6)) << 4); }

// Load rows [0, N) of NM head slices (64 wide) into LDS images of ROWS rows,
// zero-filling rows >= N.  All global loads of the thread are issued before the
// first LDS write (one latency, not one per chunk); rows >= N load a clamped
// valid row and are zeroed in registers.
template <int ROWS, int NTHR, int NM>
__device__ __forceinline__ void at_load(char* const (&img)[NM], const bf16* const (&src)[NM],
                                        const int64_t (&ld)[NM], int N) {
  constexpr int TOTAL = ROWS * 8, PER = (TOTAL + NTHR - 1) / NTHR;
  bf16x8 v[NM][PER];
#pragma unroll
  for (int mtx = 0; mtx < NM; ++mtx)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = threadIdx.x + u * NTHR;
      const int row = min(idx >> 3, N - 1), c = idx & 7;
      if (idx < TOTAL) v[mtx][u] = *reinterpret_cast<const bf16x8*>(src[mtx] + (int64_t)row * ld[mtx] + c * 8);
    }
#pragma unroll
  for (int mtx = 0; mtx < NM; ++mtx)
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = threadIdx.x + u * NTHR;
      const int row = idx >> 3, c = idx & 7;
      if (idx < TOTAL) {
        bf16x8 w = v[mtx][u];
        if (row >= N) {
#pragma unroll
          for (int t = 0; t < 8; ++t) w[t] = (bf16)0.f;
        }
        *reinterpret_cast<bf16x8*>(img[mtx] + at_off(row, c)) = w;
      }
    }
}

constexpr int AT_THREADS = 512;  // 8 waves per (batch, head)
constexpr int AT_WAVES = AT_THREADS / 64;

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  return bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
}

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------
// Per-lane LDS offsets.  Tiles start at multiples of 16 (row fragments) or 32
// (transposed fragments) rows, which leaves (row & 6) -- the swizzle -- a
// function of the lane only, so every fragment address is a lane constant plus
// a wave-uniform tile offset (row0 * 128).
// ---------------------------------------------------------------------------
struct AtOffsets {
  int row[2];   // row fragment, k-substep kk (d 0..31 / 32..63)
  int tr[4];    // transposed fragment, d-tile dt, rows 4g+q (+16 rows: + 2048)
  __device__ __forceinline__ AtOffsets(int lane) {
    const int l15 = lane & 15, g = lane >> 4, q = l15 >> 2, p = l15 & 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) row[kk] = l15 * 128 + (((kk * 4 + g) ^ (l15 & 6)) << 4);
    const int ra = 4 * g + q;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) tr[dt] = ra * 128 + (((2 * dt + (p >> 1)) ^ (ra & 6)) << 4) + (p & 1) * 8;
  }
};
__device__ __forceinline__ bf16x8 rowf(const char* img, int row0, int off) {
  return *reinterpret_cast<const bf16x8*>(img + row0 * 128 + off);
}
__device__ __forceinline__ bf16x8 trf(const char* img, int row0, int off) {
  const char* b = img + row0 * 128 + off;
  return cat4(lds_read_tr(b), lds_read_tr(b + 16 * 128));
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Diagnostic phase stamps (tools/attn_stamps.py): a separate template instance, launched only
// while vit_debug_attn_stamps() has set a buffer.  Thread 0 of a workgroup records s_memtime at
// phase boundaries and s_memrealtime at start / end into stamps[blockIdx.x * 8 + i].
static unsigned long long* g_attn_stamps = nullptr;
#define AT_STAMP(i)                                                   \
  if constexpr (STAMP) { if (threadIdx.x == 0) st[i] = __builtin_amdgcn_s_memtime(); }
#define AT_STAMP_BEGIN()                                                                          \
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                            \
  if constexpr (STAMP) { if (threadIdx.x == 0) st[5] = __builtin_amdgcn_s_memrealtime(); }        \
  AT_STAMP(0)
#define AT_STAMP_FLUSH()                                                                         \
  if constexpr (STAMP) if (threadIdx.x == 0) {                                                   \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                             \
    st[6] = __builtin_amdgcn_s_memtime();                                                        \
    st[7] = __builtin_amdgcn_s_memrealtime();                                                    \
    unsigned long long* d = stamps + (int64_t)blockIdx.x * 8;                                    \
    for (int i_ = 0; i_ < 8; ++i_) d[i_] = st[i_];                                               \
  }

// ---------------------------------------------------------------------------
// bf16 forward
// ---------------------------------------------------------------------------
template <int NT, bool STAMP = false, bool CAUSAL = false>  // key/query tiles of 16: NT = ceil(N/16)
__global__ __launch_bounds__(AT_THREADS, NT <= 14 ? 4 : 2) void attn_fwd_mfma(const bf16* __restrict__ qkv, int64_t ld_qkv, int D,
                                                     int H, int N, float scale, bf16* __restrict__ o,
                                                     int64_t ld_o, float* __restrict__ lse, int causal,
                                                     unsigned long long* __restrict__ stamps) {
  AT_STAMP_BEGIN()
  constexpr int NT2 = (NT + 1) / 2, ROWS = NT2 * 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * ROWS * 128];
  char* Kimg = smem;
  char* Vimg = smem + ROWS * 128;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const bf16* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  {
    char* const imgs[2] = {Kimg, Vimg};
    const bf16* const srcs[2] = {base + D, base + 2 * D};
    const int64_t lds_[2] = {ld_qkv, ld_qkv};
    at_load<ROWS, AT_THREADS, 2>(imgs, srcs, lds_, N);
  }
  const AtOffsets off(lane);
  __syncthreads();
  AT_STAMP(1)
  const float c2 = scale * LOG2E;
  for (int qt = wave; qt < NT; qt += AT_WAVES) {
    const int q = qt * 16 + (lane & 15);
    bf16x8 qf[2];
    {
      const int qq = min(q, N - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)qq * ld_qkv + kk * 32 + g * 8);
    }
    f32x4 s[NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) s[kt] = mfma16(rowf(Kimg, kt * 16, off.row[kk]), qf[kk], s[kt]);
      if (kt % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // bound K-fragment hoisting (VGPRs)
    }
    // keys >= N exist only in the last tile
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if ((NT - 1) * 16 + 4 * g + r >= N) s[NT - 1][r] = -INFINITY;
    if constexpr (CAUSAL) {  // key > query masked (CLIP text tower attn_mask); key 0 always survives
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kt * 16 + 4 * g + r > q) s[kt][r] = -INFINITY;
    }
    // row max / sum as 4 independent chains (one per accumulator slot r): a single chain over
    // the 4*NT scores is a 52-deep dependent VALU sequence at N = 197
    float mr[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mr[r] = fmaxf(mr[r], s[kt][r]);
    float m = fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3]));
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float mc = m * c2;
    float lr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) { float p = fexp2(fmaf(s[kt][r], c2, -mc)); s[kt][r] = p; lr[r] += p; }
    float l = (lr[0] + lr[1]) + (lr[2] + lr[3]);
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    f32x4 oacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NT2; ++ks) {
      f32x4 hi = (2 * ks + 1 < NT) ? s[2 * ks + 1 < NT ? 2 * ks + 1 : 0] : f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 pf = pack8(s[2 * ks], hi);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) oacc[dt] = mfma16(trf(Vimg, ks * 32, off.tr[dt]), pf, oacc[dt]);
      if (ks % 2 == 1) __builtin_amdgcn_sched_barrier(0);  // bound V-fragment hoisting (VGPRs)
    }
    if (q < N) {
      const float inv = 1.0f / l;
      bf16* orow = o + ((int64_t)b * N + q) * ld_o + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 ov = {(bf16)(oacc[dt][0] * inv), (bf16)(oacc[dt][1] * inv), (bf16)(oacc[dt][2] * inv),
                     (bf16)(oacc[dt][3] * inv)};
        *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = ov;
      }
      if (g == 0) lse[(int64_t)bh * N + q] = (mc + __log2f(l)) * LN2;
    }
  }
  AT_STAMP(2)
  AT_STAMP_FLUSH()
}


// ---------------------------------------------------------------------------
// fp8 forward (BASELINE configs[4]: the perturbation sweep's frozen-tower attention and the RSA
// evaluation forward).  Block-scaled OCP e4m3 operands on v_mfma_scale_f32_32x32x64_f8f6f4
// (twice the bf16 MFMA rate per clock), operand layouts probed with exact one-hot data
// (tools/probe/mfma_scale_probe.hip): lane l holds A[row l%32][k = 32(l/32) + byte] and
// B[k = 32(l/32) + byte][col l%32]; its E8M0 scale byte covers those 32 k values.
//
//   S^T = K Q^T: A = K (rows = keys, k = d), B = Q^T; one MFMA per 32-key tile (hd = 64 = K).
//     Q and K are quantised per row (all 64 d): e = the smallest exponent with
//     max|x| <= 448 * 2^e, byte = x * 2^-e rounded to e4m3, E8M0 scale 127 + e in both lane halves
//     of the row.  (One scale per row, not per 32 values: the hardware's 32-value scale blocks
//     interleave the two lane halves' bytes -- tools/probe/mfma_scale_probe.hip, test 6.)
//   P = exp(S - rowmax) in (0, 1], quantised as P * 2^8 (scale 2^-8): no block max needed.
//   O^T = V^T P^T: A = V^T (rows = d, k = keys), B = P^T straight from the S^T accumulators:
//     lane half h holds keys 4h + (r&3) + 8(r>>2) of each 32-key tile (the 32x32 C layout), so
//     the MFMA's k slots are permuted the same way for both operands; V is quantised per
//     (d, 64-key tile) into a transposed [d][keys] LDS image read 4 keys at a time.
// One workgroup (8 waves) per (b, h); each wave takes 32-query tiles.  Softmax statistics, the
// row sum and the output scaling stay f32; o is written bf16, lse f32 (natural log).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int e8m0_exp(float amax) {
  // smallest e with amax <= 448 * 2^e (448 = 1.75 * 2^8), clamped to the E8M0 range
  const uint32_t bits = __float_as_uint(amax);
  const int E = (int)((bits >> 23) & 255) - 127;
  if (((bits >> 23) & 255) == 0) return -127;  // 0 / denormal
  const int e = (bits & 0x7fffff) <= 0x600000 ? E - 8 : E - 7;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}
__device__ __forceinline__ float inv_exp2i(int e) {  // 2^-e, exact for e in [-127, 126]
  return e >= 127 ? 0.f : __uint_as_float((uint32_t)(e == -127 ? 254 : 127 - e) << 23);
}
// 4 floats -> 4 e4m3 bytes (round to nearest even; |x| <= 448 by construction)
__device__ __forceinline__ int pack_fp8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int F8_THREADS = 512, F8_WAVES = 8;
__device__ __forceinline__ int f8_koff(int key, int c) { return key * 64 + ((c ^ ((key >> 2) & 1)) << 4); }

template <typename T> __device__ __forceinline__ void load8f(const T* p, float* x);
template <> __device__ __forceinline__ void load8f<bf16>(const bf16* p, float* x) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = (float)v[u];
}
template <> __device__ __forceinline__ void load8f<float>(const float* p, float* x) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int u = 0; u < 4; ++u) { x[u] = a[u]; x[4 + u] = b[u]; }
}

template <int NKT, typename T>  // 64-key tiles: keys padded to NKT * 64; T = the qkv / o dtype
__global__ __launch_bounds__(F8_THREADS, 2) void attn_fwd_fp8(const T* __restrict__ qkv, int64_t ld_qkv, int D,
                                                             int H, int N, float scale, T* __restrict__ o,
                                                             int64_t ld_o, float* __restrict__ lse, int causal) {
  constexpr int KEYS = NKT * 64, VROW = KEYS + 4;  // V^T rows padded: conflict-free transposed writes
  __shared__ __attribute__((aligned(16))) unsigned char Kimg[KEYS * 64];
  __shared__ __attribute__((aligned(16))) unsigned char Vt[64 * VROW];
  __shared__ unsigned char Ksc[KEYS * 2];
  __shared__ unsigned char Vsc[64 * NKT];
  const int bh = blockIdx.x, b = bh / H, hh = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T* base = qkv + (int64_t)b * N * ld_qkv + hh * 64;

  // K: two adjacent lanes per key (one 32-wide d half each), one scale per key row
  for (int t = threadIdx.x; t < KEYS * 2; t += F8_THREADS) {
    const int key = t >> 1, half = t & 1;
    float x[32];
    if (key < N) {
      const T* src = base + (int64_t)key * ld_qkv + D + half * 32;
#pragma unroll
      for (int c = 0; c < 4; ++c) load8f<T>(src + c * 8, x + c * 8);
    } else {
#pragma unroll
      for (int u = 0; u < 32; ++u) x[u] = 0.f;
    }
    float amax = 0.f;
#pragma unroll
    for (int u = 0; u < 32; ++u) amax = fmaxf(amax, fabsf(x[u]));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));  // the row's other half (KEYS * 2 is a multiple of 64)
    const int e = e8m0_exp(amax);
    const float inv = inv_exp2i(e);
    int w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) w[u] = pack_fp8x4(x[4 * u] * inv, x[4 * u + 1] * inv, x[4 * u + 2] * inv, x[4 * u + 3] * inv);
    typedef int i32x4_ __attribute__((ext_vector_type(4)));
    *reinterpret_cast<i32x4_*>(Kimg + f8_koff(key, 2 * half)) = i32x4_{w[0], w[1], w[2], w[3]};
    *reinterpret_cast<i32x4_*>(Kimg + f8_koff(key, 2 * half + 1)) = i32x4_{w[4], w[5], w[6], w[7]};
    Ksc[key * 2 + half] = (unsigned char)(e + 127);
  }
  // V: wave per 64-key tile, lane = d
  for (int kt = wave; kt < NKT; kt += F8_WAVES) {
    float x[64];
    const T* src = base + 2 * D + lane;
#pragma unroll
    for (int u = 0; u < 64; ++u) {
      const int key = kt * 64 + u;
      x[u] = key < N ? (float)src[(int64_t)key * ld_qkv] : 0.f;
    }
    float amax = 0.f;
#pragma unroll
    for (int u = 0; u < 64; ++u) amax = fmaxf(amax, fabsf(x[u]));
    const int e = e8m0_exp(amax);
    const float inv = inv_exp2i(e);
#pragma unroll
    for (int u = 0; u < 16; ++u)
      *reinterpret_cast<int*>(Vt + lane * VROW + kt * 64 + 4 * u) =
          pack_fp8x4(x[4 * u] * inv, x[4 * u + 1] * inv, x[4 * u + 2] * inv, x[4 * u + 3] * inv);
    Vsc[lane * NKT + kt] = (unsigned char)(e + 127);
  }
  __syncthreads();

  const float c2 = scale * LOG2E;
  const int h = lane >> 5, l31 = lane & 31;
  const int nqt = (N + 31) / 32;
  for (int qt = wave; qt < nqt; qt += F8_WAVES) {
    const int q = qt * 32 + l31;
    // Q^T fragment: this lane's 32 d values (block h) of query q
    i32x8 qf;
    int qsc;
    {
      const T* src = base + (int64_t)min(q, N - 1) * ld_qkv + h * 32;
      float x[32];
#pragma unroll
      for (int c = 0; c < 4; ++c) load8f<T>(src + c * 8, x + c * 8);
      float amax = 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) amax = fmaxf(amax, fabsf(x[u]));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));  // the query's other lane half: one scale per row
      const int e = e8m0_exp(amax);
      const float inv = inv_exp2i(e);
#pragma unroll
      for (int u = 0; u < 8; ++u) qf[u] = pack_fp8x4(x[4 * u] * inv, x[4 * u + 1] * inv, x[4 * u + 2] * inv, x[4 * u + 3] * inv);
      qsc = e + 127;
    }
    // online softmax over 64-key tiles (two S^T MFMAs each): only one tile's scores are live
    float m = -INFINITY, l = 0.f;
    f32x16 oacc[2] = {};
#pragma unroll 1
    for (int kt = 0; kt < NKT; ++kt) {
      f32x16 s[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int key = (2 * kt + u) * 32 + l31;
        typedef int i32x4_ __attribute__((ext_vector_type(4)));
        const i32x4_ lo = *reinterpret_cast<const i32x4_*>(Kimg + f8_koff(key, 2 * h));
        const i32x4_ hi = *reinterpret_cast<const i32x4_*>(Kimg + f8_koff(key, 2 * h + 1));
        const i32x8 kf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        f32x16 z = {};
        s[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(kf, qf, z, 0, 0, 0, Ksc[key * 2 + h], 0, qsc);
      }
      // rows of s[u]: key (2kt+u)*32 + 4h + (r&3) + 8(r>>2); column: query q
      float mt = -INFINITY;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = (2 * kt + u) * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
          if (key >= N || (causal && key > q)) s[u][r] = -INFINITY;
          mt = fmaxf(mt, s[u][r]);
        }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt);  // finite from the first tile on: key 0 is never masked
      const float alpha = fexp2((m - mn) * c2);  // first tile: m = -inf -> 0
      m = mn;
      const float mc = m * c2;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) oacc[dt] *= alpha;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(s[u][r], c2, -mc));
          s[u][r] = p;
          l += p;
        }
      i32x8 pf;  // P^T fragment: byte j = tile (j/16), register j%16, times 2^8
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        const f32x16& t = s[w >> 2];
        const int r = 4 * (w & 3);
        pf[w] = pack_fp8x4(t[r] * 256.f, t[r + 1] * 256.f, t[r + 2] * 256.f, t[r + 3] * 256.f);
      }
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int d = dt * 32 + l31;
        const unsigned char* row = Vt + d * VROW + kt * 64 + 4 * h;
        i32x8 vf;
#pragma unroll
        for (int w = 0; w < 8; ++w) vf[w] = *reinterpret_cast<const int*>(row + (w >> 2) * 32 + 8 * (w & 3));
        oacc[dt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(vf, pf, oacc[dt], 0, 0, 0, Vsc[d * NKT + kt], 0,
                                                                   127 - 8);
      }
    }
    l += __shfl_xor(l, 32, 64);
    const float mc = m * c2;
    if (q < N) {
      const float inv = 1.0f / l;
      T* orow = o + ((int64_t)b * N + q) * ld_o + hh * 64;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int mq = 0; mq < 4; ++mq) {
          const int d = dt * 32 + 4 * h + 8 * mq;
          const f32x4 ov = {oacc[dt][4 * mq] * inv, oacc[dt][4 * mq + 1] * inv, oacc[dt][4 * mq + 2] * inv,
                            oacc[dt][4 * mq + 3] * inv};
          if constexpr (sizeof(T) == 2) *reinterpret_cast<bf16x4*>(orow + d) = bf16x4{(bf16)ov[0], (bf16)ov[1], (bf16)ov[2], (bf16)ov[3]};
          else *reinterpret_cast<f32x4*>(orow + d) = ov;
        }
      if (h == 0 && lse) lse[(int64_t)bh * N + q] = (mc + __log2f(l)) * LN2;
    }
  }
}

// qkv-bias gradient partials of one (b, h): sum this workgroup's rows of dq (or dk, dv)
// -- per lane over its rows, across the 16 lanes of a row group, across the 8 waves
// through LDS (reused after the main loop) -- into out[0..63] (and out[D..] for dk,
// out[2D..] for dv when NOUT = 2).
template <int NOUT>
__device__ __forceinline__ void bias_flush(f32x4 (&c0)[4], f32x4 (*c1)[4], char* smem, float* out, int D) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  float* red = reinterpret_cast<float*>(smem);  // [NOUT][AT_WAVES][64]
  __syncthreads();                              // every wave is done reading the LDS images
#pragma unroll
  for (int o = 0; o < NOUT; ++o) {
    f32x4 (&c)[4] = o == 0 ? c0 : *c1;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = c[dt][t];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if ((lane & 15) == 0) red[(o * AT_WAVES + wave) * 64 + dt * 16 + 4 * g + t] = v;
      }
  }
  __syncthreads();
  if (threadIdx.x < 64 * NOUT) {
    const int o = threadIdx.x >> 6, d = threadIdx.x & 63;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < AT_WAVES; ++w) sum += red[(o * AT_WAVES + w) * 64 + d];
    out[(NOUT == 1 ? 0 : (o + 1) * D) + d] = sum;
  }
}

// Column sums of a 16-row fragment set c[dt][t] (rows = lane & 15, column dt*16 + 4g + t),
// reduced over the 16 rows and kept compressed: lane l ends up owning column
// (l15 >> 2) * 16 + 4g + (l15 & 3), one register instead of sixteen.
__device__ __forceinline__ float colsum16(const f32x4 (&c)[4], int lane) {
  const int l15 = lane & 15;
  float own = 0.f;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = c[dt][t];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (l15 == dt * 4 + t) own = v;
    }
  return own;
}
__device__ __forceinline__ int colsum16_col(int lane) {
  const int l15 = lane & 15;
  return (l15 >> 2) * 16 + 4 * (lane >> 4) + (l15 & 3);
}
// Flush per-lane compressed column sums (own[o] for output o) of the 8 waves into out.
template <int NOUT>
__device__ __forceinline__ void bias_flush_c(const float (&own)[NOUT], char* smem, float* out, int D) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* red = reinterpret_cast<float*>(smem);  // [NOUT][AT_WAVES][64]
  __syncthreads();                              // every wave is done reading the LDS images
#pragma unroll
  for (int o = 0; o < NOUT; ++o) red[(o * AT_WAVES + wave) * 64 + colsum16_col(lane)] = own[o];
  __syncthreads();
  if (threadIdx.x < 64 * NOUT) {
    const int o = threadIdx.x >> 6, d = threadIdx.x & 63;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < AT_WAVES; ++w) sum += red[(o * AT_WAVES + w) * 64 + d];
    out[(NOUT == 1 ? 0 : (o + 1) * D) + d] = sum;
  }
}

// ---------------------------------------------------------------------------
// bf16 backward, two kernels per (b, h) so each holds only half the head in LDS
// (57 KiB -> two workgroups per CU); N > 224 (CLIP ViT-L/14's 257 tokens), else attn_bwd_fused:
//   attn_bwd_dq  : LDS K, V; each wave owns query tiles (Q, dO, O from global),
//                  computes delta = rowsum(dO*O) (written for the other kernel),
//                  recomputes S^T, dP^T over all keys, accumulates dQ.
//   attn_bwd_dkv : LDS Q, dO (+ lse, delta); each wave owns key tiles (K, V from
//                  global), recomputes S, dP over all queries, accumulates dK, dV.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(AT_THREADS, 4) void attn_bwd_dq(const bf16* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                            int N, float scale, const bf16* __restrict__ o,
                                                            int64_t ld_o, const bf16* __restrict__ dout, int64_t ld_do,
                                                            const float* __restrict__ lse, float* __restrict__ delta_out,
                                                            bf16* __restrict__ dqkv, int64_t ld_dqkv,
                                                            float* __restrict__ bias_part, int causal) {
  constexpr int NT2 = (NT + 1) / 2, ROWS = NT2 * 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * ROWS * 128];
  char* Kimg = smem;
  char* Vimg = Kimg + ROWS * 128;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const bf16* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  {
    char* const imgs[2] = {Kimg, Vimg};
    const bf16* const srcs[2] = {base + D, base + 2 * D};
    const int64_t lds_[2] = {ld_qkv, ld_qkv};
    at_load<ROWS, AT_THREADS, 2>(imgs, srcs, lds_, N);
  }
  const AtOffsets off(lane);
  __syncthreads();
  const float c2 = scale * LOG2E;
  f32x4 cs[4];  // column sums of dq (qkv-bias gradient), this lane's rows
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) cs[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int qt = wave; qt < NT; qt += AT_WAVES) {
    const int q = qt * 16 + (lane & 15);
    const int qc = min(q, N - 1);
    bf16x8 qf[2], of[2];
    float dl = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)qc * ld_qkv + kk * 32 + g * 8);
      of[kk] = *reinterpret_cast<const bf16x8*>(dout + ((int64_t)b * N + qc) * ld_do + h * 64 + kk * 32 + g * 8);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(o + ((int64_t)b * N + qc) * ld_o + h * 64 + kk * 32 + g * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) dl = fmaf((float)of[kk][e], (float)ov[e], dl);
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    const float l2 = lse[(int64_t)bh * N + qc] * LOG2E;
    if (g == 0 && q < N) delta_out[(int64_t)bh * N + q] = dl;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kp = 0; kp < NT2; ++kp) {
      f32x4 ds[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kt = 2 * kp + u;
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, dpacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sacc = mfma16(rowf(Kimg, kt * 16, off.row[kk]), qf[kk], sacc);
          dpacc = mfma16(rowf(Vimg, kt * 16, off.row[kk]), of[kk], dpacc);
        }
        const bool edge = (kt + 1) * 16 > N;  // wave-uniform: only the last tiles hold padded keys
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = fexp2(fmaf(sacc[r], c2, -l2));
          if (edge && kt * 16 + 4 * g + r >= N) pv = 0.f;
          if (causal && kt * 16 + 4 * g + r > q) pv = 0.f;
          ds[u][r] = pv * (dpacc[r] - dl);
        }
      }
      const bf16x8 dsf = pack8(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(trf(Kimg, kp * 32, off.tr[dt]), dsf, dq[dt]);
    }
    if (q < N) {
      bf16* row = dqkv + ((int64_t)b * N + q) * ld_dqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 qv = {(bf16)(dq[dt][0] * scale), (bf16)(dq[dt][1] * scale), (bf16)(dq[dt][2] * scale),
                     (bf16)(dq[dt][3] * scale)};
        *reinterpret_cast<bf16x4*>(row + dt * 16 + 4 * g) = qv;
        cs[dt] += dq[dt] * scale;
      }
    }
  }
  if (bias_part) bias_flush<1>(cs, nullptr, smem, bias_part + (int64_t)b * 3 * D + h * 64, D);
}

template <int NT>
__global__ __launch_bounds__(AT_THREADS, 4) void attn_bwd_dkv(const bf16* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                             int N, float scale, const bf16* __restrict__ dout,
                                                             int64_t ld_do, const float* __restrict__ lse,
                                                             const float* __restrict__ delta_in, bf16* __restrict__ dqkv,
                                                             int64_t ld_dqkv, float* __restrict__ bias_part,
                                                             int causal) {
  constexpr int NT2 = (NT + 1) / 2, ROWS = NT2 * 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * ROWS * 128 + 2 * ROWS * 4];
  char* Qimg = smem;
  char* Oimg = Qimg + ROWS * 128;  // dO
  float* lse2 = reinterpret_cast<float*>(Oimg + ROWS * 128);
  float* delta = lse2 + ROWS;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const bf16* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  const bf16* dob = dout + (int64_t)b * N * ld_do + h * 64;
  {
    char* const imgs[2] = {Qimg, Oimg};
    const bf16* const srcs[2] = {base, dob};
    const int64_t lds_[2] = {ld_qkv, ld_do};
    at_load<ROWS, AT_THREADS, 2>(imgs, srcs, lds_, N);
  }
  for (int q = threadIdx.x; q < ROWS; q += AT_THREADS) {
    delta[q] = (q < N) ? delta_in[(int64_t)bh * N + q] : 0.f;
    lse2[q] = (q < N) ? lse[(int64_t)bh * N + q] * LOG2E : INFINITY;
  }
  const AtOffsets off(lane);
  __syncthreads();
  const float c2 = scale * LOG2E;
  float cs[2] = {0.f, 0.f};  // compressed column sums of dk, dv (qkv-bias gradient), colsum16 layout
  for (int kt = wave; kt < NT; kt += AT_WAVES) {
    const int key = kt * 16 + (lane & 15);
    const bool kvalid = key < N;
    const int kc = min(key, N - 1);
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)kc * ld_qkv + D + kk * 32 + g * 8);
      vf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)kc * ld_qkv + 2 * D + kk * 32 + g * 8);
    }
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[dt] = dv[dt]; }
#pragma unroll 1  // unroll 2 spills ~300 VGPRs at the 128-register budget
    for (int qp = 0; qp < NT2; ++qp) {
      f32x4 p[2], ds[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * qp + u;
        f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, dpacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          sacc = mfma16(rowf(Qimg, qt * 16, off.row[kk]), kf[kk], sacc);
          dpacc = mfma16(rowf(Oimg, qt * 16, off.row[kk]), vf[kk], dpacc);
        }
        const f32x4 l2 = *reinterpret_cast<const f32x4*>(lse2 + qt * 16 + 4 * g);
        const f32x4 dl = *reinterpret_cast<const f32x4*>(delta + qt * 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = kvalid ? fexp2(fmaf(sacc[r], c2, -l2[r])) : 0.f;
          if (causal && key > qt * 16 + 4 * g + r) pv = 0.f;
          p[u][r] = pv;
          ds[u][r] = pv * (dpacc[r] - dl[r]);
        }
      }
      const bf16x8 pf = pack8(p[0], p[1]), dsf = pack8(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(trf(Oimg, qp * 32, off.tr[dt]), pf, dv[dt]);
        dk[dt] = mfma16(trf(Qimg, qp * 32, off.tr[dt]), dsf, dk[dt]);
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      dk[dt] = kvalid ? dk[dt] * scale : f32x4{0.f, 0.f, 0.f, 0.f};
      if (!kvalid) dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (kvalid) {
      bf16* row = dqkv + ((int64_t)b * N + key) * ld_dqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 kv = {(bf16)dk[dt][0], (bf16)dk[dt][1], (bf16)dk[dt][2], (bf16)dk[dt][3]};
        bf16x4 vv = {(bf16)dv[dt][0], (bf16)dv[dt][1], (bf16)dv[dt][2], (bf16)dv[dt][3]};
        *reinterpret_cast<bf16x4*>(row + D + dt * 16 + 4 * g) = kv;
        *reinterpret_cast<bf16x4*>(row + 2 * D + dt * 16 + 4 * g) = vv;
      }
    }
    if (bias_part) {  // wave-uniform
      cs[0] += colsum16(dk, lane);
      cs[1] += colsum16(dv, lane);
    }
  }
  if (bias_part) bias_flush_c<2>(cs, smem, bias_part + (int64_t)b * 3 * D + h * 64, D);
}

// ---------------------------------------------------------------------------
// bf16 backward fused into one kernel per (b, h) for N <= 224 (NT <= 14 tiles of 16): one
// workgroup of NT waves, so each wave owns exactly one key tile in phase 1 and one query tile
// in phase 2.  q, k, v, o, dO are read once and S, dP computed once (the two-kernel form
// recomputes both and reads q, k, v, dO twice).
//   prologue: Q, dO -> LDS images; delta = rowsum(dO * O) (O straight from global) and lse -> LDS;
//             wave w holds key tile w's K, V rows in registers.
//   phase 1 : wave w: S, dP of its 16 keys against every query (the attn_bwd_dkv loop) ->
//             dK, dV; dS^T goes to LDS as NT column tiles [key row][16 queries] bf16, the layout
//             the transposed read of phase 2 takes conflict-free (16 rows x 32 B per group).
//   phase 2 : the K tiles replace the Q image; wave w: dQ of its 16 queries = dS K over all keys
//             (A = K^T and B = dS^T from the same transposed-read pattern: same k-slot order).
// LDS at N = 197: 2 x 28 KiB images + 13 x 7 KiB dS^T tiles + lse/delta = 149 KiB (1 WG/CU).
// ---------------------------------------------------------------------------
template <int NT> struct BwdF {
  static constexpr int NT2 = (NT + 1) / 2, ROWS = NT2 * 32, THREADS = NT * 64;
  static constexpr int IMG = ROWS * 128, DST = ROWS * 32;
  static constexpr int LDS = 2 * IMG + NT * DST + 2 * ROWS * 4;
};

template <int NT, bool CAUSAL = false, bool STAMP = false>
__global__ __launch_bounds__(NT * 64, (NT + 3) / 4) void attn_bwd_fused(
    const bf16* __restrict__ qkv, int64_t ld_qkv, int D, int H, int N, float scale, const bf16* __restrict__ o,
    int64_t ld_o, const bf16* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse,
    float* __restrict__ delta_out, bf16* __restrict__ dqkv, int64_t ld_dqkv, float* __restrict__ bias_part,
    unsigned long long* __restrict__ stamps) {
  AT_STAMP_BEGIN()
  using F = BwdF<NT>;
  constexpr int NT2 = F::NT2, ROWS = F::ROWS, NTHR = F::THREADS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qimg = smem;  // Q in phase 1, K in phase 2
  char* Oimg = smem + F::IMG;  // dO
  char* dST = smem + 2 * F::IMG;
  float* lse2 = reinterpret_cast<float*>(dST + NT * F::DST);
  float* delta = lse2 + ROWS;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l15 = lane & 15;
  const bf16* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  const bf16* dob = dout + (int64_t)b * N * ld_do + h * 64;
  const bf16* obase = o + (int64_t)b * N * ld_o + h * 64;

  // ---- prologue: this wave's key tile (registers), Q / dO images, delta, lse
  const int key = wave * 16 + l15;
  const bool kvalid = key < N;
  bf16x8 kf[2], vf[2];
  {
    const int kc = min(key, N - 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)kc * ld_qkv + D + kk * 32 + g * 8);
      vf[kk] = *reinterpret_cast<const bf16x8*>(base + (int64_t)kc * ld_qkv + 2 * D + kk * 32 + g * 8);
    }
  }
  {
    constexpr int TOTAL = ROWS * 8, PER = (TOTAL + NTHR - 1) / NTHR;
    bf16x8 qv[PER], dv8[PER], ov[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * NTHR;
      const int row = min(idx >> 3, N - 1), c = idx & 7;
      if (idx < TOTAL) {
        qv[u] = *reinterpret_cast<const bf16x8*>(base + (int64_t)row * ld_qkv + c * 8);
        dv8[u] = *reinterpret_cast<const bf16x8*>(dob + (int64_t)row * ld_do + c * 8);
        ov[u] = *reinterpret_cast<const bf16x8*>(obase + (int64_t)row * ld_o + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int idx = tid + u * NTHR;
      const int row = idx >> 3, c = idx & 7;
      const bool in = idx < TOTAL, live = in && row < N;
      float dl = 0.f;
      if (live) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dl = fmaf((float)dv8[u][e], (float)ov[u][e], dl);
      }
      // the 8 chunks of a row sit in 8 consecutive lanes (NTHR % 8 == 0): reduce outside the branch
      dl += __shfl_xor(dl, 1, 64);
      dl += __shfl_xor(dl, 2, 64);
      dl += __shfl_xor(dl, 4, 64);
      if (in) {
        bf16x8 qw = qv[u], dw = dv8[u];
        if (!live) {
#pragma unroll
          for (int t = 0; t < 8; ++t) { qw[t] = (bf16)0.f; dw[t] = (bf16)0.f; }
        }
        *reinterpret_cast<bf16x8*>(Qimg + at_off(row, c)) = qw;
        *reinterpret_cast<bf16x8*>(Oimg + at_off(row, c)) = dw;
        if (c == 0) {
          // negated row constants: the initial S / dP accumulators of phase 1
          delta[row] = -dl;
          lse2[row] = live ? -lse[(int64_t)bh * N + row] / scale : -INFINITY;
          if (live) delta_out[(int64_t)bh * N + row] = dl;
        }
      }
    }
    // dS^T rows of the padded keys [NT*16, ROWS) are read by phase 2's last key pair: zero them
    constexpr int PAD = (ROWS - NT * 16) * 32 / 16;  // 16-B chunks per column tile
    if constexpr (PAD > 0) {
      for (int i = tid; i < NT * PAD; i += NTHR) {
        const int t = i / PAD, r = i - t * PAD;
        *reinterpret_cast<f32x4*>(dST + t * F::DST + NT * 16 * 32 + r * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  const AtOffsets off(lane);
  __syncthreads();
  AT_STAMP(1)
  const float c2 = scale * LOG2E;

  // ---- phase 1: wave = key tile
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) { dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[dt] = dv[dt]; }
  char* dsw = dST + key * 32 + g * 8;  // this lane's dS^T slot (queries 4g..4g+3 of a column tile)
#pragma unroll
  for (int qp = 0; qp < NT2; ++qp) {
    f32x4 p[2], ds[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int qt = 2 * qp + u;
      // row constants as the initial accumulators: S' = QK^T - lse/scale (-inf on padded keys),
      // dP' = dO V^T - delta, so p = exp2(c2 S') and dS = p dP' (two VALU ops per element)
      const f32x4 nl = *reinterpret_cast<const f32x4*>(lse2 + qt * 16 + 4 * g);
      f32x4 sacc = kvalid ? nl : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      f32x4 dpacc = *reinterpret_cast<const f32x4*>(delta + qt * 16 + 4 * g);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        sacc = mfma16(rowf(Qimg, qt * 16, off.row[kk]), kf[kk], sacc);
        dpacc = mfma16(rowf(Oimg, qt * 16, off.row[kk]), vf[kk], dpacc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = fexp2(sacc[r] * c2);
        if constexpr (CAUSAL) { if (key > qt * 16 + 4 * g + r) pv = 0.f; }
        p[u][r] = pv;
        ds[u][r] = pv * dpacc[r];
      }
      if (qt < NT) {  // wave-uniform (the padded tile of an odd NT has no column tile)
        const bf16x4 w = {(bf16)ds[u][0], (bf16)ds[u][1], (bf16)ds[u][2], (bf16)ds[u][3]};
        *reinterpret_cast<bf16x4*>(dsw + qt * F::DST) = w;
      }
    }
    const bf16x8 pf = pack8(p[0], p[1]), dsf = pack8(ds[0], ds[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      dv[dt] = mfma16(trf(Oimg, qp * 32, off.tr[dt]), pf, dv[dt]);
      dk[dt] = mfma16(trf(Qimg, qp * 32, off.tr[dt]), dsf, dk[dt]);
    }
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    dk[dt] = kvalid ? dk[dt] * scale : f32x4{0.f, 0.f, 0.f, 0.f};
    if (!kvalid) dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (kvalid) {
    bf16* row = dqkv + ((int64_t)b * N + key) * ld_dqkv + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 kv = {(bf16)dk[dt][0], (bf16)dk[dt][1], (bf16)dk[dt][2], (bf16)dk[dt][3]};
      bf16x4 vv = {(bf16)dv[dt][0], (bf16)dv[dt][1], (bf16)dv[dt][2], (bf16)dv[dt][3]};
      *reinterpret_cast<bf16x4*>(row + D + dt * 16 + 4 * g) = kv;
      *reinterpret_cast<bf16x4*>(row + 2 * D + dt * 16 + 4 * g) = vv;
    }
  }
  float cs[3] = {0.f, 0.f, 0.f};  // compressed column sums of dq, dk, dv (qkv-bias gradient)
  if (bias_part) {
    cs[1] = colsum16(dk, lane);
    cs[2] = colsum16(dv, lane);
  }
  __syncthreads();  // every wave is done with Q, dO and has written its dS^T rows
  AT_STAMP(2)

  // ---- phase 2: K tiles over the Q image (padded rows: zeros), wave = query tile
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 w = kf[kk];
    if (!kvalid) {
#pragma unroll
      for (int t = 0; t < 8; ++t) w[t] = (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(Qimg + at_off(key, kk * 4 + g)) = w;
  }
  __syncthreads();
  AT_STAMP(3)
  {
    const int q = wave * 16 + l15;
    const char* dsr = dST + wave * F::DST + (4 * g + (l15 >> 2)) * 32 + (l15 & 3) * 8;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp = 0; kp < NT2; ++kp) {
      const bf16x8 sf = cat4(lds_read_tr(dsr + kp * 32 * 32), lds_read_tr(dsr + kp * 32 * 32 + 16 * 32));
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(trf(Qimg, kp * 32, off.tr[dt]), sf, dq[dt]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = q < N ? dq[dt] * scale : f32x4{0.f, 0.f, 0.f, 0.f};
    if (q < N) {
      bf16* row = dqkv + ((int64_t)b * N + q) * ld_dqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 qv4 = {(bf16)dq[dt][0], (bf16)dq[dt][1], (bf16)dq[dt][2], (bf16)dq[dt][3]};
        *reinterpret_cast<bf16x4*>(row + dt * 16 + 4 * g) = qv4;
      }
    }
    if (bias_part) cs[0] = colsum16(dq, lane);
  }
  if (bias_part) {  // [3][NT][64] partials through LDS, then one 64-column row per output
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 3; ++t) red[(t * NT + wave) * 64 + colsum16_col(lane)] = cs[t];
    __syncthreads();
    for (int i = tid; i < 3 * 64; i += NTHR) {
      const int t = i >> 6, d = i & 63;
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NT; ++w) sum += red[(t * NT + w) * 64 + d];
      bias_part[(int64_t)b * 3 * D + t * D + h * 64 + d] = sum;
    }
  }
  AT_STAMP(4)
  AT_STAMP_FLUSH()
}

// ---------------------------------------------------------------------------
// f32 forward on v_mfma_f32_16x16x4_f32 (CLIP-HBA at the reference's fp32 precision, NEWP:274;
// config C3): one workgroup (8 waves) per (b, h), K and V of the head in LDS as f32 (<= 2 x 72 KiB,
// N <= 288), wave = query tile of 16.  Products are exact f32 (the MFMA's f32 form), accumulation f32.
//   S^T = K Q^T: A = K (row = key), B = Q^T; the 4 k-slots of lane group g take head dims 16g + ks, so a
//     lane reads 16 consecutive floats of its key row (4 x ds_read_b128) and holds Q[query][16g..16g+15]
//     in registers.  Output: lane (l15, g) holds S[query l15][key 4g + r] -- the bf16 kernel's layout.
//   O^T = V^T P^T: B = P^T straight from the softmax registers (k-slot g at step (kt, r) is key
//     kt*16 + 4g + r, the key the lane already holds); A row m of d-tile dt is head dim 4m + dt, so one
//     ds_read_b128 of V[key][4*l15 .. 4*l15+3] feeds the 4 d-tiles, and a lane ends with
//     O[query l15][16g .. 16g+15].
// K image: 16-B chunk c of row r at chunk position c ^ kswz(r) -- conflict-free for the four
// ds_read_b128 of a key tile (each 16-lane group covers 16 rows and two chunk columns); V image plain
// row-major (a group reads one row and its 4th-next, disjoint banks).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int kswz(int r) {
  const int x = r & 15;
  return x ^ ((((x >> 2) ^ (x >> 3)) & 1) << 2);
}

template <int NT>
__global__ __launch_bounds__(512) void attn_fwd_f32mfma(const float* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                        int N, float scale, float* __restrict__ o, int64_t ld_o,
                                                        float* __restrict__ lse, int causal) {
  constexpr int ROWS = NT * 16, KG = 4;  // key tiles per K-register group
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Kimg = reinterpret_cast<float*>(smem);
  float* Vimg = Kimg + ROWS * 64;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l15 = lane & 15;
  const float* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  // K, V -> LDS (rows >= N zero)
  for (int i = tid; i < ROWS * 16; i += 512) {
    const int r = i >> 4, c = i & 15;
    f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = kv;
    if (r < N) {
      kv = *reinterpret_cast<const f32x4*>(base + (int64_t)r * ld_qkv + D + c * 4);
      vv = *reinterpret_cast<const f32x4*>(base + (int64_t)r * ld_qkv + 2 * D + c * 4);
    }
    *reinterpret_cast<f32x4*>(Kimg + r * 64 + ((c ^ kswz(r)) << 2)) = kv;
    *reinterpret_cast<f32x4*>(Vimg + r * 64 + c * 4) = vv;
  }
  __syncthreads();
  const float c2 = scale * LOG2E;
  for (int qt = wave; qt < NT; qt += 8) {
    const int q = qt * 16 + l15;
    float qf[16];
    {
      const float* qr = base + (int64_t)min(q, N - 1) * ld_qkv + 16 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(qr + 4 * j);
        qf[4 * j] = v[0]; qf[4 * j + 1] = v[1]; qf[4 * j + 2] = v[2]; qf[4 * j + 3] = v[3];
      }
    }
    f32x4 s[NT];
#pragma unroll
    for (int k0 = 0; k0 < NT; k0 += KG) {
      float kf[KG][16];
#pragma unroll
      for (int u = 0; u < KG; ++u) {
        if (k0 + u < NT) {
          const int r = (k0 + u) * 16 + l15;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(Kimg + r * 64 + (((4 * g + j) ^ kswz(r)) << 2));
            kf[u][4 * j] = v[0]; kf[u][4 * j + 1] = v[1]; kf[u][4 * j + 2] = v[2]; kf[u][4 * j + 3] = v[3];
          }
          s[k0 + u] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int ks = 0; ks < 16; ++ks)
#pragma unroll
        for (int u = 0; u < KG; ++u)
          if (k0 + u < NT) s[k0 + u] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[u][ks], qf[ks], s[k0 + u], 0, 0, 0);
    }
    // keys >= N exist only in the last tile
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if ((NT - 1) * 16 + 4 * g + r >= N) s[NT - 1][r] = -INFINITY;
    if (causal) {
#pragma unroll
      for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kt * 16 + 4 * g + r > q) s[kt][r] = -INFINITY;
    }
    float mr[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mr[r] = fmaxf(mr[r], s[kt][r]);
    float m = fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3]));
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float mc = m * c2;
    float lr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) { const float p = fexp2(fmaf(s[kt][r], c2, -mc)); s[kt][r] = p; lr[r] += p; }
    float l = (lr[0] + lr[1]) + (lr[2] + lr[3]);
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    f32x4 oacc[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(Vimg + (kt * 16 + 4 * g + r) * 64 + 4 * l15);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(v[dt], s[kt][r], oacc[dt], 0, 0, 0);
      }
      if (kt % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // bound V-read hoisting (VGPRs)
    }
    if (q < N) {
      const float inv = 1.0f / l;
      float* orow = o + ((int64_t)b * N + q) * ld_o + h * 64 + 16 * g;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        *reinterpret_cast<f32x4*>(orow + 4 * rr) =
            f32x4{oacc[0][rr] * inv, oacc[1][rr] * inv, oacc[2][rr] * inv, oacc[3][rr] * inv};
      if (g == 0 && lse) lse[(int64_t)bh * N + q] = (mc + __log2f(l)) * LN2;
    }
  }
}

// ---------------------------------------------------------------------------
// f32 backward on v_mfma_f32_16x16x4_f32 (N <= 288, head_dim 64), the same operand algebra as the f32
// forward: two kernels, each with two head images in LDS (kswz chunk swizzle, read both by rows -- 4
// ds_read_b128 of 16 consecutive floats -- and by columns -- one ds_read_b128 of chunk l15 of row
// 4g + r, the A operand of the 4 d-tiles whose row m is head dim 4m + dt).
//   dq : wave = query tile, K and V images; S^T and dP^T with the lane's query in registers, so a lane
//        holds keys 4g + r of query l15; dQ^T += K^T dS^T, B = dS^T from registers.  Writes delta.
//   dkv: wave = key tile, Q and dO images; S and dP with the wave's key tile in registers (a lane
//        holds queries 4g + r of key l15); dV^T += dO^T P, dK^T += Q^T dS, B from registers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void f32_img_load(float* img, const float* src, int64_t ld, int N, int rows, int tid,
                                             int nthr) {
  for (int i = tid; i < rows * 16; i += nthr) {
    const int r = i >> 4, c = i & 15;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r < N) v = *reinterpret_cast<const f32x4*>(src + (int64_t)r * ld + c * 4);
    *reinterpret_cast<f32x4*>(img + r * 64 + ((c ^ kswz(r)) << 2)) = v;
  }
}
// row r of a swizzled image: the 16 floats [16g, 16g + 16) (4 chunks)
__device__ __forceinline__ void f32_row16(const float* img, int r, int g, float (&x)[16]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * 64 + (((4 * g + j) ^ kswz(r)) << 2));
    x[4 * j] = v[0]; x[4 * j + 1] = v[1]; x[4 * j + 2] = v[2]; x[4 * j + 3] = v[3];
  }
}
__device__ __forceinline__ f32x4 f32_chunk(const float* img, int r, int c) {
  return *reinterpret_cast<const f32x4*>(img + r * 64 + ((c ^ kswz(r)) << 2));
}
__device__ __forceinline__ void f32_glob16(const float* p, float (&x)[16]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p + 4 * j);
    x[4 * j] = v[0]; x[4 * j + 1] = v[1]; x[4 * j + 2] = v[2]; x[4 * j + 3] = v[3];
  }
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int NT>
__global__ __launch_bounds__(512) void attn_bwd_dq_f32mfma(const float* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                           int N, float scale, const float* __restrict__ o, int64_t ld_o,
                                                           const float* __restrict__ dout, int64_t ld_do,
                                                           const float* __restrict__ lse, float* __restrict__ delta_out,
                                                           float* __restrict__ dqkv, int64_t ld_dqkv, int causal) {
  constexpr int ROWS = NT * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Kimg = reinterpret_cast<float*>(smem);
  float* Vimg = Kimg + ROWS * 64;
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l15 = lane & 15;
  const float* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  f32_img_load(Kimg, base + D, ld_qkv, N, ROWS, tid, 512);
  f32_img_load(Vimg, base + 2 * D, ld_qkv, N, ROWS, tid, 512);
  __syncthreads();
  const float c2 = scale * LOG2E;
  for (int qt = wave; qt < NT; qt += 8) {
    const int q = qt * 16 + l15, qc = min(q, N - 1);
    float qf[16], df[16], of[16];
    f32_glob16(base + (int64_t)qc * ld_qkv + 16 * g, qf);
    f32_glob16(dout + ((int64_t)b * N + qc) * ld_do + h * 64 + 16 * g, df);
    f32_glob16(o + ((int64_t)b * N + qc) * ld_o + h * 64 + 16 * g, of);
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) dl = fmaf(df[j], of[j], dl);
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    if (q < N && g == 0) delta_out[(int64_t)bh * N + q] = dl;
    const float l2 = q < N ? lse[(int64_t)bh * N + q] * LOG2E : INFINITY;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kt = 0; kt < NT; ++kt) {
      float kf[16], vf[16];
      f32_row16(Kimg, kt * 16 + l15, g, kf);
      f32_row16(Vimg, kt * 16 + l15, g, vf);
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = st;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        st = mfma4(kf[ks], qf[ks], st);   // S^T[key 4g + r][query l15]
        dpt = mfma4(vf[ks], df[ks], dpt);
      }
      f32x4 ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 16 + 4 * g + r;
        float p = key < N ? fexp2(fmaf(st[r], c2, -l2)) : 0.f;
        if (causal && key > q) p = 0.f;
        ds[r] = p * (dpt[r] - dl);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x4 a = f32_chunk(Kimg, kt * 16 + 4 * g + r, l15);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma4(a[dt], ds[r], dq[dt]);
      }
    }
    if (q < N) {
      float* row = dqkv + ((int64_t)b * N + q) * ld_dqkv + h * 64 + 16 * g;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        *reinterpret_cast<f32x4*>(row + 4 * rr) =
            f32x4{dq[0][rr] * scale, dq[1][rr] * scale, dq[2][rr] * scale, dq[3][rr] * scale};
    }
  }
}

template <int NT>
__global__ __launch_bounds__(512) void attn_bwd_dkv_f32mfma(const float* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                            int N, float scale, const float* __restrict__ dout,
                                                            int64_t ld_do, const float* __restrict__ lse,
                                                            const float* __restrict__ delta, float* __restrict__ dqkv,
                                                            int64_t ld_dqkv, int causal) {
  constexpr int ROWS = NT * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Qimg = reinterpret_cast<float*>(smem);
  float* Oimg = Qimg + ROWS * 64;  // dO
  float* l2s = Oimg + ROWS * 64;   // lse * log2(e) per query (+inf past N)
  float* dls = l2s + ROWS;         // delta per query
  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l15 = lane & 15;
  const float* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  f32_img_load(Qimg, base, ld_qkv, N, ROWS, tid, 512);
  f32_img_load(Oimg, dout + (int64_t)b * N * ld_do + h * 64, ld_do, N, ROWS, tid, 512);
  for (int i = tid; i < ROWS; i += 512) {
    l2s[i] = i < N ? lse[(int64_t)bh * N + i] * LOG2E : INFINITY;
    dls[i] = i < N ? delta[(int64_t)bh * N + i] : 0.f;
  }
  __syncthreads();
  const float c2 = scale * LOG2E;
  for (int kt = wave; kt < NT; kt += 8) {
    const int key = kt * 16 + l15, kc = min(key, N - 1);
    const bool kvalid = key < N;
    float kf[16], vf[16];
    f32_glob16(base + (int64_t)kc * ld_qkv + D + 16 * g, kf);
    f32_glob16(base + (int64_t)kc * ld_qkv + 2 * D + 16 * g, vf);
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }
#pragma unroll 1
    for (int qt = 0; qt < NT; ++qt) {
      float qf[16], df[16];
      f32_row16(Qimg, qt * 16 + l15, g, qf);
      f32_row16(Oimg, qt * 16 + l15, g, df);
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dpc = sc;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        sc = mfma4(qf[ks], kf[ks], sc);   // S[query 4g + r][key l15]
        dpc = mfma4(df[ks], vf[ks], dpc);
      }
      const f32x4 l2 = *reinterpret_cast<const f32x4*>(l2s + qt * 16 + 4 * g);
      const f32x4 dl = *reinterpret_cast<const f32x4*>(dls + qt * 16 + 4 * g);
      f32x4 p, ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = kvalid ? fexp2(fmaf(sc[r], c2, -l2[r])) : 0.f;
        if (causal && key > qt * 16 + 4 * g + r) pv = 0.f;
        p[r] = pv;
        ds[r] = pv * (dpc[r] - dl[r]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f32x4 ao = f32_chunk(Oimg, qt * 16 + 4 * g + r, l15), aq = f32_chunk(Qimg, qt * 16 + 4 * g + r, l15);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[dt] = mfma4(ao[dt], p[r], dv[dt]);
          dk[dt] = mfma4(aq[dt], ds[r], dk[dt]);
        }
      }
    }
    if (kvalid) {
      float* row = dqkv + ((int64_t)b * N + key) * ld_dqkv + h * 64 + 16 * g;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        *reinterpret_cast<f32x4*>(row + D + 4 * rr) =
            f32x4{dk[0][rr] * scale, dk[1][rr] * scale, dk[2][rr] * scale, dk[3][rr] * scale};
        *reinterpret_cast<f32x4*>(row + 2 * D + 4 * rr) = f32x4{dv[0][rr], dv[1][rr], dv[2][rr], dv[3][rr]};
      }
    }
  }
}

// ---------------------------------------------------------------------------
// generic (f32 compute, f32 or bf16 storage) path: 4 lanes per query / key,
// each owning 16 of the 64 head dims; keys / queries streamed through LDS.
// ---------------------------------------------------------------------------
constexpr int GCH = 64;  // rows per LDS chunk

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_generic(const T* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                        int N, float scale, T* __restrict__ o, int64_t ld_o,
                                                        float* __restrict__ lse, int causal) {
  __shared__ float Ks[GCH][65], Vs[GCH][65];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, qi = blockIdx.x * 64 + (t >> 2), u = t & 3;
  const T* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  float qv[16], acc[16];
  const bool valid = qi < N;
#pragma unroll
  for (int d = 0; d < 16; ++d) { qv[d] = valid ? (float)base[(int64_t)qi * ld_qkv + u * 16 + d] * scale : 0.f; acc[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < N; j0 += GCH) {
    __syncthreads();
    for (int idx = t; idx < GCH * 64; idx += 256) {
      int r = idx >> 6, d = idx & 63, j = j0 + r;
      Ks[r][d] = j < N ? (float)base[(int64_t)j * ld_qkv + D + d] : 0.f;
      Vs[r][d] = j < N ? (float)base[(int64_t)j * ld_qkv + 2 * D + d] : 0.f;
    }
    __syncthreads();
    const int jn = min(GCH, N - j0);
    for (int r = 0; r < jn; ++r) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) s = fmaf(qv[d], Ks[r][u * 16 + d], s);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if (causal && j0 + r > qi) s = -INFINITY;  // key 0 comes first, so m is finite from then on
      float mn = fmaxf(m, s);
      float corr = __expf(m - mn), p = __expf(s - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] = acc[d] * corr + p * Vs[r][u * 16 + d];
      m = mn;
    }
  }
  if (!valid) return;
  const float inv = 1.f / l;
  T* orow = o + ((int64_t)b * N + qi) * ld_o + h * 64 + u * 16;
#pragma unroll
  for (int d = 0; d < 16; ++d) orow[d] = (T)(acc[d] * inv);
  if (u == 0) lse[(int64_t)bh * N + qi] = m + logf(l);
}

// q-parallel: delta_i = dO_i . O_i ; dQ_i = scale * sum_j p_ij (dO_i.v_j - delta_i) k_j
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_dq_generic(const T* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                           int N, float scale, const T* __restrict__ o,
                                                           int64_t ld_o, const T* __restrict__ dout, int64_t ld_do,
                                                           const float* __restrict__ lse, float* __restrict__ delta_out,
                                                           T* __restrict__ dqkv, int64_t ld_dqkv, int causal) {
  __shared__ float Ks[GCH][65], Vs[GCH][65];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, qi = blockIdx.x * 64 + (t >> 2), u = t & 3;
  const T* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  const bool valid = qi < N;
  float qv[16], dov[16], acc[16];
  float dl = 0.f;
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    qv[d] = valid ? (float)base[(int64_t)qi * ld_qkv + u * 16 + d] * scale : 0.f;
    dov[d] = valid ? (float)dout[((int64_t)b * N + qi) * ld_do + h * 64 + u * 16 + d] : 0.f;
    float ov = valid ? (float)o[((int64_t)b * N + qi) * ld_o + h * 64 + u * 16 + d] : 0.f;
    dl = fmaf(dov[d], ov, dl);
    acc[d] = 0.f;
  }
  dl += __shfl_xor(dl, 1, 64);
  dl += __shfl_xor(dl, 2, 64);
  const float L = valid ? lse[(int64_t)bh * N + qi] : 0.f;
  for (int j0 = 0; j0 < N; j0 += GCH) {
    __syncthreads();
    for (int idx = t; idx < GCH * 64; idx += 256) {
      int r = idx >> 6, d = idx & 63, j = j0 + r;
      Ks[r][d] = j < N ? (float)base[(int64_t)j * ld_qkv + D + d] : 0.f;
      Vs[r][d] = j < N ? (float)base[(int64_t)j * ld_qkv + 2 * D + d] : 0.f;
    }
    __syncthreads();
    const int jn = min(GCH, N - j0);
    for (int r = 0; r < jn; ++r) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) { s = fmaf(qv[d], Ks[r][u * 16 + d], s); dp = fmaf(dov[d], Vs[r][u * 16 + d], dp); }
      s += __shfl_xor(s, 1, 64); s += __shfl_xor(s, 2, 64);
      dp += __shfl_xor(dp, 1, 64); dp += __shfl_xor(dp, 2, 64);
      float ds = (causal && j0 + r > qi) ? 0.f : __expf(s - L) * (dp - dl);
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] = fmaf(ds, Ks[r][u * 16 + d], acc[d]);
    }
  }
  if (!valid) return;
  if (u == 0) delta_out[(int64_t)bh * N + qi] = dl;
  T* row = dqkv + ((int64_t)b * N + qi) * ld_dqkv + h * 64 + u * 16;
#pragma unroll
  for (int d = 0; d < 16; ++d) row[d] = (T)(acc[d] * scale);
}

// key-parallel: dV_j = sum_i p_ij dO_i ; dK_j = scale * sum_i ds_ij q_i
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_dkv_generic(const T* __restrict__ qkv, int64_t ld_qkv, int D, int H,
                                                            int N, float scale, const T* __restrict__ dout,
                                                            int64_t ld_do, const float* __restrict__ lse,
                                                            const float* __restrict__ delta, T* __restrict__ dqkv,
                                                            int64_t ld_dqkv, int causal) {
  __shared__ float Qs[GCH][65], Os[GCH][65];
  __shared__ float Ls[GCH], Dl[GCH];
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int t = threadIdx.x, kj = blockIdx.x * 64 + (t >> 2), u = t & 3;
  const T* base = qkv + (int64_t)b * N * ld_qkv + h * 64;
  const bool valid = kj < N;
  float kv[16], vv[16], dk[16], dv[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    kv[d] = valid ? (float)base[(int64_t)kj * ld_qkv + D + u * 16 + d] : 0.f;
    vv[d] = valid ? (float)base[(int64_t)kj * ld_qkv + 2 * D + u * 16 + d] : 0.f;
    dk[d] = 0.f; dv[d] = 0.f;
  }
  for (int i0 = 0; i0 < N; i0 += GCH) {
    __syncthreads();
    for (int idx = t; idx < GCH * 64; idx += 256) {
      int r = idx >> 6, d = idx & 63, i = i0 + r;
      Qs[r][d] = i < N ? (float)base[(int64_t)i * ld_qkv + d] : 0.f;
      Os[r][d] = i < N ? (float)dout[((int64_t)b * N + i) * ld_do + h * 64 + d] : 0.f;
    }
    if (t < GCH) {
      int i = i0 + t;
      Ls[t] = i < N ? lse[(int64_t)bh * N + i] : 0.f;
      Dl[t] = i < N ? delta[(int64_t)bh * N + i] : 0.f;
    }
    __syncthreads();
    const int in = min(GCH, N - i0);
    for (int r = 0; r < in; ++r) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) { s = fmaf(Qs[r][u * 16 + d], kv[d], s); dp = fmaf(Os[r][u * 16 + d], vv[d], dp); }
      s += __shfl_xor(s, 1, 64); s += __shfl_xor(s, 2, 64);
      dp += __shfl_xor(dp, 1, 64); dp += __shfl_xor(dp, 2, 64);
      float p = (causal && kj > i0 + r) ? 0.f : __expf(s * scale - Ls[r]);
      float ds = p * (dp - Dl[r]);
#pragma unroll
      for (int d = 0; d < 16; ++d) { dv[d] = fmaf(p, Os[r][u * 16 + d], dv[d]); dk[d] = fmaf(ds, Qs[r][u * 16 + d], dk[d]); }
    }
  }
  if (!valid) return;
  T* row = dqkv + ((int64_t)b * N + kj) * ld_dqkv + h * 64 + u * 16;
#pragma unroll
  for (int d = 0; d < 16; ++d) { row[D + d] = (T)(dk[d] * scale); row[2 * D + d] = (T)dv[d]; }
}

// delta[(b*H + h)*N + n] = sum_d dO[b*N+n][h*64+d] * O[b*N+n][h*64+d]; 16 lanes
// per (row, head), 4 dims per lane (8-B loads), shuffle-reduced.
template <typename T>
__global__ __launch_bounds__(256) void attn_delta_kernel(const T* __restrict__ o, int64_t ld_o,
                                                         const T* __restrict__ dout, int64_t ld_do, int B, int H,
                                                         int N, float* __restrict__ delta) {
  const int64_t pair = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int l = threadIdx.x & 15;
  const bool ok = pair < (int64_t)B * N * H;
  float s = 0.f;
  int64_t row = 0;
  int h = 0;
  if (ok) {
    row = pair / H;
    h = (int)(pair - row * H);
    const T* op = o + row * ld_o + h * 64 + l * 4;
    const T* dp = dout + row * ld_do + h * 64 + l * 4;
#pragma unroll
    for (int t = 0; t < 4; ++t) s = fmaf((float)op[t], (float)dp[t], s);
  }
#pragma unroll
  for (int m = 8; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (ok && l == 0) {
    const int b = (int)(row / N), n = (int)(row - (int64_t)b * N);
    delta[((int64_t)b * H + h) * N + n] = s;
  }
}

// ---------------------------------------------------------------------------
template <int NT>
static int fwd_mfma(const void* qkv, int64_t ld_qkv, int D, int B, int H, int N, float scale, int causal, void* o,
                    int64_t ld_o, float* lse, hipStream_t s) {
  // the causal mask is a compile-time choice: as a runtime flag its per-score compares and selects
  // stayed in the unmasked kernel's softmax loop (≈130 of ≈400 VALU instructions per query tile)
  if (causal)
    hipLaunchKernelGGL((attn_fwd_mfma<NT, false, true>), dim3(B * H), dim3(AT_THREADS), 0, s, (const bf16*)qkv, ld_qkv,
                       D, H, N, scale, (bf16*)o, ld_o, lse, causal, nullptr);
  else if (g_attn_stamps)
    hipLaunchKernelGGL((attn_fwd_mfma<NT, true>), dim3(B * H), dim3(AT_THREADS), 0, s, (const bf16*)qkv, ld_qkv, D, H,
                       N, scale, (bf16*)o, ld_o, lse, causal, g_attn_stamps);
  else
    hipLaunchKernelGGL((attn_fwd_mfma<NT>), dim3(B * H), dim3(AT_THREADS), 0, s, (const bf16*)qkv, ld_qkv, D, H, N,
                       scale, (bf16*)o, ld_o, lse, causal, nullptr);
  VIT_CHECK_LAUNCH();
  return 0;
}
// VIT_ATTN_F32_GENERIC=1: the scalar-FMA f32 forward instead of the f32 MFMA kernel (A/B runs)
static bool attn_f32_generic() {
  static const int v = [] { const char* e = getenv("VIT_ATTN_F32_GENERIC"); return e && *e == '1' ? 1 : 0; }();
  return v != 0;
}
template <int NT>
static int fwd_f32mfma(const void* qkv, int64_t ld_qkv, int D, int B, int H, int N, float scale, int causal, void* o,
                       int64_t ld_o, float* lse, hipStream_t s) {
  constexpr int lds = 2 * NT * 16 * 64 * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_f32mfma<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL((attn_fwd_f32mfma<NT>), dim3(B * H), dim3(512), lds, s, (const float*)qkv, ld_qkv, D, H, N, scale,
                     (float*)o, ld_o, lse, causal);
  VIT_CHECK_LAUNCH();
  return 0;
}
template <int NT>
static int bwd_f32mfma(const void* qkv, int64_t ld_qkv, int D, int B, int H, int N, float scale, int causal,
                       const void* o, int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, float* delta,
                       void* dqkv, int64_t ld_dqkv, hipStream_t s) {
  constexpr int img = NT * 16 * 64 * 4, lds_dq = 2 * img, lds_dkv = 2 * img + 2 * NT * 16 * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq_f32mfma<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_dq);
    (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_f32mfma<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_dkv);
    attr = true;
  }
  hipLaunchKernelGGL((attn_bwd_dq_f32mfma<NT>), dim3(B * H), dim3(512), lds_dq, s, (const float*)qkv, ld_qkv, D, H, N,
                     scale, (const float*)o, ld_o, (const float*)dout, ld_do, lse, delta, (float*)dqkv, ld_dqkv, causal);
  VIT_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_dkv_f32mfma<NT>), dim3(B * H), dim3(512), lds_dkv, s, (const float*)qkv, ld_qkv, D, H,
                     N, scale, (const float*)dout, ld_do, lse, (const float*)delta, (float*)dqkv, ld_dqkv, causal);
  VIT_CHECK_LAUNCH();
  return 0;
}
// VIT_ATTN_BWD_SPLIT=1 keeps the two-kernel backward for every N (A/B runs)
// bf16 backward form for N <= 224 (vit_sdpa_bwd_variant / VIT_ATTN_BWD_SPLIT=1, A/B): 1 = whole-head fused
// (the default), 2 = the two kernels.  (Round 4's banded-query form measured 0.276 vs 0.248 ms standalone
// and -0.8 % in the step, profiles/r04/ab_attn_bwd_band.txt, and was removed in round 5.)
static int g_bwd_variant = -1;
static bool attn_bwd_split() {
  if (g_bwd_variant == 2) return true;
  static const int v = [] { const char* e = getenv("VIT_ATTN_BWD_SPLIT"); return e && *e == '1' ? 1 : 0; }();
  return v != 0;
}

template <int NT>
static int bwd_mfma(const void* qkv, int64_t ld_qkv, int D, int B, int H, int N, float scale, int causal, const void* o,
                    int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, float* delta,
                    void* dqkv, int64_t ld_dqkv, float* bias_part, hipStream_t s) {
  if constexpr (NT <= 14) {
    if (!attn_bwd_split()) {
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)attn_bwd_fused<NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  BwdF<NT>::LDS);
        (void)hipFuncSetAttribute((const void*)attn_bwd_fused<NT, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  BwdF<NT>::LDS);
        (void)hipFuncSetAttribute((const void*)attn_bwd_fused<NT, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, BwdF<NT>::LDS);
        attr = true;
      }
#define BWD_FUSED(C, S, ST)                                                                                    \
  hipLaunchKernelGGL((attn_bwd_fused<NT, C, S>), dim3(B * H), dim3(BwdF<NT>::THREADS), BwdF<NT>::LDS, s,         \
                     (const bf16*)qkv, ld_qkv, D, H, N, scale, (const bf16*)o, ld_o, (const bf16*)dout, ld_do, lse, \
                     delta, (bf16*)dqkv, ld_dqkv, bias_part, ST)
      if (causal)
        BWD_FUSED(true, false, nullptr);
      else if (g_attn_stamps)
        BWD_FUSED(false, true, g_attn_stamps);
      else
        BWD_FUSED(false, false, nullptr);
#undef BWD_FUSED
      VIT_CHECK_LAUNCH();
      return 0;
    }
  }
  hipLaunchKernelGGL((attn_bwd_dq<NT>), dim3(B * H), dim3(AT_THREADS), 0, s, (const bf16*)qkv, ld_qkv, D, H, N, scale,
                     (const bf16*)o, ld_o, (const bf16*)dout, ld_do, lse, delta, (bf16*)dqkv, ld_dqkv, bias_part, causal);
  VIT_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_dkv<NT>), dim3(B * H), dim3(AT_THREADS), 0, s, (const bf16*)qkv, ld_qkv, D, H, N, scale,
                     (const bf16*)dout, ld_do, lse, (const float*)delta, (bf16*)dqkv, ld_dqkv, bias_part, causal);
  VIT_CHECK_LAUNCH();
  return 0;
}

#define NT_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18)

extern "C" {

// diagnostic only (tools/attn_stamps.py): phase stamps of the bf16 forward / fused backward
// kernels go to buf ([B*H][8] u64) until called again with null; not part of include/vit_hip.h
int vit_debug_attn_stamps(void* buf) {
  g_attn_stamps = (unsigned long long*)buf;
  return 0;
}

// Tuning hook: the bf16 backward form (-1 = from the environment, 1 = whole-head fused (the default),
// 2 = two kernels; they agree to bf16 rounding).  0 (round 4's banded form) is gone.
int vit_sdpa_bwd_variant(int v) {
  if (v == 0 || v > 2) return (int)hipErrorInvalidValue;
  g_bwd_variant = v < 0 ? -1 : v;
  return 0;
}

// F.scaled_dot_product_attention(q, k, v) (no dropout) for head_dim 64; causal = 1
// masks key > query (OpenAI CLIP text tower attn_mask, additive -inf above the diagonal).
// qkv: [B*N, ld_qkv] with q at column h*64, k at D + h*64, v at 2D + h*64.
// o: [B*N, ld_o] (column h*64); lse: [B*H*N] f32 (natural-log, scaled scores).
int vit_sdpa_fwd(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, void* o,
                 int64_t ld_o, float* lse, float scale, int causal, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (head_dim != 64 || N <= 0 || N > 288) return (int)hipErrorInvalidValue;
  const int D = H * 64;
  if (dtype == VIT_BF16 && (ld_qkv % 8 == 0) && (ld_o % 4 == 0)) {
    int nt = (N + 15) / 16;
    switch (nt) {
#define CASE(n) case n: return fwd_mfma<n>(qkv, ld_qkv, D, B, H, N, scale, causal, o, ld_o, lse, s);
      NT_CASES(CASE)
#undef CASE
    }
  }
  if (dtype == VIT_F32 && (ld_qkv % 4 == 0) && (ld_o % 4 == 0) && !attn_f32_generic()) {
    int nt = (N + 15) / 16;
    switch (nt) {
#define CASE(n) case n: return fwd_f32mfma<n>(qkv, ld_qkv, D, B, H, N, scale, causal, o, ld_o, lse, s);
      NT_CASES(CASE)
#undef CASE
    }
  }
  dim3 grid((N + 63) / 64, B * H);
  if (dtype == VIT_BF16)
    hipLaunchKernelGGL(attn_fwd_generic<bf16>, grid, dim3(256), 0, s, (const bf16*)qkv, ld_qkv, D, H, N, scale, (bf16*)o, ld_o, lse, causal);
  else
    hipLaunchKernelGGL(attn_fwd_generic<float>, grid, dim3(256), 0, s, (const float*)qkv, ld_qkv, D, H, N, scale, (float*)o, ld_o, lse, causal);
  VIT_CHECK_LAUNCH();
  return 0;
}

// fp8 (block-scaled OCP e4m3) forward, head_dim 64, N <= 320: see attn_fwd_fp8.  qkv / o bf16
// or f32 (dtype; quantised to e4m3 inside the kernel either way); lse f32 or null.
int vit_sdpa_fwd_fp8(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, void* o,
                     int64_t ld_o, float* lse, float scale, int causal, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (head_dim != 64 || N <= 0 || N > 320 || (ld_qkv % 8) || (ld_o % 4)) return (int)hipErrorInvalidValue;
  const int D = H * 64;
  switch ((N + 63) / 64) {
#define F8(n)                                                                                                   \
  case n:                                                                                                       \
    if (dtype == VIT_BF16)                                                                                      \
      hipLaunchKernelGGL((attn_fwd_fp8<n, bf16>), dim3(B * H), dim3(F8_THREADS), 0, s, (const bf16*)qkv, ld_qkv, \
                         D, H, N, scale, (bf16*)o, ld_o, lse, causal);                                          \
    else                                                                                                        \
      hipLaunchKernelGGL((attn_fwd_fp8<n, float>), dim3(B * H), dim3(F8_THREADS), 0, s, (const float*)qkv,      \
                         ld_qkv, D, H, N, scale, (float*)o, ld_o, lse, causal);                                 \
    break;
    F8(1) F8(2) F8(3) F8(4) F8(5)
#undef F8
  }
  VIT_CHECK_LAUNCH();
  return 0;
}

// SDPA backward: writes dq/dk/dv into dqkv (same column layout as qkv).
// `delta_ws` (>= B*H*N floats) receives rowsum(dO*O) per (b, h, n).
// dbias (optional, [3D] f32) = column sums of dqkv (the qkv Linear's bias gradient);
// needs `partial` >= vit_sdpa_bwd_partial_floats(B, N, D) floats.
int vit_sdpa_bwd_partial_floats(int B, int N, int D) {
  const int64_t C = 3 * (int64_t)D;
  const int64_t mfma = B * C + (B > 64 ? (int64_t)((B + 63) / 64) * C : 0);
  const int64_t gen = 256 * C + 4 * C;  // vit_colsum on the generic path
  return (int)(mfma > gen ? mfma : gen);
}

int vit_sdpa_bwd(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, const void* o,
                 int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, void* dqkv, int64_t ld_dqkv,
                 float* delta_ws, float scale, int causal, float* dbias, float* partial, int64_t partial_floats,
                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (head_dim != 64 || N <= 0 || N > 288) return (int)hipErrorInvalidValue;
  const int D = H * 64;
  if (!delta_ws) return (int)hipErrorInvalidValue;
  // dbias == null with a partial buffer: leave the per-image [B][3D] partials for the caller (bf16 path)
  const bool part_only = !dbias && partial;
  if ((dbias || part_only) && (partial == nullptr || partial_floats < vit_sdpa_bwd_partial_floats(B, N, D)))
    return (int)hipErrorInvalidValue;
  const bool mfma_ok = dtype == VIT_BF16 && (ld_qkv % 8 == 0) && (ld_do % 8 == 0) && (ld_dqkv % 4 == 0) && (ld_o % 4 == 0);
  if (part_only && !mfma_ok) return (int)hipErrorInvalidValue;
  if (mfma_ok) {
    int nt = (N + 15) / 16;
    int rc = (int)hipErrorInvalidValue;
    switch (nt) {
#define CASE(n) case n: rc = bwd_mfma<n>(qkv, ld_qkv, D, B, H, N, scale, causal, o, ld_o, dout, ld_do, lse, delta_ws, dqkv, ld_dqkv, (dbias || part_only) ? partial : nullptr, s); break;
      NT_CASES(CASE)
#undef CASE
    }
    if (rc || !dbias) return rc;
    launch_colreduce(partial, B, 3 * D, dbias, 0, s, partial + (int64_t)B * 3 * D);
    VIT_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == VIT_F32 && (ld_qkv % 4 == 0) && (ld_do % 4 == 0) && (ld_dqkv % 4 == 0) && (ld_o % 4 == 0) &&
      !attn_f32_generic()) {
    int nt = (N + 15) / 16, rc = (int)hipErrorInvalidValue;
    switch (nt) {
#define CASE(n) case n: rc = bwd_f32mfma<n>(qkv, ld_qkv, D, B, H, N, scale, causal, o, ld_o, dout, ld_do, lse, delta_ws, dqkv, ld_dqkv, s); break;
      NT_CASES(CASE)
#undef CASE
    }
    if (rc) return rc;
    if (dbias) return vit_colsum(dtype, B * N, 3 * D, dqkv, ld_dqkv, dbias, partial, partial_floats, 0, stream);
    return 0;
  }
  dim3 grid((N + 63) / 64, B * H);
#define GEN(T)                                                                                               \
  hipLaunchKernelGGL(attn_bwd_dq_generic<T>, grid, dim3(256), 0, s, (const T*)qkv, ld_qkv, D, H, N, scale,    \
                     (const T*)o, ld_o, (const T*)dout, ld_do, lse, delta_ws, (T*)dqkv, ld_dqkv, causal);    \
  VIT_CHECK_LAUNCH();                                                                                        \
  hipLaunchKernelGGL(attn_bwd_dkv_generic<T>, grid, dim3(256), 0, s, (const T*)qkv, ld_qkv, D, H, N, scale,   \
                     (const T*)dout, ld_do, lse, delta_ws, (T*)dqkv, ld_dqkv, causal);
  if (dtype == VIT_BF16) { GEN(bf16) } else { GEN(float) }
#undef GEN
  VIT_CHECK_LAUNCH();
  if (dbias) return vit_colsum(dtype, B * N, 3 * D, dqkv, ld_dqkv, dbias, partial, partial_floats, 0, stream);
  return 0;
}

}  // extern "C"
