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
#include "reduce.hpp"
#include <stdlib.h>
#include <string.h>
#include <type_traits>

#include "gemm_lds.hpp"
#include "gemm_epi.hpp"
// build-time switches of the bf16 epilogue forms (A/B builds: -DVIT_PAIR16=0 etc.)
#ifndef VIT_PAIR16
#define VIT_PAIR16 1
#endif
#ifndef VIT_PLAIN16
#define VIT_PLAIN16 1
#endif
#ifndef VIT_GBWD_PREFETCH
#define VIT_GBWD_PREFETCH 1
#endif
#ifndef VIT_SPLIT_ISSUE
#define VIT_SPLIT_ISSUE 1
#endif
#ifndef VIT_SPLIT_ISSUE1
#define VIT_SPLIT_ISSUE1 1
#endif

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
__device__ __forceinline__ f32x4 epi4(const Epi& e, int i, int j, f32x4 v, int z = 0) {
  if (e.bias) {
    f32x4 b = *reinterpret_cast<const f32x4*>(e.bias + j);
    v += b;
  }
  if constexpr (EPI == EPI_STORE) {
    store4<TO>((TO*)e.C + e.slab * z + (int64_t)i * e.ldc + j, v);
    return v;
  } else if constexpr (EPI == EPI_ACC) {
    TO* c = (TO*)e.C + (int64_t)i * e.ldc + j;
    store4<TO>(c, v + load4<TO>(c));
    return v;
  } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
    // act and act' of the pre-activation rounded to the storage type (the value a
    // stored-pre design would have differentiated)
    f32x4 a, d;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float pr = (float)(TO)v[t];
      float ga, gd;
      if constexpr (EPI == EPI_BIAS_GELU) gelu_fast_both(pr, ga, gd);
      else quick_gelu_both(pr, ga, gd);
      a[t] = ga;
      d[t] = gd;
    }
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, d);
    store4<TO>((TO*)e.aux_out + (int64_t)i * e.ldc + j, a);
    return v;
  } else if constexpr (EPI == EPI_RESID) {
    f32x4 r = load4<float>((const float*)e.aux + (int64_t)i * e.ld_aux + j);
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, v + r);
    return v;
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    v *= load4<TA>((const TA*)e.aux + (int64_t)i * e.ld_aux + j);
    store4<TO>((TO*)e.C + (int64_t)i * e.ldc + j, v);
  } else if constexpr (EPI == EPI_PATCH) {
    int b = i / e.n_patch, p = i - b * e.n_patch;
    int64_t row = (int64_t)b * (e.n_patch + 1) + 1 + p;
    f32x4 ps = *reinterpret_cast<const f32x4*>(e.pos + (int64_t)(1 + p) * e.ldc + j);
    store4<TO>((TO*)e.C + row * e.ldc + j, v + ps);
    return v;
  }
  return v;
}



// ---------------------------------------------------------------------------
// Row-contiguous epilogue (the bf16 fast kernels): V = 16 / sizeof(TO) consecutive
// columns j..j+V-1 of row i per thread, so every global load and store is 16 B and
// a wave's instruction covers whole 512-B row segments (the MFMA fragment layout
// gives 8-B pieces of 16 different rows per instruction: store-issue-bound).
// ---------------------------------------------------------------------------
template <int V> struct VecF { f32x4 q[V / 4]; };

template <typename T, int V> __device__ __forceinline__ void vload(const T* p, VecF<V>& v);
template <> __device__ __forceinline__ void vload<float, 4>(const float* p, VecF<4>& v) {
  v.q[0] = *reinterpret_cast<const f32x4*>(p);
}
template <> __device__ __forceinline__ void vload<float, 8>(const float* p, VecF<8>& v) {
  v.q[0] = *reinterpret_cast<const f32x4*>(p);
  v.q[1] = *reinterpret_cast<const f32x4*>(p + 4);
}
template <> __device__ __forceinline__ void vload<bf16, 8>(const bf16* p, VecF<8>& v) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
  v.q[0] = f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
  v.q[1] = f32x4{(float)x[4], (float)x[5], (float)x[6], (float)x[7]};
}
template <> __device__ __forceinline__ void vload<bf16, 4>(const bf16* p, VecF<4>& v) {
  const bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
  v.q[0] = f32x4{(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
}
template <typename T, int V> __device__ __forceinline__ void vstore(T* p, const VecF<V>& v);
template <> __device__ __forceinline__ void vstore<float, 4>(float* p, const VecF<4>& v) {
  *reinterpret_cast<f32x4*>(p) = v.q[0];
}
template <> __device__ __forceinline__ void vstore<bf16, 8>(bf16* p, const VecF<8>& v) {
  const bf16x8 o = {(bf16)v.q[0][0], (bf16)v.q[0][1], (bf16)v.q[0][2], (bf16)v.q[0][3],
                    (bf16)v.q[1][0], (bf16)v.q[1][1], (bf16)v.q[1][2], (bf16)v.q[1][3]};
  *reinterpret_cast<bf16x8*>(p) = o;
}

// Epilogue math on V columns; returns (in v) the value whose column sum a fused
// bias gradient wants (what was stored as C, before a GELU activation).
template <int EPI, typename TO, typename TA, int V>
__device__ __forceinline__ void epi_vec(const Epi& e, int i, int j, VecF<V>& v, int z) {
  if (e.bias) {
    VecF<V> b;
    vload<float, V>(e.bias + j, b);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) v.q[q] += b.q[q];
  }
  if constexpr (EPI == EPI_STORE) {
    vstore<TO, V>((TO*)e.C + e.slab * z + (int64_t)i * e.ldc + j, v);
  } else if constexpr (EPI == EPI_ACC) {
    TO* c = (TO*)e.C + (int64_t)i * e.ldc + j;
    VecF<V> o;
    vload<TO, V>(c, o);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) o.q[q] += v.q[q];
    vstore<TO, V>(c, o);
  } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
    VecF<V> a, d;
#pragma unroll
    for (int q = 0; q < V / 4; ++q)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float pr = (float)(TO)v.q[q][t];  // pre-activation rounded to the storage type
        float ga, gd;
        if constexpr (EPI == EPI_BIAS_GELU) gelu_fast_both(pr, ga, gd);
        else quick_gelu_both(pr, ga, gd);
        a.q[q][t] = ga;
        d.q[q][t] = gd;
      }
    vstore<TO, V>((TO*)e.C + (int64_t)i * e.ldc + j, d);
    vstore<TO, V>((TO*)e.aux_out + (int64_t)i * e.ldc + j, a);
  } else if constexpr (EPI == EPI_RESID) {
    VecF<V> r;
    vload<float, V>((const float*)e.aux + (int64_t)i * e.ld_aux + j, r);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) r.q[q] += v.q[q];
    vstore<TO, V>((TO*)e.C + (int64_t)i * e.ldc + j, r);
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    VecF<V> dact;
    vload<TA, V>((const TA*)e.aux + (int64_t)i * e.ld_aux + j, dact);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) v.q[q] *= dact.q[q];
    vstore<TO, V>((TO*)e.C + (int64_t)i * e.ldc + j, v);
  } else if constexpr (EPI == EPI_PATCH) {
    const int b = i / e.n_patch, p = i - b * e.n_patch;
    const int64_t row = (int64_t)b * (e.n_patch + 1) + 1 + p;
    VecF<V> ps;
    vload<float, V>(e.pos + (int64_t)(1 + p) * e.ldc + j, ps);
#pragma unroll
    for (int q = 0; q < V / 4; ++q) ps.q[q] += v.q[q];
    vstore<TO, V>((TO*)e.C + row * e.ldc + j, ps);
  }
}

// LDS bytes the staged epilogue of a BM x BN tile needs: one WM-row band of f32
// accumulators (rows padded by 16 B) + the column-sum reduction rows.
template <class C, typename TO> struct EpiLds {
  static constexpr int V = 16 / (int)sizeof(TO);
  static constexpr int ROWB = C::BN * 4 + 16;
  static constexpr int CPR = C::BN / V;           // V-column chunks per row
  static constexpr int RL = C::THREADS / CPR;     // rows in flight per sweep
  static constexpr int STAGE = C::WM * ROWB;
  static constexpr int BYTES = STAGE + RL * C::BN * 4;
  static_assert(C::THREADS % CPR == 0 && C::WM % RL == 0 && 64 % RL == 0, "epilogue sweep shape");
};

// bf16 epilogue straight from the MFMA fragments with 16-B stores (no LDS round trip).
// A lane holds C[i][4g..4g+3] of each 16-column fragment (g = lane >> 4).  For a fragment
// pair (b, b+1), one v_permlane16_swap per dword (vdst = fragment b, src = fragment b+1)
// trades lane rows g=1 / g=3 of b with rows g=0 / g=2 of b+1, after which every lane holds 8
// consecutive columns of the pair: g=0 cols 0-7, g=2 8-15, g=1 16-23, g=3 24-31 -- one
// dwordx4 store instead of two dwordx2 (the fragment-layout store tail is issue-bound).
// Needs N % 32 == 0 (whole 8-column groups).
template <int EPI, typename TO, typename TA>
__device__ __forceinline__ f32x4 epi_val(const Epi& e, int i, int j, f32x4 v, bool ok, f32x4& o0, f32x4& o1,
                                         const f32x4& bias4) {
  v += bias4;  // this lane's 4 bias values (zero without bias), loaded once per column fragment
  if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float pr = (float)(TO)v[t];  // pre-activation rounded to the storage type
      float ga, gd;
      if constexpr (EPI == EPI_BIAS_GELU) gelu_fast_both(pr, ga, gd);
      else quick_gelu_both(pr, ga, gd);
      o0[t] = gd;
      o1[t] = ga;
    }
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    v *= ok ? load4<TA>((const TA*)e.aux + (int64_t)i * e.ld_aux + j) : f32x4{0.f, 0.f, 0.f, 0.f};
    o0 = v;
  } else {  // EPI_STORE
    o0 = v;
  }
  return v;
}


template <class C, int EPI, typename TO, typename TA>
__device__ __forceinline__ void epilogue_swap(const Epi& e, const f32x4 (&acc)[C::AI][C::AJ], int i0, int j0, int wi,
                                              int wj, int lane, int M, int N) {
  static_assert(C::AJ % 2 == 0, "fragment pairs");
  constexpr bool two = EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU;
  const int g = lane >> 4;
  const int colsel = (g & 1) * 16 + (g >> 1) * 8;
  f32x4 cs[C::AJ], bias4[C::AJ];
#pragma unroll
  for (int b = 0; b < C::AJ; ++b) {
    cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int j = j0 + wj * C::WN + b * 16 + 4 * g;
    bias4[b] = (e.bias && j < N) ? *reinterpret_cast<const f32x4*>(e.bias + j) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int a = 0; a < C::AI; ++a) {
    const int i = i0 + wi * C::WM + a * 16 + (lane & 15);
    const bool row_ok = i < M;
#pragma unroll
    for (int b = 0; b < C::AJ; b += 2) {
      const int jp = j0 + wj * C::WN + b * 16;
      const int ja = jp + 4 * g, jb = jp + 16 + 4 * g;
      const bool oka = row_ok && ja < N, okb = row_ok && jb < N;
      f32x4 xa, ya, xb, yb;
      const f32x4 va = epi_val<EPI, TO, TA>(e, i, ja, acc[a][b], oka, xa, ya, bias4[b]);
      const f32x4 vb = epi_val<EPI, TO, TA>(e, i, jb, acc[a][b + 1], okb, xb, yb, bias4[b + 1]);
      if (e.csum) {
        if (oka) cs[b] += va;
        if (okb) cs[b + 1] += vb;
      }
      const bool ok = row_ok && jp + colsel < N;
      store_pair_bf16(e.C, e.ldc, i, jp + colsel, xa, xb, ok);
      if constexpr (two) store_pair_bf16(e.aux_out, e.ldc, i, jp + colsel, ya, yb, ok);
    }
    if (e.csum && (a & 3) == 3) csum_flush<C::AJ>(e, cs, i0 + wi * C::WM + (a - 3) * 16, M, N, j0 + wj * C::WN, lane);
  }
}

// Staged epilogue: for each band of WM rows (the waves of one wi), those waves
// write their f32 accumulators to LDS, then the whole workgroup sweeps the band
// row-contiguously through epi_vec.  Column sums (fused bias gradients) are
// reduced over each 64-row group through LDS and written as one partial row.
template <class C, int EPI, typename TO, typename TA>
__device__ __forceinline__ void epilogue_staged(const Epi& e, const f32x4 (&acc)[C::AI][C::AJ], char* smem, int i0,
                                                int j0, int wi, int wj, int lane, int M, int N, int z) {
  using EL = EpiLds<C, TO>;
  constexpr int V = EL::V;
  const int tid = threadIdx.x;
  const int c = tid % EL::CPR, r0 = tid / EL::CPR;
  float* red = reinterpret_cast<float*>(smem + EL::STAGE);
  const int j = j0 + c * V;
  // GELU' input gradient: the act'(pre) rows of band p + 1 (WM/RL rows of 16 B per thread) are loaded
  // before band p's round, so their HBM latency hides under that round instead of stalling the next
  constexpr int NPRE = C::WM / EL::RL;
  constexpr bool PREF = (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) && std::is_same<TA, bf16>::value &&
                        V == 8 && NPRE <= 4 && VIT_GBWD_PREFETCH;
  bf16x8 pre[PREF ? NPRE : 1], pre_next[PREF ? NPRE : 1];
  auto load_pre = [&](int p, bf16x8 (&dst)[PREF ? NPRE : 1]) {
#pragma unroll
    for (int u = 0; u < NPRE; ++u) {
      const int i = i0 + p * C::WM + r0 + u * EL::RL;
      dst[u] = (i < M && j < N) ? *reinterpret_cast<const bf16x8*>((const bf16*)e.aux + (int64_t)i * e.ld_aux + j)
                                : bf16x8{};
    }
  };
  if constexpr (PREF) load_pre(0, pre);
#pragma unroll 1
  for (int p = 0; p < C::WI; ++p) {
    if constexpr (PREF) {
      if (p + 1 < C::WI) load_pre(p + 1, pre_next);
    }
    __syncthreads();  // main-loop fragment reads / the previous band's sweep are done
    if (wi == p) {
#pragma unroll
      for (int a = 0; a < C::AI; ++a)
#pragma unroll
        for (int b = 0; b < C::AJ; ++b) {
          const int row = a * 16 + (lane & 15), col = wj * C::WN + b * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + row * EL::ROWB + col * 4) = acc[a][b];
        }
    }
    __syncthreads();
    const int ib = i0 + p * C::WM;
    VecF<V> cs;
#pragma unroll
    for (int q = 0; q < V / 4; ++q) cs.q[q] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int r = r0; r < C::WM; r += EL::RL) {
      VecF<V> v;
      const float* src = reinterpret_cast<const float*>(smem + r * EL::ROWB) + c * V;
#pragma unroll
      for (int q = 0; q < V / 4; ++q) v.q[q] = *reinterpret_cast<const f32x4*>(src + 4 * q);
      const int i = ib + r;
      if (i < M && j < N) {
        if constexpr (PREF) {  // epi_vec's GELU' branch, with the prefetched act' row
          bf16x8 d8 = pre[0];
#pragma unroll
          for (int u = 1; u < NPRE; ++u)
            if (u == (r - r0) / EL::RL) d8 = pre[u];
#pragma unroll
          for (int q = 0; q < 8; ++q) v.q[q >> 2][q & 3] *= (float)d8[q];
          vstore<TO, V>((TO*)e.C + (int64_t)i * e.ldc + j, v);
        } else {
          epi_vec<EPI, TO, TA, V>(e, i, j, v, z);
        }
        if (e.csum) {
#pragma unroll
          for (int q = 0; q < V / 4; ++q) cs.q[q] += v.q[q];
        }
      }
      if (e.csum && ((r + EL::RL) & 63) < EL::RL) {  // last row of this thread in a 64-row group
        float* rr = red + r0 * C::BN + c * V;
#pragma unroll
        for (int q = 0; q < V / 4; ++q) {
          *reinterpret_cast<f32x4*>(rr + 4 * q) = cs.q[q];
          cs.q[q] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        __syncthreads();
        const int g0 = ib + (r & ~63);
        for (int col = tid; col < C::BN; col += C::THREADS) {
          float sum = 0.f;
#pragma unroll
          for (int k = 0; k < EL::RL; ++k) sum += red[k * C::BN + col];
          if (g0 < M && j0 + col < N) e.csum[(int64_t)(g0 >> 6) * N + j0 + col] = sum;
        }
        __syncthreads();
      }
    }
    if constexpr (PREF) {
#pragma unroll
      for (int u = 0; u < NPRE; ++u) pre[u] = pre_next[u];
    }
  }
}

// GELU pair (bias + act' / act) through a bf16 LDS image of the whole tile: the pair is computed from
// the pre-activation rounded to bf16 anyway, so every wave writes bf16(acc + bias) at once (one
// barrier, half the bytes of the f32 band-by-band staging) and the workgroup then sweeps all BM rows
// row-contiguously (16-B loads / stores).  Bit-identical to epilogue_staged.
template <class C> struct Pair16 {
  static constexpr int PITCH = C::BN * 2 + 16;  // 16-B row pad: a fragment write's 16 rows hit distinct banks
  static constexpr int BYTES = C::BM * PITCH;
};
template <class C, int EPI>
__device__ __forceinline__ void epilogue_pair16(const Epi& e, const f32x4 (&acc)[C::AI][C::AJ], char* smem, int i0,
                                                int j0, int wi, int wj, int lane, int M, int N) {
  constexpr int PITCH = Pair16<C>::PITCH, CPR = C::BN / 8, RL = C::THREADS / CPR;
  static_assert(C::THREADS % CPR == 0, "sweep shape");
  const int tid = threadIdx.x, g = lane >> 4;
  __syncthreads();  // every wave's main-loop fragment reads are done
#pragma unroll
  for (int b = 0; b < C::AJ; ++b) {
    const int col = wj * C::WN + b * 16 + 4 * g;
    const f32x4 bias4 = (e.bias && j0 + col < N) ? *reinterpret_cast<const f32x4*>(e.bias + j0 + col)
                                                  : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < C::AI; ++a) {
      const f32x4 v = acc[a][b] + bias4;
      const bf16x4 pv = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      *reinterpret_cast<bf16x4*>(smem + (wi * C::WM + a * 16 + (lane & 15)) * PITCH + col * 2) = pv;
    }
  }
  __syncthreads();
  const int c = tid % CPR, j = j0 + c * 8;
  for (int r = tid / CPR; r < C::BM; r += RL) {
    const int i = i0 + r;
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(smem + r * PITCH + c * 16);
    if (i < M && j < N) {
      if constexpr (EPI == EPI_STORE) {
        *reinterpret_cast<bf16x8*>((bf16*)e.C + (int64_t)i * e.ldc + j) = x;
      } else {
        VecF<8> av, dv;
        if constexpr (EPI == EPI_BIAS_GELU) {  // two elements per call (packed FP32; same bits)
#pragma unroll
          for (int q = 0; q < 8; q += 2) {
            f32x2 ga, gd;
            gelu_fast_both2(f32x2{(float)x[q], (float)x[q + 1]}, ga, gd);
            av.q[q >> 2][q & 3] = ga.x;
            av.q[q >> 2][(q & 3) + 1] = ga.y;
            dv.q[q >> 2][q & 3] = gd.x;
            dv.q[q >> 2][(q & 3) + 1] = gd.y;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float ga, gd;
            quick_gelu_both((float)x[q], ga, gd);
            av.q[q >> 2][q & 3] = ga;
            dv.q[q >> 2][q & 3] = gd;
          }
        }
        vstore<bf16, 8>((bf16*)e.C + (int64_t)i * e.ldc + j, dv);
        vstore<bf16, 8>((bf16*)e.aux_out + (int64_t)i * e.ldc + j, av);
      }
    }
  }
}

// Scalar form for the generic kernel (ragged edges).
template <int EPI, typename TO, typename TA>
__device__ __forceinline__ void epi1(const Epi& e, int i, int j, float v) {
  if (e.bias) v += e.bias[j];
  if constexpr (EPI == EPI_STORE) {
    ((TO*)e.C)[e.slab * blockIdx.z + (int64_t)i * e.ldc + j] = (TO)v;
  } else if constexpr (EPI == EPI_ACC) {
    TO* c = (TO*)e.C + (int64_t)i * e.ldc + j;
    *c = (TO)((float)*c + v);
  } else if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) {
    const float pf = (float)(TO)v;
    float a, d;
    if constexpr (EPI == EPI_BIAS_GELU) gelu_erf_both(pf, a, d);
    else quick_gelu_both(pf, a, d);
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = (TO)d;
    ((TO*)e.aux_out)[(int64_t)i * e.ldc + j] = (TO)a;
  } else if constexpr (EPI == EPI_RESID) {
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = (TO)(v + ((const float*)e.aux)[(int64_t)i * e.ld_aux + j]);
  } else if constexpr (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) {
    v *= (float)((const TA*)e.aux)[(int64_t)i * e.ld_aux + j];
    ((TO*)e.C)[(int64_t)i * e.ldc + j] = (TO)v;
  } else if constexpr (EPI == EPI_PATCH) {
    int b = i / e.n_patch, p = i - b * e.n_patch;
    int64_t row = (int64_t)b * (e.n_patch + 1) + 1 + p;
    ((TO*)e.C)[row * e.ldc + j] = (TO)(v + e.pos[(int64_t)(1 + p) * e.ldc + j]);
  }
}

// ----------------------------------------------------------------------------
// Fast bf16 kernel, parametrised: BM x BN x BK tile, WI x WJ waves (each a
// (BM/WI) x (BN/WJ) wave tile of 16x16 accumulators), an S-deep LDS ring filled
// by global_load_lds with a counted vmcnt (S-2 k-steps stay in flight across the
// single s_barrier per k-step), optional register double-buffering of the MFMA
// fragments (DB: the next k-step's ds_reads overlap this k-step's MFMAs), OCC =
// minimum waves per SIMD (sets the VGPR budget / workgroups per CU).
// ----------------------------------------------------------------------------
namespace big {

// EPS (epilogue style): 0 = per-shape choice (LDS-staged row-contiguous stores for the bf16 256x256
// tile and the GELU epilogues), 1 = straight from the MFMA fragments (permlane16-widened 16-B bf16
// stores, 16-B f32 stores) -- no LDS, so the kernel's LDS is its ring alone and two workgroups
// share a CU: one's epilogue runs beside the other's MFMAs.
template <int BM_, int BN_, int BK_, int WI_, int WJ_, int S_, bool DB_, int OCC_, int EPS_ = 0> struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WI = WI_, WJ = WJ_, STAGES = S_, OCC = OCC_, EPS = EPS_;
  static constexpr bool DB = DB_;
  static constexpr int WAVES = WI * WJ, THREADS = WAVES * 64;
  static constexpr int WM = BM / WI, WN = BN / WJ;
  static constexpr int AI = WM / 16, AJ = WN / 16, KS = BK / 32;
  static constexpr int PIMG = BM * BK * 2, QIMG = BN * BK * 2;
  static constexpr int STAGE = PIMG + QIMG;
  static constexpr int GP = PIMG / 1024 / WAVES, GQ = QIMG / 1024 / WAVES;
  static constexpr int G = GP + GQ;  // global_load_lds per wave per stage
  static constexpr int LDS = STAGES * STAGE;
  static_assert(GP * 1024 * WAVES == PIMG && GQ * 1024 * WAVES == QIMG, "stage must split into 1-KiB pieces per wave");
  static_assert(AI % 4 == 0, "column-sum epilogue works on 64-row groups");
  static_assert(LDS <= 163840, "LDS");
};


// Stage a ROWS x BK operand tile into an LDS image; each wave issues G_OP 1-KiB
// global_load_lds.  Rows (RC) / columns (CR) past `lim` are clamped to valid
// memory; their outputs are never stored.
template <int LAY, int ROWS, int BK, int G_OP>
__device__ __forceinline__ void stage(char* img, const bf16* __restrict__ base, int64_t ld, int row0, int r0,
                                      int lim, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < G_OP; ++u) {
    const int t = wave * G_OP + u;
    const bf16* src;
    if constexpr (LAY == LAY_RC) {
      constexpr int CPR = BK / 8, RPI = 64 / CPR;
      const int row = t * RPI + lane / CPR;
      const int c = (lane % CPR) ^ rc_sw<BK>(row);
      const int grow = min(row0 + row, lim - 1);
      src = base + (int64_t)grow * ld + r0 + c * 8;
    } else {
      constexpr int CPR = ROWS / 8;  // 16-B chunks per r-row
      constexpr int RPI = 64 / CPR;  // r-rows per wave-instruction
      const int r = t * RPI + lane / CPR;
      const int c = cr_swz(lane % CPR, r);
      const int col = min(row0 + c * 8, lim - 8);
      src = base + (int64_t)(r0 + r) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(img + t * 1024), 16, 0, 0);
  }
}

// fragment of rows s*16..s*16+15, k-substep kk (16x16x32 operand, natural k order)
template <int LAY, int ROWS, int BK>
__device__ __forceinline__ bf16x8 frag(const char* img, int s, int kk, int lane) {
  if constexpr (LAY == LAY_RC) {
    return *reinterpret_cast<const bf16x8*>(img + rc_off<BK>(s * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int c = 2 * s + (p >> 1);
    const int r0 = kk * 32 + 8 * g + q;
    bf16x4 lo = lds_read_tr(img + cr_off<ROWS>(r0, c) + (p & 1) * 8);
    bf16x4 hi = lds_read_tr(img + cr_off<ROWS>(r0 + 4, c) + (p & 1) * 8);
    return cat4(lo, hi);
  }
}


// One output tile (unit w of the 1-D (split, tile) space) of the fast bf16 GEMM.
template <class C, int PL, int QL, int EPI, typename TO, typename TA>
__device__ __forceinline__ void gemm_tile(const bf16* __restrict__ P, int64_t ldp, const bf16* __restrict__ Q,
                                          int64_t ldq, int M, int N, int R, int r_chunk, const Epi& e, int w,
                                          char* smem) {
  constexpr int S = C::STAGES, BM = C::BM, BN = C::BN, BK = C::BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_j = (N + BN - 1) / BN, tiles_i = (M + BM - 1) / BM;
  const int tiles = tiles_i * tiles_j;
  const int z = w / tiles, t = w - z * tiles;
  int ti, tj;
  tile_coords(t, tiles_i, tiles_j, e.group_m, ti, tj);
  const int i0 = ti * BM, j0 = tj * BN;
  const int rb = z * r_chunk;
  const int re = min(R, rb + r_chunk);
  const int nk = (re - rb) / BK;
  const int wi = wave / C::WJ, wj = wave % C::WJ;

  f32x4 acc[C::AI][C::AJ];
#pragma unroll
  for (int a = 0; a < C::AI; ++a)
#pragma unroll
    for (int b = 0; b < C::AJ; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging sources: a k-independent per-lane byte offset of each 1-KiB piece (stage()'s
  // addressing) plus a wave-uniform base advanced per k-step, so the loads take the SGPR-base
  // form with no per-piece 64-bit address arithmetic (host side guarantees offsets < 2^32)
  uint32_t poff[C::GP], qoff[C::GQ];
  auto lane_offsets = [&](auto lay_tag, auto rows_tag, uint32_t* off, int G_OP, int64_t ld, int row0, int lim) {
    constexpr int LAY = decltype(lay_tag)::value, ROWS = decltype(rows_tag)::value;
    for (int u = 0; u < G_OP; ++u) {
      const int t = wave * G_OP + u;
      if constexpr (LAY == LAY_RC) {
        constexpr int CPR = BK / 8, RPI = 64 / CPR;
        const int row = t * RPI + lane / CPR;
        const int c = (lane % CPR) ^ rc_sw<BK>(row);
        off[u] = (uint32_t)((int64_t)min(row0 + row, lim - 1) * ld * 2 + c * 16);
      } else if constexpr (VIT_CR_HB) {
        off[u] = (uint32_t)(crh_src<ROWS>(t, lane, ld, row0, lim) * 2);
      } else {
        constexpr int CPR = ROWS / 8, RPI = 64 / CPR;
        const int r = t * RPI + lane / CPR;
        const int c = cr_swz(lane % CPR, r);
        off[u] = (uint32_t)((int64_t)r * ld * 2 + min(row0 + c * 8, lim - 8) * 2);
      }
    }
  };
  lane_offsets(std::integral_constant<int, PL>{}, std::integral_constant<int, BM>{}, poff, C::GP, ldp, i0, M);
  lane_offsets(std::integral_constant<int, QL>{}, std::integral_constant<int, BN>{}, qoff, C::GQ, ldq, j0, N);
  // part 1: the P pieces of stage k, part 2: the Q pieces, 3: both
  auto issue = [&](int k, int part = 3) {
    char* buf = smem + (k % S) * C::STAGE;
    const int r = rb + k * BK;
    const char* pb = reinterpret_cast<const char*>(P) + (PL == LAY_RC ? (int64_t)r * 2 : (int64_t)r * ldp * 2);
    const char* qb = reinterpret_cast<const char*>(Q) + (QL == LAY_RC ? (int64_t)r * 2 : (int64_t)r * ldq * 2);
    if (part & 1) {
#pragma unroll
      for (int u = 0; u < C::GP; ++u)
        __builtin_amdgcn_global_load_lds((const void*)(pb + poff[u]), LDS_PTR(buf + (wave * C::GP + u) * 1024), 16, 0,
                                         0);
    }
    if (part & 2) {
#pragma unroll
      for (int u = 0; u < C::GQ; ++u)
        __builtin_amdgcn_global_load_lds((const void*)(qb + qoff[u]), LDS_PTR(buf + C::PIMG + (wave * C::GQ + u) * 1024),
                                         16, 0, 0);
    }
  };
  // two k-substeps (BK = 64): the next stage's P pieces go out before the first substep's fragment
  // reads, its Q pieces before the second's, instead of all of them behind the barrier (the waves of a
  // SIMD reach the barrier together, so a burst of LDS-DMA issue there stalls both of their MFMA
  // streams at once: +3-8 % main loop, tools/lab/mf32_lab.py, profiles/r04/gemm_load_split_lab.jsonl)
  constexpr bool SPLIT_ISSUE = C::KS == 2 && VIT_SPLIT_ISSUE;
  // one k-substep (BK = 32): the P pieces behind the barrier, the Q pieces behind the MFMAs
  constexpr bool SPLIT_ISSUE1 = C::KS == 1 && VIT_SPLIT_ISSUE1;
  auto load_frags = [&](int k, int kk, bf16x8 (&pf)[C::AI], bf16x8 (&qf)[C::AJ]) {
    const char* cur = smem + (k % S) * C::STAGE;
#pragma unroll
    for (int b = 0; b < C::AJ; ++b) qf[b] = frag<QL, BN, BK>(cur + C::PIMG, wj * C::AJ + b, kk, lane);
#pragma unroll
    for (int a = 0; a < C::AI; ++a) pf[a] = frag<PL, BM, BK>(cur, wi * C::AI + a, kk, lane);
  };
  auto mma = [&](const bf16x8 (&pf)[C::AI], const bf16x8 (&qf)[C::AJ]) {
#pragma unroll
    for (int a = 0; a < C::AI; ++a)
#pragma unroll
      for (int b = 0; b < C::AJ; ++b) acc[a][b] = mfma16(qf[b], pf[a], acc[a][b]);
  };

  // lane part of the r-contiguous fragment addresses: rc_off(s*16 + l15, kk*4 + g) =
  // s*16*BK*2 + rc_off(l15, kk*4 + g) for the wave's first fragment s, because the swizzle
  // rc_sw(row) depends on row mod 16 only
  uint32_t rc_lane[2][C::KS];
#pragma unroll
  for (int kk = 0; kk < C::KS; ++kk) {
    rc_lane[0][kk] = (uint32_t)(wi * C::AI * 16 * BK * 2 + rc_off<BK>(lane & 15, kk * 4 + (lane >> 4)));
    rc_lane[1][kk] = (uint32_t)(wj * C::AJ * 16 * BK * 2 + rc_off<BK>(lane & 15, kk * 4 + (lane >> 4)));
  }
  // timing experiments (vit_gemm_variant(v + 100 * bits)): bit 1 drops the ring loads, bit 2 the
  // per-k-step barrier -- the main loop's ceiling without the memory system / the workgroup sync
  const bool dbg_noload = e.dbg & 1, dbg_nobar = e.dbg & 2;
  uint32_t crh_p[2][2], crh_q[2][2];  // half-blocked: [lo / hi][fragment parity], first fragment pair folded in
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      crh_p[lh][h] = crh_lane<BM>(lane, lh, h) + (uint32_t)(wi * C::AI / 2 * 1024);
      crh_q[lh][h] = C::PIMG + crh_lane<BN>(lane, lh, h) + (uint32_t)(wj * C::AJ / 2 * 1024);
    }
  if (nk > 0) {
#pragma unroll
    for (int k = 0; k < S - 1; ++k)
      if (k < nk && !dbg_noload) issue(k);
    if constexpr (!C::DB) {
      for (int kt = 0; kt < nk; ++kt) {
        wait_stages<C::G, S>(min(S - 2, nk - 1 - kt));
        if (!dbg_nobar) lds_barrier();
        const bool more = kt + S - 1 < nk && !dbg_noload;
        if (!SPLIT_ISSUE && more) issue(kt + S - 1, SPLIT_ISSUE1 ? 1 : 3);
        Unroll<C::KS>::run([&](auto kkI) {
          constexpr int kk = decltype(kkI)::value;
          if constexpr (SPLIT_ISSUE) {
            if (more) issue(kt + S - 1, kk + 1);
          }
          // asm fragment reads (no compiler vmcnt(0) for the in-flight ring loads);
          // retired before the MFMAs, so they are also done before the next barrier (WAR)
          const uint32_t cur = lds_addr(smem + (kt % S) * C::STAGE);
          bf16x8 pf[C::AI], qf[C::AJ];
          if constexpr (QL == LAY_RC) {  // fragment b = lane base + b * 16 rows (immediate)
            const uint32_t qa = cur + C::PIMG + rc_lane[1][kk];
            Unroll<C::AJ>::run([&](auto bI) {
              constexpr int b = decltype(bI)::value;
              qf[b] = asm_read128_off<b * 16 * BK * 2>(qa);
            });
          } else if constexpr (VIT_CR_HB) {
            Unroll<C::AJ>::run([&](auto bI) {
              constexpr int b = decltype(bI)::value;
              qf[b] = frag_crh<BN, kk, b>(crh_q, cur);
            });
          } else {
#pragma unroll
            for (int b = 0; b < C::AJ; ++b) qf[b] = frag_asm<QL, BN, BK>(cur + C::PIMG, wj * C::AJ + b, kk, lane);
          }
          if constexpr (PL == LAY_RC) {
            const uint32_t pa = cur + rc_lane[0][kk];
            Unroll<C::AI>::run([&](auto aI) {
              constexpr int a = decltype(aI)::value;
              pf[a] = asm_read128_off<a * 16 * BK * 2>(pa);
            });
          } else if constexpr (VIT_CR_HB) {
            Unroll<C::AI>::run([&](auto aI) {
              constexpr int a = decltype(aI)::value;
              pf[a] = frag_crh<BM, kk, a>(crh_p, cur);
            });
          } else {
#pragma unroll
            for (int a = 0; a < C::AI; ++a) pf[a] = frag_asm<PL, BM, BK>(cur, wi * C::AI + a, kk, lane);
          }
          lgkm_wait0();
          mma(pf, qf);
        });
        if constexpr (SPLIT_ISSUE1) {
          if (more) issue(kt + S - 1, 2);
        }
      }
    } else {
      static_assert(C::KS == 1, "register double-buffering is built for BK = 32");
      static_assert(!(VIT_CR_HB && (PL == LAY_CR || QL == LAY_CR)), "load_frags reads the swizzled CR image");
      // step k: make stage k+1 readable, refill slot k%S with stage k+S-1... (ring of S, S-1 ahead)
      auto step = [&](int k, const bf16x8 (&pc)[C::AI], const bf16x8 (&qc)[C::AJ], bf16x8 (&pn)[C::AI],
                      bf16x8 (&qn)[C::AJ]) {
        if (k + 1 < nk) {
          wait_stages<C::G, S>(min(S - 3, nk - 2 - k));
          lds_barrier();
          if (k + S - 1 < nk) issue(k + S - 1);
          load_frags(k + 1, 0, pn, qn);
        }
        mma(pc, qc);
      };
      bf16x8 pA[C::AI], qA[C::AJ], pB[C::AI], qB[C::AJ];
      wait_stages<C::G, S>(min(S - 2, nk - 1));
      lds_barrier();
      load_frags(0, 0, pA, qA);
      int kt = 0;
      for (; kt + 1 < nk; kt += 2) {
        step(kt, pA, qA, pB, qB);
        step(kt + 1, pB, qB, pA, qA);
      }
      if (kt < nk) step(kt, pA, qA, pB, qB);
    }
  }
  if (e.dbg & 4) {  // timing experiment: keep the accumulators live, skip the epilogue
#pragma unroll
    for (int a = 0; a < C::AI; ++a)
#pragma unroll
      for (int b = 0; b < C::AJ; ++b) asm volatile("" ::"v"(acc[a][b]));
    return;
  }
  // bf16 outputs: row-contiguous epilogue through LDS (16-B stores; dbg bit 8 forces the
  // fragment-layout one, for timing).  f32 fragments already store 16 B per lane.
  // bf16 outputs: plain stores of the smaller tiles go out as fragment pairs widened to 16-B
  // stores by permlane16_swap (N % 32 == 0; +2-5 % over staging on the N = 768 outputs); the
  // 256x256 tile and the GELU / GELU' epilogues are faster through the row-contiguous LDS
  // staging (tools/bench_kernels.py --sweep: v vs 6400 + v).  Timing flags: dbg 64 forces the
  // staged epilogue, dbg 8 the plain fragment-layout one below (8-B stores).
  // (plain bf16 stores: fragment epilogue on every tile -- the qkv forward on the 256x256 tile runs 10 %
  // faster than through the LDS staging, tools/bench_kernels.py --sweep=5,1605; the GELU pair stays staged)
  if constexpr (sizeof(TO) == 2 && (EPI == EPI_STORE ||
                                     (C::EPS == 1 && (EPI == EPI_STORE || EPI == EPI_BIAS_GELU ||
                                                      EPI == EPI_BIAS_QGELU || EPI == EPI_GELU_BWD ||
                                                      EPI == EPI_QGELU_BWD)))) {
    if constexpr (EPI == EPI_STORE && C::EPS == 0 && C::BM == 256 && C::BN == 256 &&
                  Pair16<C>::BYTES <= (C::LDS > EpiLds<C, TO>::BYTES ? C::LDS : EpiLds<C, TO>::BYTES)) {
      // the 256x256 tile: the plain bf16 store through the bf16 LDS image of the tile as well (+1-4 %
      // standalone over the fragment stores, profiles/r03/gemm_plain_store_bf16_stage_sweep.jsonl);
      // dbg 256 forces the fragment stores (A/B)
      if (VIT_PLAIN16 && !(e.dbg & (8 | 64 | 256)) && !e.csum && N % 8 == 0) {
        epilogue_pair16<C, EPI>(e, acc, smem, i0, j0, wi, wj, lane, M, N);
        return;
      }
    }
    if (!(e.dbg & (8 | 64)) && N % 32 == 0) {
      epilogue_swap<C, EPI, TO, TA>(e, acc, i0, j0, wi, wj, lane, M, N);
      return;
    }
  }
  if constexpr (sizeof(TO) == 2 && C::EPS == 0 && (EPI == EPI_STORE || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU ||
                                                    EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD)) {
    if ((e.dbg & 16) && N % 32 == 0) {  // timing experiment: the fragment (permlane16) epilogue on any tile
      epilogue_swap<C, EPI, TO, TA>(e, acc, i0, j0, wi, wj, lane, M, N);
      return;
    }
  }
  if constexpr (sizeof(TO) == 2 && C::EPS == 0 && (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) &&
                Pair16<C>::BYTES <= (C::LDS > EpiLds<C, TO>::BYTES ? C::LDS : EpiLds<C, TO>::BYTES)) {
    if (VIT_PAIR16 && !e.csum && !(e.dbg & (8 | 128)) && N % 8 == 0) {  // dbg 128: the f32 band staging (A/B)
      epilogue_pair16<C, EPI>(e, acc, smem, i0, j0, wi, wj, lane, M, N);
      return;
    }
  }
  if constexpr (sizeof(TO) == 2 && C::EPS == 0) {
    if (!(e.dbg & 8)) {
      epilogue_staged<C, EPI, TO, TA>(e, acc, smem, i0, j0, wi, wj, lane, M, N, z);
      return;
    }
  }
  // epilogue: acc[a][b] holds C[i][j..j+3] with i = lane&15, j = 4*(lane>>4)
  f32x4 cs[C::AJ];
#pragma unroll
  for (int b = 0; b < C::AJ; ++b) cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < C::AI; ++a) {
    const int i = i0 + wi * C::WM + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < C::AJ; ++b) {
      const int j = j0 + wj * C::WN + b * 16 + 4 * (lane >> 4);
      if (i < M && j < N) {
        const f32x4 v = epi4<EPI, TO, TA>(e, i, j, acc[a][b], z);
        if (e.csum) cs[b] += v;
      }
    }
    if (e.csum && (a & 3) == 3) csum_flush<C::AJ>(e, cs, i0 + wi * C::WM + (a - 3) * 16, M, N, j0 + wj * C::WN, lane);
  }
}

// 1-D grid over (split, tile): consecutive ids share an XCD after the remap, so a split's
// workgroups (same rows of P and Q) sit on one L2
template <class C, int PL, int QL, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(C::THREADS, C::OCC) void gemm_kernel(const bf16* __restrict__ P, int64_t ldp,
                                                                  const bf16* __restrict__ Q, int64_t ldq,
                                                                  int M, int N, int R, int r_chunk, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemm_tile<C, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, r_chunk, e, xcd_remap(blockIdx.x, gridDim.x), smem);
}

// ----------------------------------------------------------------------------
// Ping-pong schedule: 256x256 tile, BK = 32, 8 waves in two groups of four
// (group g owns rows g*128..g*128+127; wave w%4 owns 64 columns).  Each k-tile is
// two phases -- {ds_read fragments} barrier {MFMA cluster of 16} barrier -- and
// group 1 runs one barrier behind group 0, so on every SIMD one wave's MFMA
// cluster overlaps the other wave's LDS reads.  Operands stream through an
// S-deep ring of 32-KiB stages filled by global_load_lds, S-1 tiles ahead; each
// tile's loads are split over the two MFMA phases and retired by a counted
// vmcnt (never 0 inside the loop), raw s_barrier only.
// ----------------------------------------------------------------------------
template <int S_> struct PP {
  static constexpr int S = S_, BM = 256, BN = 256, BK = 32, THREADS = 512;
  static constexpr int PIMG = BM * BK * 2, STAGE = 2 * PIMG, LDS = S * STAGE;
  static_assert(LDS <= 163840, "LDS");
};

// s_waitcnt vmcnt(n) for a wave-uniform even n <= 14
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 2: wait_vm<2>(); break;
    case 4: wait_vm<4>(); break;
    case 6: wait_vm<6>(); break;
    case 8: wait_vm<8>(); break;
    case 10: wait_vm<10>(); break;
    case 12: wait_vm<12>(); break;
    default: wait_vm<14>(); break;
  }
}

// unit w of the (split, tile) space of one ping-pong GEMM
template <int S, int PL, int QL, int EPI, typename TO, typename TA>
__device__ __forceinline__ void pp_tile(const bf16* __restrict__ P, int64_t ldp, const bf16* __restrict__ Q,
                                        int64_t ldq, int M, int N, int R, int r_chunk, const Epi& e, int w,
                                        char* smem) {
  using C = PP<S>;
  constexpr bool CRH = VIT_CR_HB && PL == LAY_CR && QL == LAY_CR;  // half-blocked CR images (weight gradient)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wj = wave & 3;
  const int tiles_j = (N + 255) / 256, tiles_i = (M + 255) / 256;
  const int tiles = tiles_i * tiles_j;
  const int z = w / tiles, t0 = w - z * tiles;
  // walk along the longer tile dimension, so an XCD's run of consecutive units (one split) covers
  // all the short-side blocks and a band of the long side: for the 768 x 3072 fc2 weight gradient
  // (3 x 12 tiles) 18 units = 3 x 6 tiles read 9 operand blocks instead of 2 x 12 = 14
  int ti, tj;
  if (tiles_j > tiles_i) {
    tj = t0 / tiles_i;
    ti = t0 - tj * tiles_i;
  } else {
    ti = t0 / tiles_j;
    tj = t0 - ti * tiles_j;
  }
  const int i0 = ti * 256, j0 = tj * 256;
  const int rb = z * r_chunk;
  const int re = min(R, rb + r_chunk);
  const int nk = (re - rb) / 32;

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane global source pointers of this wave's 4 staging pieces (2 of P, 2 of Q),
  // advanced by one k-tile after each issue; LDS destination = slot + piece * 1 KiB
  const bf16* srcP[2];
  const bf16* srcQ[2];
  int64_t stepP, stepQ;
  {
    auto init = [&](auto lay_tag, const bf16* base, int64_t ld, int row0, int lim, const bf16* (&src)[2],
                    int64_t& step) {
      constexpr int LAY = decltype(lay_tag)::value;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = wave * 2 + u;
        if constexpr (LAY == LAY_RC) {
          const int row = t * 16 + lane / 4;
          const int c = (lane % 4) ^ rc_sw<32>(row);
          src[u] = base + (int64_t)min(row0 + row, lim - 1) * ld + rb + c * 8;
          step = 32;
        } else if constexpr (CRH) {
          src[u] = base + (int64_t)rb * ld + crh_src<256>(t, lane, ld, row0, lim);
          step = 32 * ld;
        } else {
          const int r = t * 2 + lane / 32;
          const int c = cr_swz(lane % 32, r);
          src[u] = base + (int64_t)(rb + r) * ld + min(row0 + c * 8, lim - 8);
          step = 32 * ld;
        }
      }
    };
    init(std::integral_constant<int, PL>{}, P, ldp, i0, M, srcP, stepP);
    init(std::integral_constant<int, QL>{}, Q, ldq, j0, N, srcQ, stepQ);
  }
  // issue the 4 loads of the next k-tile in sequence into ring slot k % S
  auto issue = [&](int k) {
    char* buf = smem + (k % S) * C::STAGE;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      __builtin_amdgcn_global_load_lds((const void*)srcP[u], LDS_PTR(buf + (wave * 2 + u) * 1024), 16, 0, 0);
      srcP[u] += stepP;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      __builtin_amdgcn_global_load_lds((const void*)srcQ[u], LDS_PTR(buf + C::PIMG + (wave * 2 + u) * 1024), 16, 0, 0);
      srcQ[u] += stepQ;
    }
  };
  const bool dbg_noload = e.dbg & 1, dbg_nobar = e.dbg & 2;
  auto bar = [&]() { if (!dbg_nobar) lds_barrier(); };
  uint32_t crh_p[2][2], crh_q[2][2];  // half-blocked: [lo / hi][fragment parity]
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      crh_p[lh][h] = crh_lane<256>(lane, lh, h) + (uint32_t)(grp * 4 * 1024);
      crh_q[lh][h] = C::PIMG + crh_lane<256>(lane, lh, h) + (uint32_t)(wj * 2 * 1024);
    }
  // one k-tile = two phases {reads} barrier {16 MFMA} barrier; the next tile's loads are
  // issued in the second read phase, where the partner wave's MFMAs cover their issue
  auto tile = [&](int t, bf16x8 (&qf)[4], bf16x8 (&p0)[4], bf16x8 (&p1)[4]) {
    const uint32_t cur = lds_addr(smem + (t % S) * C::STAGE);
    const bool more = t + S - 1 < nk && !dbg_noload;
    if constexpr (CRH) {
      Unroll<4>::run([&](auto bI) {
        constexpr int b = decltype(bI)::value;
        qf[b] = frag_crh<256, 0, b>(crh_q, cur);
      });
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b) qf[b] = frag_asm<QL, 256, 32>(cur + C::PIMG, wj * 4 + b, 0, lane);
    }
    if constexpr (CRH) {
      Unroll<4>::run([&](auto aI) {
        constexpr int a = decltype(aI)::value;
        p0[a] = frag_crh<256, 0, a>(crh_p, cur);
      });
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a) p0[a] = frag_asm<PL, 256, 32>(cur, grp * 8 + a, 0, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    bar();
    lgkm_wait0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(qf[b], p0[a], acc[a][b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    bar();
    if constexpr (CRH) {
      Unroll<4>::run([&](auto aI) {
        constexpr int a = decltype(aI)::value;
        p1[a] = frag_crh<256, 0, 4 + a>(crh_p, cur);
      });
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a) p1[a] = frag_asm<PL, 256, 32>(cur, grp * 8 + 4 + a, 0, lane);
    }
    if (t + 1 < nk && !dbg_noload) {  // tile t+1 landed; in flight behind it: tiles t+2.. (4 loads each)
      if (t + S - 2 < nk) wait_vm<4 * (S - 3)>();
      else wait_vm_n(4 * (nk - 2 - t));
    }
    if (more) issue(t + S - 1);  // slot (t-1) % S: every wave's reads of tile t-1 retired two phases ago
    __builtin_amdgcn_sched_barrier(0);
    bar();
    lgkm_wait0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[4 + a][b] = mfma16(qf[b], p1[a], acc[4 + a][b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    bar();
  };

  if (nk > 0) {
#pragma unroll
    for (int k = 0; k < S - 1; ++k)
      if (k < nk) issue(k);
    wait_vm_n(4 * min(S - 2, nk - 1));
    lds_barrier();
    if (grp) lds_barrier();  // stagger group 1 by one phase
    bf16x8 qA[4], pA0[4], pA1[4], qB[4], pB0[4], pB1[4];
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      tile(t, qA, pA0, pA1);
      tile(t + 1, qB, pB0, pB1);
    }
    if (t < nk) tile(t, qA, pA0, pA1);
    if (!grp) lds_barrier();  // rebalance the barrier count
  }
  if (e.dbg & 4) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) asm volatile("" ::"v"(acc[a][b]));
    return;
  }
  f32x4 cs[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = i0 + grp * 128 + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int j = j0 + wj * 64 + b * 16 + 4 * (lane >> 4);
      if (i < M && j < N) {
        const f32x4 v = epi4<EPI, TO, TA>(e, i, j, acc[a][b], z);
        if (e.csum) cs[b] += v;
      }
    }
    if (e.csum && (a & 3) == 3) csum_flush<4>(e, cs, i0 + grp * 128 + (a - 3) * 16, M, N, j0 + wj * 64, lane);
  }
}

template <int S, int PL, int QL, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(512, 1) void pp_kernel(const bf16* __restrict__ P, int64_t ldp,
                                                    const bf16* __restrict__ Q, int64_t ldq,
                                                    int M, int N, int R, int r_chunk, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  pp_tile<S, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, r_chunk, e, xcd_remap(blockIdx.x, gridDim.x), smem);
}

// Two weight gradients in one launch (grouped): units [0, nwg0) are problem 0's (split, tile)
// space, the rest problem 1's.  Both reduce over the same token rows with the same split, so
// every workgroup runs the same number of k-steps; the pair has twice the tiles of either, so
// it fills the side stream's workgroup budget with half the split (half the fp32 slab traffic).
struct PPProb {
  const bf16* P; const bf16* Q; int64_t ldp, ldq;
  int M, N, R, r_chunk, nwg;
  Epi e;
};
template <int S, int PL, int QL, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(512, 1) void pp_kernel2(PPProb a, PPProb b) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  if (w < a.nwg)
    pp_tile<S, PL, QL, EPI, TO, TA>(a.P, a.ldp, a.Q, a.ldq, a.M, a.N, a.R, a.r_chunk, a.e, w, smem);
  else
    pp_tile<S, PL, QL, EPI, TO, TA>(b.P, b.ldp, b.Q, b.ldq, b.M, b.N, b.R, b.r_chunk, b.e, w - a.nwg, smem);
}

// the configurations kept after the sweep (tools/bench_kernels.py --sweep; DESIGN.md
// lists the measured TFLOP/s per shape).  Others tried: 256x256x32 S5 with register
// double-buffering (1 WG/CU; wgrad 360-400 TF), 128x128x32 S4, 256x128x64 S3, 128x256x32 S4,
// 256x256x32 S3 / S4 (V5's waves, deeper ring: qkv forward +6 % standalone, the other shapes flat
// or slower; as the in-step weight gradient -0.4 .. -0.7 % step rate vs the ping-pong kernel).
//            BM   BN  BK WI WJ  S  DB    OCC
using V1 = Cfg<256, 128, 32, 4, 2, 3, false, 4>;  //  72 KiB, 2 WG/CU: dgrad
using V2 = Cfg<128, 128, 64, 2, 2, 2, false, 2>;  //  64 KiB, 2 WG/CU (4 waves): N = 768 forward
using V5 = Cfg<256, 256, 64, 2, 4, 2, false, 2>;  // 128 KiB, 1 WG/CU: wide forward, wgrad
using V3 = Cfg<128, 256, 32, 2, 2, 3, false, 2>;  //  72 KiB, 2 WG/CU (4 waves of 64x128)
using V4 = Cfg<256, 128, 32, 4, 2, 4, false, 4>;  //  96 KiB, 1 WG/CU, 4-deep ring
// 4 waves of 128x64 (V5's wave tile), 3-deep ring, epilogue from the fragments: 72 KiB -> 2
// workgroups per CU (one wave per SIMD each), whose epilogues overlap each other's MFMAs
using V6 = Cfg<256, 128, 32, 2, 2, 3, false, 2, 1>;
using V7 = Cfg<128, 256, 32, 2, 2, 3, false, 2, 1>;  // 4 waves of 64x128
}  // namespace big

#include "gemm_f32.inc"
#include "gemm_w4.inc"

// ----------------------------------------------------------------------------
// Generic strided kernel: any M, N, R; f32 or bf16 inputs; fp32 FMA.
//   P(i,r) = P[i*sPi + r*sPr], Q(j,r) = Q[j*sQj + r*sQr]
// ----------------------------------------------------------------------------
namespace gen {
// TK 64: a quarter of the serial k-steps of 16.  TILE 64 (4x4 outputs per thread) or
// 32 (2x2) -- the smaller tile when 64-tiles leave CUs idle (e.g. the 256-row head GEMMs).
constexpr int TK = 64;
template <int TILE, typename T, int EPI, typename TO, typename TA>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ P, int64_t sPi, int64_t sPr,
                                                   const T* __restrict__ Q, int64_t sQj, int64_t sQr,
                                                   int M, int N, int R, int r_chunk, Epi e) {
  constexpr int TM = TILE, TN = TILE, A = TILE / 16;
  __shared__ float Ps[TK][TM + 4];
  __shared__ float Qs[TK][TN + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
  const int rb = blockIdx.z * r_chunk, re = min(R, rb + r_chunk);
  float acc[A][A] = {};
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
      float pv[A], qv[A];
#pragma unroll
      for (int a = 0; a < A; ++a) pv[a] = Ps[kk][ty + 16 * a];
#pragma unroll
      for (int b = 0; b < A; ++b) qv[b] = Qs[kk][tx * A + b];
#pragma unroll
      for (int a = 0; a < A; ++a)
#pragma unroll
        for (int b = 0; b < A; ++b) acc[a][b] = fmaf(pv[a], qv[b], acc[a][b]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < A; ++a) {
    int i = i0 + ty + 16 * a;
    if (i >= M) continue;
#pragma unroll
    for (int b = 0; b < A; ++b) {
      int j = j0 + tx * A + b;
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


// ----------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------
// fast-path eligibility: bf16, 16-B aligned operands, 8-element row strides,
// reduction length a multiple of BK (callers split off a ragged tail).  An
// r-contiguous (RC) operand's row count is free (staging clamps rows past the
// edge, the epilogue guards i < M: e.g. the 66 x 77 = 5082 text-tower tokens);
// an i/j-contiguous (CR) one loads 8-wide column chunks, so it needs a multiple
// of 8; the 4-column epilogue stores need N % 4.
// big::gemm_tile addresses an RC operand through per-lane uint32 byte offsets from a k-advanced
// base: the largest one is (rows - 1) * ld * 2 plus a 64-element (128-B) chunk.  Larger operands
// are split along the rows by the dispatcher (rc_chunk_rows); the CR layouts keep offsets below
// BK rows and need no limit.
static constexpr int64_t kOffLimit = (int64_t)1 << 32;
static bool rc_offsets_fit(int rows, int64_t ld) { return (int64_t)(rows > 0 ? rows - 1 : 0) * ld * 2 + 128 < kOffLimit; }
// rows per launch for an RC operand of `ld` elements per row: a multiple of 256 (the largest BM, and
// of 64 for the column-sum partial rows) whose offsets fit; M itself when it fits
static int rc_chunk_rows(int M, int64_t ld) {
  if (rc_offsets_fit(M, ld)) return M;
  const int64_t r = ((kOffLimit - 129) / (ld * 2) + 1) / 256 * 256;  // the most rows that fit, in 256s
  return (int)(r > 0 ? r : 0);
}

static bool fast_ok(int dtype, int pl, int ql, int M, int N, int R, const void* P, const void* Q, int64_t ldp,
                    int64_t ldq) {
  if (dtype != VIT_BF16) return false;
  // an RC Q (the weights of a forward GEMM) must fit the 32-bit offsets whole; an RC P is chunked
  if (ql == LAY_RC && !rc_offsets_fit(N, ldq)) return false;
  if (pl == LAY_RC && rc_chunk_rows(M, ldp) == 0) return false;
  if ((pl == LAY_CR && M % 8) || (ql == LAY_CR && N % 8) || N % 4 || R % 32 || R <= 0) return false;
  if ((ldp % 8) || (ldq % 8)) return false;
  if (((uintptr_t)P & 15) || ((uintptr_t)Q & 15)) return false;
  return true;
}

// fp32 MFMA path (f32m::gemm_kernel): 16-B aligned operands, 4-element row strides, reduction a
// multiple of 32; a CR operand loads 4-wide column chunks (its extent a multiple of 4).
static bool fast_f32_ok(int dtype, int pl, int ql, int M, int N, int R, const void* P, const void* Q, int64_t ldp,
                        int64_t ldq) {
  if (dtype != VIT_F32) return false;
  if ((pl == LAY_CR && M % 4) || (ql == LAY_CR && N % 4) || N % 4 || R % f32m::BK || R <= 0) return false;
  if ((ldp % 4) || (ldq % 4)) return false;
  if (((uintptr_t)P & 15) || ((uintptr_t)Q & 15)) return false;
  return true;
}
// small grids (the 256-row classifier head) keep the generic kernel's 32x32 tiles: more workgroups
static bool f32_grid_ok(int M, int N, int split) {
  return (int64_t)((M + f32m::BM - 1) / f32m::BM) * ((N + f32m::BN - 1) / f32m::BN) * (split > 1 ? split : 1) >= 64;
}
static bool any_fast_ok(int dtype, int pl, int ql, int M, int N, int R, const void* P, const void* Q, int64_t ldp,
                        int64_t ldq) {
  return fast_ok(dtype, pl, ql, M, N, R, P, Q, ldp, ldq) || fast_f32_ok(dtype, pl, ql, M, N, R, P, Q, ldp, ldq);
}

static int g_variant = -1;  // -1: per-shape choice; 1, 2, 5: force big::V<n>, 8, 9: ping-pong (tuning)
static int g_dbg = 0;

// per-class override for in-step A/B runs (tools/ab_bench.sh): VIT_GEMM_{FWD,DGRAD,WGRAD}=<variant>
static int env_variant(const char* name) {
  const char* s = getenv(name);
  return s && *s ? atoi(s) : -1;
}

// per-shape choice among the kept configurations (sweep on MI355X, bs=256 ViT-B/16 shapes)
static int pick_variant(int pl, int ql, int M, int N, int R, int split, bool act_bwd) {
  static const int o_fwd = env_variant("VIT_GEMM_FWD"), o_dgrad = env_variant("VIT_GEMM_DGRAD"),
                   o_wgrad = env_variant("VIT_GEMM_WGRAD");
  const bool wgrad = split > 1 || (pl == LAY_CR && ql == LAY_CR), fwd = pl == LAY_RC && ql == LAY_RC;
  const int o = wgrad ? o_wgrad : fwd ? o_fwd : o_dgrad;
  int v;
  if (g_variant >= 0) v = g_variant % 100;
  else if (o >= 0) v = o;
  else if (wgrad) v = 8;   // wgrad: the ping-pong 256x256 kernel; 11 = w4 (4 waves of 128x128, round 5):
                           // 1.3x the ping-pong's loop ceiling but not faster with loads and epilogue, and
                           // -0.3 % in the step (profiles/r05/ab_wgrad_w4_vs_pingpong.txt, bench_wgrad_r05a.jsonl)
  else if (fwd) v = 5;     // forward: V5 (the N, R < 1536 proj / patch embedding too: +0.35 % over V2, round 3)
  else v = (act_bwd || (N <= 1024 && R <= 1024)) ? 1 : 3;  // dgrad (GELU' epilogue: V1, 2 WG/CU)
  // (round 5 removed the per-shape overrides VIT_GEMM_{FWD,DGRAD}_{SMALL,GELU}: every re-check measured
  // their other tiles slower or equal, profiles/r04/ab_dgrad_per_shape.txt, ab_dgrad_gelu_tiles_recheck.txt)
  (void)M;
  if ((v == 2 || v == 5) && R % 64) v = 1;                                 // BK = 64 configurations need 64-row chunks
  return v;
}

// rows per split-K chunk: ceil(R / split) rounded up to the k-step, so the launch never has more
// than `split` chunks (nz = ceil(R / r_chunk) <= split): every slab-size check against split * M * N
// then covers the slabs the kernel writes (R = 1025, split = 8: 192-row chunks, 6 slabs -- the
// floor(R / split) rounding gave 128 and 9 slabs)
static int r_chunk_for(int R, int split, int bk) {
  if (split < 1) split = 1;
  int c = (((R + split - 1) / split + bk - 1) / bk) * bk;
  return c > 0 ? c : bk;
}

template <class C, int PL, int QL, int EPI, typename TO, typename TA>
static int launch_big(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
                      const Epi& e, hipStream_t s) {
  constexpr int lds = (C::EPS == 1 || C::LDS > EpiLds<C, TO>::BYTES) ? C::LDS : EpiLds<C, TO>::BYTES;
  static_assert(lds <= 163840, "LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)big::gemm_kernel<C, PL, QL, EPI, TO, TA>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  if (R % C::BK) return (int)hipErrorInvalidValue;
  const int r_chunk = r_chunk_for(R, split, 64);  // one chunking for every variant (wgrad counts slabs)
  const int nz = (R + r_chunk - 1) / r_chunk;
  dim3 grid(((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN) * nz);
  hipLaunchKernelGGL((big::gemm_kernel<C, PL, QL, EPI, TO, TA>), grid, dim3(C::THREADS), lds, s,
                     (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

template <int S, int PL, int QL, int EPI, typename TO, typename TA>
static int launch_pp(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
                     const Epi& e, hipStream_t s) {
  using C = big::PP<S>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)big::pp_kernel<S, PL, QL, EPI, TO, TA>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  if (R % C::BK) return (int)hipErrorInvalidValue;
  const int r_chunk = r_chunk_for(R, split, 64);
  const int nz = (R + r_chunk - 1) / r_chunk;
  dim3 grid(((M + 255) / 256) * ((N + 255) / 256) * nz);
  hipLaunchKernelGGL((big::pp_kernel<S, PL, QL, EPI, TO, TA>), grid, dim3(C::THREADS), C::LDS, s,
                     (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

template <class C, int PL, int QL, int EPI, typename TO, typename TA>
static int launch_w4(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
                     const Epi& e, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)w4::kernel<C, PL, QL, EPI, TO, TA>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    attr = true;
  }
  if (R % w4::BK) return (int)hipErrorInvalidValue;
  const int r_chunk = r_chunk_for(R, split, 64);
  const int nz = (R + r_chunk - 1) / r_chunk;
  dim3 grid(((M + 255) / 256) * ((N + 255) / 256) * nz);
  hipLaunchKernelGGL((w4::kernel<C, PL, QL, EPI, TO, TA>), grid, dim3(C::THREADS), C::LDS, s, (const bf16*)P, ldp,
                     (const bf16*)Q, ldq, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

static int num_cus() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// g4 (gemm_g4.hip): the plain bf16 forward / input-gradient GEMMs (ep 0) and the GELU' input gradient (ep
// 1, VIT_G4_GELU).  g4_enabled(): VIT_GEMM_G4=0 sends these classes back to the 8-wave V5 / V1 / V3 kernels
// (A/B); g4_launch returns -1 for shapes it does not take.
bool g4_enabled();
int g4_launch(int q_layout, int ep, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
              const Epi& e, hipStream_t s);
// row-tile band of the tile walk per class (tile_coords); VIT_GEMM_GROUP_{FWD,DGRAD}=<row tiles> (A/B)
// Bands of 8 row tiles help the wide-output GEMMs whose weight operand does not fit beside the
// row blocks in an XCD's 4 MiB L2 (the fc1 forward GELU pair and the fc2 GELU' input gradient:
// +3.5-4.5 % standalone at the half-batch shapes, tools/bench_kernels.py --groups) but measured
// 0.5-1 % slower in the two-stream step (profiles/r03/ab_group_colbatch.txt), so the forward keeps
// the row-major walk; -1 selects that per-shape band rule.  Round 5: with the plain input gradients
// on hipBLASLt the only input gradient left here is fc2's GELU' one, and bands of 4 row tiles cut its
// operand FETCH from 288 to 74 MB raw (profiles/r05/pmc_fc2_gelu_dgrad_bands.json) and measured +0.65 %
// in the step (profiles/r05/ab_dgrad_band4.txt): the input-gradient default is 4.
static int g_group[2] = {-2, -2};  // forward, dgrad; -2 = not yet read from the environment
static int group_for(int pl, int ql, int N, int R) {
  if (g_group[0] == -2) { const int v = env_variant("VIT_GEMM_GROUP_FWD"); g_group[0] = v == -1 ? 0 : v; }
  if (g_group[1] == -2) { const int v = env_variant("VIT_GEMM_GROUP_DGRAD"); g_group[1] = v == -1 ? 4 : v; }
  const int g = (pl == LAY_RC && ql == LAY_RC) ? g_group[0] : (pl == LAY_RC && ql == LAY_CR) ? g_group[1] : 0;
  if (g >= 0) return g;
  return (N >= 2048 && (int64_t)N * R * 2 >= ((int64_t)4 << 20)) ? 8 : 0;
}

template <int PL, int QL, int EPI, typename TO, typename TA>
static int launch_fast(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R,
                       int split, const Epi& e0, hipStream_t s) {
  Epi e = e0;
  if (split <= 1) e.group_m = group_for(PL, QL, N, R);
  const int v = pick_variant(PL, QL, M, N, R, split, EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD);
  if constexpr (PL == LAY_RC && EPI == EPI_STORE && std::is_same<TO, bf16>::value) {
    // the plain bf16 forward / input gradient: g4 by default (variant 20 forces it; any other forced
    // variant, a timing flag or VIT_GEMM_G4=0 keeps the 8-wave kernels)
    if (v == 20 || (g4_enabled() && g_variant < 0 && !e.dbg)) {
      const int rc = g4_launch(QL, 0, P, ldp, Q, ldq, M, N, R, split, e, s);
      if (rc != -1) return rc;
    }
  }
  if constexpr (PL == LAY_RC && QL == LAY_RC && EPI == EPI_BIAS_GELU && std::is_same<TO, bf16>::value) {
    // the fc1 GELU pair forward: g4 when bit 1 of VIT_G4_GELU / vit_gemm_g4_gelu is set
    if (v == 20 || (g4_enabled() && g_variant < 0 && !e.dbg)) {
      const int rc = g4_launch(QL, 2, P, ldp, Q, ldq, M, N, R, split, e, s);
      if (rc != -1) return rc;
    }
  }
  if constexpr (PL == LAY_RC && QL == LAY_CR && (EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD) &&
                std::is_same<TO, bf16>::value && std::is_same<TA, bf16>::value) {
    // the GELU' input gradient (C = dY W * act'): g4 when VIT_G4_GELU=1 (or variant 20)
    if (v == 20 || (g4_enabled() && g_variant < 0 && !e.dbg)) {
      const int rc = g4_launch(QL, 1, P, ldp, Q, ldq, M, N, R, split, e, s);
      if (rc != -1) return rc;
    }
  }
  if constexpr (PL == LAY_CR && QL == LAY_CR) {  // w4 ring / load-placement A/B (tools/bench_kernels.py --sweep)
    if (v == 12) return launch_w4<w4::Cfg<4, 0>, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (v == 13) return launch_w4<w4::Cfg<4, 2>, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (v == 14) return launch_w4<w4::Cfg<3, 1>, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (v == 15) return launch_w4<w4::Cfg<5, 1>, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
  }
  switch (v) {
    case 2: return launch_big<big::V2, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 5: return launch_big<big::V5, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 3: return launch_big<big::V3, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 4: return launch_big<big::V4, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 6: return launch_big<big::V6, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 7: return launch_big<big::V7, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 8: return launch_pp<4, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 9: return launch_pp<5, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    case 11: return launch_w4<w4::Default, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
    default: return launch_big<big::V1, PL, QL, EPI, TO, TA>(P, ldp, Q, ldq, M, N, R, split, e, s);
  }
}

// Stream-K workspaces registered per (device, stream) by the host (vit_gemm_streamk_workspace): the
// cut-tile fragment images (2 x 64 KiB per workgroup) and one ticket counter per workgroup boundary.
// The device is part of the key: the null stream is handle 0 on every device.
struct SkWs { int dev; hipStream_t s; float* part; int64_t part_bytes; int* cnt; int ncnt; };
static SkWs g_sk[32];
static int g_nsk = 0;
static int stream_device(hipStream_t s) {  // the null stream: the current device
  hipDevice_t d = -1;
  return hipStreamGetDevice(s, &d) == hipSuccess ? (int)d : -1;
}
// the device query runs only when a registered handle matches (not on every f32 GEMM
// dispatch; hipStreamGetDevice is a host-side lookup, legal on a capturing stream)
static const SkWs* sk_for(hipStream_t s) {
  int d = -2;
  for (int i = 0; i < g_nsk; ++i) {
    if (g_sk[i].s != s) continue;
    if (d == -2) d = stream_device(s);
    if (g_sk[i].dev == d) return &g_sk[i];
  }
  return nullptr;
}
// fraction of the last round's workgroup slots a plain launch of `tiles` leaves empty
static double ragged_waste(int64_t tiles, int slots) {
  const int64_t rounds = (tiles + slots - 1) / slots;
  return 1.0 - (double)tiles / (double)(rounds * slots);
}

template <int PL, int QL, int EPI, typename TO>
static int launch_f32(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
                      const Epi& e, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)f32m::gemm_kernel<PL, QL, EPI, TO, float>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, f32m::LDS);
    (void)hipFuncSetAttribute((const void*)f32m::gemm_sk_kernel<PL, QL, EPI, TO, float>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, f32m::LDS + 16);
    attr = true;
  }
  const int64_t tiles = (int64_t)((M + f32m::BM - 1) / f32m::BM) * ((N + f32m::BN - 1) / f32m::BN);
  const int G = 2 * num_cus();  // two workgroups per CU
  if (split <= 1 && R % f32m::BK == 0 && tiles >= G && ragged_waste(tiles, G) > 0.03) {
    const SkWs* w = sk_for(s);
    if (w && w->ncnt >= G && w->part_bytes >= (int64_t)G * 2 * f32m::BM * f32m::BN * 4) {
      // tile-aligned rounds, then the last full round plus the remainder shared by k-steps (sharing every
      // tile by k-steps from the start was 2-7 % slower on the tall forwards, round 3; that form and the
      // VIT_GEMM_STREAMK A/B switch were removed in round 5)
      const int dp_rounds = (int)(tiles / G) - 1;
      hipLaunchKernelGGL((f32m::gemm_sk_kernel<PL, QL, EPI, TO, float>), dim3(G), dim3(f32m::THREADS),
                         f32m::LDS + 16, s, (const float*)P, ldp, (const float*)Q, ldq, M, N, R, dp_rounds, e,
                         w->part, w->cnt);
      VIT_CHECK_LAUNCH();
      return 0;
    }
  }
  const int r_chunk = r_chunk_for(R, split, f32m::BK);
  const int nz = (R + r_chunk - 1) / r_chunk;
  dim3 grid(((M + f32m::BM - 1) / f32m::BM) * ((N + f32m::BN - 1) / f32m::BN) * nz);
  hipLaunchKernelGGL((f32m::gemm_kernel<PL, QL, EPI, TO, float>), grid, dim3(f32m::THREADS), f32m::LDS, s,
                     (const float*)P, ldp, (const float*)Q, ldq, M, N, R, r_chunk, e);
  VIT_CHECK_LAUNCH();
  return 0;
}

template <typename T, int EPI, typename TO, typename TA>
static int launch_gen(const void* P, int64_t sPi, int64_t sPr, const void* Q, int64_t sQj, int64_t sQr,
                      int M, int N, int R, int split, const Epi& e, hipStream_t s) {
  const int r_chunk = r_chunk_for(R, split, gen::TK);
  int nz = (R + r_chunk - 1) / r_chunk;
  if (nz == 0) nz = 1;
  const int64_t big_tiles = (int64_t)((N + 63) / 64) * ((M + 63) / 64) * nz;
  if (big_tiles < 256) {
    dim3 grid((N + 31) / 32, (M + 31) / 32, nz);
    hipLaunchKernelGGL((gen::gemm_kernel<32, T, EPI, TO, TA>), grid, dim3(256), 0, s,
                       (const T*)P, sPi, sPr, (const T*)Q, sQj, sQr, M, N, R, r_chunk, e);
  } else {
    dim3 grid((N + 63) / 64, (M + 63) / 64, nz);
    hipLaunchKernelGGL((gen::gemm_kernel<64, T, EPI, TO, TA>), grid, dim3(256), 0, s,
                       (const T*)P, sPi, sPr, (const T*)Q, sQj, sQr, M, N, R, r_chunk, e);
  }
  VIT_CHECK_LAUNCH();
  return 0;
}

// (layout, epilogue, output type) combinations the model uses get MFMA kernels; any other
// goes to the generic kernel (keeps the instantiation count, and the build time, down).
template <int PL, int QL, int EPI, typename TO> constexpr bool fast_combo() {
  constexpr bool f32o = std::is_same<TO, float>::value;
  if (PL == LAY_RC && QL == LAY_RC)  // forward
    return EPI == EPI_STORE || ((EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_QGELU) && !f32o) ||
           ((EPI == EPI_RESID || EPI == EPI_PATCH) && f32o);
  if (PL == LAY_RC && QL == LAY_CR) return EPI == EPI_STORE || EPI == EPI_GELU_BWD || EPI == EPI_QGELU_BWD;  // dgrad
  if (PL == LAY_CR && QL == LAY_CR) return EPI == EPI_STORE && f32o;  // wgrad (f32 slabs)
  return EPI == EPI_STORE;                                           // CR x RC (raw vit_gemm)
}

// One dispatcher for all layouts/epilogues.  out_dtype selects TO; for the
// *_BWD epilogues the pre-activation has the input dtype.
template <int EPI>
static int gemm_dispatch(int dtype, int out_dtype, int pl, int ql, int M, int N, int R,
                         const void* P, int64_t ldp, const void* Q, int64_t ldq, int split,
                         const Epi& e, hipStream_t s, bool allow_fast) {
  if (M <= 0 || N <= 0) return 0;
  if (allow_fast && fast_ok(dtype, pl, ql, M, N, R, P, Q, ldp, ldq) && (e.ldc % 4 == 0) && pl == LAY_RC) {
    // an RC P past the 32-bit staging offsets: launch row chunks with every row-indexed operand
    // shifted (the patch epilogue's row remap and split slabs are not row-shiftable: generic path)
    const int rows = rc_chunk_rows(M, ldp);
    if (rows < M) {
      if (EPI == EPI_PATCH || split > 1) {
        allow_fast = false;
      } else {
        const size_t osz = out_dtype == VIT_F32 ? 4 : 2;
        const size_t asz = (EPI == EPI_RESID) ? 4 : 2;  // RESID: f32 stream; *_BWD: pre-activation (bf16 here)
        for (int r0 = 0; r0 < M; r0 += rows) {
          const int m = M - r0 < rows ? M - r0 : rows;
          Epi c = e;
          c.C = (char*)e.C + (size_t)r0 * e.ldc * osz;
          if (e.aux) c.aux = (const char*)e.aux + (size_t)r0 * e.ld_aux * asz;
          if (e.aux_out) c.aux_out = (char*)e.aux_out + (size_t)r0 * e.ldc * osz;
          if (e.csum) c.csum = e.csum + (int64_t)(r0 / 64) * N;
          const int rc = gemm_dispatch<EPI>(dtype, out_dtype, pl, ql, m, N, R, (const char*)P + (size_t)r0 * ldp * 2,
                                            ldp, Q, ldq, split, c, s, true);
          if (rc) return rc;
        }
        return 0;
      }
    }
  }
  if (allow_fast && fast_ok(dtype, pl, ql, M, N, R, P, Q, ldp, ldq) && (e.ldc % 4 == 0)) {
#define FAST(PLx, QLx)                                                                                  \
    if (out_dtype == VIT_F32) {                                                                         \
      if constexpr (fast_combo<PLx, QLx, EPI, float>()) return launch_fast<PLx, QLx, EPI, float, bf16>(P, ldp, Q, ldq, M, N, R, split, e, s); \
    } else {                                                                                            \
      if constexpr (fast_combo<PLx, QLx, EPI, bf16>()) return launch_fast<PLx, QLx, EPI, bf16, bf16>(P, ldp, Q, ldq, M, N, R, split, e, s); \
    }
    if (pl == LAY_RC && ql == LAY_RC) { FAST(LAY_RC, LAY_RC) }
    if (pl == LAY_RC && ql == LAY_CR) { FAST(LAY_RC, LAY_CR) }
    if (pl == LAY_CR && ql == LAY_CR) { FAST(LAY_CR, LAY_CR) }
    if (pl == LAY_CR && ql == LAY_RC) { FAST(LAY_CR, LAY_RC) }
#undef FAST
  }
  if (allow_fast && out_dtype == VIT_F32 && fast_f32_ok(dtype, pl, ql, M, N, R, P, Q, ldp, ldq) && (e.ldc % 4 == 0) &&
      ((uintptr_t)e.C & 15) == 0 && f32_grid_ok(M, N, split)) {
    if (pl == LAY_RC && ql == LAY_RC) return launch_f32<LAY_RC, LAY_RC, EPI, float>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (pl == LAY_RC && ql == LAY_CR) return launch_f32<LAY_RC, LAY_CR, EPI, float>(P, ldp, Q, ldq, M, N, R, split, e, s);
    if (pl == LAY_CR && ql == LAY_CR) return launch_f32<LAY_CR, LAY_CR, EPI, float>(P, ldp, Q, ldq, M, N, R, split, e, s);
    return launch_f32<LAY_CR, LAY_RC, EPI, float>(P, ldp, Q, ldq, M, N, R, split, e, s);
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
    case EPI_ACC: return gemm_dispatch<EPI_ACC>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
    case EPI_PATCH: return gemm_dispatch<EPI_PATCH>(dtype, out_dtype, pl, ql, M, N, R, P, ldp, Q, ldq, split, e, s, allow_fast);
  }
  return (int)hipErrorInvalidValue;
}

static Epi make_epi() { Epi e; memset(&e, 0, sizeof(e)); e.dbg = g_dbg; return e; }

extern "C" {

// Host-side plan of the bf16 MFMA path's 32-bit staging offsets (no GPU needed; tests):
// rows per launch for an RC operand of M rows and `ld` elements per row (M when it fits one
// launch, 0 when even 256 rows do not fit).
int vit_gemm_rc_chunk_rows(int M, int64_t ld) { return rc_chunk_rows(M, ld); }

// Stream-K workspace for the f32 MFMA GEMMs launched on `stream` (C3's 128.5-row-tile shapes; the
// null stream means the current device's): part >= 2 * CUs * 2 * 128*128 floats, counters >= 2 * CUs
// ints zero-filled before first use (the kernel leaves them zero), both on the stream's device.  part == NULL removes
// the (device, stream) entry.  Without an entry the plain one-tile-per-workgroup launch runs.
int vit_gemm_streamk_workspace(void* stream, float* part, int64_t part_bytes, int* counters, int ncounters) {
  hipStream_t s = (hipStream_t)stream;
  const int d = stream_device(s);
  for (int i = 0; i < g_nsk; ++i)
    if (g_sk[i].s == s && g_sk[i].dev == d) {
      if (part == nullptr) {
        g_sk[i] = g_sk[--g_nsk];
        return 0;
      }
      g_sk[i] = SkWs{d, s, part, part_bytes, counters, ncounters};
      return 0;
    }
  if (part == nullptr || g_nsk == 32) return 0;  // a full registry: the stream keeps the plain launch
  g_sk[g_nsk++] = SkWs{d, s, part, part_bytes, counters, ncounters};
  return 0;
}

// Tuning hook: row-tile band of the forward / dgrad tile walk (0 = row-major, -1 = per-shape default;
// tile_coords).
int vit_gemm_group(int fwd, int dgrad) { g_group[0] = fwd; g_group[1] = dgrad; return 0; }

// Tuning hook: force GEMM configuration big::V<v> (-1 restores the per-shape heuristic).
int vit_gemm_variant(int v) { g_variant = v; g_dbg = v >= 100 ? v / 100 : 0; return 0; }

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

// f32 C[M][N] (contiguous) = sum_r P(i,r) Q(j,r) split along r on the generic kernel for small outputs over
// long reductions (DoRA's factor gradients: [in x r] / [r x out] over out / in = 1024..4096 products, 24-32
// workgroups unsplit): chunks of >= 128 products into slabs[z][M][N], then one slab sum in slab order
// (deterministic).  Without room for two slabs it is the unsplit launch.
int vit_gemm_splitk(int p_layout, int q_layout, int M, int N, int R, const float* P, int64_t ldp, const float* Q,
                    int64_t ldq, float* C, float* slabs, int64_t slab_floats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  const int64_t mn = (int64_t)M * N;
  const int tiles = ((N + 31) / 32) * ((M + 31) / 32);
  int split = 256 / (tiles > 0 ? tiles : 1);
  if (split > R / 128) split = R / 128;
  if (slabs == nullptr || (mn % 4) || ((uintptr_t)slabs & 15) || ((uintptr_t)C & 15)) split = 1;
  while (split > 1 && (int64_t)split * mn > slab_floats) --split;
  Epi e = make_epi();
  if (split < 2) {
    e.C = C; e.ldc = N;
    return gemm_any(EPI_STORE, VIT_F32, VIT_F32, p_layout, q_layout, M, N, R, P, ldp, Q, ldq, 1, e, s, false);
  }
  const int r_chunk = r_chunk_for(R, split, gen::TK);
  const int nz = (R + r_chunk - 1) / r_chunk;
  e.C = slabs; e.ldc = N; e.slab = mn;
  const int rc = gemm_any(EPI_STORE, VIT_F32, VIT_F32, p_layout, q_layout, M, N, R, P, ldp, Q, ldq, split, e, s, false);
  if (rc) return rc;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((mn / 4 + 255) / 256 + 1)), dim3(256), 0, s,
                     (const float*)slabs, nz, mn, C);
  VIT_CHECK_LAUNCH();
  return 0;
}

// F.linear forward: Y[M,N] = X[M,K] W[N,K]^T + b with a fused epilogue
//   epi = EPI_STORE (Y out_dtype), EPI_BIAS_GELU / EPI_BIAS_QGELU (Y = act'(pre), act_out = act(pre)),
//   EPI_RESID (Y f32 = resid + X W^T + b; Y may alias resid).
int vit_linear_fwd(int dtype, int out_dtype, int epi, int M, int N, int K, const void* X, int64_t ldx,
                   const void* W, const float* bias, void* Y, int64_t ldy, const void* resid,
                   void* act_out, void* stream) {
  Epi e = make_epi();
  e.C = Y; e.ldc = ldy; e.bias = bias; e.aux = resid; e.ld_aux = ldy; e.aux_out = act_out;
  return gemm_any(epi, dtype, out_dtype, LAY_RC, LAY_RC, M, N, K, X, ldx, W, K, 1, e, (hipStream_t)stream);
}

// Linear input gradient: dX[M,K] = dY[M,N] W[N,K]  (epi EPI_STORE or *_GELU_BWD: times the
// act'(pre) [M,K] the forward epilogue saved).
// dbias (optional, [K] f32) = column sums of dX as written by the epilogue (the bias
// gradient of the Linear whose output gradient dX is, e.g. fc1's from fc2's dgrad with
// the GELU' epilogue); needs `partial` >= vit_linear_dgrad_partial_floats(M, K).
int vit_linear_dgrad_partial_floats(int M, int K) {
  const int rows = (M + 63) / 64;
  return (int)((int64_t)rows * K + colreduce_scratch_floats(rows, K));
}

int vit_linear_dgrad(int dtype, int out_dtype, int epi, int M, int N, int K, const void* dY, int64_t lddy,
                     const void* W, void* dX, int64_t lddx, const void* pre, float* dbias, float* partial,
                     int64_t partial_floats, int defer_reduce, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  Epi e = make_epi();
  e.C = dX; e.ldc = lddx; e.aux = pre; e.ld_aux = lddx;
  const int rows = (M + 63) / 64;
  const bool fast = any_fast_ok(dtype, LAY_RC, LAY_CR, M, K, N, dY, W, lddy, K) && (lddx % 4 == 0) &&
                    (dtype == VIT_BF16 || (out_dtype == VIT_F32 && ((uintptr_t)dX & 15) == 0 && f32_grid_ok(M, K, 1)));
  if (dbias) {
    if (partial == nullptr || partial_floats < vit_linear_dgrad_partial_floats(M, K)) return (int)hipErrorInvalidValue;
    if (fast) e.csum = partial;
  }
  int rc = gemm_any(epi, dtype, out_dtype, LAY_RC, LAY_CR, M, K, N, dY, lddy, W, K, 1, e, s);
  if (rc || !dbias || M <= 0) return rc;
  if (!fast) {  // generic path: column sums of the stored output
    if (out_dtype == VIT_BF16)
      hipLaunchKernelGGL(colsum_partial_kernel<bf16>, dim3((K + 255) / 256, rows), dim3(256), 0, s, (const bf16*)dX,
                         lddx, M, K, 64, partial);
    else
      hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3((K + 255) / 256, rows), dim3(256), 0, s, (const float*)dX,
                         lddx, M, K, 64, partial);
    VIT_CHECK_LAUNCH();
  }
  if (defer_reduce) return 0;  // the caller reduces the partials (vit_colreduce)
  launch_colreduce(partial, rows, K, dbias, 0, s, partial + (int64_t)rows * K);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Column reduction out[N] (+)= sum_z part[z][N] (second stage of fused bias gradients);
// scratch (optional) >= ceil(S/64)*N floats.
int vit_colreduce(const float* part, int S, int N, float* out, int accumulate, float* scratch, void* stream) {
  if (S <= 0 || N <= 0) return 0;
  launch_colreduce(part, S, N, out, accumulate, (hipStream_t)stream, scratch);
  VIT_CHECK_LAUNCH();
  return 0;
}

// nq (<= 3) stacked [S][N] partial matrices reduced in one launch per stage into out0..out2.
int vit_colreduce_multi(const float* part, int nq, int S, int N, float* out0, float* out1, float* out2,
                        int accumulate, float* scratch, void* stream) {
  if (nq < 1 || nq > 3 || S <= 0 || N <= 0) return nq == 0 ? 0 : (int)hipErrorInvalidValue;
  float* outs[3] = {out0, out1, out2};
  launch_colreduce_multi(part, nq, S, N, outs, accumulate, (hipStream_t)stream, scratch);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Linear weight gradient: dW[N,K] (f32) = dY[M,N]^T X[M,K], split over M into
// `split` fp32 slabs in `workspace` (>= split*N*K*4 bytes) then reduced.
int vit_linear_wgrad(int dtype, int M, int N, int K, const void* dY, int64_t lddy, const void* X,
                     int64_t ldx, float* dW, int split, void* workspace, int64_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (split < 1) split = 1;
  if (M <= 0) return (int)hipMemsetAsync(dW, 0, (size_t)N * K * 4, s);
  // the MFMA kernel takes the BK-aligned rows; a ragged tail (M % 32) is added by the generic kernel
  const int tail = M % 32;
  const bool fast = (M - tail) > 0 && any_fast_ok(dtype, LAY_CR, LAY_CR, N, K, M - tail, dY, X, lddy, ldx) &&
                    (dtype == VIT_BF16 || (((uintptr_t)dW & 15) == 0 && f32_grid_ok(N, K, split)));
  const int R0 = fast ? M - tail : M;
  if (split > 1 && (workspace == nullptr || ws_bytes < (int64_t)split * N * K * 4)) return (int)hipErrorInvalidValue;
  Epi e = make_epi();
  int rc;
  if (split == 1) {
    e.C = dW; e.ldc = K;
    rc = gemm_any(EPI_STORE, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, R0, dY, lddy, X, ldx, 1, e, s, fast);
  } else {
    e.C = workspace; e.ldc = K; e.slab = (int64_t)N * K;
    const int r_chunk = r_chunk_for(R0, split, fast ? (dtype == VIT_BF16 ? 64 : f32m::BK) : gen::TK);
    const int nz = (R0 + r_chunk - 1) / r_chunk;
    rc = gemm_any(EPI_STORE, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, R0, dY, lddy, X, ldx, split, e, s, fast);
    if (rc) return rc;
    const int64_t n = (int64_t)N * K;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n / 4 + 255) / 256 + 1)), dim3(256), 0, s,
                       (const float*)workspace, nz, n, dW);
    VIT_CHECK_LAUNCH();
  }
  if (rc || R0 == M) return rc;
  Epi t = make_epi();
  t.C = dW; t.ldc = K;
  const size_t esz = dtype == VIT_BF16 ? 2 : 4;
  return gemm_any(EPI_ACC, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, M - R0, (const char*)dY + (size_t)R0 * lddy * esz,
                  lddy, (const char*)X + (size_t)R0 * ldx * esz, ldx, 1, t, s, false);
}

// Number of fp32 slabs vit_linear_wgrad_partials writes for this shape and split.
int vit_linear_wgrad_nslabs(int dtype, int M, int N, int K, int split) {
  if (split < 1) split = 1;
  if (M <= 0) return 0;
  const int tail = M % 32;
  const int R0 = M - tail;
  if (R0 <= 0) return 1;
  const int bk = dtype == VIT_BF16 ? 64 : f32m::BK;
  const int r_chunk = r_chunk_for(R0, split, bk);
  return (R0 + r_chunk - 1) / r_chunk;
}

// Weight gradient as split-K partials only: slabs[z][N][K] (f32, z < vit_linear_wgrad_nslabs) with
// dW = sum_z slabs[z]; the caller reduces them (vit_colreduce_batch: S = nslabs, N = N*K), e.g. in
// the one reduction launch of a block's backward.  The ragged M % 32 rows are added into the last slab.
int vit_linear_wgrad_partials(int dtype, int M, int N, int K, const void* dY, int64_t lddy, const void* X,
                              int64_t ldx, int split, float* slabs, int64_t slab_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int nz = vit_linear_wgrad_nslabs(dtype, M, N, K, split);
  if (M <= 0 || nz <= 0) return (int)hipErrorInvalidValue;
  if (slabs == nullptr || slab_bytes < (int64_t)nz * N * K * 4 || ((uintptr_t)slabs & 15)) return (int)hipErrorInvalidValue;
  const int tail = M % 32;
  const int R0 = M - tail;
  Epi e = make_epi();
  e.C = slabs; e.ldc = K; e.slab = (int64_t)N * K;
  if (R0 > 0) {
    const bool fast = any_fast_ok(dtype, LAY_CR, LAY_CR, N, K, R0, dY, X, lddy, ldx) &&
                      (dtype == VIT_BF16 || f32_grid_ok(N, K, split));
    // the MFMA and generic paths chunk the rows the same way (r_chunk_for with their BK; the generic
    // TK = 64 = the bf16 BK) only on the bf16 path: elsewhere one slab per launch keeps nz exact
    if (!fast && dtype != VIT_BF16) return (int)hipErrorInvalidValue;
    const int rc = gemm_any(EPI_STORE, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, R0, dY, lddy, X, ldx, split, e, s, fast);
    if (rc) return rc;
  } else {
    const int rc = (int)hipMemsetAsync(slabs, 0, (size_t)N * K * 4, s);
    if (rc) return rc;
  }
  if (tail == 0) return 0;
  Epi t = make_epi();
  t.C = slabs + (int64_t)(nz - 1) * N * K; t.ldc = K;
  const size_t esz = dtype == VIT_BF16 ? 2 : 4;
  return gemm_any(EPI_ACC, dtype, VIT_F32, LAY_CR, LAY_CR, N, K, tail, (const char*)dY + (size_t)R0 * lddy * esz,
                  lddy, (const char*)X + (size_t)R0 * ldx * esz, ldx, 1, t, s, false);
}

// Two weight gradients over the same M token rows as ONE ping-pong launch (split-K partials only,
// slabs as vit_linear_wgrad_partials for each): dW_a[Na,Ka] = dYa^T Xa, dW_b[Nb,Kb] = dYb^T Xb.
// bf16, M % 32 == 0 and the MFMA operand rules for both; otherwise hipErrorInvalidValue (the caller
// launches them one by one).
int vit_linear_wgrad_partials2(int M, int split, int Na, int Ka, const void* dYa, int64_t lddya, const void* Xa,
                               int64_t ldxa, float* slabs_a, int64_t bytes_a, int Nb, int Kb, const void* dYb,
                               int64_t lddyb, const void* Xb, int64_t ldxb, float* slabs_b, int64_t bytes_b,
                               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (split < 1) split = 1;
  if (M <= 0 || M % 32) return (int)hipErrorInvalidValue;
  if (!fast_ok(VIT_BF16, LAY_CR, LAY_CR, Na, Ka, M, dYa, Xa, lddya, ldxa) ||
      !fast_ok(VIT_BF16, LAY_CR, LAY_CR, Nb, Kb, M, dYb, Xb, lddyb, ldxb))
    return (int)hipErrorInvalidValue;
  const int nz = vit_linear_wgrad_nslabs(VIT_BF16, M, Na, Ka, split);
  if (!slabs_a || !slabs_b || bytes_a < (int64_t)nz * Na * Ka * 4 || bytes_b < (int64_t)nz * Nb * Kb * 4 ||
      ((uintptr_t)slabs_a & 15) || ((uintptr_t)slabs_b & 15))
    return (int)hipErrorInvalidValue;
  const int r_chunk = r_chunk_for(M, split, 64);
  auto prob = [&](const void* dY, int64_t lddy, const void* X, int64_t ldx, int N, int K, float* slabs) {
    big::PPProb p;
    p.P = (const bf16*)dY; p.Q = (const bf16*)X; p.ldp = lddy; p.ldq = ldx;
    p.M = N; p.N = K; p.R = M; p.r_chunk = r_chunk;
    p.nwg = ((N + 255) / 256) * ((K + 255) / 256) * nz;
    p.e = make_epi();
    p.e.C = slabs; p.e.ldc = K; p.e.slab = (int64_t)N * K;
    return p;
  };
  const big::PPProb a = prob(dYa, lddya, Xa, ldxa, Na, Ka, slabs_a), b = prob(dYb, lddyb, Xb, ldxb, Nb, Kb, slabs_b);
  // the weight-gradient kernel pick_variant chooses: 11-15 = w4 and its ring / load-placement siblings (as
  // launch_fast maps them), anything else the ping-pong kernel (8, the default; VIT_GEMM_WGRAD A/B)
  auto pair_w4 = [&](auto cfg_tag) {
    using C = decltype(cfg_tag);
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)w4::kernel2<C, LAY_CR, LAY_CR, EPI_STORE, float, bf16>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
      attr = true;
    }
    hipLaunchKernelGGL((w4::kernel2<C, LAY_CR, LAY_CR, EPI_STORE, float, bf16>), dim3(a.nwg + b.nwg),
                       dim3(C::THREADS), C::LDS, s, a, b);
  };
  switch (pick_variant(LAY_CR, LAY_CR, Na, Ka, M, split, false)) {
    case 11: pair_w4(w4::Default{}); break;
    case 12: pair_w4(w4::Cfg<4, 0>{}); break;
    case 13: pair_w4(w4::Cfg<4, 2>{}); break;
    case 14: pair_w4(w4::Cfg<3, 1>{}); break;
    case 15: pair_w4(w4::Cfg<5, 1>{}); break;
    default: {
      using C = big::PP<4>;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)big::pp_kernel2<4, LAY_CR, LAY_CR, EPI_STORE, float, bf16>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
        attr = true;
      }
      hipLaunchKernelGGL((big::pp_kernel2<4, LAY_CR, LAY_CR, EPI_STORE, float, bf16>), dim3(a.nwg + b.nwg),
                         dim3(C::THREADS), C::LDS, s, a, b);
    }
  }
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
  float* scratch = partial_floats >= (int64_t)S * N + colreduce_scratch_floats(S, N) ? partial + (int64_t)S * N : nullptr;
  launch_colreduce(partial, S, N, out, accumulate, s, scratch);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Patch embedding forward (timm PatchEmbed Conv2d 16/16 + _pos_embed):
//   x[b*(np+1) + 1 + p][n] = U[b*np + p] . Wpe[n] + bpe[n] + pos[1+p][n]   (f32 out)
// U = unfolded patches [B*np, K] (vit_patch_unfold).  CLS rows: vit_cls_pos_fill.
int vit_patch_embed_fwd_ld(int dtype, int B, int np, int D, int K, const void* U, int64_t ldu, const void* W,
                           int64_t ldw, const float* bias, const float* pos, float* x, void* stream) {
  if (ldu < K || ldw < K) return (int)hipErrorInvalidValue;
  Epi e = make_epi();
  e.C = x; e.ldc = D; e.bias = bias; e.pos = pos; e.n_patch = np;
  return gemm_any(EPI_PATCH, dtype, VIT_F32, LAY_RC, LAY_RC, B * np, D, K, U, ldu, W, ldw, 1, e, (hipStream_t)stream);
}

int vit_patch_embed_fwd(int dtype, int B, int np, int D, int K, const void* U, const void* W,
                        const float* bias, const float* pos, float* x, void* stream) {
  return vit_patch_embed_fwd_ld(dtype, B, np, D, K, U, K, W, K, bias, pos, x, stream);
}

}  // extern "C"
