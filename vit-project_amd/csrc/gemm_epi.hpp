// The GEMM epilogue contract shared by the bf16 GEMM translation units (gemm.hip: the 8-wave / ping-pong /
// w4 kernels and the f32 MFMA path; gemm_g4.hip: the 4-wave plain-store kernel): the epilogue selector,
// its operands, the permlane-widened 16-B bf16 fragment store and the tile walk.
#pragma once
#include "common.hpp"
#include "gemm_lds.hpp"

// BIAS_GELU / BIAS_QGELU: C = act'(pre) (what the backward needs), aux_out = act(pre);
// GELU_BWD / QGELU_BWD: C = acc * aux, aux = that saved act'(pre)  (same for both).
enum { EPI_STORE = 0, EPI_BIAS_GELU = 1, EPI_RESID = 2, EPI_GELU_BWD = 3, EPI_PATCH = 4,
       EPI_BIAS_QGELU = 5, EPI_QGELU_BWD = 6, EPI_ACC = 7 };
struct Epi {
  void* C; int64_t ldc;
  const float* bias;        // [N] or null
  const void* aux; int64_t ld_aux;  // EPI_RESID: f32 residual;  *_BWD: pre-activation (T)
  void* aux_out;            // BIAS_GELU: activation output (T, ld = ldc)
  const float* pos;         // EPI_PATCH: pos_embed [seq, N]
  int n_patch;              // EPI_PATCH: patches per image (seq = n_patch + 1)
  int64_t slab;             // split-r: element offset of slab z
  float* csum;              // optional column sums of the epilogue output: [ceil(M/64)][N] partials (64-row groups)
  int group_m;              // > 0: tiles walk column-major inside bands of group_m row tiles (L2 reuse of Q columns)
  int dbg;                  // timing experiments only (vit_gemm_variant(v + 100*bits)): 1 = no in-loop loads, 2 = no in-loop barriers, 4 = no epilogue, 16 = fragment epilogue
};

// bf16 fragment-pair store: a lane holds C[i][4g..4g+3] of two 16-column fragments (g = lane >> 4); one
// v_permlane16_swap per dword (vdst = fragment b, src = fragment b+1) trades lane rows g=1 / g=3 of b with
// rows g=0 / g=2 of b+1, after which every lane holds 8 consecutive columns of the pair: g=0 cols 0-7,
// g=2 8-15, g=1 16-23, g=3 24-31 -- one dwordx4 store instead of two dwordx2.
__device__ __forceinline__ void store_pair_bf16(void* base, int64_t ldc, int i, int col, const f32x4& x,
                                                const f32x4& y, bool ok) {
  const bf16x4 px = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
  const bf16x4 py = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x2 ux = __builtin_bit_cast(u32x2, px), uy = __builtin_bit_cast(u32x2, py);
  const auto r0 = __builtin_amdgcn_permlane16_swap(ux[0], uy[0], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(ux[1], uy[1], false, false);
  if (ok) *reinterpret_cast<u32x4*>((bf16*)base + (int64_t)i * ldc + col) = u32x4{r0[0], r1[0], r0[1], r1[1]};
}


// Column sums of a wave's epilogue outputs over one 64-row group (4 accumulator
// rows of 16): cs[b] holds this lane's partial for columns j..j+3 of fragment b;
// reduce over the 16 lanes of each row group and store one partial row.
template <int AJ>
__device__ __forceinline__ void csum_flush(const Epi& e, f32x4 (&cs)[AJ], int row0, int M, int N, int jbase, int lane) {
#pragma unroll
  for (int b = 0; b < AJ; ++b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float v = cs[b][t];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      cs[b][t] = v;
    }
    const int j = jbase + b * 16 + 4 * (lane >> 4);
    if ((lane & 15) == 0 && row0 < M && j < N)
      *reinterpret_cast<f32x4*>(e.csum + (int64_t)(row0 >> 6) * N + j) = cs[b];
    cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

namespace big {
// Tile t of a tiles_i x tiles_j grid.  group_m == 0: row-major (consecutive t share a row tile,
// so the P rows stay in the XCD's L2 while every Q column block streams past).  group_m > 0:
// bands of group_m row tiles walked column-major, so the workgroups an XCD runs at once cover
// group_m row tiles x a few column tiles and both operand blocks fit its 4 MiB L2.
__device__ __forceinline__ void tile_coords(int t, int tiles_i, int tiles_j, int group_m, int& ti, int& tj) {
  if (group_m <= 0) {
    ti = t / tiles_j;
    tj = t - ti * tiles_j;
    return;
  }
  const int per = group_m * tiles_j;
  const int g = t / per, r = t - g * per;
  const int first = g * group_m;
  const int gsz = min(tiles_i - first, group_m);
  tj = r / gsz;
  ti = first + (r - tj * gsz);
}

}  // namespace big
