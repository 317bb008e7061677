// Lab kernel (not product code): the V5 forward main loop (256x256x64 tile, 8 waves of 128x64, 2-stage
// global_load_lds ring, RC x RC) with v_mfma_f32_32x32x16_bf16 (MF = 32) or v_mfma_f32_16x16x32_bf16
// (MF = 16), to compare their main-loop rates.  32x32x16 holds the SIMD's issue for 8 of its 32 cycles
// (16x16x32: 8 of 16), so half the issue slots per FLOP go to MFMAs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I vit-project_amd/csrc tools/lab/mf32_lab.hip -o tools/lab/libmf32_lab.so
// mode 0: bf16 store (+bias), 1: no epilogue, 2: no loads in the k-loop and no epilogue.
#include "common.hpp"
#include "gemm_lds.hpp"

using namespace big;
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MF> struct MC {
  static constexpr int FR = MF;                 // rows of one fragment
  static constexpr int AI = 128 / MF, AJ = 64 / MF;
  static constexpr int KSUB = 64 / (MF == 32 ? 16 : 32);  // MFMA k-substeps per 64-deep k-step
};

template <int MF, int LP = 0>
__device__ __forceinline__ void lab_body(const bf16* __restrict__ P, const bf16* __restrict__ Q,
                                         const float* __restrict__ bias, bf16* __restrict__ C, int M, int N, int K,
                                         int mode) {
  using T = MC<MF>;
  constexpr int BK = 64, STAGE = 65536, PIMG = 32768;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / 4, wj = wave % 4;
  const int tiles_j = N / 256;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int i0 = t / tiles_j * 256, j0 = (t % tiles_j) * 256;
  const int nk = K / BK;
  uint32_t poff[4], qoff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = (wave * 4 + u) * 8 + lane / 8;
    const int c = (lane % 8) ^ rc_sw<BK>(row);
    poff[u] = (uint32_t)((int64_t)min(i0 + row, M - 1) * K * 2 + c * 16);
    qoff[u] = (uint32_t)((int64_t)(j0 + row) * K * 2 + c * 16);
  }
  // piece p (0..7) of k-step k: 0-3 of P, 4-7 of Q
  auto piece = [&](int k, int p) {
    char* buf = smem + (k & 1) * STAGE;
    if (p < 4) {
      const char* pb = reinterpret_cast<const char*>(P) + (int64_t)k * BK * 2;
      __builtin_amdgcn_global_load_lds((const void*)(pb + poff[p]), LDS_PTR(buf + (wave * 4 + p) * 1024), 16, 0, 0);
    } else {
      const char* qb = reinterpret_cast<const char*>(Q) + (int64_t)k * BK * 2;
      __builtin_amdgcn_global_load_lds((const void*)(qb + qoff[p - 4]), LDS_PTR(buf + PIMG + (wave * 4 + p - 4) * 1024),
                                       16, 0, 0);
    }
  };
  auto issue = [&](int k) {
#pragma unroll
    for (int p = 0; p < 8; ++p) piece(k, p);
  };
  // lane base of the k-substep s fragment read (rows = fragment base + lane row; the swizzle depends on
  // the row mod 16 only, a lane constant for 16- / 32-aligned fragment bases)
  uint32_t lb[2][T::KSUB];
#pragma unroll
  for (int s = 0; s < T::KSUB; ++s) {
    const int r = MF == 32 ? (lane & 31) : (lane & 15);
    const int ch = MF == 32 ? 2 * s + (lane >> 5) : 4 * s + (lane >> 4);
    lb[0][s] = (uint32_t)(wi * 128 * 128 + rc_off<BK>(r, ch));
    lb[1][s] = (uint32_t)(PIMG + wj * 64 * 128 + rc_off<BK>(r, ch));
  }
  using Acc = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  Acc acc[T::AI][T::AJ];
#pragma unroll
  for (int a = 0; a < T::AI; ++a)
#pragma unroll
    for (int b = 0; b < T::AJ; ++b) acc[a][b] = Acc{};
  const bool noload = mode == 2;
  if (!noload) issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<0>();
    lds_barrier();
    const bool more = kt + 1 < nk && !noload;
    if (LP == 0 && more) issue(kt + 1);
    const uint32_t cur = lds_addr(smem + (kt & 1) * STAGE);
    Unroll<T::KSUB>::run([&](auto sI) {
      constexpr int s = decltype(sI)::value;
      bf16x8 pf[T::AI], qf[T::AJ];
      if constexpr (LP == 4) {  // P pieces before the first substep's reads, Q pieces after the last MFMAs
        if (more && s == 0) {
#pragma unroll
          for (int p = 0; p < 4; ++p) piece(kt + 1, p);
        }
      }
      if constexpr (LP == 1) {
        if (more) {
#pragma unroll
          for (int p = 0; p < 8 / T::KSUB; ++p) piece(kt + 1, s * (8 / T::KSUB) + p);
        }
      }
      Unroll<T::AJ>::run([&](auto bI) {
        constexpr int b = decltype(bI)::value;
        qf[b] = asm_read128_off<b * MF * 128>(cur + lb[1][s]);
      });
      Unroll<T::AI>::run([&](auto aI) {
        constexpr int a = decltype(aI)::value;
        pf[a] = asm_read128_off<a * MF * 128>(cur + lb[0][s]);
      });
      lgkm_wait0();
      constexpr int NM = T::AI * T::AJ, PPS = 8 / T::KSUB;  // MFMAs, pieces per substep
#pragma unroll
      for (int a = 0; a < T::AI; ++a)
#pragma unroll
        for (int b = 0; b < T::AJ; ++b) {
          if constexpr (MF == 32) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qf[b], pf[a], acc[a][b], 0, 0, 0);
          else acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[b], pf[a], acc[a][b], 0, 0, 0);
          if constexpr (LP == 2) {
            constexpr int dummy = 0; (void)dummy;
            const int m = a * T::AJ + b;
            if ((m + 1) % (NM / PPS) == 0 && more) {
              __builtin_amdgcn_sched_barrier(0);
              piece(kt + 1, s * PPS + (m + 1) / (NM / PPS) - 1);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (LP == 4) {
        if (more && s == T::KSUB - 1) {
#pragma unroll
          for (int p = 4; p < 8; ++p) piece(kt + 1, p);
        }
      }
      if constexpr (LP == 3) {  // after this substep's MFMAs: substep s's share of the pieces
        if (more) {
#pragma unroll
          for (int p = 0; p < PPS; ++p) piece(kt + 1, s * PPS + p);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  }
  if (mode != 0) {
#pragma unroll
    for (int a = 0; a < T::AI; ++a)
#pragma unroll
      for (int b = 0; b < T::AJ; ++b) asm volatile("" ::"v"(acc[a][b]));
    return;
  }
  // 8-B stores of 4 consecutive columns
#pragma unroll
  for (int a = 0; a < T::AI; ++a)
#pragma unroll
    for (int b = 0; b < T::AJ; ++b) {
      if constexpr (MF == 32) {
        const int i = i0 + wi * 128 + a * 32 + (lane & 31);
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const int j = j0 + wj * 64 + b * 32 + 8 * rg + 4 * (lane >> 5);
          const f32x4 bb = bias ? *reinterpret_cast<const f32x4*>(bias + j) : f32x4{0.f, 0.f, 0.f, 0.f};
          const bf16x4 o = {(bf16)(acc[a][b][4 * rg] + bb[0]), (bf16)(acc[a][b][4 * rg + 1] + bb[1]),
                            (bf16)(acc[a][b][4 * rg + 2] + bb[2]), (bf16)(acc[a][b][4 * rg + 3] + bb[3])};
          if (i < M) *reinterpret_cast<bf16x4*>(C + (int64_t)i * N + j) = o;
        }
      } else {
        const int i = i0 + wi * 128 + a * 16 + (lane & 15);
        const int j = j0 + wj * 64 + b * 16 + 4 * (lane >> 4);
        const f32x4 bb = bias ? *reinterpret_cast<const f32x4*>(bias + j) : f32x4{0.f, 0.f, 0.f, 0.f};
        const bf16x4 o = {(bf16)(acc[a][b][0] + bb[0]), (bf16)(acc[a][b][1] + bb[1]), (bf16)(acc[a][b][2] + bb[2]),
                          (bf16)(acc[a][b][3] + bb[3])};
        if (i < M) *reinterpret_cast<bf16x4*>(C + (int64_t)i * N + j) = o;
      }
    }
}

__global__ __launch_bounds__(512, 1) void lab_k32(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                  int N, int K, int mode) {
  lab_body<32>(P, Q, bias, C, M, N, K, mode);
}
__global__ __launch_bounds__(512, 1) void lab_k16(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                  int N, int K, int mode) {
  lab_body<16>(P, Q, bias, C, M, N, K, mode);
}
__global__ __launch_bounds__(512, 1) void lab_k16b(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                   int N, int K, int mode) {
  lab_body<16, 1>(P, Q, bias, C, M, N, K, mode);
}
__global__ __launch_bounds__(512, 1) void lab_k16d(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                   int N, int K, int mode) {
  lab_body<16, 3>(P, Q, bias, C, M, N, K, mode);
}
__global__ __launch_bounds__(512, 1) void lab_k16e(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                   int N, int K, int mode) {
  lab_body<16, 4>(P, Q, bias, C, M, N, K, mode);
}
__global__ __launch_bounds__(512, 1) void lab_k16c(const bf16* P, const bf16* Q, const float* bias, bf16* C, int M,
                                                   int N, int K, int mode) {
  lab_body<16, 2>(P, Q, bias, C, M, N, K, mode);
}

extern "C" int lab_gemm(int mf, int M, int N, int K, const void* X, const void* W, const float* bias, void* C, int mode,
                        void* stream) {
  if (N % 256 || K % 64 || M <= 0) return 1;
  const int grid = ((M + 255) / 256) * (N / 256);
  auto k = mf == 32 ? lab_k32 : mf == 17 ? lab_k16b : mf == 18 ? lab_k16c : mf == 19 ? lab_k16d : mf == 20 ? lab_k16e : lab_k16;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), 131072, (hipStream_t)stream, (const bf16*)X, (const bf16*)W, bias,
                     (bf16*)C, M, N, K, mode);
  return (int)hipGetLastError();
}
