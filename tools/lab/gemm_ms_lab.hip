// Multi-tile forward GEMM with deferred stores (bf16, P and Q both r-contiguous: Y = X W^T + b).
//
// Why: on the one-tile-per-workgroup 256x256 kernel (gemm.hip V5) the epilogue runs after the
// k-loop with nothing to overlap it (the tile's accumulators fill half the register file, so a
// second workgroup cannot share the CU): 26-45 % of a K = 768 forward is its store tail
// (tools/bench_kernels.py --sweep=5,405).  Here a workgroup runs several tiles (w, w + G, ...):
// at the end of a tile its accumulators are packed to bf16 in registers (bias added; the GELU
// pair keeps the pre-activation) and the 16-B stores of that tile are issued during the first
// k-steps of the next one, under its MFMAs; the next tile's first operand stage is loaded during
// the last k-step of the current one, so the pipeline does not drain between tiles either.
//
// Tile BM x 256 x 64 (BM = 256 or 192), 8 waves as 2 x 4 (wave tile BM/2 x 64), a 2-stage
// global_load_lds ring (the RC image layout and fragment reads of gemm.hip's gemm_tile), the
// bias vector staged once into the LDS left over by the ring.  Same k-order as gemm_tile, so the
// results are bit-identical to the V5 kernel for the same epilogue.
#include "common.hpp"
#include "gemm_lds.hpp"

namespace ms {
using namespace big;

enum { MS_STORE = 0, MS_BIAS_GELU = 1 };  // values of gemm.hip's EPI_STORE / EPI_BIAS_GELU

struct Args {
  const bf16* P; int64_t ldp;  // X [M][K]
  const bf16* Q; int64_t ldq;  // W [N][K]
  int M, N, K;
  bf16* C; int64_t ldc;        // STORE: Y;  BIAS_GELU: GELU'(pre)
  bf16* C2;                    // BIAS_GELU: GELU(pre) (ld = ldc)
  const float* bias;           // [N] or null
};

template <int BM_, int PRE_> struct Cfg {
  static constexpr int BM = BM_, BN = 256, BK = 64, WI = 2, WJ = 4, S = 2, WAVES = 8, THREADS = 512;
  static constexpr int WM = BM / WI, WN = BN / WJ, AI = WM / 16, AJ = WN / 16, KS = BK / 32;
  static constexpr int PIMG = BM * BK * 2, QIMG = BN * BK * 2, STAGE = PIMG + QIMG, RING = S * STAGE;
  static constexpr int GP = PIMG / 1024 / WAVES, GQ = QIMG / 1024 / WAVES;
  static constexpr int NGRP = AI * AJ / 2;                 // 16-B store groups (fragment pairs) per wave
  static constexpr int PRE = PRE_;                         // groups stored at once at the end of a tile
  static constexpr int GPS = 2;                            // store groups per store-carrying k-step
  static constexpr int NSTEP = (NGRP - PRE) / GPS;         // k-steps that carry the previous tile's stores
  static constexpr int BIAS_FLOATS = (163840 - RING) / 4;  // bias entries that fit beside the ring
  static constexpr int PH = BM == 256 ? 2 : 1;             // parts the P fragment reads come in
  static_assert(GP * 1024 * WAVES == PIMG && GQ * 1024 * WAVES == QIMG, "1-KiB pieces per wave");
  static_assert(PRE + GPS * NSTEP == NGRP, "store groups spread evenly over NSTEP k-steps");
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// two column fragments (b, b+1) of one row -> this lane's 8 consecutive bf16 (gemm.hip store_pair_bf16)
__device__ __forceinline__ u32x4 pack_pair(const f32x4& x, const f32x4& y) {
  const bf16x4 px = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
  const bf16x4 py = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
  const u32x2 ux = __builtin_bit_cast(u32x2, px), uy = __builtin_bit_cast(u32x2, py);
  const auto r0 = __builtin_amdgcn_permlane16_swap(ux[0], uy[0], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(ux[1], uy[1], false, false);
  return u32x4{r0[0], r1[0], r0[1], r1[1]};
}

template <int BM, int PRE, int EPI, int QL>
__global__ __launch_bounds__(512, 1) void gemm_ms_kernel(Args a) {
  using C = Cfg<BM, PRE>;
  constexpr int BK = C::BK, AI = C::AI, AJ = C::AJ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / C::WJ, wj = wave % C::WJ;
  const int M = a.M, N = a.N;
  const int tiles_j = N / C::BN, tiles_i = (M + BM - 1) / BM, tiles = tiles_i * tiles_j;
  const int G = gridDim.x, w = xcd_remap(blockIdx.x, G);
  const int ntile = w < tiles ? (tiles - w + G - 1) / G : 0;
  const int nk = a.K / BK;

  float* sbias = reinterpret_cast<float*>(smem + C::RING);
  if (a.bias)
    for (int j = tid * 4; j < N; j += C::THREADS * 4)
      *reinterpret_cast<f32x4*>(sbias + j) = *reinterpret_cast<const f32x4*>(a.bias + j);

  // per-lane byte offsets of this wave's staging pieces (gemm_tile's RC addressing), per tile
  uint32_t poff[C::GP], qoff[C::GQ];
  auto set_tile = [&](int t, int& i0, int& j0) {
    const int ti = t / tiles_j, tj = t - ti * tiles_j;
    i0 = ti * BM;
    j0 = tj * C::BN;
#pragma unroll
    for (int u = 0; u < C::GP; ++u) {
      const int row = (wave * C::GP + u) * 8 + lane / 8;
      const int c = (lane % 8) ^ rc_sw<BK>(row);
      poff[u] = (uint32_t)((int64_t)min(i0 + row, M - 1) * a.ldp * 2 + c * 16);
    }
#pragma unroll
    for (int u = 0; u < C::GQ; ++u) {
      if constexpr (QL == LAY_RC) {
        const int row = (wave * C::GQ + u) * 8 + lane / 8;
        const int c = (lane % 8) ^ rc_sw<BK>(row);
        qoff[u] = (uint32_t)((int64_t)(j0 + row) * a.ldq * 2 + c * 16);
      } else {  // half-blocked CR image (gemm_lds.hpp): W [R][N] read as 16-row x 64-B pieces
        qoff[u] = (uint32_t)(crh_src<C::BN>(wave * C::GQ + u, lane, a.ldq, j0, N) * 2);
      }
    }
  };
  auto issue = [&](int k, int slot) {
    char* buf = smem + slot * C::STAGE;
    const char* pb = reinterpret_cast<const char*>(a.P) + (int64_t)k * BK * 2;
    const char* qb = reinterpret_cast<const char*>(a.Q) + (int64_t)k * BK * 2 * (QL == LAY_RC ? 1 : a.ldq);
#pragma unroll
    for (int u = 0; u < C::GP; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(pb + poff[u]), LDS_PTR(buf + (wave * C::GP + u) * 1024), 16, 0, 0);
#pragma unroll
    for (int u = 0; u < C::GQ; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(qb + qoff[u]), LDS_PTR(buf + C::PIMG + (wave * C::GQ + u) * 1024),
                                       16, 0, 0);
  };
  uint32_t rc_lane[2][C::KS];
#pragma unroll
  for (int kk = 0; kk < C::KS; ++kk) {
    rc_lane[0][kk] = (uint32_t)(wi * AI * 16 * BK * 2 + rc_off<BK>(lane & 15, kk * 4 + (lane >> 4)));
    rc_lane[1][kk] = (uint32_t)(wj * AJ * 16 * BK * 2 + rc_off<BK>(lane & 15, kk * 4 + (lane >> 4)));
  }
  uint32_t crh_q[2][2];  // CR Q: [lo / hi read][fragment parity], this wave's first fragment pair folded in
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) crh_q[lh][h] = C::PIMG + crh_lane<C::BN>(lane, lh, h) + (uint32_t)(wj * AJ / 2 * 1024);

  f32x4 acc[AI][AJ];
  u32x4 pk[AI][AJ / 2];  // the previous tile's outputs (STORE) / bf16 pre-activations (GELU), 16-B store layout
  int pi0 = 0, pj0 = 0;  // that tile's origin
  bool pending = false;
  const int g4 = lane >> 4;
  const int colsel = (g4 & 1) * 16 + (g4 >> 1) * 8;

  // store group g (fragment pair bp of accumulator row ai) of the tile at (ti0, tj0) from v
  auto store_vals = [&](auto gI, const u32x4& v, int ti0, int tj0) {
    constexpr int g = decltype(gI)::value;
    constexpr int ai = g / (AJ / 2), bp = g % (AJ / 2);
    const int i = ti0 + wi * C::WM + ai * 16 + (lane & 15);
    const int64_t off = (int64_t)i * a.ldc + tj0 + wj * C::WN + bp * 32 + colsel;
    if (i < M) {
      if constexpr (EPI == MS_STORE) {
        *reinterpret_cast<u32x4*>(a.C + off) = v;
      } else {
        const bf16x8 x = __builtin_bit_cast(bf16x8, v);
        bf16x8 d, y;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float ga, gd;
          gelu_fast_both((float)x[q], ga, gd);
          d[q] = (bf16)gd;
          y[q] = (bf16)ga;
        }
        *reinterpret_cast<bf16x8*>(a.C + off) = d;
        *reinterpret_cast<bf16x8*>(a.C2 + off) = y;
      }
    }
  };
  auto store_group = [&](auto gI) {
    constexpr int g = decltype(gI)::value;
    store_vals(gI, pk[g / (AJ / 2)][g % (AJ / 2)], pi0, pj0);
  };
  constexpr int SPG = EPI == MS_STORE ? 1 : 2;  // global stores per group

  // one k-step's MFMAs from ring slot `slot`; the P fragments are read in PH parts (PH = 2 on the
  // 256-row tile: 16 fewer fragment registers live beside the deferred stores)
  auto mma_step = [&](int slot) {
    constexpr int AH = AI / C::PH;
    const uint32_t cur = lds_addr(smem + slot * C::STAGE);
    Unroll<C::KS>::run([&](auto kkI) {
      constexpr int kk = decltype(kkI)::value;
      bf16x8 qf[AJ];
      if constexpr (QL == LAY_RC) {
        const uint32_t qa = cur + C::PIMG + rc_lane[1][kk];
        Unroll<AJ>::run([&](auto bI) {
          constexpr int b = decltype(bI)::value;
          qf[b] = asm_read128_off<b * 16 * BK * 2>(qa);
        });
      } else {
        Unroll<AJ>::run([&](auto bI) {
          constexpr int b = decltype(bI)::value;
          qf[b] = frag_crh<C::BN, kk, b>(crh_q, cur);
        });
      }
      const uint32_t pa = cur + rc_lane[0][kk];
      Unroll<C::PH>::run([&](auto hI) {
        constexpr int h = decltype(hI)::value;
        bf16x8 pf[AH];
        Unroll<AH>::run([&](auto aI) {
          constexpr int ai = decltype(aI)::value;
          pf[ai] = asm_read128_off<(h * AH + ai) * 16 * BK * 2>(pa);
        });
        lgkm_wait0();
#pragma unroll
        for (int x = 0; x < AH; ++x)
#pragma unroll
          for (int y = 0; y < AJ; ++y) acc[h * AH + x][y] = mfma16(qf[y], pf[x], acc[h * AH + x][y]);
        __builtin_amdgcn_sched_barrier(0);  // the next fragment reads stay behind these MFMAs (register budget)
      });
    });
  };

  if (ntile > 0) {
    int i0, j0;
    set_tile(w, i0, j0);
    issue(0, 0);
    int slot = 0;
    for (int u = 0; u < ntile; ++u) {
#pragma unroll
      for (int x = 0; x < AI; ++x)
#pragma unroll
        for (int y = 0; y < AJ; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
      // one k-step: stage kt landed (vmcnt: the NA stores issued behind its loads may remain),
      // barrier (every wave's reads of the other slot are done), next stage into the other slot
      auto step = [&](int kt, auto naI) {
        wait_vm<decltype(naI)::value>();
        lds_barrier();
        if (kt + 1 < nk) {
          issue(kt + 1, slot ^ 1);
        } else if (u + 1 < ntile) {  // the next tile's first stage, under this k-step's MFMAs
          set_tile(w + (u + 1) * G, i0, j0);
          issue(0, slot ^ 1);
        }
      };
      using Z = std::integral_constant<int, 0>;
      using NPRE = std::integral_constant<int, C::PRE * SPG>;  // stores behind stage 0's loads
      using NGPS = std::integral_constant<int, C::GPS * SPG>;  // stores behind a carrying step's loads
      Unroll<C::NSTEP>::run([&](auto kI) {
        constexpr int kt = decltype(kI)::value;
        if (!pending) step(kt, Z{});
        else if constexpr (kt == 0) step(kt, NPRE{});
        else step(kt, NGPS{});
        if (pending) {
          Unroll<C::GPS>::run([&](auto sI) {
            store_group(std::integral_constant<int, C::PRE + kt * C::GPS + decltype(sI)::value>{});
          });
        }
        mma_step(slot);
        slot ^= 1;
      });
      for (int kt = C::NSTEP; kt < nk; ++kt) {
        if (kt == C::NSTEP && pending) {
          if constexpr (C::NSTEP == 0) step(kt, NPRE{});
          else step(kt, NGPS{});
        } else {
          step(kt, Z{});
        }
        mma_step(slot);
        slot ^= 1;
      }
      // this tile's epilogue into registers: + bias, bf16, 16-B store layout; the first PRE groups go
      // out at once (fewer registers held across the next tile's first k-steps)
      const int ci0 = (w + u * G) / tiles_j * BM, cj0 = ((w + u * G) % tiles_j) * C::BN;
      Unroll<AJ / 2>::run([&](auto bI) {
        constexpr int bp = decltype(bI)::value;
        f32x4 b0 = f32x4{0.f, 0.f, 0.f, 0.f}, b1 = b0;
        if (a.bias) {
          const int j = cj0 + wj * C::WN + bp * 32 + 4 * g4;
          b0 = *reinterpret_cast<const f32x4*>(sbias + j);
          b1 = *reinterpret_cast<const f32x4*>(sbias + j + 16);
        }
        Unroll<AI>::run([&](auto xI) {
          constexpr int x = decltype(xI)::value, g = x * (AJ / 2) + bp;
          const u32x4 v = pack_pair(acc[x][2 * bp] + b0, acc[x][2 * bp + 1] + b1);
          if constexpr (g < C::PRE) store_vals(std::integral_constant<int, g>{}, v, ci0, cj0);
          else pk[x][bp] = v;
        });
      });
      pi0 = ci0;
      pj0 = cj0;
      pending = true;
    }
    // the last tile's stores
    Unroll<C::NGRP - C::PRE>::run([&](auto gI) { store_group(std::integral_constant<int, C::PRE + decltype(gI)::value>{}); });
  }
}

}  // namespace ms

template <int BM, int PRE, int EPI, int QL>
static int launch_ms(const ms::Args& a, int grid, hipStream_t s) {
  using C = ms::Cfg<BM, PRE>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)ms::gemm_ms_kernel<BM, PRE, EPI, QL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  if (a.K / C::BK <= C::NSTEP || (a.bias && a.N > C::BIAS_FLOATS)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((ms::gemm_ms_kernel<BM, PRE, EPI, QL>), dim3(grid), dim3(C::THREADS), 163840, s, a);
  VIT_CHECK_LAUNCH();
  return 0;
}

// the kept configurations: (bm, stores deferred) -> PRE
template <int EPI, int QL>
static int launch_ms_cfg(int cfg, const ms::Args& a, int grid, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_ms<192, 0, EPI, QL>(a, grid, s);    // 192 rows, every store deferred
    case 1: return launch_ms<256, 16, EPI, QL>(a, grid, s);   // 256 rows, stores at the tile's end (not waited on)
    case 2: return launch_ms<256, 12, EPI, QL>(a, grid, s);   // 256 rows, a quarter of the stores deferred
    case 3: return launch_ms<192, 12, EPI, QL>(a, grid, s);   // 192 rows, stores at the tile's end
    default: return (int)hipErrorInvalidValue;
  }
}

extern "C" {

// Y = X W^T (+ bias) in bf16 on the multi-tile kernel.  wl = 0: W is [N][K] (a forward, F.linear);
// wl = 1: W is [K][N] (an input gradient dX = dY W, X = dY, the layout read through the half-blocked
// CR image).  epi 0 = store Y (C), 1 = GELU pair (C = GELU'(pre), C2 = GELU(pre); wl = 0 only).
// cfg: 0 = 192-row tiles with every store deferred into the next tile's k-steps, 1 = 256-row tiles
// storing at the tile's end without waiting, 2 = 256-row tiles with a quarter deferred, 3 = 192-row
// tiles storing at the end.  grid = workgroups (each runs tiles w, w + grid, ...; <= 0 or > tiles: one
// per tile).  Returns hipErrorInvalidValue outside the kernel's contract: N % 256, K % 64, more k-steps
// than the deferred stores take, 8-element row strides, 16-B aligned pointers, N * 4 B of bias beside
// the ring, 32-bit staging offsets.
int vit_gemm_ms(int epi, int wl, int cfg, int M, int N, int K, const void* X, int64_t ldx, const void* W,
                int64_t ldw, const float* bias, void* C, int64_t ldc, void* C2, int grid, void* stream) {
  if (M <= 0 || N % 256 || K % 64 || K <= 0 || (ldx | ldw | ldc) % 8 || cfg < 0 || cfg > 3)
    return (int)hipErrorInvalidValue;
  if ((wl != 0 && wl != 1) || (epi != 0 && epi != 1) || (epi == 1 && (wl == 1 || C2 == nullptr)))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)X | (uintptr_t)W | (uintptr_t)C | (uintptr_t)C2) & 15) return (int)hipErrorInvalidValue;
  if ((int64_t)(M - 1) * ldx * 2 + 128 >= ((int64_t)1 << 32)) return (int)hipErrorInvalidValue;
  if (wl == 0 ? (int64_t)(N - 1) * ldw * 2 + 128 >= ((int64_t)1 << 32) : (int64_t)64 * ldw * 2 >= ((int64_t)1 << 32))
    return (int)hipErrorInvalidValue;
  ms::Args a{(const bf16*)X, ldx, (const bf16*)W, ldw, M, N, K, (bf16*)C, ldc, (bf16*)C2, bias};
  const int bm = (cfg == 1 || cfg == 2) ? 256 : 192;
  const int tiles = ((M + bm - 1) / bm) * (N / 256);
  if (grid <= 0 || grid > tiles) grid = tiles;
  hipStream_t s = (hipStream_t)stream;
  if (wl == 1) return launch_ms_cfg<0, LAY_CR>(cfg, a, grid, s);
  return epi == 1 ? launch_ms_cfg<1, LAY_RC>(cfg, a, grid, s) : launch_ms_cfg<0, LAY_RC>(cfg, a, grid, s);
}

}  // extern "C"
