// Lab kernel (not product code): the w4 main loop (csrc/gemm_w4.inc: interleaved next-k-step fragment
// reads, asm MFMAs on AGPR accumulators) with a narrower wave tile, so that TWO workgroups share a CU and
// one's epilogue runs beside the other's MFMAs: 4 waves of 128 x WN (WN = 64: 128 accumulator registers),
// tile 256 x 2WN, an S-deep ring of (256 + 2WN) x 32 bf16 stages.  RC x RC (forward) or RC x CR (input
// gradient), bf16 output through the fragment layout (8-B stores) with an optional bias, or f32 out.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I vit-project_amd/csrc tools/lab/w4b_lab.hip -o tools/lab/libw4b_lab.so
// dbg bits: 1 no ring loads in the k-loop, 4 no epilogue.
#include "common.hpp"
#include "gemm_lds.hpp"

using namespace big;

__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int QL, int WN, int S, int OCC>
__global__ __launch_bounds__(256, OCC) void w4b_kernel(const bf16* __restrict__ P, int64_t ldp, const bf16* __restrict__ Q,
                                                       int64_t ldq, int M, int N, int R, const float* __restrict__ bias,
                                                       bf16* __restrict__ C, int dbg) {
  constexpr int BK = 32, BN = 2 * WN, AJ = WN / 16;
  constexpr int PIMG = 256 * BK * 2, QIMG = BN * BK * 2, STAGE = PIMG + QIMG;
  constexpr int GQ = BN / 16 / 4;  // Q pieces per wave
  constexpr int G = 4 + GQ;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_j = (N + BN - 1) / BN;
  const int ti = w / tiles_j, tj = w - ti * tiles_j;
  const int i0 = ti * 256, j0 = tj * BN;
  const int nk = R / BK;

  f32x4 acc[8][AJ];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < AJ; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* srcP[4];
  const bf16* srcQ[GQ];
  int64_t stepQ;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = wave * 4 + u;
    const int row = t * 16 + lane / 4;
    const int c = (lane % 4) ^ rc_sw<32>(row);
    srcP[u] = P + (int64_t)min(i0 + row, M - 1) * ldp + c * 8;
  }
#pragma unroll
  for (int u = 0; u < GQ; ++u) {
    const int t = wave * GQ + u;
    if constexpr (QL == LAY_RC) {
      const int row = t * 16 + lane / 4;
      const int c = (lane % 4) ^ rc_sw<32>(row);
      srcQ[u] = Q + (int64_t)min(j0 + row, N - 1) * ldq + c * 8;
      stepQ = BK;
    } else {
      srcQ[u] = Q + crh_src<BN>(t, lane, ldq, j0, N);
      stepQ = BK * ldq;
    }
  }
  auto piece = [&](int k, int u) {
    char* buf = smem + (k % S) * STAGE;
    if (u < 4) {
      __builtin_amdgcn_global_load_lds((const void*)srcP[u], LDS_PTR(buf + (wave * 4 + u) * 1024), 16, 0, 0);
      srcP[u] += BK;
    } else {
      __builtin_amdgcn_global_load_lds((const void*)srcQ[u - 4], LDS_PTR(buf + PIMG + (wave * GQ + u - 4) * 1024), 16,
                                       0, 0);
      srcQ[u - 4] += stepQ;
    }
  };
  const bool noload = dbg & 1;
  uint32_t crh_q[2][2];
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) crh_q[lh][h] = PIMG + crh_lane<BN>(lane, lh, h) + (uint32_t)(wj * (WN / 32) * 1024);
  const uint32_t rc_p = (uint32_t)(wi * 128 * 64 + rc_off<32>(lane & 15, lane >> 4));
  const uint32_t rc_q = (uint32_t)(PIMG + wj * WN * 64 + rc_off<32>(lane & 15, lane >> 4));
  constexpr int NF = 8 + AJ;
  auto read_frag = [&](auto fI, uint32_t cur, bf16x8 (&pf)[8], bf16x8 (&qf)[AJ]) {
    constexpr int f = decltype(fI)::value;
    if constexpr (f < AJ) {
      if constexpr (QL == LAY_RC) qf[f] = asm_read128_off<f * 16 * 64>(cur + rc_q);
      else qf[f] = frag_crh<BN, 0, f>(crh_q, cur);
    } else {
      constexpr int a = f - AJ;
      pf[a] = asm_read128_off<a * 16 * 64>(cur + rc_p);
    }
  };
  auto settle = [&](bf16x8 (&pf)[8], bf16x8 (&qf)[AJ]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pf[a]));
#pragma unroll
    for (int b = 0; b < AJ; ++b) asm volatile("" : "+v"(qf[b]));
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int NM = 8 * AJ;  // MFMAs per k-step
  constexpr int RD = NM / NF > 0 ? NM / NF : 1;  // MFMAs per fragment read slot
  auto kstep = [&](int t, uint32_t nxt, const bf16x8 (&pc)[8], const bf16x8 (&qc)[AJ], bf16x8 (&pn)[8],
                   bf16x8 (&qn)[AJ]) {
    const bool more = t + S < nk && !noload;
    Unroll<NM>::run([&](auto mI) {
      constexpr int m = decltype(mI)::value;
      constexpr int a = m / AJ, b = m % AJ;
      mfma_acc(acc[a][b], qc[b], pc[a]);
      if constexpr (m % RD == 0 && m / RD < NF) read_frag(std::integral_constant<int, m / RD>{}, nxt, pn, qn);
      if constexpr (m % (NM / G) == NM / G / 2 && m / (NM / G) < G) {
        if (more) piece(t + S, m / (NM / G));
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  if (!noload) {
#pragma unroll
    for (int k = 0; k < S; ++k)
      if (k < nk)
#pragma unroll
        for (int u = 0; u < G; ++u) piece(k, u);
    wait_stages<G, S>(min(S - 1, nk - 1));
  }
  lds_barrier();
  bf16x8 pA[8], qA[AJ], pB[8], qB[AJ];
  Unroll<NF>::run([&](auto fI) { read_frag(fI, lds_addr(smem), pA, qA); });
  settle(pA, qA);
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < AJ; ++b) asm volatile("" : "+a"(acc[a][b]));
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  auto iter = [&](int t, const bf16x8 (&pc)[8], const bf16x8 (&qc)[AJ], bf16x8 (&pf)[8], bf16x8 (&qf)[AJ]) {
    if (t + 1 < nk) {
      if (!noload) wait_stages<G, S>(min(S - 2, nk - 2 - t));
      lds_barrier();
    }
    kstep(t, lds_addr(smem + ((t + 1) % S) * STAGE), pc, qc, pf, qf);
    settle(pf, qf);
  };
  int t = 0;
  for (; t + 2 <= nk; t += 2) {
    iter(t, pA, qA, pB, qB);
    iter(t + 1, pB, qB, pA, qA);
  }
  if (t < nk) iter(t, pA, qA, pB, qB);
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (dbg & 4) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < AJ; ++b) asm volatile("" ::"a"(acc[a][b]));
    return;
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) {
#pragma unroll
    for (int b = 0; b < AJ; ++b) asm volatile("" : "+a"(acc[a][b]));
    const int i = i0 + wi * 128 + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < AJ; ++b) {
      const int j = j0 + wj * WN + b * 16 + 4 * (lane >> 4);
      if (i < M && j < N) {
        f32x4 v = acc[a][b];
        if (bias) v += *reinterpret_cast<const f32x4*>(bias + j);
        const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        *reinterpret_cast<bf16x4*>(C + (int64_t)i * N + j) = o;
      }
    }
  }
}

template <int QL, int WN, int S, int OCC>
static int launch(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, const float* bias,
                  void* C, int dbg, hipStream_t st) {
  constexpr int LDS = S * (256 + 2 * WN) * 32 * 2;
  auto k = w4b_kernel<QL, WN, S, OCC>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
  const int grid = ((M + 255) / 256) * ((N + 2 * WN - 1) / (2 * WN));
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), LDS, st, (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R, bias,
                     (bf16*)C, dbg);
  return (int)hipGetLastError();
}

// lay 0: forward Y[M,N] = P[M,R] Q[N,R]^T; lay 1: input gradient Y[M,N] = P[M,R] Q[R,N] (Q CR).
// cfg: 1 = WN 64, S 3, 2 WG/CU (72 KiB); 2 = WN 64, S 4, 2 WG/CU (96 KiB: LDS-limited to 1); 3 = WN 128, S 4,
// 1 WG/CU (the w4 tile with bf16 fragment stores)
extern "C" int lab_w4b(int lay, int cfg, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R,
                       const float* bias, void* C, int dbg, void* stream) {
  if (R % 32 || M <= 0 || N % 4) return 1;
  hipStream_t st = (hipStream_t)stream;
#define L4(W, S_, O)                                                                           \
  return lay ? launch<LAY_CR, W, S_, O>(P, ldp, Q, ldq, M, N, R, bias, C, dbg, st)              \
             : launch<LAY_RC, W, S_, O>(P, ldp, Q, ldq, M, N, R, bias, C, dbg, st);
  if (cfg == 1) { L4(64, 3, 2) }
  if (cfg == 2) { L4(64, 4, 2) }
  if (cfg == 3) { L4(128, 4, 1) }
#undef L4
  return 2;
}
