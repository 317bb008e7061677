// Lab kernel (not product code): a 256x256 bf16 GEMM tile on FOUR waves, one per SIMD, each wave owning
// a 128x128 block of the output (64 16x16 accumulators = 256 fp32 registers per lane, which the
// one-wave-per-SIMD budget of 512 registers lets live in AGPRs).  Per 32-deep k-step a wave reads 16
// fragments for 64 MFMAs (the 8-wave 128x64 tiles read 12 for 32), and the next k-step's fragment reads
// are interleaved with this k-step's MFMAs (register double buffer), so LDS reads never sit between a
// barrier and the first MFMA.  Operands: an S-deep ring of 32-KiB stages (P image 16 KiB + Q image),
// RC rows (BK = 32 swizzle) or half-blocked CR images (gemm_lds.hpp), filled by global_load_lds.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I vit-project_amd/csrc tools/lab/w4_lab.hip -o tools/lab/libw4_lab.so
// dbg bits: 1 no ring loads in the k-loop, 4 no epilogue.  LD (load placement): 0 = all pieces right
// after the barrier, 1 = one piece after every 8 MFMAs, 2 = one piece after every 4 MFMAs (first half).
#include "common.hpp"
#include "gemm_lds.hpp"

using namespace big;

// MFMA with the accumulator pinned to AGPRs ("+a"): the compiler's own MFMA (builtin) lets the register
// allocator split the 256 accumulator live ranges across VGPRs and AGPRs, which put ~500 v_accvgpr
// moves per k-loop trip.  Inline asm is invisible to the hazard recognizer: the operands are read a whole
// k-step after their LDS reads retire (lgkmcnt(0)), accumulators are re-used 64 MFMAs apart, the first
// k-step takes SrcC = 0 (no VALU write feeds SrcC), and s_nops separate the last MFMA from the epilogue.
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

template <int PL, int QL, int S, int LD, int FIX = 0>
__global__ __launch_bounds__(256, 1) void w4_kernel(const bf16* __restrict__ P, int64_t ldp, const bf16* __restrict__ Q,
                                                    int64_t ldq, int M, int N, int R, int r_chunk,
                                                    float* __restrict__ C, int dbg) {
  constexpr int BK = 32, PIMG = 256 * BK * 2, STAGE = 2 * PIMG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_j = (N + 255) / 256, tiles_i = (M + 255) / 256;
  const int tiles = tiles_i * tiles_j;
  const int z = w / tiles, t0 = w - z * tiles;
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
  const int nk = (re - rb) / BK;

  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 16 pieces per operand image, 4 per wave
  const bf16* srcP[4];
  const bf16* srcQ[4];
  int64_t stepP, stepQ;
  {
    auto init = [&](auto lay_tag, const bf16* base, int64_t ld, int row0, int lim, const bf16* (&src)[4],
                    int64_t& step) {
      constexpr int LAY = decltype(lay_tag)::value;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = wave * 4 + u;
        if constexpr (LAY == LAY_RC) {
          const int row = t * 16 + lane / 4;
          const int c = (lane % 4) ^ rc_sw<32>(row);
          src[u] = base + (int64_t)min(row0 + row, lim - 1) * ld + rb + c * 8;
          step = 32;
        } else {
          src[u] = base + (int64_t)rb * ld + crh_src<256>(t, lane, ld, row0, lim);
          step = 32 * ld;
        }
      }
    };
    init(std::integral_constant<int, PL>{}, P, ldp, i0, M, srcP, stepP);
    init(std::integral_constant<int, QL>{}, Q, ldq, j0, N, srcQ, stepQ);
  }
  // piece u (0..7) of stage k: 0-3 of P, 4-7 of Q
  auto piece = [&](int k, int u) {
    char* buf = smem + (k % S) * STAGE;
    if (u < 4) {
      __builtin_amdgcn_global_load_lds((const void*)srcP[u], LDS_PTR(buf + (wave * 4 + u) * 1024), 16, 0, 0);
      srcP[u] += stepP;
    } else {
      __builtin_amdgcn_global_load_lds((const void*)srcQ[u - 4], LDS_PTR(buf + PIMG + (wave * 4 + u - 4) * 1024), 16, 0,
                                       0);
      srcQ[u - 4] += stepQ;
    }
  };
  const bool noload = dbg & 1;

  // fragment read bases
  uint32_t crh_p[2][2], crh_q[2][2];
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      crh_p[lh][h] = crh_lane<256>(lane, lh, h) + (uint32_t)(wi * 4 * 1024);
      crh_q[lh][h] = PIMG + crh_lane<256>(lane, lh, h) + (uint32_t)(wj * 4 * 1024);
    }
  const uint32_t rc_p = (uint32_t)(wi * 128 * 64 + rc_off<32>(lane & 15, lane >> 4));
  const uint32_t rc_q = (uint32_t)(PIMG + wj * 128 * 64 + rc_off<32>(lane & 15, lane >> 4));
  // fragment f (0..15): 0-7 Q (columns), 8-15 P (rows)
  auto read_frag = [&](auto fI, uint32_t cur, bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    constexpr int f = decltype(fI)::value;
    if constexpr (f < 8) {
      if constexpr (QL == LAY_RC) qf[f] = asm_read128_off<f * 16 * 64>(cur + rc_q);
      else qf[f] = frag_crh<256, 0, f>(crh_q, cur);
    } else {
      constexpr int a = f - 8;
      if constexpr (PL == LAY_RC) pf[a] = asm_read128_off<a * 16 * 64>(cur + rc_p);
      else pf[a] = frag_crh<256, 0, a>(crh_p, cur);
    }
  };
  auto read_all = [&](uint32_t cur, bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    Unroll<16>::run([&](auto fI) { read_frag(fI, cur, pf, qf); });
  };
  // one k-step: 64 MFMAs on (pc, qc); the next k-step's 16 fragment reads (from `nxt`, if rd) after
  // MFMAs 3f+1, the next stage's pieces per LD
  // one k-step: 64 MFMAs on (pc, qc) with the next k-step's 16 fragment reads (from `nxt`) after MFMAs
  // 3f+1 -- unconditionally: past the last k-step they read a stale ring slot, which nothing uses, so the
  // loop body has no data-dependent register definitions -- and the next stage's pieces per LD
  auto kstep = [&](int t, uint32_t nxt, const bf16x8 (&pc)[8], const bf16x8 (&qc)[8], bf16x8 (&pn)[8],
                   bf16x8 (&qn)[8]) {
    const bool more = t + S < nk && !noload;
    if constexpr (LD == 0) {
      if (more) {
#pragma unroll
        for (int u = 0; u < 8; ++u) piece(t + S, u);
      }
    }
    Unroll<64>::run([&](auto mI) {
      constexpr int m = decltype(mI)::value;
      constexpr int a = m / 8, b = m % 8;
      mfma_acc(acc[a][b], qc[b], pc[a]);
      if constexpr (m % 3 == 1 && m / 3 < 16) read_frag(std::integral_constant<int, m / 3>{}, nxt, pn, qn);
      if constexpr (LD == 1 && m % 8 == 4) {
        if (more) piece(t + S, m / 8);
      }
      if constexpr (LD == 2 && m % 4 == 2 && m < 32) {
        if (more) piece(t + S, m / 4);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (FIX & 1) {  // keep this k-step's fragments live to its end (no next-read into their registers)
#pragma unroll
      for (int a = 0; a < 8; ++a) asm volatile("" ::"v"(pc[a]), "v"(qc[a]));
    }
  };

  if (nk > 0) {  // nk even (host)
    if (!noload) {
#pragma unroll
      for (int k = 0; k < S; ++k)
        if (k < nk)
#pragma unroll
          for (int u = 0; u < 8; ++u) piece(k, u);
    }
    // stage 0 landed: S-1 stages of 8 pieces may stay in flight
    if (!noload) wait_stages<8, S>(min(S - 1, nk - 1));
    lds_barrier();
    bf16x8 pA[8], qA[8], pB[8], qB[8];
    read_all(lds_addr(smem), pA, qA);
    lgkm_wait0();
    asm volatile("s_nop 4" ::: "memory");  // accumulator zeroing (VALU) -> first MFMA SrcC
    // iteration t: stage t+1 must be visible before its fragment reads (wait own pieces + barrier);
    // after the barrier every wave has retired its reads of stage t (done in iteration t-1), so
    // slot t % S takes stage t + S
    auto iter = [&](int t, const bf16x8 (&pc)[8], const bf16x8 (&qc)[8], bf16x8 (&pn)[8], bf16x8 (&qn)[8]) {
      if (t + 1 < nk) {
        if (!noload) wait_stages<8, S>(min(S - 2, nk - 2 - t));
        lds_barrier();
      }
      kstep(t, lds_addr(smem + ((t + 1) % S) * STAGE), pc, qc, pn, qn);
      if constexpr (FIX & 2) {  // the wait names every read destination: no copy of them before it
#pragma unroll
        for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pn[a]), "+v"(qn[a]));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pn[a]), "+v"(qn[a]));
        __builtin_amdgcn_sched_barrier(0);
      } else {
        lgkm_wait0();
      }
    };
    for (int t = 0; t < nk; t += 2) {
      iter(t, pA, qA, pB, qB);
      iter(t + 1, pB, qB, pA, qA);
    }
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");  // last MFMA -> accumulator reads
    __builtin_amdgcn_sched_barrier(0);
  }
  if (dbg & 4) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) asm volatile("" ::"a"(acc[a][b]));
    return;
  }
  float* out = C + (int64_t)z * M * N;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int i = i0 + wi * 128 + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + wj * 128 + b * 16 + 4 * (lane >> 4);
      if (i < M && j < N) *reinterpret_cast<f32x4*>(out + (int64_t)i * N + j) = acc[a][b];
    }
  }
}

template <int PL, int QL, int S, int LD, int FIX>
static int launch(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split, float* C,
                  int dbg, hipStream_t st) {
  const int r_chunk = ((R / split) + 63) / 64 * 64;
  const int nz = (R + r_chunk - 1) / r_chunk;
  const int grid = ((M + 255) / 256) * ((N + 255) / 256) * nz;
  auto k = w4_kernel<PL, QL, S, LD, FIX>;
  const int lds = S * 65536 / 2;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R, r_chunk, C,
                     dbg);
  return (int)hipGetLastError();
}

// lay: 0 = RC x RC (forward), 1 = CR x CR (weight gradient); cfg = S * 10 + LD
extern "C" int lab_w4(int lay, int cfg, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R,
                      int split, float* C, int dbg, void* stream) {
  if (R % 64 || M <= 0 || N <= 0) return 1;
  hipStream_t st = (hipStream_t)stream;
#define W4(S, LD, F)                                                                                \
  if (cfg == F * 100 + S * 10 + LD)                                                                 \
    return lay ? launch<LAY_CR, LAY_CR, S, LD, F>(P, ldp, Q, ldq, M, N, R, split, C, dbg, st)       \
               : launch<LAY_RC, LAY_RC, S, LD, F>(P, ldp, Q, ldq, M, N, R, split, C, dbg, st);
  W4(4, 0, 0) W4(4, 1, 0) W4(4, 2, 0) W4(3, 1, 0) W4(5, 1, 0)
  W4(4, 0, 1) W4(4, 2, 1) W4(4, 0, 2) W4(4, 2, 2) W4(4, 0, 3) W4(4, 2, 3) W4(4, 1, 3)
#undef W4
  return 2;
}
