// Lab kernel (not product code): the w4 weight-gradient tile (csrc/gemm_w4.inc: 256x256 on 4 waves of
// 128x128, asm MFMAs on AGPR accumulators, next-k-step fragment reads interleaved) with the operand stages
// moved through registers instead of LDS-DMA: per k-step each wave issues 8 global_load_dwordx4 for stage
// t+2 right after the barrier and writes them with 8 ds_write_b128 after MFMA WR, into a 3-slot ring.  The
// question: is 8 x (load + ds_write) cheaper in issue cycles on a one-wave-per-SIMD loop than 8 LDS-DMA
// pieces (the w4 lab's loads-on vs loads-off gap: 17 % on CR x CR).  CR x CR only, f32 slab output.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I vit-project_amd/csrc tools/lab/w4r_lab.hip -o tools/lab/libw4r_lab.so
#include "common.hpp"
#include "gemm_lds.hpp"

using namespace big;

__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int WR>
__global__ __launch_bounds__(256, 1) void w4r_kernel(const bf16* __restrict__ P, int64_t ldp, const bf16* __restrict__ Q,
                                                     int64_t ldq, int M, int N, int R, int r_chunk, float* __restrict__ C,
                                                     int dbg) {
  constexpr int BK = 32, PIMG = 256 * BK * 2, STAGE = 2 * PIMG, S = 3;
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

  const bf16* src[8];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = wave * 4 + u;
    src[u] = P + (int64_t)rb * ldp + crh_src<256>(t, lane, ldp, i0, M);
    src[4 + u] = Q + (int64_t)rb * ldq + crh_src<256>(t, lane, ldq, j0, N);
  }
  const int64_t stepP = BK * ldp, stepQ = BK * ldq;
  const bool noload = dbg & 1;
  i32x4 stg[8];
  auto gload = [&](bool on) {  // the next stage's 8 pieces into registers
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (on) stg[u] = *reinterpret_cast<const i32x4*>(src[u]);
      src[u] += u < 4 ? stepP : stepQ;
    }
  };
  auto lwrite = [&](int k) {  // ... and into ring slot k % S (the LDS-DMA piece layout: lane l at 16 l)
    char* buf = smem + (k % S) * STAGE;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      *reinterpret_cast<i32x4*>(buf + (u < 4 ? 0 : PIMG) + (wave * 4 + (u & 3)) * 1024 + lane * 16) = stg[u];
  };
  uint32_t crh_p[2][2], crh_q[2][2];
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      crh_p[lh][h] = crh_lane<256>(lane, lh, h) + (uint32_t)(wi * 4 * 1024);
      crh_q[lh][h] = PIMG + crh_lane<256>(lane, lh, h) + (uint32_t)(wj * 4 * 1024);
    }
  auto read_frag = [&](auto fI, uint32_t cur, bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    constexpr int f = decltype(fI)::value;
    if constexpr (f < 8) qf[f] = frag_crh<256, 0, f>(crh_q, cur);
    else pf[f - 8] = frag_crh<256, 0, f - 8>(crh_p, cur);
  };
  auto settle = [&](bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pf[a]), "+v"(qf[a]));
    asm volatile("s_nop 1" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // k-step t: MFMAs on (pc, qc); reads of stage t+1 after MFMAs 3f+1; stage t+2's global loads at the top,
  // its LDS writes after MFMA WR (slot (t+2) % 3 was last read in k-step t-1, before this k-step's barrier)
  auto kstep = [&](int t, uint32_t nxt, const bf16x8 (&pc)[8], const bf16x8 (&qc)[8], bf16x8 (&pn)[8],
                   bf16x8 (&qn)[8]) {
    const bool more = t + 2 < nk && !noload;
    if (more) gload(true);
    __builtin_amdgcn_sched_barrier(0);
    Unroll<64>::run([&](auto mI) {
      constexpr int m = decltype(mI)::value;
      constexpr int a = m / 8, b = m % 8;
      mfma_acc(acc[a][b], qc[b], pc[a]);
      if constexpr (m % 3 == 1 && m / 3 < 16) read_frag(std::integral_constant<int, m / 3>{}, nxt, pn, qn);
      if constexpr (m == WR) {
        if (more) lwrite(t + 2);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  if (!noload) {
    gload(true);
    lwrite(0);
    if (nk > 1) {
      gload(true);
      lwrite(1);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();
  bf16x8 pA[8], qA[8], pB[8], qB[8];
  Unroll<16>::run([&](auto fI) { read_frag(fI, lds_addr(smem), pA, qA); });
  settle(pA, qA);
#pragma unroll
  for (int a = 0; a < 8; ++a)
    asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                      "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  auto iter = [&](int t, const bf16x8 (&pc)[8], const bf16x8 (&qc)[8], bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    if (t + 1 < nk) lds_barrier();  // stage t+1's writes (k-step t-1, waited by its settle) visible
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
      for (int b = 0; b < 8; ++b) asm volatile("" ::"a"(acc[a][b]));
    return;
  }
  float* out = C + (int64_t)z * M * N;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                      "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
    const int i = i0 + wi * 128 + a * 16 + (lane & 15);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + wj * 128 + b * 16 + 4 * (lane >> 4);
      if (i < M && j < N) *reinterpret_cast<f32x4*>(out + (int64_t)i * N + j) = acc[a][b];
    }
  }
}

template <int WR>
static int launch(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split, float* C,
                  int dbg, hipStream_t st) {
  const int r_chunk = ((R + split - 1) / split + 63) / 64 * 64;
  const int nz = (R + r_chunk - 1) / r_chunk;
  const int grid = ((M + 255) / 256) * ((N + 255) / 256) * nz;
  constexpr int lds = 3 * 32768;
  (void)hipFuncSetAttribute((const void*)w4r_kernel<WR>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(w4r_kernel<WR>, dim3(grid), dim3(256), lds, st, (const bf16*)P, ldp, (const bf16*)Q, ldq, M, N, R,
                     r_chunk, C, dbg);
  return (int)hipGetLastError();
}

// CR x CR: C[split][M][N] slabs, sum = P^T Q over R rows; cfg = the MFMA after which the LDS writes go
extern "C" int lab_w4r(int cfg, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
                       float* C, int dbg, void* stream) {
  if (R % 64 || M <= 0 || N <= 0) return 1;
  hipStream_t st = (hipStream_t)stream;
  if (cfg == 40) return launch<40>(P, ldp, Q, ldq, M, N, R, split, C, dbg, st);
  if (cfg == 52) return launch<52>(P, ldp, Q, ldq, M, N, R, split, C, dbg, st);
  if (cfg == 60) return launch<60>(P, ldp, Q, ldq, M, N, R, split, C, dbg, st);
  return 2;
}
