// ----------------------------------------------------------------------------
// g4 (round 6): the plain bf16 forward (+ f32 bias) and input-gradient GEMMs of the step on FOUR waves
// -- one per SIMD, each owning a 128x128 block of a 256x256 output tile (64 16x16 accumulators = 256
// AGPRs per lane, pinned by inline-asm MFMAs as in gemm_w4.inc) -- with a 64-deep k-step and two 64-KiB
// LDS stages.  This replaces the hipBLASLt dispatch of round 5 (ABI 9 -> 10).
//
// Why this shape: one wave per SIMD reads 32 fragments per 128 MFMAs (the 8-wave
// V5 tile reads 48), and a BK = 64 stage is filled by 1-KiB LDS-DMA pieces of 8 rows x 128 B -- whole
// cache lines (BK = 32 pieces are 16 half lines: twice the lines per instruction for the address path).
//
// One k-step ("iteration" g of the workgroup's stage stream) is 128 MFMAs (slots m = 0..127; 0..63 on
// the k-substep-0 fragments X, 64..127 on the k-substep-1 fragments Y) with everything else at fixed
// slots between them:
//   m 0..15   the 16 Y fragment reads of stage g (its LDS slot g % 2), one after each MFMA;
//   m 24      s_waitcnt lgkmcnt(0) + s_barrier: every wave's reads of stage g are done, so slot g % 2
//             takes stage g + 2;
//   m 26..116 the 16 LDS-DMA pieces of stage g + 2 (8 P, 8 Q per wave), one every 6 MFMAs;
//   m 96      s_waitcnt vmcnt(12) (stage g + 1 landed; the 12 pieces of stage g + 2 issued so far may
//             stay in flight) + s_barrier, then the 16 X fragment reads of stage g + 1 (slot
//             (g + 1) % 2) after MFMAs 96..111;
//   end       s_waitcnt lgkmcnt(0): X is complete before the loop's back edge.
// So a piece has ~1.2 k-steps to land, two barriers per 128 MFMAs, and no wait on LDS reads sits in
// front of an MFMA that needs them except the two drains above.
//
// Persistent stage stream: a workgroup owns a sequence of output tiles (stride walk: tiles w, w + G,
// ...; or band walk: row tile w across every column tile, the input-gradient shape N = 768) and its
// k-steps form ONE stream g = tile * nk + k, so the last two k-steps of a tile already load -- and the
// last one already reads into X -- the next tile's first stages: the epilogue's stores overlap the
// next tile's operand fetch instead of a cold prologue.
//
// Inline asm (MFMA, fragment reads) is invisible to the compiler's waitcnt pass and hazard recognizer
// (gemm_w4.inc has the rules): fragment destinations are named "+v" after the wait that covers them,
// accumulators "+a" after zeroing (s_nop 4 before the first MFMA), three s_nop 7 separate the last
// MFMA from the epilogue's accumulator reads.  Nothing in the k-step body is conditional: past the
// stream's end the loader re-issues valid addresses into the slot nothing reads any more (and the
// workgroup waits for them before it exits).
// ----------------------------------------------------------------------------
#include <stdlib.h>

#include "gemm_epi.hpp"

namespace g4 {

constexpr int BK = 64, PIMG = 256 * BK * 2, STAGE = 2 * PIMG, LDS = 2 * STAGE, THREADS = 256;
static_assert(LDS <= 163840, "LDS");

__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// a workgroup's output tiles: mode 0 strides over the row-major (or group_m-banded) tile order by the
// grid size G, mode 1 gives workgroup w row tile w and walks its column tiles
struct Walk {
  int tiles_i, tiles_j, mode, G, group_m;
};
__device__ __forceinline__ bool tile_at(const Walk& s, int w, int q, int& i0, int& j0) {
  int ti, tj;
  if (s.mode == 1) {
    if (q >= s.tiles_j) return false;
    ti = w;
    tj = q;
  } else {
    const int t = w + q * s.G;
    if (t >= s.tiles_i * s.tiles_j) return false;
    big::tile_coords(t, s.tiles_i, s.tiles_j, s.group_m, ti, tj);
  }
  i0 = ti * 256;
  j0 = tj * 256;
  return true;
}
__host__ __device__ __forceinline__ int tiles_of(const Walk& s, int w) {
  if (s.mode == 1) return s.tiles_j;
  const int t = s.tiles_i * s.tiles_j;
  return w < t ? (t - w + s.G - 1) / s.G : 0;
}

// P RC [M x R] (forward X / input-gradient dY), Q RC [N x R] (forward W) or CR [R x N] (input-gradient
// W read with a k stride); C bf16 [M x N] = P Q^T (+ f32 bias), R % 64 == 0, N % 8 == 0.
template <int QL>
__global__ __launch_bounds__(THREADS, 1) void kernel(const bf16* __restrict__ P, int64_t ldp,
                                                     const bf16* __restrict__ Q, int64_t ldq, int M, int N, int R,
                                                     Epi e, Walk s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = big::xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = tiles_of(s, w);
  if (ntiles <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int nk = R / BK;

  // ---- loader: the tile and k-step of the next stage to issue, and its per-lane source offsets
  int qL = 0, kL = 0, i0L = 0, j0L = 0;
  tile_at(s, w, 0, i0L, j0L);
  uint32_t offP[8], offQ[8];
  auto set_offsets = [&]() {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = wave * 8 + u;
      const int row = t * 8 + (lane >> 3);
      const int c = (lane & 7) ^ big::rc_sw<64>(row);
      offP[u] = (uint32_t)((int64_t)min(i0L + row, M - 1) * ldp * 2 + c * 16);
      if constexpr (QL == LAY_RC)
        offQ[u] = (uint32_t)((int64_t)min(j0L + row, N - 1) * ldq * 2 + c * 16);
      else
        offQ[u] = (uint32_t)(big::crh_src<256>(t, lane, ldq, j0L, N) * 2);
    }
  };
  set_offsets();
  const int64_t qstep = QL == LAY_RC ? (int64_t)BK * 2 : (int64_t)BK * ldq * 2;  // bytes per k-step
  // piece u (0..15) of the loader's stage (operand bases pb / qb at its k-step) into LDS slot `buf`:
  // even u = P piece u / 2, odd u = Q piece u / 2
  auto piece = [&](int u, const char* pb, const char* qb, char* buf) {
    if ((u & 1) == 0)
      __builtin_amdgcn_global_load_lds((const void*)(pb + offP[u >> 1]), LDS_PTR(buf + (wave * 8 + (u >> 1)) * 1024),
                                       16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds((const void*)(qb + offQ[u >> 1]),
                                       LDS_PTR(buf + PIMG + (wave * 8 + (u >> 1)) * 1024), 16, 0, 0);
  };
  auto pbase = [&]() { return reinterpret_cast<const char*>(P) + (int64_t)kL * BK * 2; };
  auto qbase = [&]() { return reinterpret_cast<const char*>(Q) + (int64_t)kL * qstep; };
  // past the stream's end the loader keeps re-issuing its last tile's first k-steps (valid addresses)
  // into the slot nothing reads any more, so the k-step body has no stream-end branch
  auto advance = [&]() {
    if (++kL == nk) {
      kL = 0;
      ++qL;
      if (tile_at(s, w, qL, i0L, j0L)) set_offsets();
    }
  };

  // ---- fragment reads: f 0..7 = Q fragment f (columns), 8..15 = P fragment f - 8 (rows)
  uint32_t rc_p[2], rc_q[2], crh_q[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    rc_p[kk] = (uint32_t)(wi * 128 * 128 + big::rc_off<64>(lane & 15, kk * 4 + (lane >> 4)));
    rc_q[kk] = (uint32_t)(PIMG + wj * 128 * 128 + big::rc_off<64>(lane & 15, kk * 4 + (lane >> 4)));
  }
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) crh_q[lh][h] = PIMG + big::crh_lane<256>(lane, lh, h) + (uint32_t)(wj * 4 * 1024);
  auto read_frag = [&](auto kkI, auto fI, uint32_t cur, bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    constexpr int kk = decltype(kkI)::value, f = decltype(fI)::value;
    if constexpr (f < 8) {
      if constexpr (QL == LAY_RC) qf[f] = big::asm_read128_off<f * 2048>(cur + rc_q[kk]);
      else qf[f] = big::frag_crh<256, kk, f>(crh_q, cur);
    } else {
      pf[f - 8] = big::asm_read128_off<(f - 8) * 2048>(cur + rc_p[kk]);
    }
  };
  auto settle = [&](bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pf[a]), "+v"(qf[a]));
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[8][8];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int a = 0; a < 8; ++a)
      asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                        "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
    asm volatile("s_nop 4" ::: "memory");  // accumulator writes (VALU) -> first MFMA's SrcC
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- prologue: stages 0 and 1 in flight, stage 0 landed and visible, X = its k-substep 0
  bf16x8 pX[8], qX[8], pY[8], qY[8];
  for (int st = 0; st < 2; ++st) {
    const char *pb = pbase(), *qb = qbase();
#pragma unroll
    for (int u = 0; u < 16; ++u) piece(u, pb, qb, smem + st * STAGE);
    advance();
  }
  big::wait_vm<16>();
  big::lds_barrier();
  {
    const uint32_t cur = big::lds_addr(smem);
    big::Unroll<16>::run([&](auto fI) { read_frag(std::integral_constant<int, 0>{}, fI, cur, pX, qX); });
    settle(pX, qX);
  }
  zero_acc();

  int g = 0;
  int i0 = 0, j0 = 0;
  for (int q = 0; q < ntiles; ++q) {
    tile_at(s, w, q, i0, j0);
    for (int k = 0; k < nk; ++k, ++g) {
      const char *pb = pbase(), *qb = qbase();
      char* slot = smem + (g & 1) * STAGE;
      const uint32_t cur = big::lds_addr(smem + (g & 1) * STAGE);
      const uint32_t nxt = big::lds_addr(smem + ((g + 1) & 1) * STAGE);
      big::Unroll<128>::run([&](auto mI) {
        constexpr int m = decltype(mI)::value;
        constexpr int a = (m % 64) / 8, b = m % 8;
        if constexpr (m == 24) {  // every wave's reads of stage g are done: its slot takes stage g + 2
          settle(pY, qY);
          big::lds_barrier();
        }
        if constexpr (m == 96) {  // stage g + 1 landed (this wave's pieces) and visible (barrier)
          big::wait_vm<12>();
          big::lds_barrier();
        }
        if constexpr (m < 64) mfma_acc(acc[a][b], qX[b], pX[a]);
        else mfma_acc(acc[a][b], qY[b], pY[a]);
        if constexpr (m < 16) read_frag(std::integral_constant<int, 1>{}, std::integral_constant<int, m>{}, cur, pY, qY);
        if constexpr (m >= 96 && m < 112)
          read_frag(std::integral_constant<int, 0>{}, std::integral_constant<int, m - 96>{}, nxt, pX, qX);
        if constexpr (m >= 26 && (m - 26) % 6 == 0 && (m - 26) / 6 < 16) {
          piece((m - 26) / 6, pb, qb, slot);
          if constexpr ((m - 26) / 6 == 15) advance();
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      settle(pX, qX);
    }
    // ---- epilogue of tile q: acc[a][b] holds C[i][j..j+3], i = i0 + wi*128 + 16a + lane%16,
    // j = j0 + wj*128 + 16b + 4*(lane/16); fragment pairs widened to 16-B stores (permlane16_swap)
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const int gq = lane >> 4;
    const int colsel = (gq & 1) * 16 + (gq >> 1) * 8;
    f32x4 bias4[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + wj * 128 + b * 16 + 4 * gq;
      bias4[b] = (e.bias && j < N) ? *reinterpret_cast<const f32x4*>(e.bias + j) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                        "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
      const int i = i0 + wi * 128 + a * 16 + (lane & 15);
#pragma unroll
      for (int b = 0; b < 8; b += 2) {
        const int jp = j0 + wj * 128 + b * 16;
        store_pair_bf16(e.C, e.ldc, i, jp + colsel, acc[a][b] + bias4[b], acc[a][b + 1] + bias4[b + 1],
                        i < M && jp + colsel < N);
      }
    }
    if (q + 1 < ntiles) zero_acc();
  }
  big::wait_vm<0>();  // the stream-end pieces land before the workgroup's LDS is released
}

}  // namespace g4

namespace {
// VIT_GEMM_G4 (0 = off), VIT_G4_MODE_{FWD,DGRAD} (0 stride, 1 band), VIT_G4_WGS (stride-walk grid cap)
int g_g4[4] = {-2, -2, -2, -2};
unsigned g_g4_launches = 0;  // host-side count of g4 launches (tests: the plain GEMMs took this kernel)
int g4_env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
void g4_env() {
  if (g_g4[0] != -2) return;
  g_g4[0] = g4_env_int("VIT_GEMM_G4", 1);
  g_g4[1] = g4_env_int("VIT_G4_MODE_FWD", 0);
  g_g4[2] = g4_env_int("VIT_G4_MODE_DGRAD", 1);
  g_g4[3] = g4_env_int("VIT_G4_WGS", 0);
}
int g4_cus() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}
template <int QL>
int launch(const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, const Epi& e, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)g4::kernel<QL>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::LDS);
    attr = true;
  }
  g4::Walk w;
  w.tiles_i = (M + 255) / 256;
  w.tiles_j = (N + 255) / 256;
  w.group_m = QL == LAY_RC ? e.group_m : 0;
  w.mode = g_g4[QL == LAY_RC ? 1 : 2] == 1 ? 1 : 0;
  if (w.mode == 1) {
    w.G = w.tiles_i;
  } else {
    const int tiles = w.tiles_i * w.tiles_j, cap = g_g4[3] > 0 ? g_g4[3] : g4_cus();
    w.G = tiles < cap ? tiles : cap;
  }
  hipLaunchKernelGGL((g4::kernel<QL>), dim3(w.G), dim3(g4::THREADS), g4::LDS, s, (const bf16*)P, ldp,
                     (const bf16*)Q, ldq, M, N, R, e, w);
  ++g_g4_launches;
  return (int)hipGetLastError();
}
}  // namespace

bool g4_enabled() {
  g4_env();
  return g_g4[0] != 0;
}

// the plain bf16 GEMM C = P Q^T (+ bias) on g4, or -1 when the shape is not one it takes: a split
// reduction, column sums, slab output, R % 64, N % 8 (the dispatcher then runs the 8-wave kernels)
int g4_launch(int q_layout, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
              const Epi& e, hipStream_t s) {
  g4_env();
  if (split > 1 || R <= 0 || R % g4::BK || N < 8 || N % 8 || e.csum || e.slab || M <= 0) return -1;
  return q_layout == LAY_RC ? launch<LAY_RC>(P, ldp, Q, ldq, M, N, R, e, s)
                            : launch<LAY_CR>(P, ldp, Q, ldq, M, N, R, e, s);
}

extern "C" {

// Tuning / test hook: tile walk of the forward and input-gradient classes (0 = stride, 1 = row band, -1 =
// keep) and the stride walk's workgroup cap (0 = the CU count, -1 = keep).  Returns 0.
int vit_gemm_g4_config(int fwd_mode, int dgrad_mode, int wgs) {
  g4_env();
  if (fwd_mode >= 0) g_g4[1] = fwd_mode;
  if (dgrad_mode >= 0) g_g4[2] = dgrad_mode;
  if (wgs >= 0) g_g4[3] = wgs;
  return 0;
}

// Host-side count of g4 launches since the last reset (reset != 0 zeroes it after reading).
int vit_gemm_g4_count(int reset) {
  const int n = (int)g_g4_launches;
  if (reset) g_g4_launches = 0;
  return n;
}

}  // extern "C"
