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
// accumulators are started by SrcC = 0 MFMAs in each tile's first k-step, three s_nop 7 separate the
// last MFMA from the epilogue's accumulator reads.  Nothing in the k-step body is conditional: past the
// stream's end the loader re-issues valid addresses into the slot nothing reads any more (and the
// workgroup waits for them before it exits).
// ----------------------------------------------------------------------------
#include <stdlib.h>

#include "gemm_epi.hpp"

namespace g4 {

constexpr int BK = 64, PIMG = 256 * BK * 2, THREADS = 256;  // PIMG: one operand's 256 x 64 stage image

__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// a tile's first MFMA per accumulator: SrcC = inline 0 (no accumulator zeroing pass)
__device__ __forceinline__ void mfma_zero(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

// The k-step schedule (MFMA slots, kernel comment): Y fragment reads after MFMA Y0 + YS * f (f = 0..15);
// s_waitcnt lgkmcnt(0) + barrier before MFMA B1; LDS-DMA piece u after MFMA P0 + PS * u (u = 0..15); the
// counted vmcnt + barrier before MFMA B2, then the X reads after MFMA X0 + XS * f.  Sched<0> is the product's;
// the others are stamped-instance alternatives (tools/g4_stamps.py --sched).
template <int V> struct Sched;
// PF: the 8 P pieces (the streamed activation / output-gradient rows) go out first, then the 8 Q pieces (the
// weights, L2-resident); otherwise they alternate.
// DP: LDS slots of the P operand (2, or 3: stage g + 3's P pieces go out in k-step g, two k-steps of slack for
// the HBM-streamed operand; the Q ring stays 2 deep).
// Measured (tools/g4_stamps.py, k-step cycles; profiles/r06): Sched 1 / 2 (spread or dense reads / pieces)
// slower than 0 on every shape; PF (3) -4..-7 % on the fc1 input gradient, equal elsewhere.
template <> struct Sched<0> { static constexpr int Y0 = 0, YS = 1, B1 = 24, P0 = 26, PS = 6, B2 = 96, X0 = 96, XS = 1, DP = 2; static constexpr bool PF = true; };
template <> struct Sched<1> { static constexpr int Y0 = 0, YS = 2, B1 = 36, P0 = 38, PS = 5, B2 = 88, X0 = 88, XS = 2, DP = 2; static constexpr bool PF = false; };
template <> struct Sched<2> { static constexpr int Y0 = 0, YS = 1, B1 = 20, P0 = 21, PS = 4, B2 = 96, X0 = 96, XS = 1, DP = 2; static constexpr bool PF = false; };
template <> struct Sched<3> { static constexpr int Y0 = 0, YS = 1, B1 = 24, P0 = 26, PS = 6, B2 = 96, X0 = 96, XS = 1, DP = 2; static constexpr bool PF = false; };
template <> struct Sched<4> { static constexpr int Y0 = 0, YS = 1, B1 = 24, P0 = 26, PS = 6, B2 = 96, X0 = 96, XS = 1, DP = 3; static constexpr bool PF = true; };
template <class S> constexpr int pieces_before_b2() {
  int n = 0;
  for (int u = 0; u < 16; ++u) n += (S::P0 + S::PS * u < S::B2) ? 1 : 0;
  return n;
}

// a workgroup's output tiles: mode 0 strides over the row-major (or group_m-banded) tile order by the
// grid size G, mode 1 gives workgroup w row tile w and walks its column tiles
struct Walk {
  int tiles_i, tiles_j, mode, G, group_m;
  int epi;  // 1: every tile takes the fragment epilogue (A/B of the last tile's LDS-staged one)
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

// the last tile's epilogue stages bf16(acc + bias) through a [256][PITCH] LDS image (16-B row pad: a
// fragment write's 16 rows hit distinct banks) and stores it row-contiguously
constexpr int PITCH = 256 * 2 + 16, EPI_LDS = 256 * PITCH, RING_LDS = 5 * PIMG;  // P 3 deep + Q 2 deep at most
constexpr int KERNEL_LDS = EPI_LDS > RING_LDS ? EPI_LDS : RING_LDS;
static_assert(KERNEL_LDS <= 163840 && EPI_LDS == 131072 + 4 * 1024, "LDS: the GELU' act' image = 2 stage slots + 4 pieces");
constexpr int NST = 32;  // epilogue store instructions per thread (either form), issued unconditionally

typedef int i32x4 __attribute__((ext_vector_type(4)));

// P RC [M x R] (forward X / input-gradient dY), Q RC [N x R] (forward W) or CR [R x N] (input-gradient
// W read with a k stride); C bf16 [M x N] = P Q^T (+ f32 bias), R % 64 == 0, N % 8 == 0, M * ldc * 2 < 2^31.
//
// Epilogues: a tile that is not the workgroup's last stores straight from the fragments (permlane16_swap
// pairs, 16 B per lane) while the next tile's first two stages are already loading; the last tile (every
// tile of a one-tile workgroup) stages through LDS (the stage slots are free then) and stores 512-B row
// segments.  Stores go through a buffer resource over C: a lane outside [M, N) gets an offset past
// num_records, which the hardware drops, so every thread issues exactly NST stores and the next k-step's
// counted vmcnt can let them stay in flight.
//
// STAMP (diagnostic instance, vit_debug_g4_stamps; the product launches never record): thread 0 writes
// stamps[blockIdx.x * 64 + i]: 0 / 63 s_memrealtime (100 MHz) at start / end, 1 / 62 s_memtime at start /
// end, then s_memtime per event from slot 2 on: prologue done, every k-step's start, every epilogue's
// start and end (up to slot 61).  SD >= 0 selects it, with timing switches SD & 7 (1 = no in-loop operand
// loads, 2 = no in-loop barriers, 4 = no epilogue stores; results wrong, timing only) and schedule SD >> 4.
// sums over a 16-lane row of four values, every lane getting them: xor 1, xor 2 (quad_perm), then the quads
// and the halves paired by row_half_mirror / row_mirror -- the pairs of a xor 4 / xor 8 butterfly, so the
// same sums bit for bit as csum_flush's __shfl_xor form.  Inline asm (the builtin form's adds were paired
// into v_pk_add_f32, which takes no DPP operand): four independent chains interleaved put 4 instructions
// between a DPP add and the next read of its result; the leading s_nop 1 covers the VALU write -> DPP read
// hazard for the inputs, which the asm hides from the compiler.
__device__ __forceinline__ void sum16_dpp4(f32x4& v) {
  float a = v[0], b = v[1], c = v[2], d = v[3];
#define G4_DPP4(CTRL)                                                                \
  "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"     \
  "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
  asm volatile("s_nop 1\n" G4_DPP4("quad_perm:[1,0,3,2]") G4_DPP4("quad_perm:[2,3,0,1]") G4_DPP4("row_half_mirror")
                   G4_DPP4("row_mirror")
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#undef G4_DPP4
  v = f32x4{a, b, c, d};
}

template <int QL, int SD, int EP = 0>
__global__ __launch_bounds__(THREADS, 1) void kernel(const bf16* __restrict__ P, int64_t ldp,
                                                     const bf16* __restrict__ Q, int64_t ldq, int M, int N, int R,
                                                     Epi e, Walk s, unsigned long long* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = big::xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = tiles_of(s, w);
  if (ntiles <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr bool STAMP = SD >= 0;
  constexpr int dbg = SD < 0 ? 0 : (SD & 15);  // 8 (EP 1): no act' offsets (garbage image; timing only)  // compile-time: the switches cost the timed instance nothing
  using SC = Sched<SD < 0 ? 0 : (SD >> 4)>;
  constexpr int NB2 = pieces_before_b2<SC>();
  int ev = 2;
  auto stamp = [&]() {
    if constexpr (STAMP) {
      if (tid == 0 && ev < 62) stamps[(int64_t)blockIdx.x * 64 + ev] = __builtin_amdgcn_s_memtime();
      ++ev;
    }
  };
  if constexpr (STAMP) {
    if (tid == 0) {
      stamps[(int64_t)blockIdx.x * 64 + 0] = __builtin_amdgcn_s_memrealtime();
      stamps[(int64_t)blockIdx.x * 64 + 1] = __builtin_amdgcn_s_memtime();
    }
  }
  auto barrier = [&]() {
    if constexpr (!(dbg & 2)) big::lds_barrier();
  };
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave >> 1, wj = wave & 1;
  const int nk = R / BK;
  const int s_total = ntiles * nk;  // stages of this workgroup's stream

  // ---- loaders: P and Q each keep the tile and k-step of the next stage they issue (P runs DP - 2 stages
  // ahead of Q) and that tile's per-lane source offsets.  LDS: DP = 2: two [P | Q] stage slots (the P
  // and Q images of a stage adjacent: 4 % fewer cycles per k-step on the forward than separate rings,
  // profiles/r06); DP = 3: P slots [0, 3) x PIMG, then the two Q slots.
  constexpr int DP = SC::DP;
  constexpr int PSTR = DP == 2 ? 2 * PIMG : PIMG, QOFF = DP == 2 ? PIMG : DP * PIMG, QSTR = DP == 2 ? 2 * PIMG : PIMG;
  char* const qring = smem + QOFF;
  int qP = 0, kP = 0, i0P = 0, jP = 0, qQ = 0, kQ = 0, iQ = 0, j0Q = 0;
  tile_at(s, w, 0, i0P, jP);
  tile_at(s, w, 0, iQ, j0Q);
  uint32_t offP[8], offQ[8];
  // live = false (past the stream's end): every lane re-reads the operand's first 16 B (in L2) into a slot
  // nothing reads any more, so the k-step body issues its 16 pieces unconditionally (one code path, exact
  // vmcnt counts)
  auto set_p = [&](bool live) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = (wave * 8 + u) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ big::rc_sw<64>(row);
      const uint32_t op = (uint32_t)((int64_t)min(i0P + row, M - 1) * ldp * 2 + c * 16);
      offP[u] = live ? op : 0u;
    }
  };
  auto set_q = [&](bool live) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = wave * 8 + u;
      uint32_t oq;
      if constexpr (QL == LAY_RC) {
        const int row = t * 8 + (lane >> 3);
        const int c = (lane & 7) ^ big::rc_sw<64>(row);
        oq = (uint32_t)((int64_t)min(j0Q + row, N - 1) * ldq * 2 + c * 16);
      } else {
        oq = (uint32_t)(big::crh_src<256>(t, lane, ldq, j0Q, N) * 2);
      }
      offQ[u] = live ? oq : 0u;
    }
  };
  set_p(true);
  set_q(true);
  const int64_t qstep = QL == LAY_RC ? (int64_t)BK * 2 : (int64_t)BK * ldq * 2;  // bytes per k-step
  // EP 1 (GELU' input gradient, one tile per workgroup): the two stages past the stream's end carry the
  // tile's act' image instead of re-reads, in the epilogue's [256][PITCH] bf16 layout: the stage slots hold
  // image bytes [0, 128 KiB) (the slot aux stage a fills, (s_total + a) % 2, bytes [64 KiB * slot, + 64
  // KiB); P pieces the first half of a slot, Q pieces the second), one more piece per wave (after the
  // first aux k-step's second barrier) the last 4 KiB.  The DMA source picks the 16 B of LDS chunk p:
  // image row p / 33, chunk p % 33 (32 = the row pad: any valid address).
  const int ldaux2 = (int)e.ld_aux * 2;  // < 2^24 (g4_launch): 24-bit multiplies below
  auto aux_off = [&](int p) {
    const int row = (p * 1986) >> 16;  // p / 33 for p < 8448 (the image's chunks)
    const int c = min(p - row * 33, 31);
    return __umul24((unsigned)min(i0P + row, M - 1), (unsigned)ldaux2) + (unsigned)min(jP + c * 8, N - 8) * 2u;
  };
  auto set_aux = [&](uint32_t (&off)[8], int half, int a) {
    const int slot = (s_total + a) & 1;
#pragma unroll
    for (int u = 0; u < 8; ++u) off[u] = aux_off(slot * 4096 + (half * 32 + wave * 8 + u) * 64 + lane);
  };
  auto pbase = [&]() {
    if constexpr (EP == 1) {
      if (qP >= ntiles) return reinterpret_cast<const char*>(e.aux);
    }
    return reinterpret_cast<const char*>(P) + (int64_t)kP * BK * 2;
  };
  auto qbase = [&]() {
    if constexpr (EP == 1) {
      if (qQ >= ntiles) return reinterpret_cast<const char*>(e.aux);
    }
    return reinterpret_cast<const char*>(Q) + (int64_t)kQ * qstep;
  };
  auto piece_p = [&](int u, const char* pb, char* buf) {
    __builtin_amdgcn_global_load_lds((const void*)(pb + offP[u]), LDS_PTR(buf + (wave * 8 + u) * 1024), 16, 0, 0);
  };
  auto piece_q = [&](int u, const char* qb, char* buf) {
    __builtin_amdgcn_global_load_lds((const void*)(qb + offQ[u]), LDS_PTR(buf + (wave * 8 + u) * 1024), 16, 0, 0);
  };
  auto advance_p = [&]() {
    if (++kP == nk) {
      kP = 0;
      ++qP;
      set_p(tile_at(s, w, qP, i0P, jP));
    }
    if constexpr (EP == 1) {
      if (!(dbg & 8) && qP == ntiles && kP < 2) set_aux(offP, 0, kP);  // i0P / jP stay the last tile's
    }
  };
  auto advance_q = [&]() {
    if (++kQ == nk) {
      kQ = 0;
      ++qQ;
      set_q(tile_at(s, w, qQ, iQ, j0Q));
    }
    if constexpr (EP == 1) {
      if (!(dbg & 8) && qQ == ntiles && kQ < 2) set_aux(offQ, 1, kQ);
    }
  };

  // ---- fragment reads: f 0..7 = Q fragment f (columns), 8..15 = P fragment f - 8 (rows)
  uint32_t rc_p[2], rc_q[2], crh_q[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    rc_p[kk] = (uint32_t)(wi * 128 * 128 + big::rc_off<64>(lane & 15, kk * 4 + (lane >> 4)));
    rc_q[kk] = (uint32_t)(wj * 128 * 128 + big::rc_off<64>(lane & 15, kk * 4 + (lane >> 4)));
  }
#pragma unroll
  for (int lh = 0; lh < 2; ++lh)
#pragma unroll
    for (int h = 0; h < 2; ++h) crh_q[lh][h] = big::crh_lane<256>(lane, lh, h) + (uint32_t)(wj * 4 * 1024);
  // cp / cq: the LDS byte addresses of the P / Q slot the fragments come from
  auto read_frag = [&](auto kkI, auto fI, uint32_t cp, uint32_t cq, bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    constexpr int kk = decltype(kkI)::value, f = decltype(fI)::value;
    if constexpr (f < 8) {
      if constexpr (QL == LAY_RC) qf[f] = big::asm_read128_off<f * 2048>(cq + rc_q[kk]);
      else qf[f] = big::frag_crh<256, kk, f>(crh_q, cq);
    } else {
      pf[f - 8] = big::asm_read128_off<(f - 8) * 2048>(cp + rc_p[kk]);
    }
  };
  auto settle = [&](bf16x8 (&pf)[8], bf16x8 (&qf)[8]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int a = 0; a < 8; ++a) asm volatile("" : "+v"(pf[a]), "+v"(qf[a]));
    __builtin_amdgcn_sched_barrier(0);
  };

  // accumulators: defined (as garbage, no instruction) here; every tile's first k-step writes them with
  // SrcC = 0 MFMAs (mfma_zero), so no tile pays a 256-instruction zeroing pass
  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
    asm volatile("" : "=a"(acc[a][0]), "=a"(acc[a][1]), "=a"(acc[a][2]), "=a"(acc[a][3]), "=a"(acc[a][4]),
                      "=a"(acc[a][5]), "=a"(acc[a][6]), "=a"(acc[a][7]));

  // epilogue stores: C through a buffer resource, out-of-range lanes dropped by the range check
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc(e.C, (short)0, (int)((int64_t)M * e.ldc * 2), 0x00020000);
  auto store16 = [&](i32x4 v, int i, int col, bool ok) {
    const int off = ok ? (int)(((int64_t)i * e.ldc + col) * 2) : (int)0x80000000;
    if constexpr (!(dbg & 4)) __builtin_amdgcn_raw_buffer_store_b128(v, crs, off, 0, 0);
  };

  // ---- prologue: P stages 0..DP-1 and Q stages 0, 1 in flight, stage 0 landed and visible, X = its k-substep 0
  bf16x8 pX[8], qX[8], pY[8], qY[8];
  auto issue_p = [&](char* buf) {
    const char* pb = pbase();
#pragma unroll
    for (int u = 0; u < 8; ++u) piece_p(u, pb, buf);
    advance_p();
  };
  auto issue_q = [&](char* buf) {
    const char* qb = qbase();
#pragma unroll
    for (int u = 0; u < 8; ++u) piece_q(u, qb, buf);
    advance_q();
  };
  issue_p(smem);
  issue_q(qring);
  issue_p(smem + PSTR);  // stage 1 (or, on a one-stage stream, the stream-end re-read into a free slot)
  issue_q(qring + QSTR);
  if constexpr (DP == 3) {
    issue_p(smem + 2 * PSTR);
    big::wait_vm<24>();
  } else {
    big::wait_vm<16>();
  }
  big::lds_barrier();
  {
    const uint32_t cp = big::lds_addr(smem), cq = big::lds_addr(qring);
    big::Unroll<16>::run([&](auto fI) { read_frag(std::integral_constant<int, 0>{}, fI, cp, cq, pX, qX); });
    settle(pX, qX);
  }
  stamp();

  int g = 0, gp = 0;  // stage index and its P slot (g % DP)
  int i0 = 0, j0 = 0;
  for (int q = 0; q < ntiles; ++q) {
    tile_at(s, w, q, i0, j0);
    // one k-step of stage g (FIRST: the tile's first; it is peeled off the loop below, so the steady-state
    // loop is one code path whose fragment registers need no copies at its back edge)
    auto step = [&](auto firstI, bool stores) {
      stamp();
      const char *pb = pbase(), *qb = qbase();
      // this k-step reads P slot gp = g % DP and Q slot g % 2; stage g + DP's P pieces and stage g + 2's Q
      // pieces go into those slots after the first barrier, stage g + 1 comes from the next ones
      const int gp1 = gp + 1 == DP ? 0 : gp + 1;
      char* const pslot = smem + gp * PSTR;
      char* const qslot = qring + (g & 1) * QSTR;
      const uint32_t cp = big::lds_addr(pslot), cq = big::lds_addr(qslot);
      const uint32_t np = big::lds_addr(smem + gp1 * PSTR), nq = big::lds_addr(qring + ((g + 1) & 1) * QSTR);
      // one k-step; FIRST: the tile's first (its k-substep-0 MFMAs start the accumulators from 0)
      auto kstep = [&](auto firstI) {
        constexpr bool FIRST = decltype(firstI)::value;
        big::Unroll<128>::run([&](auto mI) {
          constexpr int m = decltype(mI)::value;
          constexpr int a = (m % 64) / 8, b = m % 8;
          if constexpr (m == SC::B1) {  // every wave's reads of stage g are done: its slot takes stage g + 2
            settle(pY, qY);
            barrier();
          }
          if constexpr (m == SC::B2) {  // stage g + 1 landed (this wave's pieces; counted) and visible (barrier)
            if (FIRST && stores) big::wait_vm<NB2 + NST>();  // the stores went out after stage g + 1's pieces
            else big::wait_vm<NB2>();
            barrier();
          }
          if constexpr (m < 64 && FIRST) mfma_zero(acc[a][b], qX[b], pX[a]);
          else if constexpr (m < 64) mfma_acc(acc[a][b], qX[b], pX[a]);
          else mfma_acc(acc[a][b], qY[b], pY[a]);
          if constexpr (m >= SC::Y0 && (m - SC::Y0) % SC::YS == 0 && (m - SC::Y0) / SC::YS < 16)
            read_frag(std::integral_constant<int, 1>{}, std::integral_constant<int, (m - SC::Y0) / SC::YS>{}, cp, cq, pY, qY);
          if constexpr (m >= SC::X0 && (m - SC::X0) % SC::XS == 0 && (m - SC::X0) / SC::XS < 16)
            read_frag(std::integral_constant<int, 0>{}, std::integral_constant<int, (m - SC::X0) / SC::XS>{}, np, nq, pX, qX);
          if constexpr (EP == 1 && m == SC::B2 + 1) {
            if (g + 2 == s_total)  // aux stage 0's k-step, after its second barrier: the next k-step's wait counts it
              __builtin_amdgcn_global_load_lds((const void*)(pb + aux_off(8192 + wave * 64 + lane)),
                                               LDS_PTR(smem + 131072 + wave * 1024), 16, 0, 0);
          }
          if constexpr (m >= SC::P0 && (m - SC::P0) % SC::PS == 0 && (m - SC::P0) / SC::PS < 16) {
            constexpr int u = (m - SC::P0) / SC::PS;
            constexpr int v = SC::PF ? u : (u & 1) * 8 + (u >> 1);  // 0..7 P pieces, 8..15 Q pieces
            if constexpr (!(dbg & 1)) {
              if constexpr (v < 8) piece_p(v, pb, pslot);
              else piece_q(v - 8, qb, qslot);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        settle(pX, qX);  // inside each instance: no fragment is live-in to the join with a read in flight
      };
      kstep(firstI);
      advance_p();  // the loaders move to stages g + DP + 1 and g + 3 (issued in the next k-step)
      advance_q();
      gp = gp1;
      ++g;
    };
    step(std::true_type{}, q > 0);  // q > 0: the previous tile's NST fragment-epilogue stores are in flight
    for (int k = 1; k < nk; ++k) step(std::false_type{}, false);
    // ---- epilogue of tile q: acc[a][b] holds C[i][j..j+3], i = i0 + wi*128 + 16a + lane%16,
    // j = j0 + wj*128 + 16b + 4*(lane/16)
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp();
    const int gq = lane >> 4;
    if constexpr (EP == 1) {
      // the tile origin re-defined here: nothing derived from it is hoisted above the k-step loop (the
      // column-partial addresses would be, and spill)
      int ti0 = i0, tj0 = j0, el = lane;
      asm volatile("" : "+s"(ti0), "+s"(tj0), "+v"(el));
      const int eg = el >> 4, e15 = el & 15;
      // C = bf16(acc * act'), the product written over its act' in the LDS image, then 512-B row segments
      // out; e.csum: per 64-row group column partials of the f32 products (the 8-wave kernels' fragment
      // epilogue order: a lane's 4 rows in order, then the 16-lane butterfly)
      auto mark = [&](int k) {  // stamped instance: phases of this epilogue in slots 50..52
        if constexpr (STAMP) {
          if (tid == 0) stamps[(int64_t)blockIdx.x * 64 + 50 + k] = __builtin_amdgcn_s_memtime();
        }
      };
      big::wait_vm<0>();
      big::lds_barrier();
      mark(0);
      f32x4 cs[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                          "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
        const int r = wi * 128 + a * 16 + e15;
        const float rowin = ti0 + r < M ? 1.f : 0.f;  // rows past M (clamped copies of row M - 1) add nothing
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          char* const p = smem + r * PITCH + (wj * 128 + b * 16 + 4 * eg) * 2;
          const bf16x4 d = *reinterpret_cast<const bf16x4*>(p);
          const f32x4 v = acc[a][b] * f32x4{(float)d[0], (float)d[1], (float)d[2], (float)d[3]};
          *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
#pragma unroll
          for (int t = 0; t < 4; ++t) cs[b][t] = __builtin_fmaf(v[t], rowin, cs[b][t]);  // = cs + v, or cs
        }
        if ((a & 3) == 3) {  // one partial row per 64-row group
          const int row0 = ti0 + wi * 128 + (a - 3) * 16;
#pragma unroll
          for (int b = 0; b < 8; ++b) {
            sum16_dpp4(cs[b]);
            const int j = tj0 + wj * 128 + b * 16 + 4 * eg;
            if (e.csum && e15 == 0 && row0 < M && j < N)
              *reinterpret_cast<f32x4*>(e.csum + (int64_t)(row0 >> 6) * N + j) = cs[b];
            cs[b] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      big::lds_barrier();
      mark(1);
      const int c = el & 31, r0 = wave * 2 + (el >> 5);
      const int col = tj0 + c * 8;
#pragma unroll 8
      for (int p = 0; p < NST; ++p) {
        const int r = r0 + 8 * p;
        const i32x4 v = *reinterpret_cast<const i32x4*>(smem + r * PITCH + c * 16);
        store16(v, i0 + r, col, ti0 + r < M && col < N);
      }
      stamp();
      continue;
    }
    f32x4 bias4[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int j = j0 + wj * 128 + b * 16 + 4 * gq;
      bias4[b] = (e.bias && j < N) ? *reinterpret_cast<const f32x4*>(e.bias + j) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // a tile that is not the workgroup's last: fragment pairs widened to 16-B stores (permlane16_swap; lane
    // group gq then holds 8 columns of the pair).  The last tile (staged): once the stream-end pieces have
    // landed and every wave's reads retired (wait + barrier) the stage slots are free, so the tile goes
    // through a bf16 LDS image and out in 512-B row segments.
    const bool staged = EP == 2 || !(q + 1 < ntiles || s.epi == 1);  // EP 2: one tile per workgroup
    if (staged) {
      big::wait_vm<0>();
      big::lds_barrier();
    }
    const int colsel = (gq & 1) * 16 + (gq >> 1) * 8;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      asm volatile("" : "+a"(acc[a][0]), "+a"(acc[a][1]), "+a"(acc[a][2]), "+a"(acc[a][3]), "+a"(acc[a][4]),
                        "+a"(acc[a][5]), "+a"(acc[a][6]), "+a"(acc[a][7]));
      const int r = wi * 128 + a * 16 + (lane & 15), i = i0 + r;
#pragma unroll
      for (int b = 0; b < 8; b += 2) {
        const f32x4 x = acc[a][b] + bias4[b], y = acc[a][b + 1] + bias4[b + 1];
        const bf16x4 px = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
        const bf16x4 py = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
        if (staged) {
          char* row = smem + r * PITCH + (wj * 128 + b * 16 + 4 * gq) * 2;
          *reinterpret_cast<bf16x4*>(row) = px;
          *reinterpret_cast<bf16x4*>(row + 32) = py;
        } else {
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          const u32x2 ux = __builtin_bit_cast(u32x2, px), uy = __builtin_bit_cast(u32x2, py);
          const auto r0 = __builtin_amdgcn_permlane16_swap(ux[0], uy[0], false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(ux[1], uy[1], false, false);
          const int col = j0 + wj * 128 + b * 16 + colsel;
          store16(i32x4{(int)r0[0], (int)r1[0], (int)r0[1], (int)r1[1]}, i, col, i < M && col < N);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one accumulator row at a time
    }
    if (staged) {
      big::lds_barrier();
      const int c = tid & 31, r0 = tid >> 5;
      const int col = j0 + c * 8;
      if constexpr (EP == 2) {
        // fc1's GELU pair: from the bf16 pre image (pre = bf16(acc + bias), as the 8-wave kernels' staged
        // pair epilogue), C = GELU'(pre) and aux_out = GELU(pre) (gelu_fast_both), both 512-B row segments
        const __amdgpu_buffer_rsrc_t ars =
            __builtin_amdgcn_make_buffer_rsrc(e.aux_out, (short)0, (int)((int64_t)M * e.ldc * 2), 0x00020000);
#pragma unroll 4
        for (int p = 0; p < NST; ++p) {
          const int r = r0 + 8 * p;
          const bf16x8 x = *reinterpret_cast<const bf16x8*>(smem + r * PITCH + c * 16);
          bf16x8 av, dv;
#pragma unroll
          for (int t = 0; t < 8; t += 2) {
            f32x2 ga, gd;
            gelu_fast_both2(f32x2{(float)x[t], (float)x[t + 1]}, ga, gd);
            av[t] = (bf16)ga.x;
            av[t + 1] = (bf16)ga.y;
            dv[t] = (bf16)gd.x;
            dv[t + 1] = (bf16)gd.y;
          }
          const bool ok = i0 + r < M && col < N;
          store16(__builtin_bit_cast(i32x4, dv), i0 + r, col, ok);
          const int off = ok ? (int)(((int64_t)(i0 + r) * e.ldc + col) * 2) : (int)0x80000000;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, av), ars, off, 0, 0);
        }
      } else {
#pragma unroll 8
        for (int p = 0; p < NST; ++p) {
          const int r = r0 + 8 * p;
          const i32x4 v = *reinterpret_cast<const i32x4*>(smem + r * PITCH + c * 16);
          store16(v, i0 + r, col, i0 + r < M && col < N);
        }
      }
    }
    stamp();
  }
  if (s.epi == 1) big::wait_vm<0>();  // the stream-end pieces land before the workgroup's LDS is released
  if constexpr (STAMP) {
    if (tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamps[(int64_t)blockIdx.x * 64 + 62] = __builtin_amdgcn_s_memtime();
      stamps[(int64_t)blockIdx.x * 64 + 63] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

}  // namespace g4

namespace {
// VIT_GEMM_G4 (0 = off), VIT_G4_MODE_{FWD,DGRAD} (0 stride, 1 band, 2 stride on tiles_i workgroups), VIT_G4_WGS (stride-walk grid cap),
// VIT_G4_TPW (stride walk: at most this many tiles per workgroup, 0 = no limit)
int g_g4[7] = {-2, -2, -2, -2, -2, -2, -2};
int g_g4_dbg = 0;  // timing switches of the stamped instance (vit_debug_g4_stamps)
unsigned g_g4_launches = 0;  // host-side count of g4 launches (tests: the plain GEMMs took this kernel)
unsigned long long* g_g4_stamps = nullptr;  // vit_debug_g4_stamps: launch the stamped instance
int g4_env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
void g4_env() {
  if (g_g4[0] != -2) return;
  g_g4[0] = g4_env_int("VIT_GEMM_G4", 1);
  g_g4[1] = g4_env_int("VIT_G4_MODE_FWD", 0);
  g_g4[2] = g4_env_int("VIT_G4_MODE_DGRAD", 2);  // 2: +1.1 / +1.3 % over the row bands (two same-box A/Bs)
  g_g4[3] = g4_env_int("VIT_G4_WGS", 0);
  g_g4[4] = g4_env_int("VIT_G4_TPW", 1);  // in the step one tile per workgroup measured best for the
                                          // forward (7267 vs 7061-7091 img/s for 2, 3, 3.8 tiles / CU)
  g_g4[5] = g4_env_int("VIT_G4_EPI", 0);
  g_g4[6] = g4_env_int("VIT_G4_GELU", 1);  // the GELU' input gradient on g4 (EP 1): +0.5 % in the step
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
int launch(int ep, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, const Epi& e, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if constexpr (QL == LAY_CR) {
      (void)hipFuncSetAttribute((const void*)g4::kernel<QL, -1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
      (void)hipFuncSetAttribute((const void*)g4::kernel<QL, 0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
      (void)hipFuncSetAttribute((const void*)g4::kernel<QL, 8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
    } else {
      (void)hipFuncSetAttribute((const void*)g4::kernel<QL, -1, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
      (void)hipFuncSetAttribute((const void*)g4::kernel<QL, 0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
    }
    for (const void* k : {(const void*)g4::kernel<QL, -1>, (const void*)g4::kernel<QL, 0>, (const void*)g4::kernel<QL, 1>,
                          (const void*)g4::kernel<QL, 2>, (const void*)g4::kernel<QL, 4>, (const void*)g4::kernel<QL, 16>,
                          (const void*)g4::kernel<QL, 32>, (const void*)g4::kernel<QL, 48>, (const void*)g4::kernel<QL, 64>})
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g4::KERNEL_LDS);
    attr = true;
  }
  g4::Walk w;
  w.tiles_i = (M + 255) / 256;
  w.tiles_j = (N + 255) / 256;
  w.group_m = QL == LAY_RC ? e.group_m : 0;
  w.epi = g_g4[5];
  const int wm = g_g4[QL == LAY_RC ? 1 : 2];
  w.mode = wm == 1 ? 1 : 0;
  if (w.mode == 1) {
    w.G = w.tiles_i;
  } else if (wm == 2) {  // stride walk on tiles_i workgroups (A/B): band mode's footprint, but the WGs
    w.G = w.tiles_i;     // running together cover a band's column tiles (its dY rows shared in L2)
  } else {
    const int tiles = w.tiles_i * w.tiles_j, cap = g_g4[3] > 0 ? g_g4[3] : g4_cus();
    w.G = tiles < cap ? tiles : cap;
    if (g_g4[4] > 0 && w.G < (tiles + g_g4[4] - 1) / g_g4[4]) w.G = (tiles + g_g4[4] - 1) / g_g4[4];
  }
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(w.G), dim3(g4::THREADS), g4::KERNEL_LDS, s, (const bf16*)P, ldp, (const bf16*)Q, ldq,
                       M, N, R, e, w, g_g4_stamps);
  };
  if constexpr (QL == LAY_CR) {
    if (ep == 1) {  // the GELU' input gradient (g4_launch checked it): one tile per workgroup, bands of group_m
      w.mode = 0;
      w.group_m = e.group_m;
      w.G = w.tiles_i * w.tiles_j;
      if (g_g4_stamps && g_g4_dbg == 8) go(g4::kernel<QL, 8, 1>);
      else if (g_g4_stamps) go(g4::kernel<QL, 0, 1>);
      else go(g4::kernel<QL, -1, 1>);
      ++g_g4_launches;
      return (int)hipGetLastError();
    }
  } else {
    if (ep == 2) {  // the fc1 GELU pair forward: one tile per workgroup, the forward's tile order
      w.mode = 0;
      w.group_m = e.group_m;
      w.G = w.tiles_i * w.tiles_j;
      if (g_g4_stamps) go(g4::kernel<QL, 0, 2>);
      else go(g4::kernel<QL, -1, 2>);
      ++g_g4_launches;
      return (int)hipGetLastError();
    }
  }
  if (!g_g4_stamps) {
    go(g4::kernel<QL, -1>);
  } else {
    switch (g_g4_dbg) {  // the stamped instances built: schedules 0-3, and schedule 0 with each timing switch
      case 1: go(g4::kernel<QL, 1>); break;
      case 2: go(g4::kernel<QL, 2>); break;
      case 4: go(g4::kernel<QL, 4>); break;
      case 16: go(g4::kernel<QL, 16>); break;
      case 32: go(g4::kernel<QL, 32>); break;
      case 48: go(g4::kernel<QL, 48>); break;
      case 64: go(g4::kernel<QL, 64>); break;
      default: go(g4::kernel<QL, 0>); break;
    }
  }
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
int g4_launch(int q_layout, int ep, const void* P, int64_t ldp, const void* Q, int64_t ldq, int M, int N, int R, int split,
              const Epi& e, hipStream_t s) {
  g4_env();
  if (split > 1 || R <= 0 || R % g4::BK || N < 8 || N % 8 || e.slab || M <= 0) return -1;
  if ((int64_t)M * e.ldc * 2 >= ((int64_t)1 << 31) || e.ldc % 8) return -1;  // buffer-store offsets are int32
  if (ep == 2) {  // fc1 GELU pair forward: C = GELU'(pre), aux_out = GELU(pre), pre = bf16(P Q^T + bias)
    if (!(g_g4[6] & 2) || q_layout != LAY_RC || !e.aux_out || e.csum) return -1;
    return launch<LAY_RC>(2, P, ldp, Q, ldq, M, N, R, e, s);
  }
  if (ep == 1) {  // GELU' input gradient: C = (P Q^T) * aux, column partials allowed; no bias
    if (!(g_g4[6] & 1) || q_layout != LAY_CR || !e.aux || e.bias || R < 2 * g4::BK || e.ld_aux % 8 || ((uintptr_t)e.aux & 15) ||
        e.ld_aux >= (1 << 23) || M >= (1 << 24) ||  // aux_off's 24-bit multiplies
        (int64_t)M * e.ld_aux * 2 >= ((int64_t)1 << 31))
      return -1;
    return launch<LAY_CR>(1, P, ldp, Q, ldq, M, N, R, e, s);
  }
  if (e.csum) return -1;
  return q_layout == LAY_RC ? launch<LAY_RC>(0, P, ldp, Q, ldq, M, N, R, e, s)
                            : launch<LAY_CR>(0, P, ldp, Q, ldq, M, N, R, e, s);
}

extern "C" {

// Tuning / test hook: tile walk of the forward and input-gradient classes (0 = stride, 1 = row band, 2 = stride
// over tiles_i persistent workgroups (the input gradients' default), -1 = keep), the stride walk's workgroup cap (0 = the CU count, -1 = keep) and its tiles per workgroup (the
// grid grows to ceil(tiles / tpw) workgroups; 0 = no limit, -1 = keep).  Returns 0.
int vit_gemm_g4_config(int fwd_mode, int dgrad_mode, int wgs, int tpw) {
  g4_env();
  if (fwd_mode >= 0) g_g4[1] = fwd_mode;
  if (dgrad_mode >= 0) g_g4[2] = dgrad_mode;
  if (wgs >= 0) g_g4[3] = wgs;
  if (tpw >= 0) g_g4[4] = tpw;
  return 0;
}

// Diagnostic (not in the header): while buf != NULL every g4 launch runs the stamped instance, writing
// 64 stamps per workgroup into buf (>= grid * 64 * 8 bytes; see g4::kernel); dbg = timing switches | 16 *
// schedule (the instances built: 0, 1, 2, 4, 16, 32, 48, 64).
int vit_debug_g4_stamps(void* buf, int dbg) {
  g_g4_stamps = (unsigned long long*)buf;
  g_g4_dbg = dbg;
  return 0;
}

// Tuning / test hook: which GELU GEMMs run on g4 (bit 0: the GELU' input gradient, bit 1: the fc1 GELU pair
// forward; the rest stay on the 8-wave kernels); -1 keeps.  Returns the previous mask.
int vit_gemm_g4_gelu(int on) {
  g4_env();
  const int prev = g_g4[6];
  if (on >= 0) g_g4[6] = on;
  return prev;
}

// Host-side count of g4 launches since the last reset (reset != 0 zeroes it after reading).
int vit_gemm_g4_count(int reset) {
  const int n = (int)g_g4_launches;
  if (reset) g_g4_launches = 0;
  return n;
}

}  // extern "C"
