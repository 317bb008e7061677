// LDS image layouts and low-level primitives shared by the bf16 MFMA GEMM kernels (gemm.hip,
// gemm_ms.hip): swizzled / half-blocked operand images, inline-asm fragment reads with immediate
// offsets, counted vmcnt waits, barriers and the XCD-aware workgroup remap.
#pragma once
#include "common.hpp"
#include <type_traits>

enum { LAY_RC = 0, LAY_CR = 1 };

namespace big {

// r-contiguous image, BK=32: 64-B rows, chunk c at row*64 + ((c ^ h(row)) << 4),
// h(row) = (row & 1) | ((row >> 1) & 2).  BK=64: 128-B rows, chunk c at
// row*128 + ((c ^ ((row >> 1) & 7)) << 4).  Both conflict-free for the 16x16x32
// ds_read_b128 fragment pattern (tests/test_lds_layouts.py).
template <int BK> __device__ __forceinline__ int rc_sw(int row) {
  if constexpr (BK == 32) return (row & 1) | ((row >> 1) & 2);
  else return (row >> 1) & 7;
}
template <int BK> __device__ __forceinline__ int rc_off(int row, int c) {
  return row * (BK * 2) + ((c ^ rc_sw<BK>(row)) << 4);
}
// r-strided image: BK r-rows x COLS (COLS*2-byte rows), chunk c at
// r*COLS*2 + (((c & ~15) | ((c & 15) ^ f(r))) << 4), f(r) = ((r&3)<<2)|((r>>2)&3):
// conflict-free for the two ds_read_b64_tr_b16 of a fragment (rows 8g+q, 8g+4+q).
__device__ __forceinline__ int cr_f(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int cr_swz(int c, int r) { return (c & ~15) | ((c & 15) ^ cr_f(r)); }
template <int COLS> __device__ __forceinline__ int cr_off(int r, int c) { return r * COLS * 2 + (cr_swz(c, r) << 4); }

// Fragment reads as inline asm: the compiler cannot see them as LDS reads, so it
// does not put an s_waitcnt vmcnt(0) (for the in-flight global_load_lds writes it
// cannot prove disjoint) in front of them.  The caller orders them: a counted
// vmcnt + barrier before (data landed), lgkm_wait0() before the first use.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)LDS_PTR(p);
}
__device__ __forceinline__ bf16x8 asm_read128(uint32_t a) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return __builtin_bit_cast(bf16x8, v);
}
// the same read with a compile-time byte offset in the instruction's 16-bit offset field: the
// fragments of one wave differ from each other only by such constants (below), so the loop
// needs one address VGPR per k-substep instead of one v_add per fragment read
template <int OFF> __device__ __forceinline__ bf16x8 asm_read128_off(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds_read offset field");
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x8, v);
}
template <int N> struct Unroll {
  template <class F> __device__ __forceinline__ static void run(F&& f) {
    Unroll<N - 1>::run(f);
    f(std::integral_constant<int, N - 1>{});
  }
};
template <> struct Unroll<0> {
  template <class F> __device__ __forceinline__ static void run(F&&) {}
};
__device__ __forceinline__ bf16x4 asm_read_tr(uint32_t a) {
  i32x2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return __builtin_bit_cast(bf16x4, v);
}
template <int LAY, int ROWS, int BK>
__device__ __forceinline__ bf16x8 frag_asm(uint32_t img, int s, int kk, int lane) {
  if constexpr (LAY == LAY_RC) {
    return asm_read128(img + rc_off<BK>(s * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int c = 2 * s + (p >> 1);
    const int r0 = kk * 32 + 8 * g + q;
    bf16x4 lo = asm_read_tr(img + cr_off<ROWS>(r0, c) + (p & 1) * 8);
    bf16x4 hi = asm_read_tr(img + cr_off<ROWS>(r0 + 4, c) + (p & 1) * 8);
    return cat4(lo, hi);
  }
}

// transposed 8-B LDS read with a compile-time byte offset in the instruction's offset field
template <int OFF> __device__ __forceinline__ bf16x4 asm_read_tr_off(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds_read offset field");
  i32x2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x4, v);
}
// Half-blocked CR image (gemm_tile, pp_tile; VIT_CR_HB=0 restores the swizzled rows of stage/frag):
// one 1-KiB piece per (16-row k-block, 32-column fragment pair) -- the piece one global_load_lds
// fills, reading 16 rows x 64 contiguous bytes like the RC staging.  Inside a piece k-row rr owns
// 64 B; fragment h (0 / 1) of the pair sits in 32-B half h ^ (rr >> 3 & 1), which puts each
// transposed read's 32-lane group (k-rows {0-3, 8-11} or {4-7, 12-15}) on all 64 banks once.  A
// fragment read is a lane base (one per fragment parity) plus an immediate (pair, k-substep): no
// per-read address arithmetic, which the swizzled-row image needed (its XOR mixes the fragment
// index with the lane's row).
#ifndef VIT_CR_HB
#define VIT_CR_HB 1
#endif
template <int ROWS>
__device__ __forceinline__ int64_t crh_src(int t, int lane, int64_t ld, int row0, int lim) {
  constexpr int FP = ROWS / 32;  // fragment pairs per 16-row k-block
  const int kb = t / FP, s2 = t - kb * FP;
  const int rr = lane >> 2, h = ((lane >> 1) & 1) ^ ((rr >> 3) & 1);
  return (int64_t)(kb * 16 + rr) * ld + min(row0 + s2 * 32 + h * 16 + (lane & 1) * 8, lim - 8);
}
// byte offset of this lane's 8 B (lo = 0 / hi = 1 read) of a fragment with parity h, k-substep 0
template <int ROWS> __device__ __forceinline__ uint32_t crh_lane(int lane, int hi, int h) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int rr = 8 * (g & 1) + q + 4 * hi;
  return (uint32_t)((g >> 1) * (ROWS / 32) * 1024 + 64 * rr + 32 * (h ^ ((rr >> 3) & 1)) + 8 * p);
}
// fragment S (relative to an even first fragment folded into the bases) at k-substep KK
template <int ROWS, int KK, int S>
__device__ __forceinline__ bf16x8 frag_crh(const uint32_t (&base)[2][2], uint32_t cur) {
  constexpr int OFF = (2 * KK * (ROWS / 32) + S / 2) * 1024;
  return cat4(asm_read_tr_off<OFF>(cur + base[0][S & 1]), asm_read_tr_off<OFF>(cur + base[1][S & 1]));
}

__device__ __forceinline__ void lgkm_wait0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  // bijective: blocks that share an XCD (bid % 8) get a contiguous range of ids
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7, k = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most n stages (of G loads each) of this wave remain in flight
template <int G, int S>
__device__ __forceinline__ void wait_stages(int n) {
  if constexpr (S >= 6) { if (n >= 5) { wait_vm<5 * G>(); return; } }
  if constexpr (S >= 5) { if (n >= 4) { wait_vm<4 * G>(); return; } }
  if constexpr (S >= 4) { if (n >= 3) { wait_vm<3 * G>(); return; } }
  if constexpr (S >= 3) { if (n >= 2) { wait_vm<2 * G>(); return; } }
  if (n >= 1) { wait_vm<G>(); return; }
  wait_vm<0>();
}
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace big
