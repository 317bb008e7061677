// Probe of the gfx950 block-scaled MFMA operand layouts (v_mfma_scale_f32_32x32x64_f8f6f4 and
// v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 operands) with exact one-hot data:
//   1. A one-hot at (lane, byte), B = ones  -> the output row of that A element
//   2. B one-hot at (lane, byte), A = ones  -> the output column of that B element
//   3. A one-hot (row r, k) x B one-hot (k', col c) under the hypothesis
//        A: lane l holds A[row l % R][k = KB * (l / R) + byte]   (R = 32 or 16, KB = 32)
//        B: lane l holds B[k = KB * (l / R) + byte][col l % R]
//      -> C[r][c] == 1 exactly when k == k'
//   4. the E8M0 scale: scale_a = 128 on one lane doubles exactly that lane's elements.
//   5/6. which bytes a scale covers.  Result (gfx950): the pairing above holds, but the 32-value
//      k-block a lane's scale belongs to is NOT that lane's 32 bytes: for 32x32x64, k-block s (scale
//      of lane 32s + row) covers bytes [16s, 16s+16) of BOTH lane halves (so the hardware k index of
//      lane half h, byte j is 32*(j/16) + 16h + j%16); for 16x16x128, bytes [16s', ..) of all four
//      lane groups.  A kernel whose two lane halves of a row carry different scales must place its
//      data by that order; one scale per row (the same in every lane of the row) is order-free.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe/mfma_scale_probe.hip -o tools/probe/mfma_scale_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr unsigned char ONE = 0x38;  // e4m3fn 1.0

// per wave: A bytes [64 lanes][32], B bytes [64][32], scales [64] x 2 -> C [64 lanes][16] (32x32) or [4] (16x16)
template <int BIG>
__global__ void probe(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* C) {
  const int w = blockIdx.x, l = threadIdx.x;
  v8i a, b;
  const int* pa = reinterpret_cast<const int*>(A + ((size_t)w * 64 + l) * 32);
  const int* pb = reinterpret_cast<const int*>(B + ((size_t)w * 64 + l) * 32);
  for (int i = 0; i < 8; ++i) { a[i] = pa[i]; b[i] = pb[i]; }
  if constexpr (BIG) {
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa[w * 64 + l], 0, sb[w * 64 + l]);
    for (int i = 0; i < 16; ++i) C[((size_t)w * 64 + l) * 16 + i] = c[i];
  } else {
    v4f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa[w * 64 + l], 0, sb[w * 64 + l]);
    for (int i = 0; i < 4; ++i) C[((size_t)w * 64 + l) * 16 + i] = c[i];
  }
}

// standard C/D maps (cdna_hip_programming.md): 32x32: row = (reg&3) + 8*(reg>>2) + 4*(lane>>5), col = lane&31;
// 16x16: row = 4*(lane>>4) + reg, col = lane&15
static void cpos(int big, int lane, int reg, int& row, int& col) {
  if (big) { row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); col = lane & 31; }
  else { row = 4 * (lane >> 4) + reg; col = lane & 15; }
}

template <int BIG>
static int run(const char* name) {
  const int R = BIG ? 32 : 16, NREG = BIG ? 16 : 4, KB = 32, K = BIG ? 64 : 128;
  const int W = 64 * 32;  // one wave per (lane, byte)
  std::vector<unsigned char> A((size_t)W * 64 * 32), B((size_t)W * 64 * 32);
  std::vector<int> sa((size_t)W * 64, 127), sb((size_t)W * 64, 127);
  std::vector<float> C((size_t)W * 64 * 16);
  unsigned char *dA, *dB; int *dsa, *dsb; float* dC;
  hipMalloc(&dA, A.size()); hipMalloc(&dB, B.size()); hipMalloc(&dsa, sa.size() * 4); hipMalloc(&dsb, sb.size() * 4);
  hipMalloc(&dC, C.size() * 4);
  auto go = [&]() {
    hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa.data(), sa.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb.data(), sb.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe<BIG>, dim3(W), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
  };
  auto find = [&](int w, int& row, int& col, int& n, float& v) {
    n = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < NREG; ++r) {
        float x = C[((size_t)w * 64 + l) * 16 + r];
        if (x != 0.f) { ++n; v = x; cpos(BIG, l, r, row, col); }
      }
  };
  int bad = 0;
  // 1. A rows
  for (int w = 0; w < W; ++w) {
    const int L = w / 32, p = w % 32;
    for (int l = 0; l < 64; ++l) for (int q = 0; q < 32; ++q) {
      A[((size_t)w * 64 + l) * 32 + q] = (l == L && q == p) ? ONE : 0;
      B[((size_t)w * 64 + l) * 32 + q] = ONE;
    }
  }
  go();
  for (int w = 0; w < W; ++w) {
    const int L = w / 32;
    int n = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < NREG; ++r) {
        float x = C[((size_t)w * 64 + l) * 16 + r];
        int row, col; cpos(BIG, l, r, row, col);
        if (x != 0.f) { ++n; if (row != L % R || x != 1.f) ++bad; }
      }
    if (n != R) ++bad;  // the row is 1 in every column
  }
  printf("%s A-row map (row = lane %% %d): %s\n", name, R, bad ? "MISMATCH" : "ok");
  int bad1 = bad;
  // 2. B cols
  bad = 0;
  for (int w = 0; w < W; ++w) {
    const int L = w / 32, p = w % 32;
    for (int l = 0; l < 64; ++l) for (int q = 0; q < 32; ++q) {
      B[((size_t)w * 64 + l) * 32 + q] = (l == L && q == p) ? ONE : 0;
      A[((size_t)w * 64 + l) * 32 + q] = ONE;
    }
  }
  go();
  for (int w = 0; w < W; ++w) {
    const int L = w / 32;
    int n = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < NREG; ++r) {
        float x = C[((size_t)w * 64 + l) * 16 + r];
        int row, col; cpos(BIG, l, r, row, col);
        if (x != 0.f) { ++n; if (col != L % R || x != 1.f) ++bad; }
      }
    if (n != R) ++bad;
  }
  printf("%s B-col map (col = lane %% %d): %s\n", name, R, bad ? "MISMATCH" : "ok");
  int bad2 = bad;
  // 3. k pairing: wave w -> A element (row 3, k = w % K), B element (k' = (w * 7 + (w / K)) % K, col 5)
  bad = 0;
  int matches = 0;
  for (int w = 0; w < W; ++w) {
    const int ka = w % K, kb = (w / K) % 2 ? ka : (w * 7 + 3) % K;
    for (int l = 0; l < 64; ++l) for (int q = 0; q < 32; ++q) {
      const int rowA = l % R, kA = KB * (l / R) + q, kB = KB * (l / R) + q, colB = l % R;
      A[((size_t)w * 64 + l) * 32 + q] = (rowA == 3 && kA == ka) ? ONE : 0;
      B[((size_t)w * 64 + l) * 32 + q] = (colB == 5 && kB == kb) ? ONE : 0;
    }
  }
  go();
  for (int w = 0; w < W; ++w) {
    const int ka = w % K, kb = (w / K) % 2 ? ka : (w * 7 + 3) % K;
    int row = -1, col = -1, n; float v = 0;
    find(w, row, col, n, v);
    if (ka == kb) { ++matches; if (n != 1 || row != 3 || col != 5 || v != 1.f) ++bad; }
    else if (n != 0) ++bad;
  }
  printf("%s k pairing (A: k = %d*(lane/%d)+byte, B same): %s (%d matching pairs checked)\n", name, KB, R,
         bad ? "MISMATCH" : "ok", matches);
  int bad3 = bad;
  // 4. scales: all ones; lane 0's scale_a = 128 (x2), lane (R) scale_b = 129 (x4)
  bad = 0;
  for (int w = 0; w < 1; ++w)
    for (int l = 0; l < 64; ++l) for (int q = 0; q < 32; ++q) {
      A[((size_t)w * 64 + l) * 32 + q] = ONE;
      B[((size_t)w * 64 + l) * 32 + q] = ONE;
    }
  sa[0] = 128; sb[R] = 129;
  go();
  // C[r][c] = sum_k a*b*sa*sb: row 0 gets k in [0,32) doubled; col 0 gets k in [32,64) x4
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < NREG; ++r) {
      int row, col; cpos(BIG, l, r, row, col);
      float want = 0;
      for (int k = 0; k < K; ++k) {
        float s = 1;
        if (row == 0 && k / KB == 0) s *= 2;
        if (col == 0 && k / KB == 1) s *= 4;
        want += s;
      }
      if (C[(size_t)l * 16 + r] != want) ++bad;
    }
  printf("%s E8M0 scale per lane (its 32 k values): %s\n", name, bad ? "MISMATCH" : "ok");
  // 5. the full scale-lane map: wave w < 64 doubles A's scale on lane w, wave 64 + w B's on lane w;
  //    A = B = ones.  With K = 2 (32x32x64) or 4 (16x16x128) k-blocks of 32, output C[r][c] = sum over
  //    blocks of s_a(r, blk) * s_b(blk, c) * 32: the doubled lane shows which (row, block) it scales.
  {
    int bad5 = 0;
    const int NB = K / KB;
    for (int w = 0; w < 128; ++w)
      for (int l = 0; l < 64; ++l) {
        for (int q = 0; q < 32; ++q) { A[((size_t)w * 64 + l) * 32 + q] = ONE; B[((size_t)w * 64 + l) * 32 + q] = ONE; }
        sa[w * 64 + l] = (w < 64 && l == w) ? 128 : 127;
        sb[w * 64 + l] = (w >= 64 && l == w - 64) ? 128 : 127;
      }
    go();
    for (int w = 0; w < 128; ++w) {
      const int L = w % 64;
      // hypothesis: lane L scales row/col L % R, block L / R
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < NREG; ++r) {
          int row, col; cpos(BIG, l, r, row, col);
          float want = 0;
          for (int blk = 0; blk < NB; ++blk) {
            float sc = 1;
            if (w < 64 && row == L % R && blk == L / R) sc = 2;
            if (w >= 64 && col == L % R && blk == L / R) sc = 2;
            want += 32 * sc;
          }
          if (C[((size_t)w * 64 + l) * 16 + r] != want) ++bad5;
        }
    }
    printf("%s scale lane map (lane L -> row/col L %% %d, k-block L / %d): %s\n", name, R, R, bad5 ? "MISMATCH" : "ok");
    bad += bad5;
  }
  // 6. which BYTES a k-block's scale covers: A nonzero only in bytes [16g, 16g+16) of lane 0 (row 0),
  //    B = ones, every lane's scale 1 except lane R*s (the scale of k-block s) = 2: the row-0 sum tells
  //    whether bytes 16g.. of lane 0 belong to k-block s.  Printed as a table (informational).
  for (int g = 0; g < 2; ++g) {
    printf("%s lane-0 bytes [%d,%d) scaled by the scale of k-block:", name, 16 * g, 16 * g + 16);
    for (int sblk = 0; sblk < K / KB; ++sblk) {
      for (int l = 0; l < 64; ++l) {
        for (int q = 0; q < 32; ++q) {
          A[(size_t)l * 32 + q] = (l == 0 && q / 16 == g) ? ONE : 0;
          B[(size_t)l * 32 + q] = ONE;
        }
        sa[l] = (l == R * sblk) ? 128 : 127;
        sb[l] = 127;
      }
      go();
      int row, col; cpos(BIG, 0, 0, row, col);  // lane 0 reg 0 = C[0][0]
      if (C[0] == 32.f) printf(" %d", sblk);
    }
    printf("\n");
  }
  hipFree(dA); hipFree(dB); hipFree(dsa); hipFree(dsb); hipFree(dC);
  return bad1 + bad2 + bad3 + bad;
}

int main() {
  int bad = run<1>("32x32x64") + run<0>("16x16x128");
  printf(bad ? "PROBE FAILED\n" : "PROBE OK\n");
  return bad ? 1 : 0;
}
