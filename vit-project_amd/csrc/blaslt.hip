// hipBLASLt for the plain bf16 GEMMs of the step (no epilogue beyond a bias), where the vendor
// library measured faster in the step than the hand-written kernels: the forwards of qkv, proj and
// fc2 (+ f32 bias) and the input gradients dX = dY W of qkv, fc1 and proj.  Bit-identical to the
// kernels in gemm.hip at every step shape (tests/test_gpu_kernels.py::test_blaslt_plain_gemms_match_kernels:
// f32 accumulation in the same k order); step +1.9 % with the input gradients, +2.6 % with both
// classes, in a same-box A/B (profiles/r05/ab_hipblaslt.txt).  Its gfx950 kernels for these shapes
// run 4 waves of 128x128 on 256x256 (or 256x192 / 192x256) tiles, stream-K for the forwards, and
// the input gradients as one workgroup per 256-row band walking the N = 768 output columns
// (197 workgroups at bs=256): beside the side stream's weight gradients they hold fewer CUs than our
// 2-workgroup-per-CU V3 / V1 launches (1182 workgroups).  Everything with a fused epilogue (GELU pair,
// GELU', residual, column sums, split-K slabs, stream-K f32) stays on the kernels in gemm.hip, and so do
// the weight gradients: the library's f32-output dW GEMMs ran 228-591 vs 596-841 TFLOP/s and -10.7 % in
// the step (profiles/r05/hipblaslt_wgrad_negative.txt).
//
// Column-major mapping (hipBLASLt is column-major; our matrices are row-major):
//   dgrad  dX[M,K] = dY[M,N] W[N,K]      ->  dX^T (K x M) = W^T (K x N, "A", op N) * dY^T (N x M, "B", op N)
//   fwd    Y[M,N]  = X[M,K] W[N,K]^T + b ->  Y^T (N x M)  = W (N x K: A stored K x N, op T) * X^T (K x M, op N),
//                                            bias along the N rows (HIPBLASLT_EPILOGUE_BIAS, f32)
// f32 accumulation, bf16 in / out.  Plans (descriptors + the heuristic's first algorithm) are built
// on first use per (device, kind, shape, strides) -- outside graph capture: a shape first seen
// while capturing is left to the hand-written kernels -- and reused.  The handle and each stream's
// workspace come from vit_blaslt_workspace (the host registers them once per (device, stream),
// like the f32 stream-K workspace), so no call here allocates device memory.
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <map>
#include <tuple>

#include "common.hpp"

namespace {

constexpr int LT_MAX_DEV = 16;
hipblasLtHandle_t g_lt[LT_MAX_DEV] = {};

struct LtWs { int dev; hipStream_t s; void* p; int64_t bytes; };
LtWs g_lt_ws[64];
int g_lt_nws = 0;

// which classes go to the library: bit 0 forward (bias), bit 1 input gradient; VIT_GEMM_LIB (A/B, default 3)
int g_lt_mask = -1;
int lt_mask() {
  if (g_lt_mask < 0) {
    const char* e = getenv("VIT_GEMM_LIB");
    g_lt_mask = e ? atoi(e) : 3;
  }
  return g_lt_mask;
}

int cur_device() {
  int d = -1;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

const LtWs* lt_ws_for(int dev, hipStream_t s) {
  for (int i = 0; i < g_lt_nws; ++i)
    if (g_lt_ws[i].dev == dev && g_lt_ws[i].s == s) return &g_lt_ws[i];
  return nullptr;
}

struct LtPlan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
};
using LtKey = std::tuple<int, int, int, int, int, int64_t, int64_t, int64_t, int64_t, int>;  // dev kind m n k lda ldb ldc ws bias
std::map<LtKey, LtPlan> g_lt_plans;

// kind 0: forward (A = W op T, bias), 1: input gradient (A = W op N)
const LtPlan* lt_plan(int dev, int kind, int m, int n, int k, int64_t lda, int64_t ldb, int64_t ldc, int64_t ws,
                      bool bias, hipStream_t s) {
  const LtKey key{dev, kind, m, n, k, lda, ldb, ldc, ws, bias ? 1 : 0};
  auto it = g_lt_plans.find(key);
  if (it != g_lt_plans.end()) return it->second.ok ? &it->second : nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  LtPlan p;
  const hipblasOperation_t ta = kind == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  bool ok = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) == HIPBLAS_STATUS_SUCCESS;
  if (bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) == HIPBLAS_STATUS_SUCCESS;
    ok = ok && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) ==
                   HIPBLAS_STATUS_SUCCESS;
  }
  // A: kind 0 stored K x N (ld lda) read transposed; kind 1 stored m x k = K x N (ld lda).  B: k x n.
  const uint64_t ar = kind == 0 ? (uint64_t)k : (uint64_t)m, ac = kind == 0 ? (uint64_t)m : (uint64_t)k;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ar, ac, lda) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, (uint64_t)k, (uint64_t)n, ldb) == HIPBLAS_STATUS_SUCCESS;
  ok = ok && hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, (uint64_t)m, (uint64_t)n, ldc) == HIPBLAS_STATUS_SUCCESS;
  if (ok) {
    hipblasLtMatmulPreference_t pref = nullptr;
    const uint64_t wsb = (uint64_t)ws;
    ok = hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)) ==
             HIPBLAS_STATUS_SUCCESS;
    hipblasLtMatmulHeuristicResult_t res[1];
    int nres = 0;
    ok = ok && hipblasLtMatmulAlgoGetHeuristic(g_lt[dev], p.desc, p.a, p.b, p.c, p.c, pref, 1, res, &nres) ==
                   HIPBLAS_STATUS_SUCCESS && nres > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS &&
         res[0].workspaceSize <= wsb;
    if (ok) {
      p.algo = res[0].algo;
      p.ws = res[0].workspaceSize;
    }
    if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  }
  p.ok = ok;
  auto& slot = g_lt_plans[key];
  slot = p;
  return slot.ok ? &slot : nullptr;
}

// 0 = done on the library; -1 = not taken (the caller runs its own kernel); else a hip error
int lt_run(int kind, int m, int n, int k, const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
           int64_t ldc, const float* bias, hipStream_t s) {
  if (!(lt_mask() & (1 << kind))) return -1;
  if (m <= 0 || n <= 0 || k <= 0) return -1;
  const int dev = cur_device();
  if (dev < 0 || dev >= LT_MAX_DEV || !g_lt[dev]) return -1;
  const LtWs* w = lt_ws_for(dev, s);
  if (!w) return -1;
  const LtPlan* p = lt_plan(dev, kind, m, n, k, lda, ldb, ldc, w->bytes, bias != nullptr, s);
  if (!p) return -1;
  if (bias) {
    const void* bp = bias;
    if (hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)) !=
        HIPBLAS_STATUS_SUCCESS)
      return -1;
  }
  const float one = 1.f, zero = 0.f;
  const hipblasStatus_t st = hipblasLtMatmul(g_lt[dev], p->desc, &one, A, p->a, B, p->b, &zero, C, p->c, C, p->c,
                                             &p->algo, w->p, p->ws, s);
  return st == HIPBLAS_STATUS_SUCCESS ? 0 : (int)hipErrorLaunchFailure;
}

}  // namespace

// used by vit_linear_fwd / vit_linear_dgrad (gemm.hip) for bf16 in / out with no fused epilogue
int vit_lt_linear_fwd(int M, int N, int K, const void* X, int64_t ldx, const void* W, const float* bias, void* Y,
                      int64_t ldy, hipStream_t s) {
  return lt_run(0, N, M, K, W, K, X, ldx, Y, ldy, bias, s);
}
int vit_lt_linear_dgrad(int M, int N, int K, const void* dY, int64_t lddy, const void* W, void* dX, int64_t lddx,
                        hipStream_t s) {
  return lt_run(1, K, M, N, W, K, dY, lddy, dX, lddx, nullptr, s);
}

extern "C" {

// Registers the hipBLASLt handle of the current device (created on the first call) and `stream`'s
// workspace (device memory the caller owns, >= 32 MiB recommended; nullptr / 0 unregisters the
// stream).  Until a stream is registered every GEMM on it runs the hand-written kernels.
int vit_blaslt_workspace(void* stream, void* ws, int64_t bytes) {
  const int dev = cur_device();
  if (dev < 0 || dev >= LT_MAX_DEV) return (int)hipErrorInvalidDevice;
  if (!g_lt[dev] && hipblasLtCreate(&g_lt[dev]) != HIPBLAS_STATUS_SUCCESS) {
    g_lt[dev] = nullptr;
    return (int)hipErrorNotInitialized;
  }
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < g_lt_nws; ++i)
    if (g_lt_ws[i].dev == dev && g_lt_ws[i].s == s) {
      g_lt_ws[i].p = ws;
      g_lt_ws[i].bytes = ws ? bytes : 0;
      if (!ws) g_lt_ws[i] = g_lt_ws[--g_lt_nws];
      return 0;
    }
  if (!ws) return 0;
  if (g_lt_nws >= 64) return (int)hipErrorOutOfMemory;
  g_lt_ws[g_lt_nws++] = LtWs{dev, s, ws, bytes};
  return 0;
}

// Tuning hook: which plain bf16 GEMM classes run on hipBLASLt (bit 0 forward + bias, bit 1 input
// gradient; -1 = from VIT_GEMM_LIB, default 3).  Returns the mask in force.
int vit_gemm_lib(int mask) {
  g_lt_mask = mask < 0 ? -1 : mask;
  return lt_mask();
}

}  // extern "C"
