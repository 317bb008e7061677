// DoRA adapter weight (NEWP:447-463) and its backward, plus the
// fused AdamW step the CLIP-HBA loop uses (NEWP:1181, a19).
//
//   Dn = D + (B @ A) * s          D [in, out], B [in, r], A [r, out]
//   nu[o] = ||Dn[:, o]||,  n[o] = nu[o] + 1e-8
//   W[o][i] = Dn[i][o] / n[o] * m[o]                    (returned as [out, in])
//
// Forward: 64x64 tiles compute Dn with the rank-r product in registers, write
// Dn^T (the [out, in] orientation of W) through an LDS transpose and per-tile
// column sum-of-squares; a row kernel then finishes n and W = Dn^T * m / n.
// Backward (gW = dL/dW, [out, in]):
//   c[o]   = sum_i gW[o][i] Dn[i][o]
//   dm[o]  = c[o] / n[o]
//   dDn^T  = m/n * gW - m c / (n^2 nu) * Dn^T     (row-wise, scaled by s below)
//   dB     = s * dDn A^T,   dA = s * B^T dDn       (generic GEMMs, f32)
#include "common.hpp"

extern "C" int vit_gemm(int dtype, int out_dtype, int p_layout, int q_layout, int epi, int M, int N, int R,
                        const void* P, int64_t ldp, const void* Q, int64_t ldq, void* C, int64_t ldc,
                        const float* bias, const void* aux, int64_t ld_aux, void* aux_out, int allow_fast,
                        void* stream);
extern "C" int vit_gemm_splitk(int p_layout, int q_layout, int M, int N, int R, const float* P, int64_t ldp,
                               const float* Q, int64_t ldq, float* C, float* slabs, int64_t slab_floats, void* stream);

constexpr int DT = 64;

__global__ __launch_bounds__(256) void dora_tile_kernel(int in, int out, int r, const float* __restrict__ A,
                                                        const float* __restrict__ Bm, const float* __restrict__ D,
                                                        float s, const float* __restrict__ noise,
                                                        float* __restrict__ DnT, float* __restrict__ colsq) {
  __shared__ float Bs[DT][65], As[64][DT + 1], T[DT][DT + 1];
  __shared__ float red[4][DT];
  const int i0 = blockIdx.y * DT, o0 = blockIdx.x * DT, t = threadIdx.x;
  for (int idx = t; idx < DT * 64; idx += 256) {
    int a = idx / 64, k = idx % 64;  // Bs[i][k]
    Bs[a][k] = (i0 + a < in && k < r) ? Bm[(int64_t)(i0 + a) * r + k] : 0.f;
    int kk = idx / DT, o = idx % DT;  // As[k][o]
    As[kk][o] = (kk < r && o0 + o < out) ? A[(int64_t)kk * out + o0 + o] : 0.f;
  }
  __syncthreads();
  const int ol = t & 63, ig = t >> 6;
  float sq = 0.f;
  for (int u = 0; u < 16; ++u) {
    int il = ig * 16 + u, i = i0 + il, o = o0 + ol;
    float acc = 0.f;
    for (int k = 0; k < r; ++k) acc = fmaf(Bs[il][k], As[k][ol], acc);
    float dn = 0.f;
    if (i < in && o < out) {
      const int64_t e = (int64_t)i * out + o;
      // DoRALayer.forward (NEWP:467-470): dropout(delta_D) = (B@A * s) * noise, noise = mask / (1 - p)
      dn = D[e] + (noise ? (acc * s) * noise[e] : acc * s);
    }
    T[ol][il] = dn;
    sq += dn * dn;
  }
  red[ig][ol] = sq;
  __syncthreads();
  if (t < DT && o0 + t < out) colsq[(int64_t)blockIdx.y * out + o0 + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  for (int idx = t; idx < DT * DT; idx += 256) {
    int ol2 = idx / DT, il2 = idx % DT;
    if (o0 + ol2 < out && i0 + il2 < in) DnT[(int64_t)(o0 + ol2) * in + i0 + il2] = T[ol2][il2];
  }
}

// one wave per output row o: nu, n, W[o][:] = Dn^T[o][:] * m[o] / n[o]
__global__ __launch_bounds__(256) void dora_finish_kernel(int in, int out, int ntiles, const float* __restrict__ colsq,
                                                          const float* __restrict__ m, const float* __restrict__ DnT,
                                                          float* __restrict__ W, float* __restrict__ nu_out) {
  int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= out) return;
  float s = 0.f;
  for (int z = lane; z < ntiles; z += 64) s += colsq[(int64_t)z * out + o];
  s = wave_sum(s);
  float nu = sqrtf(s), n = nu + 1e-8f, f = m[o] / n;
  for (int i = lane; i < in; i += 64) W[(int64_t)o * in + i] = DnT[(int64_t)o * in + i] * f;
  if (lane == 0 && nu_out) nu_out[o] = nu;
}

// one wave per row o: c = gW[o].DnT[o]; dm; sdDnT[o][:] = s * dDn^T
__global__ __launch_bounds__(256) void dora_bwd_row_kernel(int in, int out, const float* __restrict__ gW,
                                                           const float* __restrict__ DnT, const float* __restrict__ m,
                                                           const float* __restrict__ nu, float s,
                                                           const float* __restrict__ noise, float* __restrict__ dm,
                                                           float* __restrict__ sdDnT) {
  int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= out) return;
  float c = 0.f;
  for (int i = lane; i < in; i += 64) c = fmaf(gW[(int64_t)o * in + i], DnT[(int64_t)o * in + i], c);
  c = wave_sum(c);
  const float v = nu[o], n = v + 1e-8f, mo = m[o];
  if (lane == 0) dm[o] = c / n;
  const float a = mo / n, bcoef = (v > 0.f) ? mo * c / (n * n * v) : 0.f;
  for (int i = lane; i < in; i += 64) {
    int64_t e = (int64_t)o * in + i;
    const float g = s * (a * gW[e] - bcoef * DnT[e]);
    sdDnT[e] = noise ? g * noise[(int64_t)i * out + o] : g;
  }
}

// ---------------------------------------------------------------------------
// AdamW (torch.optim.AdamW, amsgrad off, single-tensor path): decoupled decay,
// lerp'd first moment, then p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps).
// step_size = lr / (1 - b1^step) and sqrt(1 - b2^step) are computed per tensor in
// double on the host from that tensor's own state['step'] (as torch does), so a
// resumed optimizer (load_state_dict) continues the bias correction where it was.
// They live in a separate device array (coef = {step_size, bc2_sqrt, decay, 0} of this
// tensor, decay = 1 - lr * weight_decay of its group) refreshed by one copy per step, so
// the tensor table itself never changes between steps and a replayed graph follows an
// lr schedule in both the step size and the decoupled decay.  The bf16 GEMM shadow of the parameter (if any) is written in the same pass.
// ---------------------------------------------------------------------------
struct AdamTensor { float* p; const float* g; float* m; float* v; bf16* shadow; int64_t n; const float* coef; };
struct AdamChunk { int tensor; int pad; int64_t start; };
constexpr int ADAM_CHUNK = 4096;

__global__ __launch_bounds__(256) void adamw_kernel(const AdamTensor* __restrict__ ts, const AdamChunk* __restrict__ chunks,
                                                    float b1, float b2, float eps) {
  const AdamChunk ch = chunks[blockIdx.x];
  const AdamTensor t = ts[ch.tensor];
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const int64_t end = min(t.n, ch.start + ADAM_CHUNK);
  const float step_size = t.coef[0], bc2_sqrt = t.coef[1], decay = t.coef[2];
  for (int64_t i = ch.start + threadIdx.x; i < end; i += 256) {
    float p = __fmul_rn(t.p[i], decay);
    const float g = t.g[i];
    float m = t.m[i];
    m = __fadd_rn(m, __fmul_rn(w1, __fsub_rn(g, m)));  // torch lerp, weight < 0.5 branch
    float v = __fadd_rn(__fmul_rn(t.v[i], b2), __fmul_rn(__fmul_rn(w2, g), g));
    const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2_sqrt), eps);
    p = __fsub_rn(p, __fmul_rn(step_size, __fdiv_rn(m, denom)));
    t.p[i] = p; t.m[i] = m; t.v[i] = v;
    if (t.shadow) t.shadow[i] = (bf16)p;
  }
}

extern "C" {

// W [out, in] (f32) from DoRA parameters; DnT_ws >= out*in floats (kept for the
// backward), colsq_ws >= ceil(in/64)*out floats, nu [out] saved for backward.
int vit_dora_weight_fwd(int in, int out, int r, const float* m, const float* A, const float* Bm, const float* D,
                        float scaling, const float* noise, float* W, float* nu, float* DnT_ws, float* colsq_ws,
                        void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (r > 64 || in <= 0 || out <= 0) return (int)hipErrorInvalidValue;
  int ty = (in + DT - 1) / DT;
  hipLaunchKernelGGL(dora_tile_kernel, dim3((out + DT - 1) / DT, ty), dim3(256), 0, s, in, out, r, A, Bm, D, scaling,
                     noise, DnT_ws, colsq_ws);
  VIT_CHECK_LAUNCH();
  hipLaunchKernelGGL(dora_finish_kernel, dim3((out + 3) / 4), dim3(256), 0, s, in, out, ty, colsq_ws, m, DnT_ws, W, nu);
  VIT_CHECK_LAUNCH();
  return 0;
}

// Backward of vit_dora_weight_fwd given gW = dL/dW [out, in]; DnT/nu from the forward.
// sdDnT_ws >= out*in floats.  Outputs dm [out], dA [r, out], dB [in, r] (f32, overwritten).
// ABI 7: slabs / slab_floats let the two factor GEMMs split their 1024-4096-long reductions
// (vit_gemm_splitk; slab contract in include/vit_hip.h: at most s slabs of M * N floats with
// s * M * N <= slab_floats); nullptr / 0 = the unsplit launches of vit_dora_weight_bwd.
int vit_dora_weight_bwd_ws(int in, int out, int r, const float* m, const float* A, const float* Bm, const float* gW,
                           const float* DnT, float scaling, const float* nu, float* dm, float* dA, float* dB,
                           float* sdDnT_ws, float* slabs, int64_t slab_floats, const float* noise, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(dora_bwd_row_kernel, dim3((out + 3) / 4), dim3(256), 0, s, in, out, gW, DnT, m, nu, scaling,
                     noise, dm, sdDnT_ws);
  VIT_CHECK_LAUNCH();
  // dB[i][k] = sum_o sdDnT[o][i] * A[k][o]:  P(i,o) = sdDnT[o*in + i] (CR), Q(k,o) = A[k*out + o] (RC)
  int rc = vit_gemm_splitk(1, 0, in, r, out, sdDnT_ws, in, A, out, dB, slabs, slab_floats, stream);
  if (rc) return rc;
  // dA[k][o] = sum_i B[i][k] * sdDnT[o][i]:  P(k,i) = B[i*r + k] (CR), Q(o,i) = sdDnT[o*in + i] (RC)
  return vit_gemm_splitk(1, 0, r, out, in, Bm, r, sdDnT_ws, in, dA, slabs, slab_floats, stream);
}

int vit_dora_weight_bwd(int in, int out, int r, const float* m, const float* A, const float* Bm, const float* gW,
                        const float* DnT, float scaling, const float* nu, float* dm, float* dA, float* dB,
                        float* sdDnT_ws, const float* noise, void* stream) {
  return vit_dora_weight_bwd_ws(in, out, r, m, A, Bm, gW, DnT, scaling, nu, dm, dA, dB, sdDnT_ws, nullptr, 0, noise,
                                stream);
}

// Fused AdamW over a table of AdamTensor {p, g, m, v, shadow, n, coef -> {step_size, bc2_sqrt, decay, 0}};
// chunks of 4096 elements {tensor, pad, start}.
int vit_adamw_step(const void* tensors, const void* chunks, int nchunks, float beta1, float beta2, float eps,
                   void* stream) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, (const AdamTensor*)tensors,
                     (const AdamChunk*)chunks, beta1, beta2, eps);
  VIT_CHECK_LAUNCH();
  return 0;
}
int vit_adamw_tensor_bytes(void) { return (int)sizeof(AdamTensor); }

}  // extern "C"
