/*
 * vit_hip.h -- C ABI of libvit_hip.so, the MI355X (gfx950) kernels behind the
 * ViT training step of seemadhungana/ViT-Project.
 *
 * The reference is pure Python: its hot path reaches GPU code only through
 * torch ops called from timm's VisionTransformer (external) and from its own
 * training loops.  Each entry point below replaces one of those ops; the
 * reference call site it serves is cited as FILE:LINE with
 *   VIT  = Training/vit_training/baseline/train_vit_sgd.py
 *   MEAS = Training/vit_training/single_epoch/measure_single_epoch_perturbation_effect.py
 *   NEWP = Training/functions/new_cvpr_train_behavior_things_pipeline.py
 *
 * Conventions: plain device pointers and sizes; `stream` is a hipStream_t;
 * every function returns 0 or a hipError_t code and never allocates, frees or
 * synchronises (graph-capture safe).  dtype codes: 0 = f32, 1 = bf16.
 * Row strides (ld*) are in elements.
 */
#ifndef VIT_HIP_H
#define VIT_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { VIT_DTYPE_F32 = 0, VIT_DTYPE_BF16 = 1 };
enum { VIT_LAYOUT_RC = 0, VIT_LAYOUT_CR = 1 };
enum {
  VIT_EPI_STORE = 0,      /* C = acc (+bias)                                   */
  VIT_EPI_BIAS_GELU = 1,  /* pre = acc+bias: C = gelu_erf'(pre), aux_out = gelu_erf(pre) */
  VIT_EPI_RESID = 2,      /* C (f32) = resid + acc + bias                      */
  VIT_EPI_GELU_BWD = 3,   /* C = acc * aux (aux = the gelu'(pre) BIAS_GELU saved) */
  VIT_EPI_PATCH = 4,      /* patch-embed row remap + pos_embed                 */
  VIT_EPI_BIAS_QGELU = 5, /* QuickGELU variant (OpenAI CLIP towers): C = qgelu'(pre) */
  VIT_EPI_QGELU_BWD = 6
};

int vit_abi_version(void); /* 10 (round 6): vit_blaslt_workspace / vit_gemm_lib removed -- the plain bf16
                              * forward / input-gradient GEMMs run the hand-written 4-wave kernel (csrc/
                              * gemm_g4.hip), the library links no vendor BLAS; 9: those two hooks (hipBLASLt);
                              * 8: vit_gemm_ms / vit_gemm_ms_config and the banded attention backward removed */

/* Generic MFMA GEMM C[i][j] = epi(sum_r P(i,r) Q(j,r)); layouts RC (r contiguous)
 * or CR (i/j contiguous).  Backs every nn.Linear of timm's ViT reached from
 * VIT:139 (forward) and VIT:142 (backward). */
int vit_gemm(int dtype, int out_dtype, int p_layout, int q_layout, int epi, int M, int N, int R,
             const void* P, int64_t ldp, const void* Q, int64_t ldq, void* C, int64_t ldc,
             const float* bias, const void* aux, int64_t ld_aux, void* aux_out, int allow_fast, void* stream);

/* Tuning hook: force GEMM tile configuration v (see csrc/gemm.hip big::V*; 20 = the 4-wave g4 kernel of
 * csrc/gemm_g4.hip for the plain bf16 store classes), -1 = per-shape choice (g4 for the plain bf16
 * forward / input gradient unless VIT_GEMM_G4=0). */
int vit_gemm_variant(int v);

/* Tuning hook: the forward / input-gradient GEMMs walk their tiles in bands of `fwd` / `dgrad`
 * row tiles, column-major inside a band (L2 reuse of the operand blocks); 0 = row-major (the forward
 * default), -1 = the per-shape rule (bands of 8 for wide outputs with >= 4 MiB weights).  The input
 * gradients default to bands of 4 (round 5: the fc2 GELU' one, 3.9x less operand FETCH, +0.65 %);
 * -2 restores a class's default (VIT_GEMM_GROUP_FWD / _DGRAD, else the defaults above). */
int vit_gemm_group(int fwd, int dgrad);

/* The plain bf16 forward (+ f32 bias) and input-gradient GEMMs run the 4-wave g4 kernel (csrc/gemm_g4.hip,
 * VIT:139 / VIT:142 through timm's qkv / proj / fc1 / fc2).  Tuning / test hook: its tile walk for the forward
 * and the input-gradient class (0 = stride over the tiles with min(tiles, CUs or `wgs`) persistent workgroups,
 * 1 = one workgroup per 256-row band walking the column tiles, 2 = stride over the tiles with one workgroup per
 * 256-row band, so the workgroups running together share a band's rows in L2 (the input gradients' default,
 * round 6: +1.1 / +1.3 % over 1), -1 = keep), the stride walk's workgroup cap
 * (0 = the CU count, -1 = keep) and its tiles per workgroup (grid >= ceil(tiles / tpw); 0 = no limit, -1 = keep). */
int vit_gemm_g4_config(int fwd_mode, int dgrad_mode, int wgs, int tpw);

/* Host-side count of g4 launches since the last reset (reset != 0 zeroes it); no GPU call. */
int vit_gemm_g4_count(int reset);

/* Tuning / test hook: the fc2 GELU' input gradient (vit_linear_dgrad with EPI_GELU_BWD / EPI_QGELU_BWD, bf16)
 * on g4 (1: the act' tile arrives by LDS-DMA in the two stage slots past the stream's end, products in place,
 * column partials for the fc1 bias gradient) or on the 8-wave V1 kernel (0); -1 keeps.  Returns the previous
 * setting (default VIT_G4_GELU, else 0). */
int vit_gemm_g4_gelu(int on);

/* Stream-K workspace for the fp32 MFMA GEMMs launched on `stream` (the reference-precision C3 path,
 * NEWP:274): part >= 4 * CUs * 128*128 floats, counters >= 2 * CUs ints, zero-filled before first use
 * (kernels leave them zero).  With it, an f32 GEMM whose tile count would leave a ragged last round
 * (C3's 128.5 row tiles) runs as 2 * CUs persistent workgroups sharing the k-steps equally; cut
 * tiles combine in-launch in a fixed order.  part == NULL removes the stream's entry (host-only); past
 * 32 registered streams a new stream keeps the plain launch. */
int vit_gemm_streamk_workspace(void* stream, float* part, int64_t part_bytes, int* counters, int ncounters);

/* Host-only query (no GPU call): rows per launch the bf16 MFMA path uses for a row-contiguous
 * operand of M rows x ld elements (its staging offsets are 32-bit: larger operands are split
 * into row chunks, a multiple of 256 rows each); M when one launch fits, 0 if none does. */
int vit_gemm_rc_chunk_rows(int M, int64_t ld);

/* F.linear forward, Y = X W^T + b with fused epilogue (timm Attention.qkv/proj,
 * Mlp.fc1+GELU / fc2 + residual, head; under VIT:138-139 autocast). */
int vit_linear_fwd(int dtype, int out_dtype, int epi, int M, int N, int K, const void* X, int64_t ldx,
                   const void* W, const float* bias, void* Y, int64_t ldy, const void* resid,
                   void* act_out, void* stream);

/* F.linear input gradient dX = dY W (+ GELU' epilogue) -- autograd of VIT:142.  dbias (optional) =
 * column sums of dX as stored (bias gradient of the Linear that produced dX's forward value, e.g.
 * fc1.bias from fc2's dgrad), fused into the epilogue; partial >= vit_linear_dgrad_partial_floats. */
int vit_linear_dgrad(int dtype, int out_dtype, int epi, int M, int N, int K, const void* dY, int64_t lddy,
                     const void* W, void* dX, int64_t lddx, const void* pre, float* dbias, float* partial,
                     int64_t partial_floats, int defer_reduce, void* stream);
/* defer_reduce = 1: dbias is not written; `partial` keeps its [ceil(M/64)][K] column-sum
 * partials for the caller to reduce with vit_colreduce (e.g. on another stream, off the
 * input-gradient chain). */
int vit_linear_dgrad_partial_floats(int M, int K);

/* F.linear weight gradient dW (f32) = dY^T X, split-K over rows with fp32 slabs
 * in `workspace` (>= split*N*K*4 bytes) -- autograd of VIT:142. */
int vit_linear_wgrad(int dtype, int M, int N, int K, const void* dY, int64_t lddy, const void* X,
                     int64_t ldx, float* dW, int split, void* workspace, int64_t ws_bytes, void* stream);
/* The same weight gradient as split-K partials only: slabs[z][N*K] f32 for
 * z < vit_linear_wgrad_nslabs(...), dW = sum_z slabs[z] (ragged M % 32 rows folded into the last
 * slab); the caller reduces them -- the block backward's single vit_colreduce_batch launch
 * (S = nslabs, N = N*K).  bf16, or f32 on the MFMA path. */
int vit_linear_wgrad_nslabs(int dtype, int M, int N, int K, int split);
int vit_linear_wgrad_partials(int dtype, int M, int N, int K, const void* dY, int64_t lddy, const void* X,
                              int64_t ldx, int split, float* slabs, int64_t slab_bytes, void* stream);
/* Two weight gradients of one block over the same M token rows (fc2 + fc1, or proj + qkv, from
 * the autograd of VIT:142) as ONE launch of split-K partials: slabs_a / slabs_b as
 * vit_linear_wgrad_partials for (Na, Ka) / (Nb, Kb) with the same split.  bf16, M % 32 == 0;
 * otherwise hipErrorInvalidValue and nothing is launched. */
int vit_linear_wgrad_partials2(int M, int split, int Na, int Ka, const void* dYa, int64_t lddya, const void* Xa,
                               int64_t ldxa, float* slabs_a, int64_t bytes_a, int Nb, int Kb, const void* dYb,
                               int64_t lddyb, const void* Xb, int64_t ldxb, float* slabs_b, int64_t bytes_b,
                               void* stream);

/* Column sums (bias gradients): out[N] = sum_i X[i][:] -- autograd of VIT:142. */
int vit_colsum(int dtype, int M, int N, const void* X, int64_t ld, float* out, float* partial,
               int64_t partial_floats, int accumulate, void* stream);
/* out[N] (+)= sum_z part[z][:] over S partial rows (second stage of fused bias gradients);
 * scratch optional (>= ceil(S/64)*N floats, faster for S > 64). */
int vit_colreduce(const float* part, int S, int N, float* out, int accumulate, float* scratch, void* stream);
/* nq (1..3) stacked [S][N] partial matrices (part + q*S*N) reduced into out0..out2 with one
 * launch per stage (the LayerNorm backward's dgamma | dbeta | dsum partials); scratch optional
 * (>= nq*ceil(S/64)*N floats). */
int vit_colreduce_multi(const float* part, int nq, int S, int N, float* out0, float* out1, float* out2,
                        int accumulate, float* scratch, void* stream);

/* Every deferred column reduction of one transformer block's backward (the bias gradients of
 * qkv / proj / fc1 / fc2 and the norm1 / norm2 affine gradients, autograd of VIT:142) in ONE
 * launch: jobs = njobs x {part, out, S, N, accumulate} as int64 in host memory, each
 * out[N] (+)= sum of the S rows of part [S][N].  Sums run in a fixed order (bitwise reproducible);
 * jobs with more than 64 partial rows combine 64-row chunk partials in-launch (agent-scope
 * release/acquire + a ticket counter per 256-column strip).  scratch / counters sized by
 * vit_colreduce_batch_sizes; counters zero-filled before first use (the kernel leaves them zero). */
int vit_colreduce_batch_sizes(const int64_t* jobs, int njobs, int64_t* scratch_floats, int* counters);
int vit_colreduce_batch(const int64_t* jobs, int njobs, float* scratch, int64_t scratch_floats, int* counters,
                        int ncounters, void* stream);

/* timm PatchEmbed Conv2d(3,768,16,16) as GEMM over unfolded patches, writing
 * rows b*(np+1)+1+p of the f32 token stream with pos_embed added (VIT:139). */
int vit_patch_embed_fwd(int dtype, int B, int np, int D, int K, const void* U, const void* W,
                        const float* bias, const float* pos, float* x, void* stream);
/* Conv2d 16/16 unfold: img f32 [B,C,H,W] -> U [B*np, C*ps*ps] (column = c*ps*ps+ky*ps+kx). */
int vit_patch_unfold(int dtype, int B, int C, int Hi, int Wi, int ps, const float* img, void* U, void* stream);
/* ABI 7: the same with U rows ldu >= C*ps*ps elements apart, columns [C*ps*ps, ldu) zero-filled, and the
 * patch embedding over such rows (K = the padded reduction length, W [D][ldw] zero past the real
 * columns): CLIP ViT-L/14's 3*14*14 = 588 columns padded to 608 run on the MFMA GEMM instead of the
 * scalar-FMA kernel (NEWP:274's visual conv1).  vit_copy_rows_padded builds such a W: dst[r][c] =
 * src[r][c] for c < cols, 0 up to ld_dst. */
int vit_patch_unfold_ld(int dtype, int B, int C, int Hi, int Wi, int ps, int ldu, const float* img, void* U,
                        void* stream);
int vit_patch_embed_fwd_ld(int dtype, int B, int np, int D, int K, const void* U, int64_t ldu, const void* W,
                           int64_t ldw, const float* bias, const float* pos, float* x, void* stream);
int vit_copy_rows_padded(int dtype, int rows, int cols, const void* src, int64_t ld_src, void* dst, int64_t ld_dst,
                         void* stream);
/* cat(cls_token) + pos_embed[0] into row 0 of every image (timm _pos_embed). */
int vit_cls_pos_fill(int B, int S, int D, float* x, const float* cls, const float* pos, void* stream);
/* d pos_embed [S,D] = sum_b dx[b]; d cls_token = d pos_embed[0]. */
int vit_pos_grad(int B, int S, int D, const float* dx, float* dpos, float* dcls, void* stream);

/* Tuning hook: LayerNorm backward form for D % 256 == 0 -- 1 = software-pipelined (next row's loads
 * issued before this row's stores; default), 0 = the plain row loop.  Equal to rounding. */
int vit_layer_norm_bwd_variant(int v);

/* F.layer_norm forward (timm norm1/norm2/norm, eps 1e-6), one wave per row; saves mean/rstd. */
int vit_layer_norm_fwd(int dtype_x, int dtype_y, int rows, int D, const void* x, int64_t ldx, void* y,
                       int64_t ldy, const float* w, const float* b, float* mean, float* rstd, float eps,
                       void* stream);
/* xs = x + r (f32 residual stream + a Linear's output (dtype_r bf16 or f32), bias included; xs may alias
 * x) and, when y is non-null, y = LayerNorm(xs) (dtype_y) with mean/rstd: timm Block's `x = x + attn(norm1(x))` /
 * `x = x + mlp(norm2(x))` residual adds (VIT Block.forward via timm) fused into the LayerNorm that
 * follows them (norm2 of the same block, norm1 of the next); y == null: the add alone (last block).
 * D % 256 == 0, strides % 4 == 0. */
int vit_add_layer_norm_fwd(int dtype_r, int dtype_y, int rows, int D, const float* x, int64_t ldx, const void* r,
                           int64_t ldr, float* xs, int64_t ldxs, void* y, int64_t ldy, const float* w, const float* b,
                           float* mean, float* rstd, float eps, void* stream);
/* LayerNorm backward with fused residual-gradient add, optional GEMM-dtype copy
 * of dx (optionally dropping CLS rows), dgamma/dbeta, and dsum = column sums of dx
 * (bias gradient of the Linear whose output fed the residual: proj / fc2). */
int vit_layer_norm_bwd(int dtype_x, int dtype_dy, int rows, int D, const void* x, int64_t ldx,
                       const void* dy, int64_t lddy, const float* w, const float* mean, const float* rstd,
                       const float* dres, int64_t ldres, float* dx, int64_t lddx, void* dx_copy, int64_t ld_copy,
                       int dtype_copy, int compact_np, float* dgamma, float* dbeta, float* dsum, float* partial,
                       int64_t partial_floats, int defer_reduce, void* stream);
/* defer_reduce = 1: dgamma / dbeta / dsum are not written; `partial` keeps their
 * [ceil(rows/64)][D] partials at float offsets 0, nblk*D, 2*nblk*D (followed by the
 * vit_colreduce scratch) for the caller to reduce with vit_colreduce. */
int vit_layer_norm_bwd_partial_floats(int rows, int D);
int vit_layer_norm_bwd_blocks(int rows); /* partial rows: the [nblk][D] partial blocks' nblk */

/* F.scaled_dot_product_attention(q,k,v) (timm Attention, head_dim 64, N <= 288) reading q/k/v in
 * place from the qkv GEMM output; lse [B*H*N] f32.  causal = 1 masks key > query: the CLIP text
 * tower's nn.MultiheadAttention attn_mask (NEWP:298 through the CLIP-HBA fork, external). */
int vit_sdpa_fwd(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, void* o,
                 int64_t ld_o, float* lse, float scale, int causal, void* stream);
/* fp8 scaled-dot-product attention forward (BASELINE configs[4]: the sweep's frozen CLIP tower blocks
 * and the RSA evaluation forward; replaces the same F.scaled_dot_product_attention call as
 * vit_sdpa_fwd): q/k/v quantised in-kernel to block-scaled OCP e4m3 (E8M0 scale per 32 values),
 * S = QK^T and O = PV on v_mfma_scale_f32_32x32x64_f8f6f4, softmax in f32.  dtype = qkv/o dtype
 * (VIT_BF16 or VIT_F32); head_dim 64, N <= 320; lse may be null.  Forward only. */
int vit_sdpa_fwd_fp8(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, void* o,
                     int64_t ld_o, float* lse, float scale, int causal, void* stream);
/* SDPA backward into dqkv (qkv layout). delta_ws >= B*H*N floats.  dbias (optional, [3*H*64]) =
 * column sums of dqkv (the qkv Linear's bias gradient), fused into the kernels;
 * partial >= vit_sdpa_bwd_partial_floats(B, N, H*64).  dbias == NULL with partial != NULL (bf16
 * only): the kernels leave the per-image [B][3*H*64] partial sums in `partial` for the caller to
 * reduce (vit_colreduce_batch). */
int vit_sdpa_bwd(int dtype, int B, int H, int N, int head_dim, const void* qkv, int64_t ld_qkv, const void* o,
                 int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, void* dqkv, int64_t ld_dqkv,
                 float* delta_ws, float scale, int causal, float* dbias, float* partial, int64_t partial_floats,
                 void* stream);
int vit_sdpa_bwd_partial_floats(int B, int N, int D);
/* Tuning hook: the bf16 backward form for N <= 224 (-1 = from VIT_ATTN_BWD_SPLIT, 1 = whole-head fused
 * (the default), 2 = two kernels; 0, round 4's banded form, was removed in ABI 8: hipErrorInvalidValue).
 * The two forms agree to bf16 rounding (some f32 sums are ordered differently). */
int vit_sdpa_bwd_variant(int v);

/* torch.nn.functional.cross_entropy(outputs, targets) mean (VIT:140) and its gradient. */
int vit_cross_entropy_fwd(int B, int C, const float* logits, int64_t ld, const int64_t* target, float* row_lse,
                          float* row_loss, float* loss, void* stream);
int vit_cross_entropy_bwd(int dtype_out, int B, int C, const float* logits, int64_t ld, const int64_t* target,
                          const float* row_lse, const float* grad_loss, void* dlogits, int64_t ldd, void* stream);

/* torch.optim.SGD(lr, momentum, weight_decay).step() over all parameters in one
 * launch (VIT:143-144, VIT:294-299).  tensors: {float* p; const float* g; float* buf;
 * bf16* shadow; int64 n}[], chunks: {int tensor; int pad; int64 start}[] (4096 elems). */
int vit_sgd_step(const void* tensors, const void* chunks, int nchunks, const float* lr, float momentum,
                 float weight_decay, void* stream);
int vit_sgd_chunk_size(void);
int vit_sgd_tensor_bytes(void);
int vit_sgd_chunk_bytes(void);

/* DoRALayer.weight (NEWP:447-463): W[out,in] = (m * (D + (B@A)s) / (||.||_col + 1e-8))^T,
 * and its backward (dm, dA, dB) for AdamW (NEWP:1000-1001).  noise (nullable, [in,out] like D):
 * DoRALayer.forward's train-mode dropout of delta_D (NEWP:465-481), (B@A)s * noise with
 * noise = keep-mask / (1 - p); the backward masks the delta_D gradient the same way. */
int vit_dora_weight_fwd(int in, int out, int r, const float* m, const float* A, const float* B, const float* D,
                        float scaling, const float* noise, float* W, float* nu, float* DnT_ws, float* colsq_ws,
                        void* stream);
int vit_dora_weight_bwd(int in, int out, int r, const float* m, const float* A, const float* B, const float* gW,
                        const float* DnT, float scaling, const float* nu, float* dm, float* dA, float* dB,
                        float* sdDnT_ws, const float* noise, void* stream);
/* ABI 7: the same with a split-K slab workspace (nullptr / 0 = unsplit), and the split-K GEMM it uses:
 * C [M][N] contiguous f32 = sum_r P(i,r) Q(j,r) in r-chunks of >= 128 summed in chunk order
 * (deterministic).  Slab contract (both functions): the split s is the largest with s <= 256 / tiles,
 * s <= R / 128 and s * M * N <= slab_floats, and the kernel writes at most s slabs of M * N floats
 * (chunks of ceil(R / s) rows); s < 2 runs unsplit.  DoRA's factor GEMMs are [in x r] and [r x out],
 * so 2 * max(in, out) * r floats allow a split of 2 and 2 * 256 * 1024 (the Python callers) their
 * full split at C3's in = out = 1024, r = 32. */
int vit_dora_weight_bwd_ws(int in, int out, int r, const float* m, const float* A, const float* B, const float* gW,
                           const float* DnT, float scaling, const float* nu, float* dm, float* dA, float* dB,
                           float* sdDnT_ws, float* slabs, int64_t slab_floats, const float* noise, void* stream);
int vit_gemm_splitk(int p_layout, int q_layout, int M, int N, int R, const float* P, int64_t ldp, const float* Q,
                    int64_t ldq, float* C, float* slabs, int64_t slab_floats, void* stream);
/* torch.optim.AdamW step (NEWP:1181, NEWP:1001): tensors {float* p; const float* g; float* exp_avg;
 * float* exp_avg_sq; bf16* shadow (or null); int64 n; const float* coef}[] where coef points at
 * the tensor's {step_size, bc2_sqrt, decay, 0} in device memory: step_size = lr / (1 - beta1^step),
 * bc2_sqrt = sqrt(1 - beta2^step) for that tensor's own state['step'] (so a load_state_dict
 * resume, NEWP:1189-1195, continues the bias correction) and decay = 1 - lr * weight_decay of the
 * tensor's group.  The table is fixed across steps (only the coefficients change), so a captured
 * graph can replay it under a changing lr; chunks as vit_sgd_step.  (ABI 6: decay moved from a
 * scalar argument into coef.) */
int vit_adamw_step(const void* tensors, const void* chunks, int nchunks, float beta1, float beta2, float eps,
                   void* stream);
int vit_adamw_tensor_bytes(void);

/* CLIP-HBA forward/loss around the towers (NEWP:287-304 -> clip_model(image, prompts, pos_embedding),
 * the CLIP-HBA fork, external; OpenAI-CLIP semantics assumed):
 *   token_embed   x[s*L+t] = table[tokens[s*L+t]] + pos[t]         (token_embedding + positional_embedding)
 *   gather_rows   dst[i] = src[idx[i]]  (text EOT pooling x[arange, text.argmax(-1)], CLS rows)
 *   scatter_rows  dst[idx[i]] = src[i]  (their backward; dst zeroed by the caller)
 *   rownorm       y = exp(*log_scale) x / ||x|| (feature normalisation; log_scale null = 1), and backward
 *   mse           nn.MSELoss() mean (NEWP:994, CBASE criterion) and its gradient (grad_loss null = 1) */
int vit_token_embed(int rows, int L, int D, int vocab, const int64_t* tokens, const float* table, const float* pos,
                    float* x, void* stream);
int vit_gather_rows(int n, int D, const float* src, int64_t ld_src, const int64_t* idx, float* dst, int64_t ld_dst,
                    void* stream);
int vit_scatter_rows(int n, int D, const float* src, int64_t ld_src, const int64_t* idx, float* dst, int64_t ld_dst,
                     void* stream);
int vit_rownorm_fwd(int n, int D, const float* x, const float* log_scale, float* y, float* rnorm, void* stream);
int vit_rownorm_bwd(int n, int D, const float* x, const float* dy, const float* rnorm, const float* log_scale,
                    float* dx, void* stream);
int vit_mse_fwd(int n, const float* pred, const float* target, float* loss, void* stream);
int vit_mse_bwd(int n, const float* pred, const float* target, const float* grad_loss, float* dpred, void* stream);

/* ImageNet input transforms on the GPU (VIT:32-46, MEAS:152-158): RandomResizedCrop /
 * Resize+CenterCrop with Pillow's 8-bit bilinear resampling (bit-exact), horizontal flip, ToTensor and
 * Normalize, over a ragged batch of decoded RGB uint8 images in device memory.  params = device int64
 * [B][12] (see image.hip); coeff_ws >= vit_image_coeff_bytes(B, S, kmax) bytes; out f32 [B][3][S][S]. */
int vit_image_coeff_bytes(int B, int S, int kmax);
int vit_image_transform(int B, int S, const uint8_t* src, const int64_t* params, int kmax, int max_rows,
                        int* coeff_ws, uint8_t* tmp_ws, float* out, const float* norm6, void* stream);

/* helpers */
int vit_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
int vit_zero(void* p, int64_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VIT_HIP_H */
