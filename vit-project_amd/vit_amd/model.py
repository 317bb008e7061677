"""ViT-B/16 behind timm's ``VisionTransformer`` surface, computed by HIP kernels.

Drop-in for ``timm.create_model('vit_base_patch16_224', pretrained=False,
num_classes=1000)`` as the reference uses it (VIT:283-287, MEAS:467-485):
``model(images)`` -> logits, ``model.forward_features(images)`` -> post-norm
tokens, ``model.global_pool == 'token'``, timm state_dict key names, ``.train()``
/ ``.eval()``, ``parameters()`` for the optimizer, DDP-compatible autograd.

Master parameters are fp32 ``nn.Parameter``s (what the optimizer and checkpoints
see).  In ``compute_dtype=torch.bfloat16`` (the performance path) every GEMM
weight has a bf16 shadow copy that :class:`vit_amd.optim.FusedSGD` refreshes in
the same pass as the update; any other writer (torch optimizers,
``load_state_dict``) bumps ``param._version`` and the shadow is recast before
the next forward.  ``compute_dtype=torch.float32`` is the parity path (generic
fp32 kernels, 1e-3 relative vs the CPU oracle).

Each transformer block is one autograd node (:class:`_BlockFn`), so the
backward chains HIP kernels without any torch elementwise glue: residual
gradients are fused into the LayerNorm backward, GELU' into the fc2 dgrad
epilogue, bias grads into column-sum kernels.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import torch
import torch.nn as nn

from . import _lib as L
from . import ops

# gradient side channel: a block's backward leaves the GEMM-dtype copy of the
# residual gradient it produced, keyed by the f32 tensor's storage pointer, for
# the next (earlier) block's backward to pick up instead of re-casting.
_GRAD_COPY = {}


def _take_copy(g: torch.Tensor, dtype, want_dsum: bool = False):
    """The GEMM-dtype copy of an incoming gradient (written by the producer's LayerNorm
    backward) and, with want_dsum, its column sums (None if the producer did not make them)."""
    key = (g.data_ptr(), g.numel())
    c = _GRAD_COPY.pop(key, None)
    fresh = c is not None and c[1] == g._version
    dsum = c[2] if fresh else None
    if fresh and c[0] is not None and c[0].dtype == dtype:
        out = c[0]
    elif dtype == torch.float32:
        out = g
    else:
        out = torch.empty(g.shape, dtype=dtype, device=g.device)
        ops.cast_bf16(g.contiguous(), out)
    return (out, dsum) if want_dsum else out


def _put_copy(g: torch.Tensor, copy, dsum=None):
    _GRAD_COPY[(g.data_ptr(), g.numel())] = (copy, g._version, dsum)


# Weight-gradient work of a block's backward runs on a second stream so its
# MFMA-bound main loops overlap the input-gradient chain's HBM-bound epilogues
# (GELU', residual and LayerNorm passes).  Fork = side waits on main; the block
# joins (main waits on side) before returning its gradients.  Capturable.
_SIDE = {}
_OVERLAP = [True]
# forward half-batch chains: join the two streams after every block ("block") or once after
# the block stack ("end", default)
_FWD_JOIN = [os.environ.get("VIT_FWD_JOIN", "end")]
# block backward: join the side stream (weight/bias gradients) at the end of every block
# ("block") or once, in the patch embedding's backward ("end": flat-gradient runs only)
_BWD_JOIN = [os.environ.get("VIT_BWD_JOIN", "end")]
# side-stream operands referenced until the next join (VIT_HOLD_REFS=0 only to demonstrate the race)
_HOLD_REFS = [os.environ.get("VIT_HOLD_REFS", "1") != "0"]
# images the caller's forward chain takes beyond B/2: at an even split the side chain ends
# ~0.3 ms later (bs=256).  Default B/32 (8 at bs=256): +0.8 %; 16+ falls off a GEMM tile-count
# cliff (-3 %).  profiles/r01/ab_fwd_half_split.json
_FWD_HALF_DELTA = [None if os.environ.get("VIT_FWD_HALF_DELTA") is None else int(os.environ["VIT_FWD_HALF_DELTA"])]
_HOLD = {}


# bf16: the proj / fc2 outputs are added into the f32 residual stream by the following LayerNorm
# (+2.0 % over the EPI_RESID epilogue, round 2); fp32 keeps the epilogue add unless VIT_FUSED_RESID_F32=1
# (bit-identical: the same f32 add, in the LayerNorm; C3 fp32 measured 607 vs 609 img/s)
_FUSED_RESID_F32 = [os.environ.get("VIT_FUSED_RESID_F32", "0") == "1"]


def set_wgrad_overlap(enable: bool):
    """Run weight/bias gradients on a side stream (default) or inline on the caller's stream."""
    _OVERLAP[0] = bool(enable)


# (round 5 removed the A/B switches whose other settings all measured slower or equal: VIT_FWD_STAGGER,
# VIT_WGRAD_PAIRS, VIT_SIDE_CUS -- records in profiles/r04/ab_fwd_stagger_recheck.txt,
# ab_wgrad_pairing_recheck.txt and DESIGN.md §4.6)


def fwd_split(B: int) -> int:
    """Images [0, hb) of a bf16 forward run on the caller's stream, [hb, B) on the side stream: the
    caller's chain takes 3B/64 extra images (12 at bs=256: +0.35 % over B/32 in five same-box
    pairs with the fused residual LayerNorms; 16 is a GEMM tile-count cliff)."""
    delta = 3 * B // 64 if _FWD_HALF_DELTA[0] is None else _FWD_HALF_DELTA[0]
    return min(B - 1, max(1, B // 2 + delta))


class _Side:
    def __init__(self, dev):
        self.main = torch.cuda.current_stream(dev)
        self.on = _OVERLAP[0] and dev.type == "cuda"
        if self.on:
            if dev not in _SIDE:
                _SIDE[dev] = torch.cuda.Stream(device=dev)
            self.side = _SIDE[dev]

    def run(self, fn):
        if not self.on:
            return fn()
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            return fn()

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)
            # everything the side stream was given is ordered before the caller's later work now
            _HOLD.pop(self.side, None)

    def guard(self, *ts):
        """The side stream uses these tensors, possibly after their owner drops them (deferred
        joins leave its work queued across blocks): keep them referenced until the next join,
        so the caching allocator cannot hand their memory to the caller's stream while that
        work is pending.  (Not record_stream: its deferred-free events kept the pool from
        reaching a steady state -- 15x slower steps.)"""
        if self.on and _HOLD_REFS[0]:
            _HOLD.setdefault(self.side, []).extend(t for t in ts if t is not None)


class _Shadowed:
    """Registry of bf16 shadows for GEMM weights."""

    def __init__(self):
        self.pairs = []  # (param, shadow)

    def add(self, p: nn.Parameter, dtype):
        if dtype == torch.float32:
            p._vit_shadow = None
            return
        sh = torch.empty(p.shape, dtype=dtype, device=p.device)
        p._vit_shadow = sh
        p._vit_shadow_version = -1
        self.pairs.append(p)

    def refresh(self):
        for p in self.pairs:
            if p._vit_shadow.device != p.device or p._vit_shadow.shape != p.shape:
                p._vit_shadow = torch.empty(p.shape, dtype=p._vit_shadow.dtype, device=p.device)
                p._vit_shadow_version = -1
            if p._vit_shadow_version != p._version:
                ops.cast_bf16(p.detach(), p._vit_shadow)
                p._vit_shadow_version = p._version


def cfg_defer_bwd(ctx) -> bool:
    return getattr(ctx, "defer_bwd", False)


_JOIN_QUEUED = set()  # (graph task id, device) pairs whose end-of-backward join is queued


def _queue_backward_join(dev):
    """Deferred-join backward: make sure the side stream is joined when this backward pass
    ends, even if the patch embedding's backward (the normal join point) never runs --
    ``backward(inputs=...)`` / ``autograd.grad`` that stop above it.  The dedup key is the
    current autograd graph task, so a backward that raised (its final callbacks never run) does
    not suppress the join of the next one."""
    key = (torch._C._current_graph_task_id(), dev)
    if key in _JOIN_QUEUED:
        return
    _JOIN_QUEUED.clear()  # entries of earlier graph tasks are finished (or abandoned)
    _JOIN_QUEUED.add(key)

    def _join():
        _JOIN_QUEUED.discard(key)
        _Side(dev).join()

    torch.autograd.Variable._execution_engine.queue_callback(_join)


def _gout(p: nn.Parameter) -> torch.Tensor:
    """Where a parameter's gradient is written: its slice of the model's flat
    gradient buffer (fixed addresses: one all-reduce, a static optimizer table,
    graph-capture friendly) unless a previous gradient still lives there (then a
    fresh tensor, so autograd's accumulation stays correct)."""
    fb = getattr(p, "_vit_flat_grad", None)
    if fb is not None and (p.grad is None or p.grad.data_ptr() != fb.data_ptr()):
        return fb.view(fb.shape)  # a fresh alias AccumulateGrad can steal (no copy)
    return torch.empty(p.shape, dtype=torch.float32, device=p.device)


def _w(p: nn.Parameter):
    sh = getattr(p, "_vit_shadow", None)
    return p.detach() if sh is None else sh


def _wt(p: torch.Tensor, dtype) -> torch.Tensor:
    """The GEMM-dtype operand of a weight: its bf16 shadow if it has one (model parameters),
    else a cast of the tensor itself (computed weights such as DoRALayer.weight)."""
    sh = getattr(p, "_vit_shadow", None)
    if sh is not None:
        return sh
    w = p.detach()
    if w.dtype == dtype:
        return w.contiguous()
    out = torch.empty(w.shape, dtype=dtype, device=w.device)
    ops.cast_bf16(w.contiguous(), out)
    return out


# ----------------------------------------------------------------------------
# autograd nodes
# ----------------------------------------------------------------------------

class _PatchEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, w, b, cls, pos, cfg):
        ctx.params = (w, b, cls, pos)
        ps, T = cfg["patch"], cfg["dtype"]
        B = img.shape[0]
        U = ops.patch_unfold(img.contiguous(), ps, T)
        npatch = U.shape[0] // B
        D = w.shape[0]
        x = ops.patch_embed_fwd(U, _w(w).reshape(D, -1), b.detach(), pos.detach().reshape(-1, D),
                                cls.detach().reshape(-1), B, npatch)
        ctx.save_for_backward(U)
        ctx.meta = (B, npatch, D, tuple(w.shape), T)
        return x

    @staticmethod
    def backward(ctx, dx):
        _Side(dx.device).join()  # weight-gradient work the blocks left on the side stream
        (U,) = ctx.saved_tensors
        B, npatch, D, wshape, T = ctx.meta
        dx = dx.contiguous()
        S = npatch + 1
        key = (dx.data_ptr(), dx.numel())
        c = _GRAD_COPY.pop(key, None)
        if c is not None and c[1] == dx._version and c[0].dtype == T and c[0].shape[0] == B * npatch:
            dxc = c[0]
        else:  # compact copy of the patch rows
            rows = dx.reshape(B, S, D)[:, 1:, :].reshape(B * npatch, D)
            if T == torch.float32:
                dxc = rows.contiguous()
            else:
                dxc = torch.empty(B * npatch, D, dtype=T, device=dx.device)
                ops.cast_bf16(rows.contiguous(), dxc)
        pw, pb, pc, pp = ctx.params
        dw = _gout(pw)
        ops.linear_wgrad(dxc, U, out=dw.view(D, -1), tail=True)  # alone on the GPU after the join
        db = ops.colsum(dxc, out=_gout(pb))
        dpos, dcls = _gout(pp), _gout(pc)
        ops.pos_grad(dx, B, S, D, dpos, dcls)
        return None, dw, db, dcls, dpos, None


class _BlockFn(torch.autograd.Function):
    """timm Block: x += proj(sdpa(qkv(norm1(x)))); x += fc2(gelu(fc1(norm2(x)))).

    Also the OpenAI-CLIP ResidualAttentionBlock (same dataflow: nn.MultiheadAttention's
    in_proj = qkv with the same [3, H, 64] row order, out_proj = proj, c_fc/c_proj = fc1/fc2,
    QuickGELU, LN eps 1e-5, causal mask in the text tower).  The backward computes only what
    ``ctx.needs_input_grad`` asks for: a frozen CLIP block whose only trainable input is a
    DoRA ``out_proj.weight`` (NEWP:484-544) runs the MLP/LN2 backward and one wgrad."""

    @staticmethod
    def forward(ctx, x, n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w, fc1b, fc2w, fc2b, cfg):
        B, N, D = x.shape
        H, T, eps = cfg["heads"], cfg["dtype"], cfg["eps"]
        act_epi = L.EPI_BIAS_QGELU if cfg["quick_gelu"] else L.EPI_BIAS_GELU
        M = B * N
        dev = x.device
        x2 = x.reshape(M, D)
        F = fc1w.shape[0]
        f32 = torch.float32
        h1, h2 = torch.empty(M, D, dtype=T, device=dev), torch.empty(M, D, dtype=T, device=dev)
        m1, r1, m2, r2 = (torch.empty(M, dtype=f32, device=dev) for _ in range(4))
        qkv = torch.empty(M, 3 * D, dtype=T, device=dev)
        o = torch.empty(M, D, dtype=T, device=dev)
        lse = torch.empty(B * H * N, dtype=f32, device=dev)
        xm, xo = torch.empty(M, D, dtype=f32, device=dev), torch.empty(M, D, dtype=f32, device=dev)
        # fc1's epilogue writes act = GELU(pre) for fc2 and dact = GELU'(pre) for the backward
        # (the erf is evaluated once; the fc2 dgrad epilogue is then a multiply)
        dact, act = torch.empty(M, F, dtype=T, device=dev), torch.empty(M, F, dtype=T, device=dev)
        Wqkv, Wproj, W1, W2 = _wt(qkvw, T), _wt(projw, T), _wt(fc1w, T), _wt(fc2w, T)
        causal = bool(cfg.get("causal", False))
        attn_fp8 = bool(cfg.get("attn_fp8", False))  # forward-only blocks (frozen prefix, no-grad passes)

        # fused residual adds (bf16 ViT, VisionTransformer._tokens): proj / fc2 store their bf16 output
        # (bias included) and the add into the f32 stream runs inside the next LayerNorm -- norm2 here,
        # the next block's norm1 for fc2 (this block's output xo is then written by that kernel), or
        # an add-only launch after the last block.  rs["pending"]: the previous block's (xm, fc2 out).
        rs = cfg.get("resid")
        pend = rs.get("pending") if rs is not None else None
        pb = yb = None
        if rs is not None:
            pb, yb = torch.empty(M, D, dtype=T, device=dev), torch.empty(M, D, dtype=T, device=dev)

        def ln1(sl):
            if pend is not None:
                return lambda: ops.add_layer_norm_fwd(pend[0][sl], pend[1][sl], x2[sl], n1w.detach(), n1b.detach(), eps,
                                                      out=h1[sl], mean=m1[sl], rstd=r1[sl])
            return lambda: ops.layer_norm_fwd(x2[sl], n1w.detach(), n1b.detach(), eps, T, out=h1[sl], mean=m1[sl],
                                              rstd=r1[sl])

        def chain_fused(b0, b1):
            sl = slice(b0 * N, b1 * N)
            steps = [
                ln1(sl),
                lambda: ops.linear_fwd(h1[sl], Wqkv, qkvb.detach(), out=qkv[sl]),
                lambda: ops.sdpa_fwd(qkv[sl], b1 - b0, H, N, o=o[sl], lse=lse[b0 * H * N:b1 * H * N], causal=causal,
                                     fp8=attn_fp8),
                lambda: ops.linear_fwd(o[sl], Wproj, projb.detach(), out=pb[sl]),
                lambda: ops.add_layer_norm_fwd(x2[sl], pb[sl], xm[sl], n2w.detach(), n2b.detach(), eps, out=h2[sl],
                                               mean=m2[sl], rstd=r2[sl]),
                lambda: ops.linear_fwd(h2[sl], W1, fc1b.detach(), epi=act_epi, out=dact[sl], act_out=act[sl]),
                lambda: ops.linear_fwd(act[sl], W2, fc2b.detach(), out=yb[sl]),
            ]
            if cfg.get("resid_last"):
                steps.append(lambda: ops.add_layer_norm_fwd(xm[sl], yb[sl], xo[sl]))
            return steps

        def chain(b0, b1):
            """The block over images [b0, b1) (rows b0*N .. b1*N of every tensor) as its 7 launches."""
            if rs is not None:
                return chain_fused(b0, b1)
            r0, r1_ = b0 * N, b1 * N
            sl = slice(r0, r1_)
            return [
                lambda: ops.layer_norm_fwd(x2[sl], n1w.detach(), n1b.detach(), eps, T, out=h1[sl], mean=m1[sl],
                                           rstd=r1[sl]),
                lambda: ops.linear_fwd(h1[sl], Wqkv, qkvb.detach(), out=qkv[sl]),
                lambda: ops.sdpa_fwd(qkv[sl], b1 - b0, H, N, o=o[sl], lse=lse[b0 * H * N:b1 * H * N], causal=causal,
                                     fp8=attn_fp8),
                lambda: ops.linear_fwd(o[sl], Wproj, projb.detach(), epi=L.EPI_RESID, resid=x2[sl], out=xm[sl]),
                lambda: ops.layer_norm_fwd(xm[sl], n2w.detach(), n2b.detach(), eps, T, out=h2[sl], mean=m2[sl],
                                           rstd=r2[sl]),
                lambda: ops.linear_fwd(h2[sl], W1, fc1b.detach(), epi=act_epi, out=dact[sl], act_out=act[sl]),
                lambda: ops.linear_fwd(act[sl], W2, fc2b.detach(), epi=L.EPI_RESID, resid=xm[sl], out=xo[sl]),
            ]

        def run(steps):
            for f in steps:
                f()

        side = _Side(dev)
        if side.on and B >= 2 and T != torch.float32:
            # two half-batch chains on two streams: one chain's GEMM epilogues (HBM-bound)
            # overlap the other's MFMA main loops (side.run waits for everything the caller's stream
            # has queued, so the side chain starts with the caller's)
            hb = fwd_split(B)
            mine, other = chain(0, hb), chain(hb, B)
            side.run(lambda: run(other))
            side.guard(x2, h1, m1, r1, qkv, o, lse, xm, h2, m2, r2, dact, act, xo,
                       *(t for t in (pb, yb, *(pend or ())) if t is not None))
            run(mine)
            # each half only feeds the same half of the next block: a stack of blocks joins
            # once after its last block (cfg "defer_join", ViT._tokens) instead of per block
            if not cfg.get("defer_join"):
                side.join()
        else:
            run(chain(0, B))
        if rs is not None:
            rs["pending"] = None if cfg.get("resid_last") else (xm, yb)
        ctx.save_for_backward(x2, h1, m1, r1, qkv, o, lse, xm, h2, m2, r2, dact, act)
        ctx.params = (n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w, fc1b, fc2w, fc2b)
        ctx.wops = (Wqkv, Wproj, W1, W2)
        ctx.meta = (B, N, D, H, T, cfg.get("compact_np", 0), cfg["quick_gelu"], causal)
        ctx.defer_bwd = bool(cfg.get("defer_bwd_join"))
        ctx.attn_fp8 = attn_fp8
        ctx.grad_hook = cfg.get("grad_hook")
        ctx.flat_span = cfg.get("flat_span")
        return xo.reshape(B, N, D)

    @staticmethod
    def backward(ctx, dxo):
        x2, h1, m1, r1, qkv, o, lse, xm, h2, m2, r2, dact, act = ctx.saved_tensors
        n1w, n1b, qkvw, qkvb, projw, projb, n2w, n2b, fc1w, fc1b, fc2w, fc2b = ctx.params
        Wqkv, Wproj, W1, W2 = ctx.wops
        B, N, D, H, T, compact_np, qg, causal = ctx.meta
        ng = ctx.needs_input_grad
        M = B * N
        dev = dxo.device
        dxo = dxo.contiguous().reshape(M, D)
        dxo_c, dxo_sum = _take_copy(dxo, T, want_dsum=True)
        gelu_bwd = L.EPI_QGELU_BWD if qg else L.EPI_GELU_BWD
        side = _Side(dev)
        need_mlp_in = any(ng[0:11])     # anything upstream of fc2 (its input gradient path)
        need_attn = any(ng[0:5])        # anything upstream of proj
        need_h1 = any(ng[0:3])
        if need_attn and ctx.attn_fp8:
            raise RuntimeError("this block's attention ran in fp8 (forward only); its backward needs the bf16 "
                               "forward: enable fp8 attention only for frozen blocks / no-grad passes")
        # gradient buffers are taken on the main stream (allocator ownership), filled on the side stream
        g = [None] * 13
        dpre = dxm = dxm_c = do = dqkv = None
        for i, p in ((1, n1w), (2, n1b), (3, qkvw), (4, qkvb), (5, projw), (6, projb), (7, n2w), (8, n2b),
                     (9, fc1w), (10, fc1b), (11, fc2w), (12, fc2b)):
            if ng[i]:
                g[i] = _gout(p)
        # MLP.  Bias gradients are column sums fused into the kernels that produce each
        # gradient: fc2.bias from the upstream LayerNorm backward (side channel), fc1.bias
        # from the GELU' dgrad epilogue, proj.bias from LN2 backward, qkv.bias from SDPA backward.
        # every deferred column reduction of this block goes into ONE launch at its end (side stream)
        # every bias / LayerNorm-affine reduction and the weight gradients' split-K slab sums of this block
        # in one batched launch (vit_colreduce_batch) on the side stream
        rb = rbw = ops.ColBatch()
        if ng[12]:
            if dxo_sum is not None:  # the upstream LayerNorm backward's column sums (side stream)
                rb.add(dxo_sum.view(1, D), 1, D, g[12])
            else:
                ops.colsum(dxo_c, out=g[12])
        # weight gradients in pairs over the same token rows (fc2 + fc1, proj + qkv): one grouped
        # launch each, half the split-K slabs of two launches
        pair_mlp = rbw is not None and ng[11] and ng[9] and need_mlp_in
        if ng[11] and not pair_mlp:
            side.run(lambda: ops.linear_wgrad(dxo_c, act, out=g[11], reduce_on=rbw))
        dx = None
        if need_mlp_in:
            dpre = ops.linear_dgrad(dxo_c, W2, out_dtype=T, epi=gelu_bwd, pre=dact, dbias=g[10], reduce_on=rb)
            if pair_mlp:
                side.run(lambda: ops.linear_wgrad_pair((dxo_c, act, g[11]), (dpre, h2, g[9]), rbw))
            elif ng[9]:
                side.run(lambda: ops.linear_wgrad(dpre, h2, out=g[9], reduce_on=rbw))
        if any(ng[0:9]):
            dh2 = ops.linear_dgrad(dpre, W1, out_dtype=T)
            dxm = torch.empty(M, D, dtype=torch.float32, device=dev)
            dxm_c = dxm if T == torch.float32 else torch.empty(M, D, dtype=T, device=dev)
            ops.layer_norm_bwd(xm, D, dh2, n2w.detach(), m2, r2, dxm, D, M, dres=dxo, ldres=D,
                               dx_copy=None if T == torch.float32 else dxm_c, ld_copy=D, dgamma=g[7], dbeta=g[8],
                               dsum=g[6], reduce_on=rb)
            # attention
            # block 0 (the patch rows' block, last in the backward): its last weight gradients are the tail
            tail = bool(compact_np)
            pair_attn = rbw is not None and ng[5] and ng[3] and need_attn
            if ng[5] and not pair_attn:
                side.run(lambda: ops.linear_wgrad(dxm_c, o, out=g[5], tail=tail, reduce_on=rbw))
            if need_attn:
                do = ops.linear_dgrad(dxm_c, Wproj, out_dtype=T)
                dqkv = ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dbias=g[4], causal=causal,
                                    reduce_on=rb)
                if pair_attn:
                    side.run(lambda: ops.linear_wgrad_pair((dxm_c, o, g[5]), (dqkv, h1, g[3]), rbw, tail=tail))
                elif ng[3]:
                    side.run(lambda: ops.linear_wgrad(dqkv, h1, out=g[3], tail=tail, reduce_on=rbw))
            if need_h1:
                dh1 = ops.linear_dgrad(dqkv, Wqkv, out_dtype=T)
                dx = torch.empty(M, D, dtype=torch.float32, device=dev)
                if compact_np:
                    dx_c = torch.empty(B * compact_np, D, dtype=T, device=dev)
                else:
                    dx_c = None if T == torch.float32 or not ng[0] else torch.empty(M, D, dtype=T, device=dev)
                # column sums of dx = the upstream block's fc2.bias gradient (not needed below the first block)
                dsum = None if (compact_np or not ng[0]) else torch.empty(D, dtype=torch.float32, device=dev)
                ops.layer_norm_bwd(x2, D, dh1, n1w.detach(), m1, r1, dx, D, M, dres=dxm, ldres=D, dx_copy=dx_c,
                                   ld_copy=D, compact_np=compact_np, dgamma=g[1], dbeta=g[2], dsum=dsum,
                                   reduce_on=rb)
                if ng[0] and (dx_c is not None or dsum is not None):
                    _put_copy(dx, dx_c, dsum)
        side.run(rb.launch)
        side.guard(*rb.parts)
        side.guard(dxo, dxo_c, dxo_sum, x2, h1, m1, r1, qkv, o, lse, xm, h2, m2, r2, dact, act,
                   *(v for v in (dpre, dxm, dxm_c, do, dqkv, dx) if v is not None))
        if cfg_defer_bwd(ctx):
            _queue_backward_join(dev)
        # (not the gradients g: they alias the persistent flat buffer, and AccumulateGrad must be
        # able to steal them -- an extra reference makes it copy before the side stream wrote them)
        if ctx.grad_hook is not None and all(ng[1:13]):
            # every gradient of this block is enqueued (side stream, after the main stream's work)
            side.run(lambda: ctx.grad_hook(*ctx.flat_span))
        if not cfg_defer_bwd(ctx):
            side.join()
        return (dx.reshape(B, N, D) if (ng[0] and dx is not None) else None, *g[1:], None)


class _HeadFn(torch.autograd.Function):
    """final norm on the CLS rows only (global_pool='token') + classifier head, f32."""

    @staticmethod
    def forward(ctx, x, nw, nb, hw, hb, cfg):
        B, N, D = x.shape
        xc, mc, rc = ops.layer_norm_fwd(x, nw.detach(), nb.detach(), cfg["eps"], torch.float32, rows=B, ldx=N * D)
        logits = ops.linear_fwd(xc, hw.detach(), hb.detach(), out_dtype=torch.float32)
        ctx.save_for_backward(x, xc, mc, rc)
        ctx.params = (nw, nb, hw, hb)
        ctx.meta = (B, N, D, cfg["dtype"])
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        x, xc, mc, rc = ctx.saved_tensors
        nw, nb, hw, hb = ctx.params
        B, N, D, T = ctx.meta
        dlogits = dlogits.contiguous().to(torch.float32)
        dxc = ops.linear_dgrad(dlogits, hw.detach(), out_dtype=torch.float32)
        dhw = ops.linear_wgrad(dlogits, xc, out=_gout(hw))
        dhb = ops.colsum(dlogits, out=_gout(hb))
        dx = ops.zero_(torch.empty(B, N, D, dtype=torch.float32, device=x.device))
        dx_c = None
        if T != torch.float32:
            dx_c = ops.zero_(torch.empty(B * N, D, dtype=T, device=x.device))
        dnw, dnb = _gout(nw), _gout(nb)
        dsum = torch.empty(D, dtype=torch.float32, device=x.device)  # last block's fc2.bias gradient
        ops.layer_norm_bwd(x, N * D, dxc, nw.detach(), mc, rc, dx, N * D, B, dx_copy=dx_c, ld_copy=N * D,
                           dgamma=dnw, dbeta=dnb, dsum=dsum)
        _put_copy(dx, dx_c, dsum)
        return dx, dnw, dnb, dhw, dhb, None


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        logits = logits.contiguous().to(torch.float32)
        loss, row_lse = ops.cross_entropy_fwd(logits, target.contiguous())
        ctx.save_for_backward(logits, target, row_lse)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, row_lse = ctx.saved_tensors
        return ops.cross_entropy_bwd(logits, target, row_lse, g), None


def cross_entropy(logits, target):
    """F.cross_entropy(logits, target) (mean), fused softmax-CE fwd/bwd kernels."""
    L.require_gpu(logits)
    return _CrossEntropyFn.apply(logits, target)


# ----------------------------------------------------------------------------
# modules (timm key layout)
# ----------------------------------------------------------------------------

class PatchEmbed(nn.Module):
    def __init__(self, img_size, patch_size, in_chans, embed_dim):
        super().__init__()
        self.img_size, self.patch_size = img_size, patch_size
        self.num_patches = (img_size // patch_size) ** 2
        self.proj = nn.Conv2d(in_chans, embed_dim, patch_size, patch_size)


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio, eps):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=eps)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=eps)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def block_params(self):
        return (self.norm1.weight, self.norm1.bias, self.attn.qkv.weight, self.attn.qkv.bias,
                self.attn.proj.weight, self.attn.proj.bias, self.norm2.weight, self.norm2.bias,
                self.mlp.fc1.weight, self.mlp.fc1.bias, self.mlp.fc2.weight, self.mlp.fc2.bias)


class VisionTransformer(nn.Module):
    """timm ``VisionTransformer`` (class-token, pre-norm, global_pool='token')."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, num_classes=1000, embed_dim=768, depth=12,
                 num_heads=12, mlp_ratio=4.0, eps=1e-6, quick_gelu=False, compute_dtype=torch.bfloat16):
        super().__init__()
        if embed_dim // num_heads != 64:
            raise ValueError("the HIP attention kernels require head_dim 64")
        self.num_classes = num_classes
        self.embed_dim = self.num_features = embed_dim
        self.global_pool = "token"
        self.num_prefix_tokens = 1
        self.compute_dtype = compute_dtype
        self._cfg = dict(heads=num_heads, eps=eps, quick_gelu=quick_gelu, dtype=compute_dtype, patch=patch_size)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.patch_embed = PatchEmbed(img_size, patch_size, in_chans, embed_dim)
        self.pos_embed = nn.Parameter(torch.zeros(1, self.patch_embed.num_patches + 1, embed_dim))
        self.blocks = nn.Sequential(*[Block(embed_dim, num_heads, mlp_ratio, eps) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=eps)
        self.head = nn.Linear(embed_dim, num_classes)
        self._shadows = None
        self._defer_grad_join = False
        self._attn_fp8 = False
        self.init_weights()

    # timm init_weights_vit_timm; exact RNG stream differs from timm
    @torch.no_grad()
    def init_weights(self, seed=None):
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        nn.init.trunc_normal_(self.pos_embed, std=0.02, generator=g)
        nn.init.normal_(self.cls_token, std=1e-6, generator=g)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02, generator=g)
                nn.init.zeros_(m.bias)

    def load_oracle_params(self, params: "OrderedDict[str, torch.Tensor]"):
        """Copy a timm-keyed fp32 state dict (e.g. the oracle's) into this model."""
        self.load_state_dict(params, strict=True)

    # -- device / dtype plumbing --------------------------------------------------
    def _ensure_shadows(self):
        dev = self.cls_token.device
        if self._shadows is None or self._shadows_device != dev:
            self._shadows = _Shadowed()
            self._shadows_device = dev
            ws = [self.patch_embed.proj.weight]
            for blk in self.blocks:
                ws += [blk.attn.qkv.weight, blk.attn.proj.weight, blk.mlp.fc1.weight, blk.mlp.fc2.weight]
            for p in ws:
                self._shadows.add(p, self.compute_dtype)
        self._shadows.refresh()

    def use_flat_grads(self, enable: bool = True):
        """Write every gradient into one flat fp32 buffer (backward order: head
        first, patch embed last) -- ``flat_grad`` is what a data-parallel
        all-reduce reduces (vit_amd.parallel)."""
        params = list(self.parameters())
        if not enable:
            for p in params:
                p._vit_flat_grad = None
            self.flat_grad = None
            return None
        order = [self.norm.weight, self.norm.bias, self.head.weight, self.head.bias]
        for blk in reversed(list(self.blocks)):
            order += list(reversed(blk.block_params()))
        pe = self.patch_embed.proj
        order += [pe.weight, pe.bias, self.cls_token, self.pos_embed]
        assert len(order) == len(params) and {id(p) for p in order} == {id(p) for p in params}
        n = sum(p.numel() for p in order)
        flat = torch.zeros(n, dtype=torch.float32, device=self.cls_token.device)
        off = 0
        self.flat_grad_slices = []
        for p in order:
            p._vit_flat_grad = flat[off:off + p.numel()].view(p.shape)
            self.flat_grad_slices.append((off, p.numel()))
            off += p.numel()
        self.flat_grad = flat
        # each block's parameters are contiguous in the buffer: its span for an overlapped all-reduce
        ends = {}
        off = 0
        for p in order:
            ends[id(p)] = (off, off + p.numel())
            off += p.numel()
        for blk in self.blocks:
            spans = [ends[id(p)] for p in blk.block_params()]
            blk._flat_span = (min(s for s, _ in spans), max(e for _, e in spans))
        return flat

    def set_deferred_grad_join(self, enable: bool = True):
        """Let the block backwards leave their weight-gradient kernels queued on the side stream
        until the end of the backward (one join instead of one per block: +0.5 % at bs=256).
        Only for callers that read gradients after ``backward()`` returns (the fused optimizers,
        ``parallel.OverlappedGradReduce``, ``allreduce_flat``) -- not under ``DDP(model)`` or
        with gradient hooks, which read ``.grad`` during the backward on the caller's stream."""
        self._defer_grad_join = bool(enable)

    def set_attention_fp8(self, enable: bool = True):
        """Run attention as block-scaled e4m3 MFMA (vit_sdpa_fwd_fp8) in forward passes that build no
        autograd graph (``torch.no_grad()``: validation, ``compute_rsa_score``'s embeddings) --
        BASELINE configs[4].  Training forwards keep the bf16 kernels their backward needs."""
        self._attn_fp8 = bool(enable)

    def set_grad_ready_hook(self, fn):
        """fn(lo, hi) is called by each block's backward once the block's gradients (the flat
        buffer's [lo, hi)) are enqueued, on the stream they were enqueued on
        (vit_amd.parallel.OverlappedGradReduce)."""
        self._grad_hook = fn

    def shadow_params(self):
        self._ensure_shadows()
        return list(self._shadows.pairs)

    # -- timm surface ----------------------------------------------------------------
    def _tokens(self, x):
        L.require_gpu(x)
        self._ensure_shadows()
        cfg = dict(self._cfg)
        pe = self.patch_embed
        x = _PatchEmbedFn.apply(x.to(torch.float32), pe.proj.weight, pe.proj.bias, self.cls_token, self.pos_embed,
                                cfg)
        n = len(self.blocks)
        cfg["defer_join"] = _FWD_JOIN[0] == "end"
        # Opt-in (set_deferred_grad_join, used by bench.py / OverlappedGradReduce): gradients in
        # the flat buffer are only read after backward (optimizer / all-reduce), so the blocks may
        # leave their weight-gradient work pending until the patch embedding's backward (or the
        # end of the backward pass, _queue_backward_join).  Not safe when something reads .grad
        # DURING the backward on the caller's stream (DDP's bucket hooks, post-accumulate-grad
        # hooks), hence off by default; also off when a .grad exists (AccumulateGrad would add
        # into it on the caller's stream).
        cfg["defer_bwd_join"] = (self._defer_grad_join and _BWD_JOIN[0] == "end"
                                 and getattr(self, "flat_grad", None) is not None
                                 and torch.is_grad_enabled() and pe.proj.weight.requires_grad
                                 and all(p.grad is None for p in self.parameters()))
        hook = getattr(self, "_grad_hook", None) if cfg["defer_bwd_join"] else None
        # fp8 attention (set_attention_fp8): forward passes that build no graph (eval / RSA)
        cfg["attn_fp8"] = self._attn_fp8 and not torch.is_grad_enabled()
        D = self.embed_dim
        if (self.compute_dtype != torch.float32 or _FUSED_RESID_F32[0]) and ops.add_layer_norm_supported(D):
            cfg["resid"] = {"pending": None}  # residual adds inside the LayerNorms (_BlockFn.forward)
        for i, blk in enumerate(self.blocks):
            bcfg = cfg if i != 0 else dict(cfg, compact_np=pe.num_patches)
            if "resid" in cfg and i == n - 1:
                bcfg = dict(bcfg, resid_last=True)
            if hook is not None:
                bcfg = dict(bcfg, grad_hook=hook, flat_span=blk._flat_span)
            x = _BlockFn.apply(x, *blk.block_params(), bcfg)
        if cfg["defer_join"]:
            _Side(x.device).join()  # the side stream's half-batch chain of the last block
        return x

    def forward_features(self, x):
        """post-norm tokens [B, N, D] (f32), as timm forward_features (MEAS:309)."""
        x = self._tokens(x)
        B, N, D = x.shape
        # full final norm (inference / RSA path; forward() only normalises CLS rows)
        y, _, _ = ops.layer_norm_fwd(x.reshape(B * N, D), self.norm.weight.detach(), self.norm.bias.detach(),
                                     self._cfg["eps"], torch.float32, need_stats=False)
        return y.reshape(B, N, D)

    def forward_head(self, feats, pre_logits=False):
        x = feats[:, 0]
        return x if pre_logits else ops.linear_fwd(x.contiguous(), self.head.weight.detach(),
                                                   self.head.bias.detach(), out_dtype=torch.float32)

    def forward(self, x):
        x = self._tokens(x)
        return _HeadFn.apply(x, self.norm.weight, self.norm.bias, self.head.weight, self.head.bias, dict(self._cfg))


_MODEL_CFGS = {
    "vit_base_patch16_224": dict(img_size=224, patch_size=16, embed_dim=768, depth=12, num_heads=12),
    "vit_large_patch16_224": dict(img_size=224, patch_size=16, embed_dim=1024, depth=24, num_heads=16),
    "vit_small_patch16_224": dict(img_size=224, patch_size=16, embed_dim=384, depth=12, num_heads=6),
}


def create_model(name: str, pretrained: bool = False, num_classes: int = 1000, compute_dtype=torch.bfloat16,
                 **kw):
    """``timm.create_model`` drop-in for the configs the reference uses (VIT:283)."""
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    if name not in _MODEL_CFGS:
        raise KeyError(f"unknown model {name}; known: {sorted(_MODEL_CFGS)}")
    cfg = dict(_MODEL_CFGS[name])
    cfg.update(kw)
    return VisionTransformer(num_classes=num_classes, compute_dtype=compute_dtype, **cfg)
