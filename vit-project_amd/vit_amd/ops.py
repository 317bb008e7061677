"""Tensor-level wrappers over the C-ABI kernels (no compute happens in Python).

Every function takes torch tensors that live on the ROCm device, launches the
HIP kernel on the current stream and returns.  These mirror the torch ops the
reference's hot path reaches through timm:

  linear_fwd / linear_dgrad / linear_wgrad   F.linear fwd / bwd  (timm Attention.qkv/proj, Mlp.fc1/fc2, head)
  layer_norm_fwd / layer_norm_bwd            F.layer_norm         (timm Block.norm1/norm2, final norm)
  sdpa_fwd / sdpa_bwd                        F.scaled_dot_product_attention
  patch_unfold + patch_embed_fwd             Conv2d(k16, s16) + cat(cls) + pos_embed (timm PatchEmbed/_pos_embed)
  cross_entropy_fwd / _bwd                   F.cross_entropy (VIT:140)
  sgd_step                                   torch.optim.SGD.step (VIT:294-299)
"""
from __future__ import annotations

import os

import torch

from . import _lib as L
from ._lib import call, ptr

_WS = {}


def workspace(name: str, nbytes: int, device) -> torch.Tensor:
    """Grow-only scratch buffer, reused across calls on the same stream."""
    key = (name, torch.device(device))
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        _WS[key] = t
    return t


def _s(t: torch.Tensor) -> int:
    return L.stream_ptr(t.device)


def _keep(t: torch.Tensor):
    """t is read by work queued on the current stream after its producer's stream moves on:
    the caching allocator must not hand its memory out again before that work ran."""
    if t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


# ----------------------------------------------------------------------------
# GEMMs
# ----------------------------------------------------------------------------

_SK = {}  # (device index, stream handle) -> (part, counters) registered with vit_gemm_streamk_workspace


def _streamk(device, stream=None):
    """Register (once per (device, stream)) the stream-K workspace the f32 MFMA GEMMs use on the
    current stream (or ``stream``).  Keyed by device too: the null stream has handle 0 on every device.
    Under graph capture an unregistered stream stays unregistered (the workspace's zero-fill would be
    captured, not run, and its memory would come from the graph's pool): the plain launch runs there.
    The two forms sum k in different orders, so an f32 GEMM that ran stream-K eagerly and as the plain
    launch in a replayed graph agree to rounding, not bit for bit -- unless the capture
    stream was registered before capture: ``register_capture_stream``."""
    st = L.stream_ptr(device) if stream is None else stream.cuda_stream
    key = (torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device(), st)
    if key in _SK or torch.cuda.is_current_stream_capturing():
        return
    g = 2 * torch.cuda.get_device_properties(device).multi_processor_count
    part = torch.empty(g * 2 * 128 * 128, dtype=torch.float32, device=device)
    cnt = torch.zeros(g, dtype=torch.int32, device=device)
    with torch.cuda.device(key[0]):
        call("vit_gemm_streamk_workspace", st, ptr(part), part.numel() * 4, ptr(cnt), g)
    _SK[key] = (part, cnt)


def register_capture_stream(stream, device=None):
    """Give ``stream`` (e.g. the side stream a ``torch.cuda.graph`` captures on) its stream-K workspace
    before capture, so the f32 GEMMs captured on it take the same form -- and the same bits -- as the
    eager launches on a registered stream."""
    _streamk(stream.device if device is None else device, stream)


def linear_fwd(x2d, w, bias=None, epi=L.EPI_STORE, out=None, out_dtype=None, resid=None, act_out=None):
    """y = epi(x @ w^T + bias).  x2d [M,K] (row stride x2d.stride(0)), w [N,K] contiguous.
    EPI_BIAS_GELU / EPI_BIAS_QGELU return (act'(pre), act(pre)) with pre = x @ w^T + bias."""
    L.require_gpu(x2d)
    M, K = x2d.shape
    N = w.shape[0]
    assert w.shape[1] == K and w.is_contiguous() and x2d.stride(1) == 1
    assert w.dtype == x2d.dtype
    if out is None:
        if epi == L.EPI_RESID:
            od = torch.float32
        else:
            od = out_dtype or x2d.dtype
        out = torch.empty(M, N, dtype=od, device=x2d.device)
    if epi in (L.EPI_BIAS_GELU, L.EPI_BIAS_QGELU):
        if act_out is None:
            act_out = torch.empty_like(out)
    if epi == L.EPI_RESID:
        assert resid is not None and resid.dtype == torch.float32 and out.dtype == torch.float32
        assert resid.stride(0) == out.stride(0)
    if x2d.dtype == torch.float32:
        _streamk(x2d.device)
    call("vit_linear_fwd", L.dt(x2d), L.dt(out), epi, M, N, K, ptr(x2d), x2d.stride(0), ptr(w), ptr(bias),
         ptr(out), out.stride(0), ptr(resid), ptr(act_out), _s(x2d))
    return (out, act_out) if epi in (L.EPI_BIAS_GELU, L.EPI_BIAS_QGELU) else out


def linear_dgrad(dy2d, w, out_dtype=torch.float32, epi=L.EPI_STORE, pre=None, out=None, dbias=None, reduce_on=None):
    """dx = dy @ w  (dy [M,N], w [N,K]); with EPI_GELU_BWD / EPI_QGELU_BWD times ``pre`` [M,K] =
    the act'(pre) the forward's BIAS_GELU epilogue saved;
    dbias [K] (optional) receives the column sums of dx (fused into the GEMM epilogue).
    ``reduce_on`` (an object with ``.run(fn)``, e.g. the model's side stream): the final
    reduction of those column sums is issued through it instead of inline."""
    M, N = dy2d.shape
    K = w.shape[1]
    assert w.shape[0] == N and w.dtype == dy2d.dtype and dy2d.stride(1) == 1
    if out is None:
        out = torch.empty(M, K, dtype=out_dtype, device=dy2d.device)
    if pre is not None:
        assert pre.stride(0) == out.stride(0)
    part, nfl = None, 0
    defer = dbias is not None and reduce_on is not None
    if dbias is not None:
        assert dbias.dtype == torch.float32 and dbias.is_contiguous() and dbias.numel() == K
        nfl = L.lib().vit_linear_dgrad_partial_floats(M, K)
        # a deferred reduction reads the partials later on another stream: own buffer
        part = (torch.empty(nfl, dtype=torch.float32, device=dy2d.device) if defer
                else workspace("dgrad_bias", nfl * 4, dy2d.device))
    if dy2d.dtype == torch.float32:
        _streamk(dy2d.device)
    call("vit_linear_dgrad", L.dt(dy2d), L.dt(out), epi, M, N, K, ptr(dy2d), dy2d.stride(0), ptr(w), ptr(out),
         out.stride(0), ptr(pre), ptr(dbias), ptr(part), nfl, int(defer), _s(dy2d))
    if defer:
        rows = (M + 63) // 64
        if isinstance(reduce_on, ColBatch):
            reduce_on.add(part, rows, K, dbias)
            return out

        def finish():
            _keep(part)
            colreduce(part, rows, K, dbias, scratch=part[rows * K:])
        reduce_on.run(finish)
    return out


def colreduce(part, S, N, out, accumulate=False, scratch=None):
    """out[N] (+)= part[:S].sum(0) (partials from a fused epilogue)."""
    call("vit_colreduce", ptr(part), S, N, ptr(out), int(accumulate), ptr(scratch), _s(out))
    return out


class ColBatch:
    """Collects the deferred column reductions of one block's backward (bias and LayerNorm-affine
    gradients from their producers' partial sums) and issues them as ONE vit_colreduce_batch launch
    (``launch``, on whatever stream is current then -- the model's side stream).  The partial
    buffers stay referenced until ``launch`` has been enqueued; the caller guards them for the
    stream (``tensors``)."""

    def __init__(self):
        self.jobs = []
        self.parts = []  # the partial buffers (guard them for the stream the launch runs on)
        self.device = None

    def add(self, part, S, N, out, accumulate=False):
        """out[N] (+)= sum of the S rows of part ([S][N] f32, contiguous rows).  Only the output's
        address is kept (gradient views must stay stealable by AccumulateGrad)."""
        if out is None or S <= 0:
            return
        assert part.dtype == torch.float32 and out.dtype == torch.float32 and part.is_contiguous()
        self.jobs.append((part.data_ptr(), out.data_ptr(), int(S), int(N), int(accumulate)))
        self.parts.append(part)
        self.device = part.device

    def launch(self):
        if not self.jobs:
            return
        import ctypes
        import numpy as np
        dev = self.device
        arr = np.array(self.jobs, dtype=np.int64).reshape(-1)
        jp = arr.ctypes.data_as(ctypes.c_void_p)
        sf, nc = ctypes.c_int64(0), ctypes.c_int(0)
        L.lib().vit_colreduce_batch_sizes(jp, len(self.jobs), ctypes.byref(sf), ctypes.byref(nc))
        scratch = workspace("colbatch", max(16, sf.value * 4), dev)
        cnt = _counters("colbatch", nc.value, dev)
        call("vit_colreduce_batch", jp, len(self.jobs), ptr(scratch), sf.value, ptr(cnt), nc.value, L.stream_ptr(dev))
        self.jobs = []


_CNT = {}


def _counters(name, n, device):
    """Grow-only int32 ticket counters, zero-filled when allocated (the kernels that use them leave
    them zero)."""
    key = (name, torch.device(device))
    t = _CNT.get(key)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 64), dtype=torch.int32, device=device)
        _CNT[key] = t
    return t


_WGRAD_WGS = [int(os.environ.get("VIT_WGRAD_WGS", "128"))]


# the backward's tail (block 0's last weight gradients, the patch embedding's): nothing else is
# left to run beside them, so they split for the whole GPU
_WGRAD_TAIL_WGS = [int(os.environ.get("VIT_WGRAD_TAIL_WGS", "256"))]


def _wgrad_split(M, N, K, wgs=None):
    """Split of the M reduction so (256x256 output tiles) x split ~ _WGRAD_WGS workgroups
    (default 128: half the CUs, so the side-stream weight gradients leave CUs to the
    input-gradient chain on the main stream -- +1.3 % step rate vs 256): fp32 slab traffic split*N*K*8 bytes stays ~10% of the
    GEMM time."""
    tiles = max(1, ((N + 255) // 256) * ((K + 255) // 256))
    want = max(1, round((wgs or _WGRAD_WGS[0]) / tiles))
    return max(1, min(want, M // 1024))


def linear_wgrad(dy2d, x2d, out=None, split=None, tail=False, reduce_on=None):
    """dW [N,K] (f32) = dy^T @ x,  dy [M,N], x [M,K].  tail: split for _WGRAD_TAIL_WGS workgroups.
    ``reduce_on`` (a ColBatch): the split-K slabs go to a buffer of their own and their sum into
    ``out`` becomes a job of that batch (no separate slab-reduce launch)."""
    M, N = dy2d.shape
    K = x2d.shape[1]
    assert x2d.shape[0] == M and x2d.dtype == dy2d.dtype
    if out is None:
        out = torch.empty(N, K, dtype=torch.float32, device=dy2d.device)
    if split is None:
        split = _wgrad_split(M, N, K, _WGRAD_TAIL_WGS[0] if tail else None)
    defer = isinstance(reduce_on, ColBatch) and split > 1 and dy2d.dtype == torch.bfloat16
    probe = WGRAD_PROBE[0]
    if probe is not None:  # bench.py: HIP events around this launch, on the stream it runs on
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    if defer:
        nz = L.lib().vit_linear_wgrad_nslabs(L.dt(dy2d), M, N, K, split)
        slabs = torch.empty(nz * N * K, dtype=torch.float32, device=dy2d.device)
        call("vit_linear_wgrad_partials", L.dt(dy2d), M, N, K, ptr(dy2d), dy2d.stride(0), ptr(x2d), x2d.stride(0),
             split, ptr(slabs), slabs.numel() * 4, _s(dy2d))
        reduce_on.add(slabs.view(nz, N * K), nz, N * K, out)
    else:
        ws = workspace("wgrad", split * N * K * 4, dy2d.device) if split > 1 else None
        call("vit_linear_wgrad", L.dt(dy2d), M, N, K, ptr(dy2d), dy2d.stride(0), ptr(x2d), x2d.stride(0), ptr(out),
             split, ptr(ws), 0 if ws is None else ws.numel(), _s(dy2d))
    if probe is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        probe.append((e0, e1, 2.0 * M * N * K, L.dt(dy2d) == L.BF16 and M % 32 == 0))
    return out


def linear_wgrad_pair(a, b, reduce_on, tail=False):
    """Two weight gradients of a block over the same token rows, a = (dy, x, out), b likewise, as
    ONE grouped launch of split-K partials whose slab sums become two jobs of ``reduce_on`` (a
    ColBatch).  The split is chosen for the pair's tiles together (half the slabs of two separate
    launches).  Falls back to two linear_wgrad calls when the pair does not meet the grouped
    kernel's rules (bf16, M % 32 == 0, MFMA operand alignment)."""
    (dya, xa, outa), (dyb, xb, outb) = a, b
    M, Na = dya.shape
    Ka, Nb, Kb = xa.shape[1], dyb.shape[1], xb.shape[1]
    ok = (isinstance(reduce_on, ColBatch) and dya.dtype == torch.bfloat16 and dyb.dtype == torch.bfloat16
          and xa.dtype == dya.dtype and xb.dtype == dyb.dtype and dyb.shape[0] == M and M % 32 == 0)
    if ok:
        tiles = ((Na + 255) // 256) * ((Ka + 255) // 256) + ((Nb + 255) // 256) * ((Kb + 255) // 256)
        wgs = _WGRAD_TAIL_WGS[0] if tail else _WGRAD_WGS[0]
        split = max(1, min(max(1, round(wgs / tiles)), M // 1024))
        nz = L.lib().vit_linear_wgrad_nslabs(L.BF16, M, Na, Ka, split)
        sa = torch.empty(nz * Na * Ka, dtype=torch.float32, device=dya.device)
        sb = torch.empty(nz * Nb * Kb, dtype=torch.float32, device=dya.device)
        probe = WGRAD_PROBE[0]
        if probe is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        rc = L.lib().vit_linear_wgrad_partials2(M, split, Na, Ka, ptr(dya), dya.stride(0), ptr(xa), xa.stride(0),
                                                ptr(sa), sa.numel() * 4, Nb, Kb, ptr(dyb), dyb.stride(0), ptr(xb),
                                                xb.stride(0), ptr(sb), sb.numel() * 4, _s(dya))
        if rc not in (0, 1):  # 1 = hipErrorInvalidValue: the pair does not fit the grouped kernel
            L.check(rc, "vit_linear_wgrad_partials2")
        if rc == 0:
            if probe is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                probe.append((e0, e1, 2.0 * M * (Na * Ka + Nb * Kb), True))
            reduce_on.add(sa.view(nz, Na * Ka), nz, Na * Ka, outa)
            reduce_on.add(sb.view(nz, Nb * Kb), nz, Nb * Kb, outb)
            return outa, outb
    linear_wgrad(dya, xa, out=outa, tail=tail, reduce_on=reduce_on)
    linear_wgrad(dyb, xb, out=outb, tail=tail, reduce_on=reduce_on)
    return outa, outb


# bench.py's live roofline of the weight-gradient GEMMs: a list to collect
# (start event, end event, flop, on the MFMA path) per vit_linear_wgrad launch, or None
WGRAD_PROBE = [None]


def colsum(x2d, out=None, accumulate=False):
    """out[N] (f32) = x.sum(0)."""
    M, N = x2d.shape
    if out is None:
        out = torch.empty(N, dtype=torch.float32, device=x2d.device)
    S = max(1, min(256, M // 64))
    nfl = (S + (S + 63) // 64) * N
    part = workspace("colsum", nfl * 4, x2d.device)
    call("vit_colsum", L.dt(x2d), M, N, ptr(x2d), x2d.stride(0), ptr(out), ptr(part), nfl, int(accumulate),
         _s(x2d))
    return out


# ----------------------------------------------------------------------------
# LayerNorm
# ----------------------------------------------------------------------------

def layer_norm_fwd(x2d, w, b, eps, out_dtype, rows=None, ldx=None, out=None, need_stats=True, mean=None, rstd=None):
    rows = x2d.shape[0] if rows is None else rows
    D = w.numel()
    ldx = x2d.stride(0) if ldx is None else ldx
    if out is None:
        out = torch.empty(rows, D, dtype=out_dtype, device=x2d.device)
    if need_stats and mean is None:
        mean = torch.empty(rows, dtype=torch.float32, device=x2d.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x2d.device)
    call("vit_layer_norm_fwd", L.dt(x2d), L.dt(out), rows, D, ptr(x2d), ldx, ptr(out), out.stride(0), ptr(w),
         ptr(b), ptr(mean), ptr(rstd), float(eps), _s(x2d))
    return out, mean, rstd


def add_layer_norm_supported(D: int) -> bool:
    """Widths ``vit_add_layer_norm_fwd`` takes: D a multiple of 256 up to 2048 (ViT-B 768, ViT-L
    1024, ViT-H 1280, ...); other widths keep the residual add in the GEMM epilogue."""
    return D % 256 == 0 and 256 <= D <= 2048


def add_layer_norm_fwd(x2d, r2d, xs, w=None, b=None, eps=1e-6, out=None, mean=None, rstd=None):
    """xs = x2d + r2d (f32 + bf16 / f32 -> f32; xs may be x2d) and, with ``out`` given, out =
    LayerNorm(xs) (bf16 / f32) with its row mean / rstd: a Linear's residual add fused into the
    LayerNorm after it."""
    assert x2d.dtype == torch.float32 and xs.dtype == torch.float32
    rows, D = xs.shape
    if out is not None:
        assert mean is not None and rstd is not None
    call("vit_add_layer_norm_fwd", L.dt(r2d), L.dt(out) if out is not None else L.dt(r2d), rows, D, ptr(x2d),
         x2d.stride(0), ptr(r2d), r2d.stride(0), ptr(xs), xs.stride(0),
         ptr(out), out.stride(0) if out is not None else 0, ptr(w), ptr(b), ptr(mean), ptr(rstd), float(eps), _s(xs))
    return xs


def layer_norm_bwd(x, ldx, dy, w, mean, rstd, dx, lddx, rows, dres=None, ldres=0, dx_copy=None, ld_copy=0,
                   compact_np=0, dgamma=None, dbeta=None, dsum=None, ws="ln_partial", reduce_on=None):
    """dsum [D] (optional) receives the column sums of dx (a Linear bias gradient).
    ``reduce_on`` (an object with ``.run(fn)``): the dgamma / dbeta / dsum reductions of the
    per-64-row partials are issued through it (e.g. on the side stream) instead of inline."""
    D = w.numel()
    part = None
    nfl = 0
    want = dgamma is not None or dsum is not None
    defer = want and reduce_on is not None
    if want:
        nfl = L.lib().vit_layer_norm_bwd_partial_floats(rows, D)
        part = (torch.empty(nfl, dtype=torch.float32, device=x.device) if defer
                else workspace(ws, nfl * 4, x.device))
    call("vit_layer_norm_bwd", L.dt(x), L.dt(dy), rows, D, ptr(x), ldx, ptr(dy), dy.stride(0), ptr(w), ptr(mean),
         ptr(rstd), ptr(dres), ldres, ptr(dx), lddx, ptr(dx_copy), ld_copy,
         L.dt(dx_copy) if dx_copy is not None else L.BF16, compact_np, ptr(dgamma), ptr(dbeta), ptr(dsum), ptr(part),
         nfl, int(defer), _s(x))
    if defer:
        nb = L.lib().vit_layer_norm_bwd_blocks(rows)
        if isinstance(reduce_on, ColBatch):
            for q, o in enumerate((dgamma, dbeta, dsum)):
                if o is not None:
                    reduce_on.add(part[q * nb * D:(q + 1) * nb * D], nb, D, o)
            return
        sc = part[3 * nb * D:]

        def finish():
            _keep(part)
            # the [dgamma | dbeta | dsum] partials are stacked: one launch per reduction stage
            if dgamma is not None:
                call("vit_colreduce_multi", ptr(part), 3 if dsum is not None else 2, nb, D, ptr(dgamma),
                     ptr(dbeta), ptr(dsum), 0, ptr(sc), _s(dgamma))
            else:
                call("vit_colreduce_multi", ptr(part[2 * nb * D:]), 1, nb, D, ptr(dsum), None, None, 0,
                     ptr(sc), _s(dsum))
        reduce_on.run(finish)


# ----------------------------------------------------------------------------
# attention
# ----------------------------------------------------------------------------

def sdpa_fwd(qkv2d, B, H, N, o=None, scale=None, lse=None, causal=False, fp8=False):
    """softmax(q k^T * scale) v per (b, h) from the fused qkv [B*N, 3D]; fp8: the block-scaled e4m3
    MFMA kernel (forward only: its lse is not the bf16 backward's)."""
    D = H * 64
    if o is None:
        o = torch.empty(B * N, D, dtype=qkv2d.dtype, device=qkv2d.device)
    if lse is None:
        lse = torch.empty(B * H * N, dtype=torch.float32, device=qkv2d.device)
    scale = 64 ** -0.5 if scale is None else scale
    name = "vit_sdpa_fwd_fp8" if fp8 else "vit_sdpa_fwd"
    call(name, L.dt(qkv2d), B, H, N, 64, ptr(qkv2d), qkv2d.stride(0), ptr(o), o.stride(0), ptr(lse),
         float(scale), int(causal), _s(qkv2d))
    return o, lse


def sdpa_bwd(qkv2d, o, do, lse, B, H, N, dqkv=None, scale=None, dbias=None, causal=False, ws="", reduce_on=None):
    """dbias [3*H*64] (optional) receives the column sums of dqkv (the qkv bias gradient).
    ``ws``: workspace-name suffix (calls running concurrently on different streams need their own).
    ``reduce_on`` (a ColBatch, bf16): the per-image bias partials are left for that batch to reduce."""
    if dqkv is None:
        dqkv = torch.empty_like(qkv2d)
    scale = 64 ** -0.5 if scale is None else scale
    delta = workspace("sdpa_delta" + ws, B * H * N * 4, qkv2d.device)
    part, nfl = None, 0
    defer = dbias is not None and isinstance(reduce_on, ColBatch) and qkv2d.dtype == torch.bfloat16
    if dbias is not None:
        nfl = L.lib().vit_sdpa_bwd_partial_floats(B, N, H * 64)
        part = (torch.empty(nfl, dtype=torch.float32, device=qkv2d.device) if defer
                else workspace("sdpa_bias" + ws, nfl * 4, qkv2d.device))
    call("vit_sdpa_bwd", L.dt(qkv2d), B, H, N, 64, ptr(qkv2d), qkv2d.stride(0), ptr(o), o.stride(0), ptr(do),
         do.stride(0), ptr(lse), ptr(dqkv), dqkv.stride(0), ptr(delta), float(scale), int(causal),
         None if defer else ptr(dbias), ptr(part), nfl, _s(qkv2d))
    if defer:
        reduce_on.add(part, B, 3 * H * 64, dbias)
    return dqkv


# ----------------------------------------------------------------------------
# patch embed, CE, casts
# ----------------------------------------------------------------------------

def patch_unfold(img, ps, dtype, ld=None):
    """U [B*np, C*ps*ps]; with ``ld`` > C*ps*ps the rows are ``ld`` wide and the extra columns zero (a
    reduction padded to the GEMM tile depth, for padded weights from :func:`pad_cols`)."""
    B, C, Hi, Wi = img.shape
    assert img.dtype == torch.float32 and img.is_contiguous()
    npatch = (Hi // ps) * (Wi // ps)
    K = C * ps * ps
    U = torch.empty(B * npatch, max(K, ld or K), dtype=dtype, device=img.device)
    call("vit_patch_unfold_ld", L.dt(U), B, C, Hi, Wi, ps, U.shape[1], ptr(img), ptr(U), _s(img))
    return U


def pad_cols(w2d, ld):
    """[rows, cols] -> [rows, ld] with columns [cols, ld) zero (vit_copy_rows_padded)."""
    rows, cols = w2d.shape
    assert w2d.stride(1) == 1 and ld >= cols
    out = torch.empty(rows, ld, dtype=w2d.dtype, device=w2d.device)
    call("vit_copy_rows_padded", L.dt(w2d), rows, cols, ptr(w2d), w2d.stride(0), ptr(out), ld, _s(w2d))
    return out


def patch_embed_fwd(U, w2d, bias, pos, cls, B, npatch):
    """x[b, 1 + p] = U[b*np + p] . w2d + bias + pos[1 + p]; U and w2d may both carry zero padding
    columns (same width)."""
    D, K = w2d.shape
    assert U.shape[1] == K and U.stride(1) == 1 and w2d.stride(1) == 1
    x = torch.empty(B, npatch + 1, D, dtype=torch.float32, device=U.device)
    call("vit_patch_embed_fwd_ld", L.dt(U), B, npatch, D, K, ptr(U), U.stride(0), ptr(w2d), w2d.stride(0),
         ptr(bias), ptr(pos), ptr(x), _s(U))
    call("vit_cls_pos_fill", B, npatch + 1, D, ptr(x), ptr(cls), ptr(pos), _s(U))
    return x


def pos_grad(dx, B, S, D, dpos, dcls):
    call("vit_pos_grad", B, S, D, ptr(dx), ptr(dpos), ptr(dcls), _s(dx))


def cross_entropy_fwd(logits, target):
    B, C = logits.shape
    assert logits.dtype == torch.float32 and target.dtype == torch.int64
    row_lse = torch.empty(B, dtype=torch.float32, device=logits.device)
    row_loss = torch.empty(B, dtype=torch.float32, device=logits.device)
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    call("vit_cross_entropy_fwd", B, C, ptr(logits), logits.stride(0), ptr(target), ptr(row_lse), ptr(row_loss),
         ptr(loss), _s(logits))
    return loss, row_lse


def cross_entropy_bwd(logits, target, row_lse, grad_loss, out_dtype=torch.float32):
    B, C = logits.shape
    d = torch.empty(B, C, dtype=out_dtype, device=logits.device)
    g = grad_loss.to(torch.float32).contiguous() if grad_loss is not None else None
    call("vit_cross_entropy_bwd", L.dt(d), B, C, ptr(logits), logits.stride(0), ptr(target), ptr(row_lse), ptr(g),
         ptr(d), d.stride(0), _s(logits))
    return d


def cast_bf16(src: torch.Tensor, dst: torch.Tensor):
    assert src.dtype == torch.float32 and dst.dtype == torch.bfloat16 and src.numel() == dst.numel()
    call("vit_cast_f32_bf16", ptr(src), ptr(dst), src.numel(), _s(src))


def zero_(t: torch.Tensor):
    call("vit_zero", ptr(t), t.numel() * t.element_size(), _s(t))
    return t


# ----------------------------------------------------------------------------
# CLIP-HBA pieces (csrc/clip.hip)
# ----------------------------------------------------------------------------

def token_embed(tokens, table, pos):
    """x [S*L, D] f32 = table[tokens] + pos[t]  (tokens int64 [S, L])."""
    S, Lq = tokens.shape
    D = table.shape[1]
    x = torch.empty(S * Lq, D, dtype=torch.float32, device=table.device)
    call("vit_token_embed", S * Lq, Lq, D, table.shape[0], ptr(tokens.contiguous()), ptr(table), ptr(pos), ptr(x),
         _s(table))
    return x


def gather_rows(src2d, idx, out=None):
    n = idx.numel()
    D = src2d.shape[1]
    if out is None:
        out = torch.empty(n, D, dtype=torch.float32, device=src2d.device)
    call("vit_gather_rows", n, D, ptr(src2d), src2d.stride(0), ptr(idx), ptr(out), out.stride(0), _s(src2d))
    return out


def scatter_rows(src2d, idx, dst2d):
    n = idx.numel()
    call("vit_scatter_rows", n, src2d.shape[1], ptr(src2d), src2d.stride(0), ptr(idx), ptr(dst2d), dst2d.stride(0),
         _s(src2d))
    return dst2d


def rownorm_fwd(x2d, log_scale=None):
    n, D = x2d.shape
    y = torch.empty_like(x2d)
    rn = torch.empty(n, dtype=torch.float32, device=x2d.device)
    call("vit_rownorm_fwd", n, D, ptr(x2d), ptr(log_scale), ptr(y), ptr(rn), _s(x2d))
    return y, rn


def rownorm_bwd(x2d, dy, rn, log_scale=None):
    n, D = x2d.shape
    dx = torch.empty_like(x2d)
    call("vit_rownorm_bwd", n, D, ptr(x2d), ptr(dy.contiguous()), ptr(rn), ptr(log_scale), ptr(dx), _s(x2d))
    return dx


def mse_fwd(pred, target):
    loss = torch.empty((), dtype=torch.float32, device=pred.device)
    call("vit_mse_fwd", pred.numel(), ptr(pred), ptr(target), ptr(loss), _s(pred))
    return loss


def mse_bwd(pred, target, grad_loss=None):
    d = torch.empty_like(pred)
    g = grad_loss.to(torch.float32).contiguous() if grad_loss is not None else None
    call("vit_mse_bwd", pred.numel(), ptr(pred), ptr(target), ptr(g), ptr(d), _s(pred))
    return d




def gemm(P, p_layout, Q, q_layout, M, N, R, out=None, out_dtype=torch.float32, bias=None):
    """Raw C[i][j] = sum_r P(i,r) Q(j,r) (+bias[j]); layouts L.LAY_RC (r contiguous) / L.LAY_CR."""
    assert P.dtype == Q.dtype and P.stride(-1) == 1 and Q.stride(-1) == 1
    if (out is None and bias is None and P.dtype == torch.float32 and out_dtype == torch.float32
            and R >= 256 and ((M + 31) // 32) * ((N + 31) // 32) < 128):
        # few output tiles over a long reduction: split it (vit_gemm_splitk, slab sum in a fixed order)
        out = torch.empty(M, N, dtype=torch.float32, device=P.device)
        ws = workspace(f"gemm_splitk:{_s(P)}", 2 * 256 * 1024 * 4, P.device).view(torch.float32)
        call("vit_gemm_splitk", p_layout, q_layout, M, N, R, ptr(P), P.stride(0), ptr(Q), Q.stride(0), ptr(out),
             ptr(ws), ws.numel(), _s(P))
        return out
    if out is None:
        out = torch.empty(M, N, dtype=out_dtype, device=P.device)
    if P.dtype == torch.float32:
        _streamk(P.device)
    call("vit_gemm", L.dt(P), L.dt(out), p_layout, q_layout, L.EPI_STORE, M, N, R, ptr(P), P.stride(0), ptr(Q),
         Q.stride(0), ptr(out), out.stride(0), ptr(bias), None, 0, None, 1, _s(P))
    return out
