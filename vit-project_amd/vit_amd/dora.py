"""DoRA adapter layer: drop-in for ``DoRALayer`` (NEWP:407-481).

Same constructor, parameter names (``m``, ``delta_D_A``, ``delta_D_B``, ``bias``),
buffer ``D`` and ``weight`` property, so ``apply_dora_to_ViT`` / the DoRA
checkpoint keys (NEWP:665-683) and ``nn.MultiheadAttention``'s use of
``out_proj.weight`` (quirk Q5) work unchanged.  The weight build
``W = m * (D + (B@A)*s) / (||.||_col + 1e-8)`` and its backward run as HIP
kernels (csrc/dora.hip).  ``forward(x)`` is ``F.linear(x, W, b)`` on
the HIP GEMM, with the reference's train-mode dropout on dD (NEWP:468) applied as a
noise multiplier inside the weight kernel (never reached on the CLIP path, where MHA
reads ``.weight``: quirk Q5, but part of the class's surface).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from ._lib import call, ptr



class _DoraWeightFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, m, A, Bm, D, scaling, noise=None):
        fin, fout = D.shape
        r = A.shape[0]
        dev = D.device
        W = torch.empty(fout, fin, dtype=torch.float32, device=dev)
        nu = torch.empty(fout, dtype=torch.float32, device=dev)
        DnT = torch.empty(fout, fin, dtype=torch.float32, device=dev)
        colsq = torch.empty(((fin + 63) // 64) * fout, dtype=torch.float32, device=dev)
        m_, A_, B_ = m.detach().contiguous(), A.detach().contiguous(), Bm.detach().contiguous()
        nz = None if noise is None else noise.detach().contiguous()
        call("vit_dora_weight_fwd", fin, fout, r, ptr(m_), ptr(A_), ptr(B_), ptr(D.contiguous()), float(scaling),
             ptr(nz), ptr(W), ptr(nu), ptr(DnT), ptr(colsq), L.stream_ptr(dev))
        ctx.save_for_backward(m_, A_, B_, DnT, nu, nz)
        ctx.scaling = scaling
        return W

    @staticmethod
    def backward(ctx, gW):
        m, A, Bm, DnT, nu, nz = ctx.saved_tensors
        fout, fin = DnT.shape
        r = A.shape[0]
        dev = DnT.device
        gW = gW.contiguous().float()
        dm = torch.empty_like(m)
        dA = torch.empty_like(A)
        dB = torch.empty_like(Bm)
        # sdDnT [out, in] f32, then the split-K slabs of the two factor GEMMs (16-B aligned)
        slab_floats = 2 * 256 * 1024
        base = -(-fout * fin // 4) * 4
        ws = ops.workspace("dora_sdDnT", (base + slab_floats) * 4, dev).view(torch.float32)
        call("vit_dora_weight_bwd_ws", fin, fout, r, ptr(m), ptr(A), ptr(Bm), ptr(gW), ptr(DnT), float(ctx.scaling),
             ptr(nu), ptr(dm), ptr(dA), ptr(dB), ptr(ws), ptr(ws[base:]), slab_floats, ptr(nz), L.stream_ptr(dev))
        return dm, dA, dB, None, None, None


class _LinearF32Fn(torch.autograd.Function):
    """F.linear(x, W, b) in fp32 on the HIP GEMMs (forward, input / weight / bias gradients)."""

    @staticmethod
    def forward(ctx, x2d, W, b):
        ctx.save_for_backward(x2d, W)
        ctx.has_b = b is not None
        return ops.linear_fwd(x2d, W.detach(), None if b is None else b.detach(), out_dtype=torch.float32)

    @staticmethod
    def backward(ctx, dy):
        x2d, W = ctx.saved_tensors
        dy = dy.contiguous().float()
        ng = ctx.needs_input_grad
        dx = ops.linear_dgrad(dy, W.detach(), out_dtype=torch.float32) if ng[0] else None
        dW = ops.linear_wgrad(dy, x2d) if ng[1] else None
        db = ops.colsum(dy) if (ctx.has_b and ng[2]) else None
        return dx, dW, db


def dora_weight(m, A, Bm, D, scaling, noise=None):
    """W [out, in] = ((D + (B@A)*s [* noise]) / (||.||_col + 1e-8) * m)^T  (NEWP:447-463; with the
    dropout noise of DoRALayer.forward, NEWP:467-468)."""
    L.require_gpu(D)
    return _DoraWeightFn.apply(m, A, Bm, D, scaling, noise)


class DoRALayer(nn.Module):
    def __init__(self, original_layer, r=8, dora_alpha=16, dora_dropout=0.1):
        super().__init__()
        self.original_layer = original_layer
        self.r = r
        self.dora_alpha = dora_alpha
        self.dora_dropout = nn.Dropout(p=dora_dropout)
        with torch.no_grad():
            W = original_layer.weight.data.clone().T      # [in, out]
            S = torch.norm(W, dim=0)
            D = W / S
        self.m = nn.Parameter(S)
        self.register_buffer("D", D)
        self.delta_D_A = nn.Parameter(torch.zeros(r, original_layer.out_features))
        self.delta_D_B = nn.Parameter(torch.zeros(original_layer.in_features, r))
        self.scaling = dora_alpha / r
        self.reset_parameters()
        if original_layer.bias is not None:
            self.bias = nn.Parameter(original_layer.bias.data.clone())
        else:
            self.bias = None

    def reset_parameters(self):
        nn.init.kaiming_uniform_(self.delta_D_A, a=math.sqrt(5))
        nn.init.kaiming_uniform_(self.delta_D_B, a=math.sqrt(5))

    @property
    def weight(self):
        return dora_weight(self.m, self.delta_D_A, self.delta_D_B, self.D, self.scaling)

    def dropout_noise(self):
        """The train-mode dropout of delta_D (NEWP:468) as a multiplier: ``nn.Dropout`` applied to a
        tensor of ones shaped like delta_D [in, out] on the same device, i.e. keep-mask / (1 - p),
        with exactly the RNG draw ``self.dora_dropout(delta_D)`` makes (same shape, device and
        generator state), so ``delta_D * noise`` is the reference's ``dropout(delta_D)`` bit for bit."""
        return self.dora_dropout(torch.ones(self.D.shape, dtype=torch.float32, device=self.D.device))

    def forward(self, x):
        """NEWP:465-481: ``F.linear(x, W, bias)`` with W rebuilt from a dropped-out delta_D in
        train mode (p > 0), from ``weight`` otherwise."""
        if self.training and self.dora_dropout.p > 0:
            W = dora_weight(self.m, self.delta_D_A, self.delta_D_B, self.D, self.scaling, self.dropout_noise())
        else:
            W = self.weight
        shp = x.shape
        y = _LinearF32Fn.apply(x.reshape(-1, shp[-1]).float().contiguous(), W, self.bias)
        return y.reshape(*shp[:-1], W.shape[0])
