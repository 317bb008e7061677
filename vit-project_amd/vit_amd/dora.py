"""DoRA adapter layer: drop-in for ``DoRALayer`` (NEWP:407-481).

Same constructor, parameter names (``m``, ``delta_D_A``, ``delta_D_B``, ``bias``),
buffer ``D`` and ``weight`` property, so ``apply_dora_to_ViT`` / the DoRA
checkpoint keys (NEWP:665-683) and ``nn.MultiheadAttention``'s use of
``out_proj.weight`` (quirk Q5) work unchanged.  The weight build
``W = m * (D + (B@A)*s) / (||.||_col + 1e-8)`` and its backward run as HIP
kernels (csrc/dora.hip).  ``forward(x)`` in eval mode is ``F.linear(x, W, b)`` on
the HIP GEMM; the reference's train-mode dropout on dD (NEWP:468) is never
reached on the CLIP path (MHA reads ``.weight``) and is not implemented.
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
    def forward(ctx, m, A, Bm, D, scaling):
        fin, fout = D.shape
        r = A.shape[0]
        dev = D.device
        W = torch.empty(fout, fin, dtype=torch.float32, device=dev)
        nu = torch.empty(fout, dtype=torch.float32, device=dev)
        DnT = torch.empty(fout, fin, dtype=torch.float32, device=dev)
        colsq = torch.empty(((fin + 63) // 64) * fout, dtype=torch.float32, device=dev)
        m_, A_, B_ = m.detach().contiguous(), A.detach().contiguous(), Bm.detach().contiguous()
        call("vit_dora_weight_fwd", fin, fout, r, ptr(m_), ptr(A_), ptr(B_), ptr(D.contiguous()), float(scaling),
             ptr(W), ptr(nu), ptr(DnT), ptr(colsq), L.stream_ptr(dev))
        ctx.save_for_backward(m_, A_, B_, DnT, nu)
        ctx.scaling = scaling
        return W

    @staticmethod
    def backward(ctx, gW):
        m, A, Bm, DnT, nu = ctx.saved_tensors
        fout, fin = DnT.shape
        r = A.shape[0]
        dev = DnT.device
        gW = gW.contiguous().float()
        dm = torch.empty_like(m)
        dA = torch.empty_like(A)
        dB = torch.empty_like(Bm)
        ws = ops.workspace("dora_sdDnT", fout * fin * 4, dev)
        call("vit_dora_weight_bwd", fin, fout, r, ptr(m), ptr(A), ptr(Bm), ptr(gW), ptr(DnT), float(ctx.scaling),
             ptr(nu), ptr(dm), ptr(dA), ptr(dB), ptr(ws), None, L.stream_ptr(dev))
        return dm, dA, dB, None, None


def dora_weight(m, A, Bm, D, scaling):
    """W [out, in] = ((D + (B@A)*s) / (||.||_col + 1e-8) * m)^T  (NEWP:447-463)."""
    L.require_gpu(D)
    return _DoraWeightFn.apply(m, A, Bm, D, scaling)


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

    def forward(self, x):
        if self.training and self.dora_dropout.p > 0:
            raise NotImplementedError("train-mode dD dropout (NEWP:468) is not on the CLIP-HBA path (quirk Q5)")
        W = self.weight
        shp = x.shape
        y = ops.linear_fwd(x.reshape(-1, shp[-1]).float().contiguous(), W, self.bias, out_dtype=torch.float32)
        return y.reshape(*shp[:-1], W.shape[0])
