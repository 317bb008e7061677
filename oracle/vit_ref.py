"""CPU fp32 oracle for the ViT training-step hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / CPU baseline.  The product path (``vit-project_amd/vit_amd``) never
imports it and fails loudly when its HIP library is missing.

This is a plain-PyTorch (CPU, fp32) restatement of what the reference runs on
its hot path.  The reference itself calls into timm (external, not vendored,
version unpinned: SURVEY.md §8c), so the model arithmetic below restates timm
``vit_base_patch16_224`` semantics and is pinned by

  * ``transformers`` ``ViTForImageClassification`` run in this container on the
    same weights (tests/golden/make_golden.py, fixture ``vit_tiny_golden.pt``
    and ``vit_b16_golden.pt``), and
  * the reference's own Python functions imported here with stubs for the
    absent third-party modules (DoRALayer.weight, behavioral_RSA,
    CosineAnnealingLRWithWarmup -> fixtures ``dora_golden.pt``,
    ``rsa_golden.npz``, ``lr_golden.json``).

Reference call sites restated (all paths under /root/reference):
  Training/vit_training/baseline/train_vit_sgd.py            (VIT)
  Training/vit_training/single_epoch/measure_single_epoch_perturbation_effect.py (MEAS)
  Training/functions/new_cvpr_train_behavior_things_pipeline.py (NEWP)
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class ViTConfig:
    """timm ``vit_base_patch16_224`` hyper-parameters (VIT:283, MEAS:467)."""
    img_size: int = 224
    patch_size: int = 16
    in_chans: int = 3
    embed_dim: int = 768
    depth: int = 12
    num_heads: int = 12
    mlp_ratio: float = 4.0
    num_classes: int = 1000
    eps: float = 1e-6           # timm LayerNorm eps for ViT
    quick_gelu: bool = False    # OpenAI-CLIP towers use QuickGELU

    @property
    def num_patches(self) -> int:
        return (self.img_size // self.patch_size) ** 2

    @property
    def seq_len(self) -> int:
        return self.num_patches + 1

    @property
    def head_dim(self) -> int:
        return self.embed_dim // self.num_heads

    @property
    def mlp_dim(self) -> int:
        return int(self.embed_dim * self.mlp_ratio)


VIT_B16 = ViTConfig()
VIT_TINY = ViTConfig(img_size=32, patch_size=16, embed_dim=128, depth=2, num_heads=2,
                     num_classes=10)


def param_shapes(cfg: ViTConfig) -> "OrderedDict[str, tuple]":
    """timm state_dict key names and shapes."""
    D, P, C = cfg.embed_dim, cfg.patch_size, cfg.in_chans
    s = OrderedDict()
    s["cls_token"] = (1, 1, D)
    s["pos_embed"] = (1, cfg.seq_len, D)
    s["patch_embed.proj.weight"] = (D, C, P, P)
    s["patch_embed.proj.bias"] = (D,)
    for i in range(cfg.depth):
        b = f"blocks.{i}."
        s[b + "norm1.weight"] = (D,)
        s[b + "norm1.bias"] = (D,)
        s[b + "attn.qkv.weight"] = (3 * D, D)
        s[b + "attn.qkv.bias"] = (3 * D,)
        s[b + "attn.proj.weight"] = (D, D)
        s[b + "attn.proj.bias"] = (D,)
        s[b + "norm2.weight"] = (D,)
        s[b + "norm2.bias"] = (D,)
        s[b + "mlp.fc1.weight"] = (cfg.mlp_dim, D)
        s[b + "mlp.fc1.bias"] = (cfg.mlp_dim,)
        s[b + "mlp.fc2.weight"] = (D, cfg.mlp_dim)
        s[b + "mlp.fc2.bias"] = (D,)
    s["norm.weight"] = (D,)
    s["norm.bias"] = (D,)
    s["head.weight"] = (cfg.num_classes, D)
    s["head.bias"] = (cfg.num_classes,)
    return s


def init_params(cfg: ViTConfig, seed: int = 0, random_affine: bool = False) -> "OrderedDict[str, torch.Tensor]":
    """Seeded timm-style init: Linear trunc_normal(0.02), zero bias,
    pos trunc_normal(0.02), cls normal(1e-6), conv default kaiming-uniform, LN (1, 0).

    ``random_affine`` perturbs LN affine params and biases so that parity tests
    exercise every term of every gradient (zero biases would hide bias bugs).
    """
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for k, shp in param_shapes(cfg).items():
        t = torch.empty(shp)
        if k == "cls_token":
            t.normal_(0.0, 1e-6, generator=g)
        elif k == "pos_embed":
            _trunc_normal(t, 0.02, g)
        elif k == "patch_embed.proj.weight":
            fan_in = shp[1] * shp[2] * shp[3]
            bound = 1.0 / math.sqrt(fan_in)
            t.uniform_(-bound, bound, generator=g)
        elif k == "patch_embed.proj.bias":
            fan_in = cfg.in_chans * cfg.patch_size ** 2
            bound = 1.0 / math.sqrt(fan_in)
            t.uniform_(-bound, bound, generator=g)
        elif k.endswith("norm1.weight") or k.endswith("norm2.weight") or k == "norm.weight":
            t.fill_(1.0)
            if random_affine:
                t.add_(torch.empty(shp).uniform_(-0.2, 0.2, generator=g))
        elif k.endswith("norm1.bias") or k.endswith("norm2.bias") or k == "norm.bias":
            t.zero_()
            if random_affine:
                t.uniform_(-0.1, 0.1, generator=g)
        elif k.endswith(".weight"):
            _trunc_normal(t, 0.02, g)
        elif k.endswith(".bias"):
            t.zero_()
            if random_affine:
                t.uniform_(-0.05, 0.05, generator=g)
        else:  # pragma: no cover
            raise KeyError(k)
        out[k] = t
    return out


def _trunc_normal(t: torch.Tensor, std: float, g: torch.Generator) -> None:
    # timm trunc_normal_(std) truncates at +-2 (absolute), i.e. at 100 sigma for 0.02:
    # effectively a plain normal.  Restated as normal + clamp.
    t.normal_(0.0, std, generator=g).clamp_(-2.0, 2.0)


# ----------------------------------------------------------------------------
# model arithmetic (timm VisionTransformer, external)
# ----------------------------------------------------------------------------

def patch_embed(p, x, cfg: ViTConfig):
    """Conv2d(k=16, s=16) -> flatten(2).transpose(1,2); prepend cls; add pos (a3, a4)."""
    y = F.conv2d(x, p["patch_embed.proj.weight"], p["patch_embed.proj.bias"], stride=cfg.patch_size)
    y = y.flatten(2).transpose(1, 2)
    cls = p["cls_token"].expand(x.shape[0], -1, -1)
    return torch.cat([cls, y], dim=1) + p["pos_embed"]


def gelu(x, cfg: ViTConfig):
    if cfg.quick_gelu:
        return x * torch.sigmoid(1.702 * x)
    return F.gelu(x)  # exact erf GELU (timm nn.GELU)


def attention(p, pre, x, cfg: ViTConfig):
    """qkv -> reshape [B,N,3,H,hd] -> permute -> softmax(q k^T * hd^-0.5) v -> proj (a7)."""
    B, N, D = x.shape
    H, hd = cfg.num_heads, cfg.head_dim
    qkv = F.linear(x, p[pre + "attn.qkv.weight"], p[pre + "attn.qkv.bias"])
    qkv = qkv.reshape(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    s = (q @ k.transpose(-2, -1)) * (hd ** -0.5)
    a = torch.softmax(s, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B, N, D)
    return F.linear(o, p[pre + "attn.proj.weight"], p[pre + "attn.proj.bias"])


def block(p, i, x, cfg: ViTConfig):
    """x += attn(norm1(x)); x += mlp(norm2(x))  (a5, a6, a8)."""
    pre = f"blocks.{i}."
    D = cfg.embed_dim
    h = F.layer_norm(x, (D,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], cfg.eps)
    x = x + attention(p, pre, h, cfg)
    h = F.layer_norm(x, (D,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], cfg.eps)
    h = gelu(F.linear(h, p[pre + "mlp.fc1.weight"], p[pre + "mlp.fc1.bias"]), cfg)
    return x + F.linear(h, p[pre + "mlp.fc2.weight"], p[pre + "mlp.fc2.bias"])


def forward_features(p, x, cfg: ViTConfig = VIT_B16):
    """timm ``forward_features`` (used at MEAS:309): post-norm tokens [B, N, D]."""
    x = patch_embed(p, x, cfg)
    for i in range(cfg.depth):
        x = block(p, i, x, cfg)
    return F.layer_norm(x, (cfg.embed_dim,), p["norm.weight"], p["norm.bias"], cfg.eps)


def forward(p, x, cfg: ViTConfig = VIT_B16):
    """timm ``forward`` (VIT:139): token pool (global_pool='token') + head (a9)."""
    f = forward_features(p, x, cfg)
    return F.linear(f[:, 0], p["head.weight"], p["head.bias"])


def cross_entropy(logits, target):
    """mean -log softmax[target] (VIT:140, a10)."""
    return F.cross_entropy(logits, target)


# ----------------------------------------------------------------------------
# optimizer step (torch.optim.SGD semantics, VIT:294-299, a11)
# ----------------------------------------------------------------------------

def sgd_step(params, grads, bufs, lr, momentum=0.9, weight_decay=1e-4, first_step=None):
    """torch.optim.SGD (dampening 0, nesterov False) restated:
    d = g + wd*p; buf = d (first step) else momentum*buf + d; p -= lr*buf."""
    for k in params:
        g = grads[k]
        d = g + weight_decay * params[k] if weight_decay != 0 else g
        if momentum != 0:
            if bufs.get(k) is None:
                bufs[k] = d.clone()
            else:
                bufs[k].mul_(momentum).add_(d)
            d = bufs[k]
        params[k].sub_(lr * d)


def train_step(p, bufs, x, y, lr, cfg: ViTConfig = VIT_B16, momentum=0.9, weight_decay=1e-4):
    """One reference step (VIT:136-144, fp32): zero_grad, fwd, CE, bwd, SGD.
    Returns (loss, grads) with grads *before* the update."""
    leaf = OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in p.items())
    loss = cross_entropy(forward(leaf, x, cfg), y)
    loss.backward()
    grads = OrderedDict((k, v.grad.detach().clone()) for k, v in leaf.items())
    with torch.no_grad():
        sgd_step(p, grads, bufs, lr, momentum, weight_decay)
    return float(loss.detach()), grads


# ----------------------------------------------------------------------------
# LR schedule (CosineAnnealingLRWithWarmup, VIT:206-244, a12, quirk Q1)
# ----------------------------------------------------------------------------

def lr_for_epoch(epoch: int, base_lr=0.1, warmup_epochs=5, max_epochs=100, eta_min=0.0) -> float:
    """LR in effect while training ``epoch``.  The scheduler is stepped only after
    each epoch (VIT:352), so epoch 0 trains at base_lr (quirk Q1); epoch e>0 trains
    at the value step() set at the end of epoch e-1 (VIT:216-228)."""
    if epoch == 0:
        return base_lr
    c = epoch - 1  # current_epoch inside the step() that produced this LR
    if c < warmup_epochs:
        return base_lr * ((c + 1) / warmup_epochs)
    progress = (c - warmup_epochs) / (max_epochs - warmup_epochs)
    return eta_min + (base_lr - eta_min) * 0.5 * (1 + math.cos(math.pi * progress))


# ----------------------------------------------------------------------------
# DoRA weight (NEWP:447-463, a16) and init (NEWP:408-441, a17)
# ----------------------------------------------------------------------------

def dora_weight(m, A, Bm, D, scaling):
    """W = ((D + (B@A)*s) / (||.||_col + 1e-8)) * m, transposed -> [out, in]."""
    delta = (Bm @ A) * scaling
    Dn = D + delta
    norms = torch.norm(Dn, dim=0, keepdim=True) + 1e-8
    return ((Dn / norms) * m).T


# ----------------------------------------------------------------------------
# RSA (behavioral_RSA NEWP:605-654 / compute_rsa_score MEAS:298-355, a14)
# ----------------------------------------------------------------------------

def model_rdm(emb: np.ndarray) -> np.ndarray:
    r = 1 - np.corrcoef(np.asarray(emb, dtype=np.float64))
    np.fill_diagonal(r, 0)
    return r


def rsa(emb: np.ndarray, ref_rdm: np.ndarray):
    from scipy.stats import spearmanr
    rdm = model_rdm(emb)
    iu = np.triu_indices_from(ref_rdm, k=1)
    rho, p = spearmanr(ref_rdm[iu], rdm[iu])
    return float(rho), float(p), rdm


def vit_flops_per_image(cfg: ViTConfig = VIT_B16) -> float:
    """Forward FLOPs per image (2 x MACs), SURVEY §8d: 35.128 GFLOP for ViT-B/16."""
    N, D, Dm, P = cfg.seq_len, cfg.embed_dim, cfg.mlp_dim, cfg.num_patches
    pe = P * D * cfg.in_chans * cfg.patch_size ** 2
    blk = N * D * 3 * D + 2 * N * N * D + N * D * D + 2 * N * D * Dm
    head = D * cfg.num_classes
    return 2.0 * (pe + cfg.depth * blk + head)
