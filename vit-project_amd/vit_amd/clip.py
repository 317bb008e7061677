"""CLIP-HBA behind the reference's module surface, computed by HIP kernels.

Drop-in for what Training/functions/new_cvpr_train_behavior_things_pipeline.py (NEWP) builds
and calls:

  * ``CLIPHBA(classnames, backbone_name, pos_embedding)`` (NEWP:268-304): ``.clip_model``,
    ``.tokenized_prompts`` [66, 1, 77], ``forward(image)`` -> float [B, 66] (forces
    ``clip_model.eval()``, caches the prompts on the image's device);
  * ``clip_model`` with OpenAI-CLIP module/state-dict names (``visual.transformer.resblocks[i]
    .attn.out_proj``, ``transformer.resblocks[i]``, ``ln_final``, ``text_projection``...), so
    ``apply_dora_to_ViT`` / ``switch_dora_layers`` (NEWP:484-544, mirrored below) and the DoRA
    checkpoint keys of ``save_dora_parameters`` (NEWP:665-683) work unchanged;
  * ``MSELoss`` (the CBASE criterion, NEWP:994) and ``FusedAdamW`` (NEWP:1181).

The CLIP-HBA fork (``src.models.CLIPs.clip_hba``) that defines ``clip_model.forward(image,
text, pos_embedding)`` is not vendored: its arithmetic is taken to be OpenAI
CLIP's (conv1 without bias, class + positional embedding, ln_pre, pre-LN blocks with
nn.MultiheadAttention + QuickGELU, LN eps 1e-5, ln_post on CLS, ``@ proj``; causal text tower,
EOT pooling, ``@ text_projection``; ``exp(logit_scale) * cos``), with ``pos_embedding=False``
dropping the visual positional embedding.  Pretrained weights come from a network download in
the reference (``load_clip_to_cpu``, NEWP:251-265): offline the model is random-initialised,
or built from a local OpenAI state dict with :func:`build_model`.

Precision: ``compute_dtype=torch.float32`` by default, as the reference runs CLIP
(``self.clip_model.float()``, NEWP:274, no autocast on this path); ``torch.bfloat16`` is an
explicit opt-in (bf16 GEMM operands and activations, f32 accumulation and LayerNorm statistics).

Compute: every tower block is the same ``_BlockFn`` as the ViT path (MFMA GEMMs with QuickGELU
epilogues, LDS-resident attention with a causal flag, wave-per-row LayerNorm).  Only the DoRA
blocks are autograd nodes with parameters that need gradients; their backward runs just the
MLP/LN2 backward and one weight gradient (``_BlockFn`` honours ``needs_input_grad``).  The
frozen text blocks in front of the first DoRA block see the same 66 prompts every step, so
their output is cached (keyed by the prompt tensor and the parameters' versions) -- the result
is bit-identical to recomputing it.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .dora import DoRALayer
from .model import _FUSED_RESID_F32, _BlockFn, _Shadowed, _gout, _wt

SOT, EOT = 49406, 49407




def _padded_weight(mod, w2, Kp):
    """``w2`` [D, K] zero-padded to [D, Kp], cached on ``mod`` until the weight (or its bf16 shadow)
    changes: the conv1 weight is frozen on the CLIP-HBA path, so this runs once."""
    p = mod.weight
    key = (w2.data_ptr(), w2.dtype, p._version, getattr(p, "_vit_shadow_version", None), Kp)
    hit = getattr(mod, "_vit_wpad", None)
    if hit is None or hit[0] != key:
        hit = (key, ops.pad_cols(w2, Kp))
        mod._vit_wpad = hit
    return hit[1]


# ----------------------------------------------------------------------------
# autograd nodes around the towers
# ----------------------------------------------------------------------------

class _PoolHeadFn(torch.autograd.Function):
    """y = LayerNorm(x[idx]) @ proj: ln_post on the CLS rows (visual) or ln_final on the EOT
    rows (text), then the [in, out] projection -- f32, the rows gathered by a HIP kernel."""

    @staticmethod
    def forward(ctx, x, idx, nw, nb, proj, eps):
        S, Lq, D = x.shape
        x2 = x.reshape(S * Lq, D)
        xg = ops.gather_rows(x2, idx)
        ln, mean, rstd = ops.layer_norm_fwd(xg, nw.detach(), nb.detach(), eps, torch.float32)
        n, E = idx.numel(), proj.shape[1]
        pj = proj.detach().contiguous()
        y = ops.gemm(ln, L.LAY_RC, pj, L.LAY_CR, n, E, D)
        ctx.save_for_backward(idx, xg, ln, mean, rstd, pj)
        ctx.params = (nw, nb)
        ctx.meta = (S, Lq, D)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, xg, ln, mean, rstd, pj = ctx.saved_tensors
        nw, nb = ctx.params
        S, Lq, D = ctx.meta
        ng = ctx.needs_input_grad
        dy = dy.contiguous().float()
        n, E = dy.shape
        dx = dnw = dnb = dproj = None
        if ng[4]:  # proj [D, E]: dproj[d][e] = sum_i ln[i][d] dy[i][e]
            dproj = ops.gemm(ln, L.LAY_CR, dy, L.LAY_CR, D, E, n)
        if ng[0] or ng[2] or ng[3]:
            dln = ops.gemm(dy, L.LAY_RC, pj, L.LAY_RC, n, D, E)  # dln = dy @ proj^T
            dxg = torch.empty(n, D, dtype=torch.float32, device=dy.device)
            dnw = _gout(nw) if ng[2] else None
            dnb = _gout(nb) if ng[3] else None
            ops.layer_norm_bwd(xg, D, dln, nw.detach(), mean, rstd, dxg, D, n, dgamma=dnw, dbeta=dnb,
                               ws="pool_ln_partial")
            if ng[0]:
                dx = ops.zero_(torch.empty(S * Lq, D, dtype=torch.float32, device=dy.device))
                ops.scatter_rows(dxg, idx, dx)
                dx = dx.reshape(S, Lq, D)
        return dx, None, dnw, dnb, dproj, None


class _ClipLogitsFn(torch.autograd.Function):
    """logits_per_image = exp(logit_scale) * (img/||img||) @ (txt/||txt||)^T."""

    @staticmethod
    def forward(ctx, img, txt, logit_scale):
        B, E = img.shape
        T = txt.shape[0]
        ls = logit_scale.detach().reshape(1).float().contiguous()
        img_s, rn_i = ops.rownorm_fwd(img.contiguous(), ls)
        txt_n, rn_t = ops.rownorm_fwd(txt.contiguous())
        logits = ops.gemm(img_s, L.LAY_RC, txt_n, L.LAY_RC, B, T, E)
        ctx.save_for_backward(img, txt, img_s, txt_n, rn_i, rn_t, ls)
        return logits

    @staticmethod
    def backward(ctx, dl):
        img, txt, img_s, txt_n, rn_i, rn_t, ls = ctx.saved_tensors
        if ctx.needs_input_grad[2]:
            raise NotImplementedError("logit_scale is frozen on the CLIP-HBA path (switch_dora_layers, NEWP:516-544)")
        dl = dl.contiguous().float()
        B, T = dl.shape
        E = img.shape[1]
        d_img = d_txt = None
        if ctx.needs_input_grad[0]:
            d_img_s = ops.gemm(dl, L.LAY_RC, txt_n, L.LAY_CR, B, E, T)          # dl @ txt_n
            d_img = ops.rownorm_bwd(img.contiguous(), d_img_s, rn_i, ls)
        if ctx.needs_input_grad[1]:
            d_txt_n = ops.gemm(dl, L.LAY_CR, img_s, L.LAY_CR, T, E, B)          # dl^T @ img_s
            d_txt = ops.rownorm_bwd(txt.contiguous(), d_txt_n, rn_t, None)
        return d_img, d_txt, None


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        pred, target = pred.contiguous().float(), target.contiguous().float()
        ctx.save_for_backward(pred, target)
        return ops.mse_fwd(pred, target)

    @staticmethod
    def backward(ctx, g):
        pred, target = ctx.saved_tensors
        return ops.mse_bwd(pred, target, g), None


def mse_loss(pred, target):
    """nn.MSELoss()(pred, target) (mean), HIP kernels (NEWP:994)."""
    L.require_gpu(pred)
    return _MSEFn.apply(pred, target)


class MSELoss(nn.Module):
    """Drop-in for the ``criterion`` object of the CLIP configs (CBASE ``nn.MSELoss()``)."""

    def forward(self, pred, target):
        return mse_loss(pred, target)


# ----------------------------------------------------------------------------
# modules (OpenAI-CLIP key layout)
# ----------------------------------------------------------------------------

class QuickGELU(nn.Module):
    """x * sigmoid(1.702 x); applied inside the c_fc GEMM epilogue, never called on its own."""


class MultiheadAttention(nn.Module):
    """nn.MultiheadAttention's parameters (in_proj_weight/bias [3W, W], out_proj Linear)."""

    def __init__(self, width, heads):
        super().__init__()
        self.num_heads = heads
        self.head_dim = width // heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * width, width))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * width))
        self.out_proj = nn.Linear(width, width)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, width, heads, causal=False):
        super().__init__()
        self.attn = MultiheadAttention(width, heads)
        self.ln_1 = nn.LayerNorm(width, eps=1e-5)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(width, 4 * width)), ("gelu", QuickGELU()),
                                              ("c_proj", nn.Linear(4 * width, width))]))
        self.ln_2 = nn.LayerNorm(width, eps=1e-5)
        self.causal = causal

    def block_params(self):
        a, m = self.attn, self.mlp
        return (self.ln_1.weight, self.ln_1.bias, a.in_proj_weight, a.in_proj_bias, a.out_proj.weight,
                a.out_proj.bias, self.ln_2.weight, self.ln_2.bias, m.c_fc.weight, m.c_fc.bias, m.c_proj.weight,
                m.c_proj.bias)

    def gemm_weights(self):
        """Weights read by GEMMs that may get a bf16 shadow (a DoRA out_proj is computed instead)."""
        ws = [self.attn.in_proj_weight, self.mlp.c_fc.weight, self.mlp.c_proj.weight]
        if isinstance(self.attn.out_proj, nn.Linear):
            ws.append(self.attn.out_proj.weight)
        return ws


class Transformer(nn.Module):
    def __init__(self, width, layers, heads, causal=False):
        super().__init__()
        self.width, self.layers = width, layers
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, causal) for _ in range(layers)])


class VisionTransformer(nn.Module):
    """OpenAI-CLIP visual tower (the ``clip_model.visual`` the reference adapts)."""

    def __init__(self, input_resolution, patch_size, width, layers, heads, output_dim):
        super().__init__()
        self.input_resolution, self.patch_size = input_resolution, patch_size
        self.conv1 = nn.Conv2d(3, width, patch_size, patch_size, bias=False)
        self.class_embedding = nn.Parameter(torch.empty(width))
        self.positional_embedding = nn.Parameter(torch.empty((input_resolution // patch_size) ** 2 + 1, width))
        self.ln_pre = nn.LayerNorm(width, eps=1e-5)
        self.transformer = Transformer(width, layers, heads)
        self.ln_post = nn.LayerNorm(width, eps=1e-5)
        self.proj = nn.Parameter(torch.empty(width, output_dim))


def _first_trainable(blocks) -> int:
    for i, b in enumerate(blocks):
        if any(p.requires_grad for p in b.parameters()):
            return i
    return len(blocks)


class CLIP(nn.Module):
    """OpenAI-CLIP (``clip.build_model`` layout) with ``forward(image, text, pos_embedding)`` as the
    CLIP-HBA fork calls it (NEWP:298) -> logits_per_image [B, T]."""

    def __init__(self, embed_dim=768, image_resolution=224, vision_layers=24, vision_width=1024, vision_patch_size=14,
                 context_length=77, vocab_size=49408, transformer_width=768, transformer_heads=12,
                 transformer_layers=12, compute_dtype=torch.float32, cache_frozen_text=True):
        super().__init__()
        if vision_width % 64 or transformer_width % 64:
            raise ValueError("the HIP attention kernels require head_dim 64")
        self.context_length = context_length
        self.compute_dtype = compute_dtype
        self.cache_frozen_text = cache_frozen_text
        self.visual = VisionTransformer(image_resolution, vision_patch_size, vision_width, vision_layers,
                                        vision_width // 64, embed_dim)
        self.transformer = Transformer(transformer_width, transformer_layers, transformer_heads, causal=True)
        self.vocab_size = vocab_size
        self.token_embedding = nn.Embedding(vocab_size, transformer_width)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, transformer_width))
        self.ln_final = nn.LayerNorm(transformer_width, eps=1e-5)
        self.text_projection = nn.Parameter(torch.empty(transformer_width, embed_dim))
        self.logit_scale = nn.Parameter(torch.ones([]) * math.log(1 / 0.07))
        self._shadows = None
        self._text_cache = None
        self.attention_fp8 = False  # set_attention_fp8
        self.initialize_parameters()

    @torch.no_grad()
    def initialize_parameters(self, seed=None):
        """OpenAI-CLIP initialize_parameters (std per tensor class); seeded when asked."""
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        nn.init.normal_(self.token_embedding.weight, std=0.02, generator=g)
        nn.init.normal_(self.positional_embedding, std=0.01, generator=g)
        v = self.visual
        vw = v.conv1.out_channels
        nn.init.normal_(v.class_embedding, std=vw ** -0.5, generator=g)
        nn.init.normal_(v.positional_embedding, std=vw ** -0.5, generator=g)
        nn.init.normal_(v.proj, std=vw ** -0.5, generator=g)
        for tr in (v.transformer, self.transformer):
            w, n = tr.width, tr.layers
            proj_std, attn_std, fc_std = (w ** -0.5) * ((2 * n) ** -0.5), w ** -0.5, (2 * w) ** -0.5
            for blk in tr.resblocks:
                nn.init.normal_(blk.attn.in_proj_weight, std=attn_std, generator=g)
                nn.init.zeros_(blk.attn.in_proj_bias)
                out = blk.attn.out_proj
                if isinstance(out, nn.Linear):
                    nn.init.normal_(out.weight, std=proj_std, generator=g)
                    nn.init.zeros_(out.bias)
                nn.init.normal_(blk.mlp.c_fc.weight, std=fc_std, generator=g)
                nn.init.normal_(blk.mlp.c_proj.weight, std=proj_std, generator=g)
        nn.init.normal_(self.text_projection, std=self.transformer.width ** -0.5, generator=g)

    # -- plumbing ---------------------------------------------------------------
    def _ensure_shadows(self):
        dev = self.logit_scale.device
        T = self.compute_dtype
        if self._shadows is None or self._shadows_device != dev:
            self._shadows = _Shadowed()
            self._shadows_device = dev
            ws = [self.visual.conv1.weight]
            for tr in (self.visual.transformer, self.transformer):
                for blk in tr.resblocks:
                    ws += blk.gemm_weights()
            for p in ws:
                self._shadows.add(p, T)
        self._shadows.refresh()

    def set_attention_fp8(self, enable: bool = True):
        """Block-scaled e4m3 attention (vit_sdpa_fwd_fp8, BASELINE configs[4]) in every block whose
        forward needs no backward: the frozen blocks in front of the first trainable one in each
        tower (CLIP-HBA trains only the DoRA blocks 22-23 / 11, NEWP:484-544) and all blocks of a
        no-grad pass (evaluation, behavioural RSA).  Trainable blocks keep bf16/f32 attention."""
        self.attention_fp8 = bool(enable)

    def _cfg(self, heads, causal, frozen=False):
        fp8 = self.attention_fp8 and (frozen or not torch.is_grad_enabled())
        return dict(heads=heads, eps=1e-5, quick_gelu=True, dtype=self.compute_dtype, causal=causal, attn_fp8=fp8)

    # -- towers -----------------------------------------------------------------
    def encode_image(self, image, pos_embedding=True):
        L.require_gpu(image)
        self._ensure_shadows()
        v = self.visual
        stem = [v.conv1.weight, v.class_embedding, v.positional_embedding, v.ln_pre.weight, v.ln_pre.bias]
        if torch.is_grad_enabled() and any(p.requires_grad for p in stem):
            raise NotImplementedError("gradients into the CLIP visual stem are not on the CLIP-HBA path "
                                      "(switch_dora_layers freezes it, NEWP:516-544)")
        T = self.compute_dtype
        B = image.shape[0]
        ps = v.patch_size
        W = v.conv1.out_channels
        # ViT-L/14's 3*14*14 = 588 patch columns are padded to a multiple of the GEMM's 32-deep k-step
        # (zeros in U and in the weight), so the patch embedding runs on the MFMA path
        K = v.conv1.in_channels * ps * ps
        Kp = -(-K // 32) * 32
        U = ops.patch_unfold(image.to(torch.float32).contiguous(), ps, T, ld=Kp)
        npatch = U.shape[0] // B
        pos = v.positional_embedding.detach()
        if not pos_embedding:
            pos = ops.zero_(torch.empty_like(pos))
        w2 = _wt(v.conv1.weight, T).reshape(W, -1)
        if Kp != K:
            w2 = _padded_weight(v.conv1, w2, Kp)
        x = ops.patch_embed_fwd(U, w2, None, pos.contiguous(), v.class_embedding.detach().contiguous(), B, npatch)
        x2, _, _ = ops.layer_norm_fwd(x.reshape(B * (npatch + 1), W), v.ln_pre.weight.detach(),
                                      v.ln_pre.bias.detach(), 1e-5, torch.float32, need_stats=False)
        x = x2.reshape(B, npatch + 1, W)
        heads = W // 64
        blocks = list(v.transformer.resblocks)
        first = _first_trainable(blocks)
        # the residual adds run inside the next LayerNorm (as the ViT blocks, model._tokens); in f32 the
        # same f32 add as the GEMM's residual epilogue, so the reference-precision result is unchanged
        rs = ({"pending": None} if ((T != torch.float32 or _FUSED_RESID_F32[0]) and ops.add_layer_norm_supported(W))
              else None)
        for i, blk in enumerate(blocks):
            cfg = self._cfg(heads, False, frozen=i < first)
            if rs is not None:
                cfg = dict(cfg, resid=rs, resid_last=i == len(blocks) - 1)
            x = _BlockFn.apply(x, *blk.block_params(), cfg)
        idx = self._cls_rows(B, npatch + 1, x.device)
        return _PoolHeadFn.apply(x, idx, v.ln_post.weight, v.ln_post.bias, v.proj, 1e-5)

    def _cls_rows(self, B, N, dev):
        key = ("cls", B, N, dev)
        c = getattr(self, "_idx_cache", {})
        if key not in c:
            c[key] = torch.arange(B, dtype=torch.int64, device=dev) * N
            self._idx_cache = c
        return c[key]

    def _text_prefix(self, text):
        """Embedding + the frozen blocks in front of the first trainable one, cached across calls
        while the prompts and those parameters are unchanged (identical result)."""
        blocks = list(self.transformer.resblocks)
        k = _first_trainable(blocks)
        emb = [self.token_embedding.weight, self.positional_embedding]
        if torch.is_grad_enabled() and any(p.requires_grad for p in emb):
            raise NotImplementedError("gradients into the CLIP token/positional embedding are not on the "
                                      "CLIP-HBA path (switch_dora_layers freezes them, NEWP:516-544)")
        params = emb + [p for b in blocks[:k] for p in b.parameters()]
        key = (text.data_ptr(), text._version, tuple(text.shape), k, self.compute_dtype, self.attention_fp8,
               tuple((p.data_ptr(), p._version) for p in params))
        if self.cache_frozen_text and self._text_cache is not None and self._text_cache[0] == key:
            return self._text_cache[1], k
        S, Lq = text.shape
        x = ops.token_embed(text, self.token_embedding.weight.detach(), self.positional_embedding.detach())
        x = x.reshape(S, Lq, -1)
        with torch.no_grad():
            for blk in blocks[:k]:
                x = _BlockFn.apply(x, *blk.block_params(), self._cfg(blk.attn.num_heads, True, frozen=True))
        if self.cache_frozen_text:
            self._text_cache = (key, x)
        return x, k

    def encode_text(self, text):
        L.require_gpu(text)
        self._ensure_shadows()
        text = text.reshape(-1, text.shape[-1])
        x, k = self._text_prefix(text)
        for blk in list(self.transformer.resblocks)[k:]:
            x = _BlockFn.apply(x, *blk.block_params(), self._cfg(blk.attn.num_heads, True))
        c = getattr(self, "_idx_cache", {})
        key = ("eot", text.data_ptr(), text._version, tuple(text.shape))
        if key not in c:
            S, Lq = text.shape
            c[key] = torch.arange(S, device=text.device) * Lq + text.argmax(dim=-1)
            self._idx_cache = c
        return _PoolHeadFn.apply(x, c[key], self.ln_final.weight, self.ln_final.bias, self.text_projection, 1e-5)

    def forward(self, image, text, pos_embedding=True):
        img = self.encode_image(image, pos_embedding)
        txt = self.encode_text(text)
        return _ClipLogitsFn.apply(img, txt, self.logit_scale)


_BACKBONES = {
    "ViT-L/14": dict(embed_dim=768, image_resolution=224, vision_layers=24, vision_width=1024, vision_patch_size=14,
                     transformer_width=768, transformer_heads=12, transformer_layers=12),
    "ViT-B/16": dict(embed_dim=512, image_resolution=224, vision_layers=12, vision_width=768, vision_patch_size=16,
                     transformer_width=512, transformer_heads=8, transformer_layers=12),
    "ViT-B/32": dict(embed_dim=512, image_resolution=224, vision_layers=12, vision_width=768, vision_patch_size=32,
                     transformer_width=512, transformer_heads=8, transformer_layers=12),
}


def build_model(state_dict, compute_dtype=torch.float32):
    """``clip.build_model`` for ViT backbones: dimensions inferred from an OpenAI state dict."""
    vw = state_dict["visual.conv1.weight"].shape[0]
    vl = len({k.split(".")[3] for k in state_dict if k.startswith("visual.transformer.resblocks.")})
    vp = state_dict["visual.conv1.weight"].shape[-1]
    grid = round((state_dict["visual.positional_embedding"].shape[0] - 1) ** 0.5)
    tw = state_dict["ln_final.weight"].shape[0]
    m = CLIP(embed_dim=state_dict["text_projection"].shape[1], image_resolution=vp * grid, vision_layers=vl,
             vision_width=vw, vision_patch_size=vp, context_length=state_dict["positional_embedding"].shape[0],
             vocab_size=state_dict["token_embedding.weight"].shape[0], transformer_width=tw,
             transformer_heads=tw // 64,
             transformer_layers=len({k.split(".")[2] for k in state_dict if k.startswith("transformer.resblocks")}),
             compute_dtype=compute_dtype)
    sd = {k: v for k, v in state_dict.items() if k not in ("input_resolution", "context_length", "vocab_size")}
    m.load_state_dict(sd)
    return m.eval()


def tokenize(text: str, context_length=77, vocab_size=49408) -> torch.Tensor:
    """Offline stand-in for ``clip.tokenize`` (the BPE vocabulary is a download): [1, L] ids as
    SOT, one id per UTF-8 byte (byte + 1, below SOT), EOT, zero padding -- same shape, same EOT
    argmax pooling.  Pass real ``clip.tokenize`` output as ``tokenized_prompts`` when available."""
    ids = [SOT] + [b + 1 for b in text.encode("utf-8")][:context_length - 2] + [EOT]
    out = torch.zeros(1, context_length, dtype=torch.int64)
    out[0, :len(ids)] = torch.tensor(ids)
    if vocab_size != 49408:  # shrunken test vocabularies: keep SOT/EOT the two largest ids
        out[0, 0] = vocab_size - 2
        out[0, len(ids) - 1] = vocab_size - 1
        out[0, 1:len(ids) - 1] = out[0, 1:len(ids) - 1] % (vocab_size - 3) + 1
    return out


class CLIPHBA(nn.Module):
    """NEWP:268-304.  ``clip_model`` / ``tokenized_prompts`` may be given (e.g. a model from
    :func:`build_model` and real ``clip.tokenize`` ids); otherwise a random-init backbone of
    ``backbone_name`` and :func:`tokenize` ids are used (no network)."""

    def __init__(self, classnames, backbone_name="ViT-L/14", pos_embedding=False, clip_model=None,
                 tokenized_prompts=None, compute_dtype=torch.float32, attention_fp8=False):
        super().__init__()
        self.num_clip = len(classnames)
        if clip_model is None:
            if backbone_name not in _BACKBONES:
                raise NotImplementedError(f"backbone {backbone_name!r}: the CLIP-HBA configs use ViT-L/14 (CBASE:16); "
                                          f"available {sorted(_BACKBONES)}")
            clip_model = CLIP(compute_dtype=compute_dtype, **_BACKBONES[backbone_name])
        self.clip_model = clip_model
        self.clip_model.float()
        if attention_fp8:  # BASELINE configs[4]: fp8 attention in the frozen / no-grad blocks
            self.clip_model.set_attention_fp8(True)
        self.pos_embedding = pos_embedding
        for p in self.clip_model.parameters():
            p.requires_grad = False
        if tokenized_prompts is None:
            tokenized_prompts = torch.stack([tokenize(c, clip_model.context_length, clip_model.vocab_size)
                                             for c in classnames])
        self.tokenized_prompts = tokenized_prompts
        self._cached_tokenized_prompts = None
        self._cached_device = None

    def forward(self, image):
        if self.clip_model.training:
            self.clip_model.eval()
        device = image.device
        if self._cached_tokenized_prompts is None or self._cached_device != device:
            self._cached_tokenized_prompts = self.tokenized_prompts.to(device)
            self._cached_device = device
        pred_score = self.clip_model(image, self._cached_tokenized_prompts, self.pos_embedding)
        return pred_score.float()


# ----------------------------------------------------------------------------
# DoRA placement / freezing (NEWP:484-548), same semantics on these modules
# ----------------------------------------------------------------------------

def apply_dora_to_ViT(model, n_vision_layers=1, n_transformer_layers=1, r=8, dora_dropout=0.1, seed=123):
    """Replace ``attn.out_proj`` of the last n visual / text blocks with :class:`DoRALayer`
    (NEWP:484-513; ``seed`` is accepted and unused, as in the reference)."""
    mm = model.module if isinstance(model, nn.DataParallel) else model
    for idx in range(-n_vision_layers, 0):
        blk = mm.clip_model.visual.transformer.resblocks[idx]
        blk.attn.out_proj = DoRALayer(blk.attn.out_proj, r=r, dora_dropout=dora_dropout)
    for idx in range(-n_transformer_layers, 0):
        blk = mm.clip_model.transformer.resblocks[idx]
        blk.attn.out_proj = DoRALayer(blk.attn.out_proj, r=r, dora_dropout=dora_dropout)
    mm.clip_model._shadows = None  # the GEMM-weight registry changes with the modules


def switch_dora_layers(model, freeze_all=True, dora_state=True):
    """NEWP:516-544: freeze everything, then (un)freeze m / delta_D_A / delta_D_B of DoRA layers."""
    for _, p in model.named_parameters():
        p.requires_grad = not freeze_all
    if freeze_all:
        def rec(module):
            for child in module.children():
                if isinstance(child, DoRALayer):
                    child.m.requires_grad = dora_state
                    child.delta_D_A.requires_grad = dora_state
                    child.delta_D_B.requires_grad = dora_state
                    if child.bias is not None:
                        child.bias.requires_grad = False
                else:
                    rec(child)
        rec(model.module if isinstance(model, nn.DataParallel) else model)


def count_trainable_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
