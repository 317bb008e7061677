"""CPU fp32 oracle for the CLIP-HBA DoRA training step.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / CPU baseline.  The product path (``vit-project_amd/vit_amd``) never
imports it.

What the reference runs (NEWP = Training/functions/new_cvpr_train_behavior_things_pipeline.py):
  CLIPHBA.forward (NEWP:287-304) -> clip_model(image, prompts[66,1,77], pos_embedding).float()
  with DoRALayer (NEWP:407-481) as ``attn.out_proj`` of the last 2 visual blocks and the
  last text block (apply_dora_to_ViT NEWP:484-513), everything else frozen
  (switch_dora_layers NEWP:516-544), nn.MSELoss (NEWP:994), AdamW (NEWP:1181).

``clip_model`` comes from the CLIP-HBA fork ``src.models.CLIPs.clip_hba`` which is NOT
vendored.  The tower arithmetic below restates OpenAI-CLIP ViT-L/14
semantics as an ASSUMPTION: conv1 without bias, class embedding + positional embedding,
ln_pre, pre-LN ResidualAttentionBlocks (nn.MultiheadAttention, QuickGELU, LN eps 1e-5),
ln_post on the CLS row, ``@ proj``; a causal text tower with EOT (argmax token id)
pooling, ``@ text_projection``; ``exp(logit_scale) * cos`` -> logits_per_image [B, T].
``pos_embedding=False`` is taken to drop the visual positional embedding (the fork's
flag semantics are unknown).  End-to-end parity for config C3 is therefore UNPINNED
against the fork; what IS pinned (tests/golden/make_golden.py -> clip_golden.pt):
  * the block arithmetic against torch.nn.MultiheadAttention (the module OpenAI CLIP
    uses), and
  * the reference's own CLIPHBA.forward, DoRALayer, apply_dora_to_ViT,
    switch_dora_layers and count_trainable_parameters, imported from /root/reference and
    applied to a torch.nn CLIP built from the same parameters, with torch's MSELoss +
    AdamW for the step.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class CLIPConfig:
    """OpenAI-CLIP hyper-parameters (ViT-L/14 defaults: SURVEY §2.2 config 3)."""
    image_resolution: int = 224
    vision_patch: int = 14
    vision_width: int = 1024
    vision_layers: int = 24
    vision_heads: int = 16
    embed_dim: int = 768
    context_length: int = 77
    vocab_size: int = 49408
    text_width: int = 768
    text_layers: int = 12
    text_heads: int = 12
    eps: float = 1e-5

    @property
    def grid(self) -> int:
        return self.image_resolution // self.vision_patch

    @property
    def vision_tokens(self) -> int:
        return self.grid ** 2 + 1


CLIP_L14 = CLIPConfig()
# parity-test size: head_dim 64 like the real towers, 17 visual tokens, 16 text tokens
CLIP_TINY = CLIPConfig(image_resolution=32, vision_patch=8, vision_width=128, vision_layers=3, vision_heads=2,
                       embed_dim=96, context_length=16, vocab_size=64, text_width=128, text_layers=2, text_heads=2)


def _block_shapes(pre: str, w: int) -> "OrderedDict[str, tuple]":
    return OrderedDict([
        (pre + "attn.in_proj_weight", (3 * w, w)), (pre + "attn.in_proj_bias", (3 * w,)),
        (pre + "attn.out_proj.weight", (w, w)), (pre + "attn.out_proj.bias", (w,)),
        (pre + "ln_1.weight", (w,)), (pre + "ln_1.bias", (w,)),
        (pre + "mlp.c_fc.weight", (4 * w, w)), (pre + "mlp.c_fc.bias", (4 * w,)),
        (pre + "mlp.c_proj.weight", (w, 4 * w)), (pre + "mlp.c_proj.bias", (w,)),
        (pre + "ln_2.weight", (w,)), (pre + "ln_2.bias", (w,)),
    ])


def param_shapes(cfg: CLIPConfig) -> "OrderedDict[str, tuple]":
    """OpenAI-CLIP state-dict keys (clip.build_model layout) and shapes."""
    vw, tw = cfg.vision_width, cfg.text_width
    s = OrderedDict()
    s["positional_embedding"] = (cfg.context_length, tw)
    s["text_projection"] = (tw, cfg.embed_dim)
    s["logit_scale"] = ()
    s["visual.class_embedding"] = (vw,)
    s["visual.positional_embedding"] = (cfg.vision_tokens, vw)
    s["visual.proj"] = (vw, cfg.embed_dim)
    s["visual.conv1.weight"] = (vw, 3, cfg.vision_patch, cfg.vision_patch)
    s["visual.ln_pre.weight"] = (vw,)
    s["visual.ln_pre.bias"] = (vw,)
    for i in range(cfg.vision_layers):
        s.update(_block_shapes(f"visual.transformer.resblocks.{i}.", vw))
    s["visual.ln_post.weight"] = (vw,)
    s["visual.ln_post.bias"] = (vw,)
    for i in range(cfg.text_layers):
        s.update(_block_shapes(f"transformer.resblocks.{i}.", tw))
    s["token_embedding.weight"] = (cfg.vocab_size, tw)
    s["ln_final.weight"] = (tw,)
    s["ln_final.bias"] = (tw,)
    return s


def init_params(cfg: CLIPConfig, seed: int = 0) -> "OrderedDict[str, torch.Tensor]":
    """Seeded OpenAI-CLIP-style init (initialize_parameters: normal with the std of each
    tensor class); LN affine and biases perturbed so every gradient term is exercised.
    Deterministic on the CPU generator (the fixtures store a checksum)."""
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for k, shp in param_shapes(cfg).items():
        t = torch.empty(shp)
        w = cfg.vision_width if k.startswith("visual.") else cfg.text_width
        if k == "logit_scale":
            t.fill_(math.log(1 / 0.07))
        elif k.endswith("ln_1.weight") or k.endswith("ln_2.weight") or k.endswith("ln_pre.weight") \
                or k.endswith("ln_post.weight") or k == "ln_final.weight":
            t.fill_(1.0).add_(torch.empty(shp).uniform_(-0.2, 0.2, generator=g))
        elif k.endswith(".bias") or k.endswith("_bias"):
            t.uniform_(-0.05, 0.05, generator=g)
        elif k in ("visual.positional_embedding", "visual.class_embedding", "visual.proj"):
            t.normal_(0.0, w ** -0.5, generator=g)
        elif k == "positional_embedding":
            t.normal_(0.0, 0.01, generator=g)
        elif k == "token_embedding.weight":
            t.normal_(0.0, 0.02, generator=g)
        elif k == "text_projection":
            t.normal_(0.0, w ** -0.5, generator=g)
        elif k == "visual.conv1.weight":
            fan_in = shp[1] * shp[2] * shp[3]
            t.uniform_(-1 / math.sqrt(fan_in), 1 / math.sqrt(fan_in), generator=g)
        else:  # in_proj / out_proj / c_fc / c_proj weights
            t.normal_(0.0, w ** -0.5 * 0.5, generator=g)
        out[k] = t
    return out


def synthetic_prompts(n: int, cfg: CLIPConfig, seed: int = 0) -> torch.Tensor:
    """[n, 1, L] int64 token ids shaped like clip.tokenize output: SOT, random ids, EOT
    (the largest id, so argmax finds it), zero padding.  The BPE tokenizer itself is out of
    scope (SURVEY §2 row 12 needs only the 66 x 77 id tensor)."""
    g = torch.Generator().manual_seed(seed)
    L, V = cfg.context_length, cfg.vocab_size
    sot, eot = V - 2, V - 1
    out = torch.zeros(n, 1, L, dtype=torch.int64)
    for i in range(n):
        k = int(torch.randint(1, L - 2, (1,), generator=g))
        out[i, 0, 0] = sot
        out[i, 0, 1:1 + k] = torch.randint(1, V - 2, (k,), generator=g)
        out[i, 0, 1 + k] = eot
    return out


# ----------------------------------------------------------------------------
# tower arithmetic (OpenAI CLIP model.py semantics, assumed; see module docstring)
# ----------------------------------------------------------------------------

def quick_gelu(x):
    return x * torch.sigmoid(1.702 * x)


def attention(p, pre, x, heads, out_w, causal):
    """nn.MultiheadAttention(x, x, x, attn_mask) with batch-first x [B, N, W]."""
    B, N, W = x.shape
    hd = W // heads
    qkv = F.linear(x, p[pre + "attn.in_proj_weight"], p[pre + "attn.in_proj_bias"])
    qkv = qkv.reshape(B, N, 3, heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    s = (q @ k.transpose(-2, -1)) * (hd ** -0.5)
    if causal:
        s = s + torch.full((N, N), float("-inf")).triu_(1)
    o = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(B, N, W)
    return F.linear(o, out_w, p[pre + "attn.out_proj.bias"])


def block(p, pre, x, heads, eps, out_w, causal=False):
    W = x.shape[-1]
    h = F.layer_norm(x, (W,), p[pre + "ln_1.weight"], p[pre + "ln_1.bias"], eps)
    x = x + attention(p, pre, h, heads, out_w, causal)
    h = F.layer_norm(x, (W,), p[pre + "ln_2.weight"], p[pre + "ln_2.bias"], eps)
    h = quick_gelu(F.linear(h, p[pre + "mlp.c_fc.weight"], p[pre + "mlp.c_fc.bias"]))
    return x + F.linear(h, p[pre + "mlp.c_proj.weight"], p[pre + "mlp.c_proj.bias"])


def dora_weight(m, A, Bm, D, scaling):
    """DoRALayer.weight (NEWP:447-463): ((D + (B@A)*s) / (||.||_col + 1e-8) * m)^T."""
    Dn = D + (Bm @ A) * scaling
    return ((Dn / (torch.norm(Dn, dim=0, keepdim=True) + 1e-8)) * m).T


def _out_w(p, dora, pre):
    key = "clip_model." + pre + "attn.out_proj"
    if dora is not None and key + ".m" in dora:
        d = dora
        return dora_weight(d[key + ".m"], d[key + ".delta_D_A"], d[key + ".delta_D_B"], d[key + ".D"],
                           d[key + ".scaling"])
    return p[pre + "attn.out_proj.weight"]


def encode_image(p, image, cfg: CLIPConfig, dora=None, pos_embedding=True):
    vw = cfg.vision_width
    x = F.conv2d(image, p["visual.conv1.weight"], None, stride=cfg.vision_patch)
    x = x.flatten(2).transpose(1, 2)
    cls = p["visual.class_embedding"].reshape(1, 1, vw).expand(x.shape[0], 1, vw)
    x = torch.cat([cls, x], dim=1)
    if pos_embedding:
        x = x + p["visual.positional_embedding"]
    x = F.layer_norm(x, (vw,), p["visual.ln_pre.weight"], p["visual.ln_pre.bias"], cfg.eps)
    for i in range(cfg.vision_layers):
        pre = f"visual.transformer.resblocks.{i}."
        x = block(p, pre, x, cfg.vision_heads, cfg.eps, _out_w(p, dora, pre))
    x = F.layer_norm(x[:, 0], (vw,), p["visual.ln_post.weight"], p["visual.ln_post.bias"], cfg.eps)
    return x @ p["visual.proj"]


def encode_text(p, text, cfg: CLIPConfig, dora=None):
    tw = cfg.text_width
    x = p["token_embedding.weight"][text] + p["positional_embedding"]
    for i in range(cfg.text_layers):
        pre = f"transformer.resblocks.{i}."
        x = block(p, pre, x, cfg.text_heads, cfg.eps, _out_w(p, dora, pre), causal=True)
    x = F.layer_norm(x, (tw,), p["ln_final.weight"], p["ln_final.bias"], cfg.eps)
    return x[torch.arange(x.shape[0]), text.argmax(dim=-1)] @ p["text_projection"]


def forward(p, image, text, cfg: CLIPConfig, dora=None, pos_embedding=True):
    """clip_model(image, prompts, pos_embedding) -> logits_per_image [B, T] (CLIPHBA.forward
    NEWP:298, prompts [T, 1, L] squeezed to [T, L])."""
    text = text.reshape(-1, text.shape[-1])
    img = encode_image(p, image, cfg, dora, pos_embedding)
    txt = encode_text(p, text, cfg, dora)
    img = img / img.norm(dim=1, keepdim=True)
    txt = txt / txt.norm(dim=1, keepdim=True)
    return p["logit_scale"].exp() * img @ txt.t()


# ----------------------------------------------------------------------------
# DoRA placement, loss and optimizer step (NEWP:484-544, 994, 1001, 1181)
# ----------------------------------------------------------------------------

def dora_targets(cfg: CLIPConfig, n_vision_layers=2, n_transformer_layers=1):
    """Block prefixes whose out_proj apply_dora_to_ViT replaces (NEWP:492-513)."""
    v = [f"visual.transformer.resblocks.{cfg.vision_layers + i}." for i in range(-n_vision_layers, 0)]
    t = [f"transformer.resblocks.{cfg.text_layers + i}." for i in range(-n_transformer_layers, 0)]
    return v + t


def init_dora(p, cfg: CLIPConfig, r=32, alpha=16, seed=0, n_vision_layers=2, n_transformer_layers=1):
    """DoRALayer.__init__ (NEWP:408-441) for each target: D = W0^T/||W0^T||_col, m = ||.||_col,
    A, B kaiming_uniform(a=sqrt 5) -> U(+-1/sqrt(fan_in)) (fan_in = out for A [r,out],
    r for B [in,r]); keys as save_dora_parameters writes them (NEWP:665-683)."""
    g = torch.Generator().manual_seed(seed)
    d = OrderedDict()
    for pre in dora_targets(cfg, n_vision_layers, n_transformer_layers):
        W = p[pre + "attn.out_proj.weight"].T
        S = torch.norm(W, dim=0)
        key = "clip_model." + pre + "attn.out_proj"
        fin, fout = W.shape
        d[key + ".m"] = S.clone()
        d[key + ".D"] = W / S
        d[key + ".delta_D_A"] = torch.empty(r, fout).uniform_(-1 / math.sqrt(fout), 1 / math.sqrt(fout), generator=g)
        d[key + ".delta_D_B"] = torch.empty(fin, r).uniform_(-1 / math.sqrt(r), 1 / math.sqrt(r), generator=g)
        d[key + ".scaling"] = alpha / r
    return d


def trainable_keys(dora):
    return [k for k in dora if k.endswith((".m", ".delta_D_A", ".delta_D_B"))]


def adamw_step(params, grads, state, lr=3e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
    """torch.optim.AdamW (default hyper-parameters, NEWP:1181) restated."""
    b1, b2 = betas
    for k in params:
        st = state.setdefault(k, {"step": 0, "m": torch.zeros_like(params[k]), "v": torch.zeros_like(params[k])})
        st["step"] += 1
        t = st["step"]
        params[k].mul_(1 - lr * weight_decay)
        st["m"].mul_(b1).add_(grads[k], alpha=1 - b1)
        st["v"].mul_(b2).addcmul_(grads[k], grads[k], value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        denom = (st["v"].sqrt() / math.sqrt(bc2)).add_(eps)
        params[k].addcdiv_(st["m"], denom, value=-lr / bc1)


def train_step(p, dora, state, image, text, target, cfg: CLIPConfig, lr=3e-4, pos_embedding=True):
    """One CLIP-HBA step (NEWP:985-1001, fp32): zero_grad, fwd, MSE, bwd, AdamW on the DoRA
    parameters.  Returns (loss, predictions, grads) with grads before the update."""
    keys = trainable_keys(dora)
    leaf = OrderedDict((k, (v.detach().clone().requires_grad_(True) if k in keys else v)) for k, v in dora.items())
    pred = forward(p, image, text, cfg, leaf, pos_embedding)
    loss = F.mse_loss(pred, target)
    loss.backward()
    grads = OrderedDict((k, leaf[k].grad.detach().clone()) for k in keys)
    with torch.no_grad():
        adamw_step(OrderedDict((k, dora[k]) for k in keys), grads, state, lr=lr)
    return float(loss.detach()), pred.detach(), grads


def visual_flops_per_image(cfg: CLIPConfig = CLIP_L14) -> float:
    """Visual-tower forward FLOPs per image (2 x MACs): 162 GFLOP for ViT-L/14."""
    N, W = cfg.vision_tokens, cfg.vision_width
    pe = cfg.grid ** 2 * W * 3 * cfg.vision_patch ** 2
    blk = N * W * 3 * W + 2 * N * N * W + N * W * W + 2 * N * W * 4 * W
    return 2.0 * (pe + cfg.vision_layers * blk + W * cfg.embed_dim)


def text_flops(cfg: CLIPConfig = CLIP_L14, n_prompts=66) -> float:
    N, W = cfg.context_length, cfg.text_width
    blk = N * W * 3 * W + 2 * N * N * W + N * W * W + 2 * N * W * 4 * W
    return 2.0 * n_prompts * (cfg.text_layers * blk + W * cfg.embed_dim)
