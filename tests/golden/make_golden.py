"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (NOT on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden.py

What it pins:
  1. The oracle's ViT restatement (oracle/vit_ref.py) against ``transformers``
     ViTForImageClassification on identical weights (timm is absent; transformers
     is an independent implementation of the same architecture).  Fixtures:
     vit_tiny_golden.pt (full grads) and vit_b16_golden.pt (bs=2 logits, CLS
     features, per-parameter grad norms + slices).
  2. The reference's own Python, imported from /root/reference with stub modules
     for the absent third-party packages (torchvision, timm, the CLIP-HBA fork):
       - DoRALayer.weight + autograd grads  (NEWP:407-463)    -> dora_golden.pt
       - behavioral_RSA                      (NEWP:605-654)    -> rsa_golden.npz
       - CosineAnnealingLRWithWarmup         (VIT:206-244)     -> lr_golden.json
       - CLIPHBA.forward + DoRALayer + apply_dora_to_ViT + switch_dora_layers +
         count_trainable_parameters (NEWP:268-304, 407-548) wrapped around a torch.nn
         OpenAI-CLIP (nn.MultiheadAttention blocks) built from oracle/clip_ref.py's
         parameters, one MSE + AdamW step                    -> clip_golden.pt
       - shuffle_targets (NEWP:731-779) and the random-target / window rules of
         train_model (NEWP:843-927), CPU generator          -> perturb_golden.pt
     The reference source itself is never copied; only input/output vectors are.
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types
from collections import OrderedDict

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import vit_ref as R  # noqa: E402
from oracle import clip_ref as CR  # noqa: E402

REF = "/root/reference"


def _stub_reference_imports():
    for name in ["torchvision", "torchvision.transforms", "torchvision.datasets", "timm", "src",
                 "src.models", "src.models.CLIPs", "src.models.CLIPs.clip_hba",
                 "src.models.clip_hba_utils"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]
    sys.modules["src.models.CLIPs.clip_hba"].clip = types.SimpleNamespace()
    sys.path.insert(0, os.path.join(REF, "Training"))
    sys.path.insert(0, os.path.join(REF, "Training", "vit_training", "baseline"))


# ----------------------------------------------------------------------------
# 1. ViT restatement vs transformers
# ----------------------------------------------------------------------------

def to_hf(p, cfg):
    from transformers import ViTConfig as HFC, ViTForImageClassification
    hc = HFC(hidden_size=cfg.embed_dim, num_hidden_layers=cfg.depth, num_attention_heads=cfg.num_heads,
             intermediate_size=cfg.mlp_dim, hidden_act="gelu", layer_norm_eps=cfg.eps,
             image_size=cfg.img_size, patch_size=cfg.patch_size, num_channels=cfg.in_chans,
             num_labels=cfg.num_classes, qkv_bias=True, hidden_dropout_prob=0.0,
             attention_probs_dropout_prob=0.0)
    m = ViTForImageClassification(hc).eval()
    D = cfg.embed_dim
    sd = OrderedDict()
    sd["vit.embeddings.cls_token"] = p["cls_token"]
    sd["vit.embeddings.position_embeddings"] = p["pos_embed"]
    sd["vit.embeddings.patch_embeddings.projection.weight"] = p["patch_embed.proj.weight"]
    sd["vit.embeddings.patch_embeddings.projection.bias"] = p["patch_embed.proj.bias"]
    for i in range(cfg.depth):
        b, h = f"blocks.{i}.", f"vit.layers.{i}."   # transformers 5.x key layout
        w, bb = p[b + "attn.qkv.weight"], p[b + "attn.qkv.bias"]
        for j, n in enumerate(["q_proj", "k_proj", "v_proj"]):
            sd[h + f"attention.{n}.weight"] = w[j * D:(j + 1) * D]
            sd[h + f"attention.{n}.bias"] = bb[j * D:(j + 1) * D]
        sd[h + "attention.o_proj.weight"] = p[b + "attn.proj.weight"]
        sd[h + "attention.o_proj.bias"] = p[b + "attn.proj.bias"]
        sd[h + "layernorm_before.weight"] = p[b + "norm1.weight"]
        sd[h + "layernorm_before.bias"] = p[b + "norm1.bias"]
        sd[h + "layernorm_after.weight"] = p[b + "norm2.weight"]
        sd[h + "layernorm_after.bias"] = p[b + "norm2.bias"]
        sd[h + "mlp.fc1.weight"] = p[b + "mlp.fc1.weight"]
        sd[h + "mlp.fc1.bias"] = p[b + "mlp.fc1.bias"]
        sd[h + "mlp.fc2.weight"] = p[b + "mlp.fc2.weight"]
        sd[h + "mlp.fc2.bias"] = p[b + "mlp.fc2.bias"]
    sd["vit.layernorm.weight"] = p["norm.weight"]
    sd["vit.layernorm.bias"] = p["norm.bias"]
    sd["classifier.weight"] = p["head.weight"]
    sd["classifier.bias"] = p["head.bias"]
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("pooler" in k for k in missing), missing
    return m


def vit_fixture(cfg, B, seed, full_grads):
    torch.manual_seed(seed)
    p = R.init_params(cfg, seed=seed, random_affine=True)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, cfg.in_chans, cfg.img_size, cfg.img_size, generator=g)
    y = torch.randint(0, cfg.num_classes, (B,), generator=g)
    with torch.no_grad():
        logits = R.forward(p, x, cfg)
        feats = R.forward_features(p, x, cfg)
        hf = to_hf(p, cfg)
        hf_logits = hf(pixel_values=x).logits
        hf_feats = hf.vit(pixel_values=x).last_hidden_state
    rel = (logits - hf_logits).abs().max() / hf_logits.abs().max()
    relf = (feats - hf_feats).abs().max() / hf_feats.abs().max()
    print(f"  oracle vs transformers: logits rel {rel:.3e}, features rel {relf:.3e}")
    assert rel < 1e-5 and relf < 1e-5
    bufs = {}
    pc = OrderedDict((k, v.clone()) for k, v in p.items())
    loss, grads = R.train_step(pc, bufs, x, y, lr=0.1, cfg=cfg)
    # grads against transformers autograd too
    hf.zero_grad()
    hl = torch.nn.functional.cross_entropy(hf(pixel_values=x).logits, y)
    hl.backward()
    gq = hf.vit.layers[0].attention.q_proj.weight.grad
    D = cfg.embed_dim
    relg = (grads["blocks.0.attn.qkv.weight"][:D] - gq).abs().max() / gq.abs().max()
    print(f"  oracle vs transformers: loss {loss:.6f} vs {float(hl):.6f}, blk0 q-grad rel {relg:.3e}")
    assert relg < 1e-4
    fx = {"seed": seed, "B": B, "cfg": cfg.__dict__, "x_sum": float(x.sum()), "y": y,
          "param_checksum": {k: float(v.double().sum()) for k, v in p.items()},
          "logits": logits, "hf_logits": hf_logits, "cls_features": feats[:, 0].clone(),
          "loss": loss, "hf_loss": float(hl),
          "grad_norm": {k: float(v.norm()) for k, v in grads.items()},
          "grad_slice": {k: v.flatten()[:64].clone() for k, v in grads.items()},
          "param_after_slice": {k: v.flatten()[:64].clone() for k, v in pc.items()}}
    if full_grads:
        fx["grads"] = grads
        fx["features"] = feats
        fx["params_after"] = pc
    return fx


# ----------------------------------------------------------------------------
# 2. reference functions imported from /root/reference
# ----------------------------------------------------------------------------

def dora_fixture():
    _stub_reference_imports()
    import functions.new_cvpr_train_behavior_things_pipeline as NEWP
    out = {}
    for (fin, fout, r) in [(96, 80, 8), (1024, 1024, 32), (768, 768, 32)]:
        torch.manual_seed(1234 + fin)
        base = torch.nn.Linear(fin, fout)
        layer = NEWP.DoRALayer(base, r=r, dora_alpha=16, dora_dropout=0.1)
        W = layer.weight
        gW = torch.randn_like(W)
        (W * gW).sum().backward()
        rec = {"in": fin, "out": fout, "r": r, "scaling": layer.scaling,
               "m": layer.m.detach().clone(), "A": layer.delta_D_A.detach().clone(),
               "B": layer.delta_D_B.detach().clone(), "D": layer.D.clone(), "gW": gW,
               "W": W.detach().clone(), "dm": layer.m.grad.clone(),
               "dA": layer.delta_D_A.grad.clone(), "dB": layer.delta_D_B.grad.clone(),
               "bias": layer.bias.detach().clone()}
        if fin > 100:  # keep the committed file small: inputs are regenerated from the seed
            rec = {k: v for k, v in rec.items() if k in ("in", "out", "r", "scaling")}
            rec.update({"seed": 1234 + fin, "W_sum": float(W.double().sum()),
                        "W_abs": float(W.double().abs().sum()), "W_row0": W[0, :64].detach().clone(),
                        "dm": layer.m.grad.clone(), "dA_norm": float(layer.delta_D_A.grad.norm()),
                        "dB_norm": float(layer.delta_D_B.grad.norm()),
                        "dA_slice": layer.delta_D_A.grad[0, :64].clone(),
                        "dB_slice": layer.delta_D_B.grad[0, :32].clone()})
        out[f"{fin}x{fout}r{r}"] = rec
    # trainable-parameter count of the CLIP-HBA DoRA setup (log: 183040)
    out["clip_trainable"] = 2 * (1024 + 32 * 1024 + 1024 * 32) + (768 + 32 * 768 + 768 * 32)
    return out


def dora_forward_fixture():
    """DoRALayer.forward in train mode (NEWP:465-481: dropout on delta_D) through the reference's own
    class on CPU, with x / bias gradients.  The dropout noise it drew is recovered by re-seeding and
    drawing nn.Dropout on ones of delta_D's shape (same RNG consumption); the fixture checks that
    the reference output equals the noise-multiplier restatement, and stores the noise so the GPU
    test can feed the identical mask to the HIP kernels."""
    _stub_reference_imports()
    import functions.new_cvpr_train_behavior_things_pipeline as NEWP
    torch.manual_seed(77)
    base = torch.nn.Linear(96, 80)
    layer = NEWP.DoRALayer(base, r=8, dora_alpha=16, dora_dropout=0.1)
    layer.train()
    x = torch.randn(6, 96, requires_grad=True)
    gy = torch.randn(6, 80)
    torch.manual_seed(78)
    y = layer(x)
    (y * gy).sum().backward()
    torch.manual_seed(78)
    noise = layer.dora_dropout(torch.ones(96, 80))
    with torch.no_grad():
        dD = (layer.delta_D_B @ layer.delta_D_A) * layer.scaling * noise
        Dn = layer.D + dD
        W = (Dn / (torch.norm(Dn, dim=0, keepdim=True) + 1e-8) * layer.m).T
        y2 = torch.nn.functional.linear(x, W, layer.bias)
    assert torch.equal(y2, y.detach()), (y2 - y).abs().max()
    assert (noise == 0).any() and ((noise == 0) | (noise == noise.max())).all()
    return {"m": layer.m.detach().clone(), "A": layer.delta_D_A.detach().clone(),
            "B": layer.delta_D_B.detach().clone(), "D": layer.D.clone(), "bias": layer.bias.detach().clone(),
            "scaling": layer.scaling, "noise": noise, "x": x.detach().clone(), "gy": gy, "y": y.detach().clone(),
            "dx": x.grad.clone(), "dm": layer.m.grad.clone(), "dA": layer.delta_D_A.grad.clone(),
            "dB": layer.delta_D_B.grad.clone(), "dbias": layer.bias.grad.clone()}


def rsa_fixture():
    _stub_reference_imports()
    import scipy.io
    import functions.new_cvpr_train_behavior_things_pipeline as NEWP
    rng = np.random.default_rng(7)
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for name, dim in [("clip66", 66), ("vit768", 768)]:
            emb = rng.standard_normal((48, dim)).astype(np.float32)
            ref = rng.integers(0, 12, size=(48, 48)).astype(np.float64) / 11.0  # ties on purpose
            ref = (ref + ref.T) / 2
            np.fill_diagonal(ref, 0)
            mat = os.path.join(td, f"{name}.mat")
            scipy.io.savemat(mat, {"RDM48_triplet": ref})

            class DS(torch.utils.data.Dataset):
                RDM48_triplet_dir = mat

                def __len__(self):
                    return 48

                def __getitem__(self, i):
                    return f"img{i:02d}", torch.from_numpy(emb[i])

            loader = torch.utils.data.DataLoader(DS(), batch_size=8, shuffle=False)
            rho, p, rdm = NEWP.behavioral_RSA(torch.nn.Identity(), loader, "cpu", logger=None)
            res[f"{name}_emb"] = emb
            res[f"{name}_ref"] = ref
            res[f"{name}_rho"] = np.float64(rho)
            res[f"{name}_p"] = np.float64(p)
            res[f"{name}_rdm"] = rdm
    return res


def lr_fixture():
    _stub_reference_imports()
    import train_vit_sgd as VIT
    net = torch.nn.Linear(2, 2)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    sch = VIT.CosineAnnealingLRWithWarmup(opt, warmup_epochs=5, max_epochs=100, eta_min=0)
    lrs = []
    for _ in range(100):
        lrs.append(opt.param_groups[0]["lr"])  # LR used while training this epoch
        sch.step()
    return {"base_lr": 0.1, "warmup_epochs": 5, "max_epochs": 100, "lr_per_epoch": lrs}


# ----------------------------------------------------------------------------
# 3. CLIP-HBA: reference wrapper + DoRA functions around a torch.nn OpenAI-CLIP
# ----------------------------------------------------------------------------

class _TorchBlock(torch.nn.Module):
    """OpenAI-CLIP ResidualAttentionBlock on torch.nn.MultiheadAttention (sequence-first)."""

    def __init__(self, w, heads, mask):
        super().__init__()
        self.attn = torch.nn.MultiheadAttention(w, heads)
        self.ln_1 = torch.nn.LayerNorm(w)
        self.mlp = torch.nn.Sequential(OrderedDict([("c_fc", torch.nn.Linear(w, 4 * w)), ("gelu", _QuickGELU()),
                                                    ("c_proj", torch.nn.Linear(4 * w, w))]))
        self.ln_2 = torch.nn.LayerNorm(w)
        self.attn_mask = mask

    def forward(self, x):
        m = None if self.attn_mask is None else self.attn_mask.to(x.dtype)
        x = x + self.attn(self.ln_1(x), self.ln_1(x), self.ln_1(x), need_weights=False, attn_mask=m)[0]
        return x + self.mlp(self.ln_2(x))


class _QuickGELU(torch.nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class _Seq(torch.nn.Module):
    def __init__(self, w, layers, heads, mask):
        super().__init__()
        self.resblocks = torch.nn.Sequential(*[_TorchBlock(w, heads, mask) for _ in range(layers)])


class _TorchCLIP(torch.nn.Module):
    def __init__(self, cfg):
        super().__init__()
        vw, tw, L = cfg.vision_width, cfg.text_width, cfg.context_length
        self.cfg = cfg
        self.visual = torch.nn.Module()
        self.visual.conv1 = torch.nn.Conv2d(3, vw, cfg.vision_patch, cfg.vision_patch, bias=False)
        self.visual.class_embedding = torch.nn.Parameter(torch.empty(vw))
        self.visual.positional_embedding = torch.nn.Parameter(torch.empty(cfg.vision_tokens, vw))
        self.visual.ln_pre = torch.nn.LayerNorm(vw)
        self.visual.transformer = _Seq(vw, cfg.vision_layers, cfg.vision_heads, None)
        self.visual.ln_post = torch.nn.LayerNorm(vw)
        self.visual.proj = torch.nn.Parameter(torch.empty(vw, cfg.embed_dim))
        self.transformer = _Seq(tw, cfg.text_layers, cfg.text_heads, torch.empty(L, L).fill_(float("-inf")).triu_(1))
        self.token_embedding = torch.nn.Embedding(cfg.vocab_size, tw)
        self.positional_embedding = torch.nn.Parameter(torch.empty(L, tw))
        self.ln_final = torch.nn.LayerNorm(tw)
        self.text_projection = torch.nn.Parameter(torch.empty(tw, cfg.embed_dim))
        self.logit_scale = torch.nn.Parameter(torch.ones([]))

    def forward(self, image, text, pos_embedding):
        v = self.visual
        x = v.conv1(image).flatten(2).permute(0, 2, 1)
        x = torch.cat([v.class_embedding + torch.zeros(x.shape[0], 1, x.shape[-1]), x], dim=1)
        if pos_embedding:
            x = x + v.positional_embedding
        x = v.ln_pre(x).permute(1, 0, 2)
        x = v.transformer.resblocks(x).permute(1, 0, 2)
        img = v.ln_post(x[:, 0, :]) @ v.proj
        text = text.reshape(-1, text.shape[-1])
        t = (self.token_embedding(text) + self.positional_embedding).permute(1, 0, 2)
        t = self.transformer.resblocks(t).permute(1, 0, 2)
        t = self.ln_final(t)
        txt = t[torch.arange(t.shape[0]), text.argmax(dim=-1)] @ self.text_projection
        img = img / img.norm(dim=1, keepdim=True)
        txt = txt / txt.norm(dim=1, keepdim=True)
        return self.logit_scale.exp() * img @ txt.t()


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def clip_fixture():
    _stub_reference_imports()
    import functions.new_cvpr_train_behavior_things_pipeline as NEWP
    cfg = CR.CLIP_TINY
    seed, B, T, r = 21, 3, 5, 8
    p = CR.init_params(cfg, seed=seed)
    tclip = _TorchCLIP(cfg)
    missing, unexpected = tclip.load_state_dict(p, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    g = torch.Generator().manual_seed(seed + 1)
    image = torch.randn(B, 3, cfg.image_resolution, cfg.image_resolution, generator=g)
    prompts = CR.synthetic_prompts(T, cfg, seed=seed + 2)
    target = torch.randn(B, T, generator=g) * 3.0 + 1.0
    # the reference wrapper, constructed without load_clip_to_cpu (network download)
    m = NEWP.CLIPHBA.__new__(NEWP.CLIPHBA)
    torch.nn.Module.__init__(m)
    m.num_clip, m.clip_model, m.pos_embedding = T, tclip.float(), True
    m.tokenized_prompts, m._cached_tokenized_prompts, m._cached_device = prompts, None, None
    for q in m.clip_model.parameters():
        q.requires_grad = False
    torch.manual_seed(seed + 3)
    NEWP.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=r, dora_dropout=0.1)
    NEWP.switch_dora_layers(m, freeze_all=True, dora_state=True)
    count = NEWP.count_trainable_parameters(m)
    names = sorted(n for n, q in m.named_parameters() if q.requires_grad)
    # oracle DoRA init must agree with the reference's on m and D; A/B are copied over
    dora = CR.init_dora(p, cfg, r=r, seed=seed + 4)
    for n, mod in m.named_modules():
        if isinstance(mod, NEWP.DoRALayer):
            key = n
            assert _rel(mod.m.detach(), dora[key + ".m"]) < 1e-6 and _rel(mod.D, dora[key + ".D"]) < 1e-6, key
            with torch.no_grad():
                mod.delta_D_A.copy_(dora[key + ".delta_D_A"])
                mod.delta_D_B.copy_(dora[key + ".delta_D_B"])
            assert mod.scaling == dora[key + ".scaling"]
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    opt.zero_grad()
    pred = m(image)
    loss = torch.nn.MSELoss()(pred, target)
    loss.backward()
    grads = {n: q.grad.detach().clone() for n, q in m.named_parameters() if q.requires_grad}
    opt.step()
    after = {n: q.detach().clone() for n, q in m.named_parameters() if q.requires_grad}
    # oracle against the reference-wrapped torch.nn model
    state = {}
    d2 = OrderedDict((k, v.clone() if torch.is_tensor(v) else v) for k, v in dora.items())
    oloss, opred, ograds = CR.train_step(p, d2, state, image, prompts, target, cfg, lr=3e-4)
    print(f"  oracle vs reference CLIPHBA: pred rel {_rel(opred, pred.detach()):.3e}, "
          f"loss {oloss:.6f} vs {float(loss):.6f}")
    assert _rel(opred, pred.detach()) < 1e-5
    for k in grads:
        assert _rel(ograds[k], grads[k]) < 1e-4, (k, _rel(ograds[k], grads[k]))
        assert _rel(d2[k], after[k]) < 1e-6, k
    return {"seed": seed, "B": B, "T": T, "r": r, "cfg": cfg.__dict__,
            "param_checksum": {k: float(v.double().sum()) for k, v in p.items()},
            "image": image, "prompts": prompts, "target": target, "pred": pred.detach(), "loss": float(loss),
            "grads": grads, "dora_after": after, "trainable_count": count, "trainable_names": names,
            "dora_A_init": {k: dora[k] for k in dora if k.endswith(".delta_D_A")},
            "dora_B_init": {k: dora[k] for k in dora if k.endswith(".delta_D_B")}}


def perturb_fixture():
    """shuffle_targets with a seeded CPU generator (NEWP:731-779, called at NEWP:959) and
    the random_target draw (NEWP:919-927) on CPU generators; window rule NEWP:844-847."""
    _stub_reference_imports()
    import functions.new_cvpr_train_behavior_things_pipeline as NEWP
    out = {"shuffle": [], "random_target": []}
    targets = torch.randn(64, 66, generator=torch.Generator().manual_seed(5))
    for (seed, run, batch) in [(0, 1, 0), (0, 37, 3), (1, 98, 22), (0, 136, 7)]:
        s = seed + run * 1000 + batch
        gen = torch.Generator()
        gen.manual_seed(s)
        out["shuffle"].append({"seed": s, "out": NEWP.shuffle_targets(targets, generator=gen)})
        gen = torch.Generator()
        gen.manual_seed(s)
        out["random_target"].append({"seed": s, "normal": torch.randn(targets.shape, dtype=torch.float32,
                                                                    generator=gen)})
    out["targets"] = targets
    return out


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    only = sys.argv[1:]
    if only:  # e.g. `make_golden.py clip perturb`: regenerate just those fixtures
        for name in only:
            fn = {"clip": (clip_fixture, "clip_golden.pt"), "perturb": (perturb_fixture, "perturb_golden.pt"),
                  "dora_fwd": (dora_forward_fixture, "dora_forward_golden.pt")}[name]
            torch.save(fn[0](), os.path.join(HERE, fn[1]))
        return
    print("ViT tiny fixture")
    torch.save(vit_fixture(R.VIT_TINY, B=3, seed=11, full_grads=True), os.path.join(HERE, "vit_tiny_golden.pt"))
    print("ViT-B/16 fixture (bs=2)")
    torch.save(vit_fixture(R.VIT_B16, B=2, seed=0, full_grads=False), os.path.join(HERE, "vit_b16_golden.pt"))
    print("DoRA fixture (reference DoRALayer)")
    torch.save(dora_fixture(), os.path.join(HERE, "dora_golden.pt"))
    torch.save(dora_forward_fixture(), os.path.join(HERE, "dora_forward_golden.pt"))
    print("RSA fixture (reference behavioral_RSA)")
    np.savez(os.path.join(HERE, "rsa_golden.npz"), **rsa_fixture())
    print("LR fixture (reference CosineAnnealingLRWithWarmup)")
    with open(os.path.join(HERE, "lr_golden.json"), "w") as f:
        json.dump(lr_fixture(), f, indent=1)
    print("CLIP-HBA fixture (reference CLIPHBA/DoRA around torch.nn CLIP)")
    torch.save(clip_fixture(), os.path.join(HERE, "clip_golden.pt"))
    print("perturbation fixture (reference shuffle_targets)")
    torch.save(perturb_fixture(), os.path.join(HERE, "perturb_golden.pt"))
    print("done")


if __name__ == "__main__":
    main()
