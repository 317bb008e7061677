"""CPU: pin the oracle (oracle/vit_ref.py) against the committed golden fixtures.

The fixtures come from transformers' ViT (independent implementation of timm's
architecture) and from the reference's own DoRALayer / behavioral_RSA /
CosineAnnealingLRWithWarmup imported from /root/reference (tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import vit_ref as R


def _load(golden_dir, name):
    return torch.load(os.path.join(golden_dir, name), weights_only=True)


def test_tiny_vit_matches_transformers_and_fixture(golden_dir):
    fx = _load(golden_dir, "vit_tiny_golden.pt")
    cfg = R.ViTConfig(**fx["cfg"])
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    for k, v in p.items():  # RNG stream unchanged
        assert abs(float(v.double().sum()) - fx["param_checksum"][k]) < 1e-6 * max(1.0, abs(fx["param_checksum"][k]))
    g = torch.Generator().manual_seed(fx["seed"] + 1)
    x = torch.randn(fx["B"], cfg.in_chans, cfg.img_size, cfg.img_size, generator=g)
    y = torch.randint(0, cfg.num_classes, (fx["B"],), generator=g)
    assert torch.equal(y, fx["y"])
    logits = R.forward(p, x, cfg)
    torch.testing.assert_close(logits, fx["logits"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(logits, fx["hf_logits"], rtol=1e-4, atol=1e-5)
    bufs = {}
    loss, grads = R.train_step(p, bufs, x, y, lr=0.1, cfg=cfg)
    assert abs(loss - fx["hf_loss"]) < 1e-5
    for k in grads:
        torch.testing.assert_close(grads[k], fx["grads"][k], rtol=1e-4, atol=1e-7)
        torch.testing.assert_close(p[k], fx["params_after"][k], rtol=1e-5, atol=1e-7)


def test_vit_b16_fixture(golden_dir):
    fx = _load(golden_dir, "vit_b16_golden.pt")
    cfg = R.ViTConfig(**fx["cfg"])
    assert cfg == R.VIT_B16
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    n = sum(v.numel() for v in p.values())
    assert n == 86_567_656  # SURVEY §4 known answer
    g = torch.Generator().manual_seed(fx["seed"] + 1)
    x = torch.randn(fx["B"], 3, 224, 224, generator=g)
    with torch.no_grad():
        logits = R.forward(p, x, cfg)
    torch.testing.assert_close(logits, fx["hf_logits"], rtol=1e-4, atol=1e-5)


def test_flops_per_image():
    f = R.vit_flops_per_image(R.VIT_B16)
    assert abs(f / 1e9 - 35.128) < 0.01, f


def test_lr_schedule_matches_reference(golden_dir):
    with open(os.path.join(golden_dir, "lr_golden.json")) as f:
        fx = json.load(f)
    for e, lr in enumerate(fx["lr_per_epoch"]):
        assert abs(R.lr_for_epoch(e, fx["base_lr"], fx["warmup_epochs"], fx["max_epochs"]) - lr) < 1e-12
    assert fx["lr_per_epoch"][0] == 0.1  # quirk Q1


def test_dora_oracle_matches_reference(golden_dir):
    fx = _load(golden_dir, "dora_golden.pt")
    rec = fx["96x80r8"]
    m = rec["m"].clone().requires_grad_(True)
    A = rec["A"].clone().requires_grad_(True)
    Bm = rec["B"].clone().requires_grad_(True)
    W = R.dora_weight(m, A, Bm, rec["D"], rec["scaling"])
    torch.testing.assert_close(W, rec["W"], rtol=1e-6, atol=1e-7)
    (W * rec["gW"]).sum().backward()
    torch.testing.assert_close(m.grad, rec["dm"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(A.grad, rec["dA"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(Bm.grad, rec["dB"], rtol=1e-5, atol=1e-7)
    assert fx["clip_trainable"] == 183040  # training_run37 log line 62


def test_rsa_oracle_and_host_rsa_match_reference(golden_dir):
    import vit_amd.rsa as HR
    fx = np.load(os.path.join(golden_dir, "rsa_golden.npz"))
    for name in ["clip66", "vit768"]:
        emb, ref = fx[f"{name}_emb"], fx[f"{name}_ref"]
        rho, p, rdm = R.rsa(emb, ref)
        assert abs(rho - float(fx[f"{name}_rho"])) < 1e-12
        np.testing.assert_allclose(rdm, fx[f"{name}_rdm"], rtol=1e-12, atol=1e-12)
        rho2, p2, rdm2 = HR.rsa(emb, ref)
        assert abs(rho2 - float(fx[f"{name}_rho"])) < 1e-12
        assert abs(p2 - float(fx[f"{name}_p"])) <= 1e-9 * max(1e-300, abs(float(fx[f"{name}_p"]))) + 1e-300
        np.testing.assert_allclose(rdm2, fx[f"{name}_rdm"], rtol=1e-12, atol=1e-12)


def test_host_spearman_ties_against_scipy():
    from scipy.stats import spearmanr
    import vit_amd.rsa as HR
    rng = np.random.default_rng(3)
    for _ in range(5):
        a = rng.integers(0, 7, 200).astype(float)
        b = rng.standard_normal(200)
        r1, p1 = HR.spearman(a, b)
        r2, p2 = spearmanr(a, b)
        assert abs(r1 - r2) < 1e-12 and abs(p1 - p2) < 1e-10


def test_sgd_restatement_matches_torch():
    torch.manual_seed(0)
    p = {"a": torch.randn(50), "b": torch.randn(7, 3)}
    q = {k: torch.nn.Parameter(v.clone()) for k, v in p.items()}
    opt = torch.optim.SGD(q.values(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    bufs = {}
    for step in range(3):
        grads = {k: torch.randn_like(v) for k, v in p.items()}
        R.sgd_step(p, grads, bufs, lr=0.1)
        for k in q:
            q[k].grad = grads[k].clone()
        opt.step()
        for k in p:
            torch.testing.assert_close(p[k], q[k].detach(), rtol=1e-6, atol=1e-7)


def test_dora_forward_fixture_is_the_noise_restatement(golden_dir):
    """dora_forward_golden.pt (the reference DoRALayer.forward in train mode, NEWP:465-481) equals
    W = m * (D + (B@A)s * noise) / (||.||_col + 1e-8), y = x W^T + b with the recorded noise --
    the restatement the HIP kernels implement (tests/test_gpu_kernels.py feeds them this noise)."""
    import torch
    fx = torch.load(os.path.join(golden_dir, "dora_forward_golden.pt"), weights_only=True)
    dD = (fx["B"] @ fx["A"]) * fx["scaling"] * fx["noise"]
    Dn = fx["D"] + dD
    W = (Dn / (torch.norm(Dn, dim=0, keepdim=True) + 1e-8) * fx["m"]).T
    assert torch.equal(torch.nn.functional.linear(fx["x"], W, fx["bias"]), fx["y"])
    keep = fx["noise"] != 0
    assert 0.8 < keep.float().mean().item() < 0.97 and torch.allclose(fx["noise"][keep], torch.tensor(1 / 0.9))


def test_fp8_attention_restatement_known_answers():
    """oracle/attn_fp8_ref.py: E8M0 block exponents (smallest e with amax <= 448 * 2^e), e4m3
    rounding, and the restated fp8 attention's distance from exact attention on random inputs."""
    import torch
    from oracle import attn_fp8_ref as F8
    a = torch.tensor([448.0, 449.0, 1.0, 0.0, 1e-30, 1.75 * 2 ** 11, 1.76 * 2 ** 11])
    assert F8.e8m0_exp(a).tolist() == [0, 1, -8, -127, -108, 3, 4]
    x = torch.tensor([[1.0, 0.1, 447.0, 3.3] * 16])
    xq = F8.quant_rows(x)
    assert xq[0, 0] == 1.0 and xq[0, 2] == 448.0 and abs(xq[0, 1] - 0.1) < 0.0079
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(1, 2, 197, 64, generator=g) for _ in range(3))
    o, lse = F8.sdpa_fp8(q, k, v)
    ex = F8.exact_sdpa(q, k, v)
    assert (o - ex).abs().max() / ex.abs().max() < 0.12
    assert torch.nn.functional.cosine_similarity(o.flatten(), ex.flatten(), dim=0) > 0.997
