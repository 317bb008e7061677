"""GPU: the fp8 attention forward (BASELINE configs[4]; vit_sdpa_fwd_fp8, block-scaled OCP e4m3 on
v_mfma_scale_f32_32x32x64_f8f6f4) against

  * its CPU restatement (oracle/attn_fp8_ref.py: same block scales, same e4m3 rounding, the same
    64-key-tile online softmax): mean |o - o_ref| <= 1e-4 and max <= 3e-2 of max|o_ref| (what is
    left: f32 summation order, and exp() ulps that can flip one P element's e4m3 rounding), lse 1e-4;
  * exact attention (float64 SDPA, what timm computes): max error <= 0.12 of max|o|,
    cosine >= 0.997 (measured ~0.04-0.08 / >= 0.9986 on random q, k, v);
  * the north_star RSA bar: rho on 48 synthetic images within +-0.005 of the bf16 / fp32 paths,
    for ViT-B/16 (compute_rsa_score's CLS features, MEAS:298-355) and for CLIP-HBA ViT-L/14
    (behavioral_RSA's 66-D predictions, NEWP:605-654; frozen blocks in fp8, fp32 elsewhere).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import attn_fp8_ref as F8  # noqa: E402
from oracle import vit_ref as R  # noqa: E402

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _qkv(B, H, N, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    q, k, v = (torch.randn(B, H, N, 64, generator=g) * s for s in (1.0, 1.3, 0.7))
    q, k, v = (t.to(dtype).float() for t in (q, k, v))
    D = H * 64
    pack = lambda t: t.permute(0, 2, 1, 3).reshape(B * N, D)
    qkv = torch.cat([pack(q), pack(k), pack(v)], 1).to(dtype)
    return q, k, v, qkv


@pytest.mark.parametrize("B,H,N,causal", [(2, 2, 197, False), (2, 3, 77, True), (1, 2, 257, False),
                                          (1, 1, 300, False), (3, 2, 16, False), (1, 2, 64, True)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sdpa_fp8_matches_restatement_and_bound(B, H, N, causal, dtype):
    from vit_amd import ops
    q, k, v, qkv = _qkv(B, H, N, seed=N + B, dtype=dtype)
    o, lse = ops.sdpa_fwd(qkv.to(DEV), B, H, N, causal=causal, fp8=True)
    torch.cuda.synchronize()
    got = o.float().cpu().reshape(B, N, H, 64).permute(0, 2, 1, 3)
    ref, ref_lse = F8.sdpa_fp8(q, k, v, causal=causal)
    scale = ref.abs().max().item()
    d = (got - ref.to(dtype).float()).abs()  # o is stored in the qkv dtype
    # an exp() ulp can flip one P element's e4m3 rounding (one ulp = 1/16 of that p): rare, bounded
    assert d.max().item() <= 3e-2 * scale and d.mean().item() <= 1e-4 * scale, (d.max().item(), d.mean().item())
    assert (lse.cpu().reshape(B, H, N) - ref_lse).abs().max().item() <= 1e-4 * ref_lse.abs().max().item() + 1e-5
    ex = F8.exact_sdpa(q, k, v, causal=causal)
    err = (got - ex).abs().max().item() / ex.abs().max().item()
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ex.flatten(), dim=0).item()
    assert err <= 0.12 and cos >= 0.997, (err, cos)


def test_vit_rsa_fp8_attention_within_north_star():
    """ViT-B/16 RSA (compute_rsa_score, MEAS:298) with fp8 attention in the no-grad embedding pass:
    rho within +-0.005 of the bf16 path and of the fp32 oracle."""
    import vit_amd
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=5, random_affine=True)
    g = torch.Generator().manual_seed(9)
    imgs = torch.randn(48, 3, 224, 224, generator=g)
    rng = np.random.default_rng(11)
    ref = rng.random((48, 48))
    ref = (ref + ref.T) / 2
    np.fill_diagonal(ref, 0)
    with torch.no_grad():
        emb_o = torch.cat([R.forward_features(p, imgs[i:i + 8], cfg)[:, 0] for i in range(0, 48, 8)]).numpy()
    rho_o, _, _ = R.rsa(emb_o, ref)
    m = vit_amd.create_model("vit_base_patch16_224", compute_dtype=torch.bfloat16)
    m.load_state_dict(p)
    m = m.to(DEV).eval()
    rho_bf16, _ = vit_amd.rsa.compute_rsa_score(m, imgs.to(DEV), ref)
    m.set_attention_fp8(True)
    rho_fp8, _ = vit_amd.rsa.compute_rsa_score(m, imgs.to(DEV), ref)
    assert abs(rho_fp8 - rho_bf16) <= 0.005 and abs(rho_fp8 - rho_o) <= 0.005, (rho_fp8, rho_bf16, rho_o)
    # training forwards keep the bf16 attention (the backward needs it)
    x = imgs[:2].to(DEV)
    m.train()
    vit_amd.cross_entropy(m(x), torch.tensor([1, 2], device=DEV)).backward()


def test_clip_behavioral_rsa_fp8_attention_within_north_star():
    """CLIP-HBA ViT-L/14 (fp32, the reference's precision) with fp8 attention in the frozen blocks:
    the behavioural RSA (NEWP:605-654) on 48 synthetic images within +-0.005 of the fp32 model,
    and a training step runs (the DoRA blocks keep fp32 attention)."""
    import vit_amd
    from vit_amd import sweep as S
    torch.manual_seed(0)
    m = vit_amd.CLIPHBA(["c%d" % i for i in range(66)], "ViT-L/14", pos_embedding=True)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    m = m.to(DEV)
    g = torch.Generator().manual_seed(3)
    imgs = torch.randn(48, 3, 224, 224, generator=g).to(DEV)
    a = np.random.default_rng(1).random((48, 48))
    ref = (a + a.T) / 2
    np.fill_diagonal(ref, 0)
    rho32, _ = S.behavioral_rsa(m, imgs, ref)
    m.clip_model.set_attention_fp8(True)
    rho8, _ = S.behavioral_rsa(m, imgs, ref)
    assert abs(rho8 - rho32) <= 0.005, (rho8, rho32)
    opt = vit_amd.FusedAdamW([q for q in m.parameters() if q.requires_grad], lr=3e-4)
    loss = vit_amd.mse_loss(m(imgs[:4]), torch.randn(4, 66, device=DEV))
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
