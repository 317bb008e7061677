"""GPU: parity of the path bench.py times, at bench.py's own shapes and schedule.

bench.py's step (VIT:132-147): ViT-B/16, bs=256, compute_dtype bf16, flat gradients,
deferred weight-gradient join, the forward as two half-batch chains on two streams
(images [0, 140) on the caller's stream, [140, 256) on the side stream at the default
VIT_FWD_HALF_DELTA = 3B/64, model.fwd_split: M = 27 580 / 22 852 token rows, ragged GEMM tiles).

  (a) per-image logits and CLS features for images on both sides of the chain split
      {0, 1, hb-1, hb, 254, 255} against the CPU fp32 oracle run on those images alone
      (the forward is per-image independent): max error <= 3e-2 of the row's scale and
      cosine >= 0.999;
  (b) every parameter gradient of the bs=256 bf16 step against the HIP fp32 path on the same
      batch (the fp32 path is pinned to the golden fixtures at 1e-3 in test_gpu_parity.py):
      per-tensor cosine >= 0.999 and norm within 2 %;
  (d) the fp32 HIP path that (b) trusts, at the same bs=256 batch, against the oracle itself:
      all 256 logit rows, the loss and every parameter gradient within 1e-3 relative (north_star),
      the oracle's gradient accumulated over 16-image chunks (the mean CE is the mean of the
      chunks' means, so the chunked sum is the bs=256 gradient and the CPU memory stays small);
  (c) a 30-step bs=32 SGD loss trajectory (lr 0.02 = the reference's warm-up epoch-1 LR,
      momentum 0.9, wd 1e-4) in bf16 against the fp32 HIP path: every step within 1 % (a
      0.01-nat floor once the memorised batch's loss nears 0), and the 30-step parameter change
      of every tensor with cosine >= 0.99 between the two.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vit_ref as R  # noqa: E402

DEV = "cuda"
B = 256
from vit_amd import model as _VM  # noqa: E402
_HB = _VM.fwd_split(B)
IDX = [0, 1, _HB - 1, _HB, 254, 255]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bench_model(p, dtype):
    import vit_amd
    m = vit_amd.create_model("vit_base_patch16_224", num_classes=1000, compute_dtype=dtype)
    m.load_state_dict(p)
    m = m.to(DEV)
    m.use_flat_grads(True)
    m.set_deferred_grad_join(True)
    return m


def _grads(m, x, y):
    import vit_amd
    m.zero_grad(set_to_none=True)
    logits = m(x)
    vit_amd.cross_entropy(logits, y).backward()
    torch.cuda.synchronize()
    return logits.detach().float().cpu(), {k: q.grad.detach().float().cpu().clone() for k, q in m.named_parameters()}


@pytest.fixture(scope="module")
def batch():
    p = R.init_params(R.VIT_B16, seed=17, random_affine=True)
    g = torch.Generator().manual_seed(18)
    x = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randint(0, 1000, (B,), generator=g)
    return p, x, y


def _row_check(got, ref, what):
    for r, i in enumerate(IDX):
        a, b = got[r].flatten(), ref[r].flatten()
        err = (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)
        cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
        assert err <= 3e-2 and cos >= 0.999, (what, i, err, cos)


def test_bench_shape_logits_and_cls_match_oracle(batch):
    """(a): the bs=256 two-chain bf16 forward, rows on both chains, against the oracle."""
    from vit_amd import model as VM
    p, x, y = batch
    assert VM._FWD_HALF_DELTA[0] is None and VM._FWD_JOIN[0] == "end"  # bench defaults
    m = _bench_model(p, torch.bfloat16)
    xd, yd = x.to(DEV), y.to(DEV)
    logits, _ = _grads(m, xd, yd)               # the training forward (head on the CLS rows)
    with torch.no_grad():
        feats = m.forward_features(xd)[:, 0].float().cpu()
        ref_logits = R.forward(p, x[IDX], R.VIT_B16)
        ref_feats = R.forward_features(p, x[IDX], R.VIT_B16)[:, 0]
    _row_check(logits[IDX], ref_logits, "logits")
    _row_check(feats[IDX], ref_feats, "cls")


def test_bench_shape_gradients_match_f32_path(batch):
    """(b): every gradient of the bench step (bs=256 bf16) against the fp32 HIP path."""
    p, x, y = batch
    xd, yd = x.to(DEV), y.to(DEV)
    _, g16 = _grads(_bench_model(p, torch.bfloat16), xd, yd)
    _, g32 = _grads(_bench_model(p, torch.float32), xd, yd)
    assert g16.keys() == g32.keys() and len(g16) == 152
    worst = []
    for k in g16:
        a, b = g16[k].flatten(), g32[k].flatten()
        cos = torch.nn.functional.cosine_similarity(a.double(), b.double(), dim=0).item()
        nr = a.norm().item() / (b.norm().item() + 1e-30)
        worst.append((cos, nr, k))
        assert cos >= 0.999 and abs(nr - 1) <= 0.02, (k, cos, nr)
    print("worst cosine", min(worst))


def test_bf16_loss_trajectory_tracks_f32_30_steps():
    """(c): 30 SGD steps at bs=32, bf16 vs the fp32 HIP path, loss within 1 % at every step."""
    import vit_amd
    p = R.init_params(R.VIT_B16, seed=19, random_affine=True)
    g = torch.Generator().manual_seed(20)
    x = torch.randn(32, 3, 224, 224, generator=g).to(DEV)
    y = torch.randint(0, 1000, (32,), generator=g).to(DEV)
    traj, delta = {}, {}
    for dt in (torch.bfloat16, torch.float32):
        m = _bench_model(p, dt)
        opt = vit_amd.FusedSGD(m.parameters(), lr=0.02, momentum=0.9, weight_decay=1e-4)
        ls = []
        for _ in range(30):
            loss = vit_amd.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            ls.append(float(loss.item()))
        traj[dt] = ls
        delta[dt] = {k: (v.float().cpu() - p[k]) for k, v in m.state_dict().items()}
    a, b = traj[torch.bfloat16], traj[torch.float32]
    assert b[-1] < 0.1 * b[0]  # the batch is memorised within the 30 steps (7.19 -> ~0.5 by step 6)
    # 1 % relative, with a 0.01-nat floor once the loss has collapsed toward 0
    err = [abs(u - v) / max(abs(v), 1.0) for u, v in zip(a, b)]
    assert max(err) <= 0.01, list(zip(a, b))
    # drift: what 30 steps changed in every parameter tensor points the same way in both
    for k in delta[torch.float32]:
        u, v = delta[torch.bfloat16][k].flatten().double(), delta[torch.float32][k].flatten().double()
        cos = torch.nn.functional.cosine_similarity(u, v, dim=0).item()
        assert cos >= 0.99, (k, cos)


def test_f32_path_bs256_matches_oracle(batch):
    """(d): the fp32 HIP path at bs=256 (two-chain forward, ragged M = 27 580 / 22 852 tiles) against
    the oracle: logits of every image, the loss and all 152 gradients within 1e-3 relative."""
    import vit_amd
    p, x, y = batch
    m = _bench_model(p, torch.float32)
    m.zero_grad(set_to_none=True)
    logits = m(x.to(DEV))
    loss = vit_amd.cross_entropy(logits, y.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    got = {k: q.grad.detach().float().cpu() for k, q in m.named_parameters()}
    ref, ref_logits, ref_loss, C = None, [], 0.0, 16
    for c in range(0, B, C):
        leaf = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
        lg = R.forward(leaf, x[c:c + C], R.VIT_B16)
        lc = R.cross_entropy(lg, y[c:c + C])
        lc.backward()
        w = C / B
        ref_loss += w * float(lc.detach())
        ref_logits.append(lg.detach())
        gc = {k: v.grad.detach() * w for k, v in leaf.items()}
        ref = gc if ref is None else {k: ref[k] + gc[k] for k in ref}
    ref_logits = torch.cat(ref_logits)
    lerr = (logits.detach().float().cpu() - ref_logits).abs().max().item() / ref_logits.abs().max().item()
    assert lerr < 1e-3, lerr
    lv = float(loss.detach())
    assert abs(lv - ref_loss) < 1e-3 * abs(ref_loss), (lv, ref_loss)
    assert got.keys() == ref.keys() and len(got) == 152
    worst = 0.0
    for k in got:
        err = (got[k] - ref[k]).abs().max().item() / (ref[k].abs().max().item() + 1e-30)
        worst = max(worst, err)
        assert err < 1e-3, (k, err)
    print("logits rel", lerr, "worst gradient rel", worst)
