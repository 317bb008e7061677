"""CLIP-HBA DoRA step.

CPU (-m "not gpu"):
  * the oracle (oracle/clip_ref.py) against clip_golden.pt, which was produced by the
    reference's own CLIPHBA.forward + DoRALayer + apply_dora_to_ViT + switch_dora_layers
    around a torch.nn (nn.MultiheadAttention) OpenAI-CLIP, MSELoss and torch AdamW;
  * the product modules' surface: OpenAI-CLIP state-dict keys, DoRA placement, trainable
    parameter names and count (183 040 at ViT-L/14, the logged value; the reference's count
    for the tiny fixture model);
  * perturbation rules (vit_amd.perturb) against perturb_golden.pt (reference shuffle_targets).
GPU (-m gpu): the HIP path against the golden step.  Tolerances: f32 compute 1e-3 relative
(north_star) on predictions, loss, DoRA gradients and post-AdamW parameters; bf16 compute:
predictions 3e-2 of scale, loss 3e-2, gradients 1e-1 (bf16 GEMM operands through 3 towers).
The fork's clip_model arithmetic itself is UNPINNED (not vendored, oracle docstring).
"""
import os

import pytest
import torch

from oracle import clip_ref as CR

CFG = CR.CLIP_TINY


@pytest.fixture(scope="module")
def gold(golden_dir):
    return torch.load(os.path.join(golden_dir, "clip_golden.pt"), weights_only=True)


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _oracle_dora(gold, p):
    d = CR.init_dora(p, CFG, r=gold["r"], seed=0)
    for k in d:
        if k.endswith(".delta_D_A"):
            d[k] = gold["dora_A_init"][k].clone()
        elif k.endswith(".delta_D_B"):
            d[k] = gold["dora_B_init"][k].clone()
    return d


def test_oracle_matches_reference_clip_hba_step(gold):
    p = CR.init_params(CFG, seed=gold["seed"])
    for k, v in p.items():
        ref = gold["param_checksum"][k]
        assert abs(float(v.double().sum()) - ref) <= 1e-6 * max(1.0, abs(ref)), k
    d = _oracle_dora(gold, p)
    loss, pred, grads = CR.train_step(p, d, {}, gold["image"], gold["prompts"], gold["target"], CFG, lr=3e-4)
    assert _rel(pred, gold["pred"]) < 1e-5
    assert abs(loss - gold["loss"]) <= 1e-5 * abs(gold["loss"])
    for k, g in gold["grads"].items():
        assert _rel(grads[k], g) < 1e-4, k
        assert _rel(d[k], gold["dora_after"][k]) < 1e-6, k


def _tiny_clip(dtype=torch.float32):
    from vit_amd import clip
    return clip.CLIP(embed_dim=CFG.embed_dim, image_resolution=CFG.image_resolution, vision_layers=CFG.vision_layers,
                     vision_width=CFG.vision_width, vision_patch_size=CFG.vision_patch,
                     context_length=CFG.context_length, vocab_size=CFG.vocab_size, transformer_width=CFG.text_width,
                     transformer_heads=CFG.text_heads, transformer_layers=CFG.text_layers, compute_dtype=dtype)


def _hba(gold, dtype):
    import vit_amd
    cm = _tiny_clip(dtype)
    cm.load_state_dict(CR.init_params(CFG, seed=gold["seed"]), strict=True)
    m = vit_amd.CLIPHBA([f"c{i}" for i in range(gold["T"])], "ViT-L/14", pos_embedding=True, clip_model=cm,
                        tokenized_prompts=gold["prompts"])
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=gold["r"], dora_dropout=0.1)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    with torch.no_grad():
        for n, q in m.named_parameters():
            if n.endswith(".delta_D_A"):
                q.copy_(gold["dora_A_init"][n])
            elif n.endswith(".delta_D_B"):
                q.copy_(gold["dora_B_init"][n])
    return m


def test_module_surface_matches_reference(gold):
    import vit_amd
    m = _hba(gold, torch.float32)
    assert vit_amd.count_trainable_parameters(m) == gold["trainable_count"]
    assert sorted(n for n, q in m.named_parameters() if q.requires_grad) == gold["trainable_names"]
    keys = m.state_dict().keys()
    for blk in ("clip_model.visual.transformer.resblocks.2", "clip_model.transformer.resblocks.1"):
        for s in ("m", "delta_D_A", "delta_D_B"):
            assert f"{blk}.attn.out_proj.{s}" in keys
    # DoRA init m, D from the base out_proj (NEWP:416-425) agree with the oracle's
    d = CR.init_dora(CR.init_params(CFG, seed=gold["seed"]), CFG, r=gold["r"], seed=0)
    sd = m.state_dict()
    for k in d:
        if k.endswith(".m") or k.endswith(".D"):
            assert _rel(sd[k], d[k]) < 1e-6, k


def test_vit_l14_trainable_count_matches_log():
    """183 040 trainable parameters (training_run37 log line 62)."""
    import vit_amd
    m = vit_amd.CLIPHBA(["x"] * 66, "ViT-L/14", pos_embedding=True)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    assert vit_amd.count_trainable_parameters(m) == 183040
    assert tuple(m.tokenized_prompts.shape) == (66, 1, 77)


def test_perturbation_rules_match_reference(golden_dir):
    from vit_amd import perturb as P
    gp = torch.load(os.path.join(golden_dir, "perturb_golden.pt"), weights_only=True)
    t = gp["targets"]
    for rec in gp["shuffle"]:
        g = torch.Generator()
        g.manual_seed(rec["seed"])
        assert torch.equal(P.shuffle_targets(t, generator=g), rec["out"])
    for rec in gp["random_target"]:
        assert torch.equal(P.random_targets(t.shape, rec["seed"], "cpu", "normal"), rec["normal"])
        assert torch.allclose(P.random_targets(t.shape, rec["seed"], "cpu", "target", 1.5, 2.0),
                              rec["normal"] * 2.0 + 1.5)
    assert P.window(1, 1) == (0, 0) and P.window(37, 4) == (36, 39)
    assert P.batch_seed(0, 37, 3) == 37003
    assert not P.in_window(35, 37, 4) and P.in_window(39, 37, 4) and not P.in_window(40, 37, 4)
    es = P.EarlyStopping(patience=2, training_run=3, perturb_length=2)
    assert [es.step(e, v) for e, v in enumerate([5.0, 4.0, 6.0, 6.0, 6.0, 6.0])] == [False] * 5 + [True]
    imgs, tg = P.perturb_batch("uniform_images", torch.randn(2, 3, 4, 4), t[:2], epoch=0, batch_idx=0,
                               training_run=1, perturb_length=1, perturb_seed=0)
    assert torch.all(imgs == 0.5) and torch.equal(tg, t[:2])


# ---------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clip_hba_step_matches_golden(gold, dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vit_amd
    m = _hba(gold, dtype).cuda()
    opt = vit_amd.FusedAdamW(m.parameters(), lr=3e-4)
    opt.zero_grad()
    pred = m(gold["image"].cuda())
    loss = vit_amd.MSELoss()(pred, gold["target"].cuda())
    loss.backward()
    grads = {n: q.grad.detach().cpu().clone() for n, q in m.named_parameters() if q.requires_grad}
    opt.step()
    torch.cuda.synchronize()
    f32 = dtype == torch.float32
    assert tuple(pred.shape) == (gold["B"], gold["T"]) and pred.dtype == torch.float32
    assert _rel(pred, gold["pred"]) < (1e-3 if f32 else 3e-2)
    assert abs(float(loss.detach()) - gold["loss"]) <= (1e-3 if f32 else 3e-2) * abs(gold["loss"])
    for n, g in gold["grads"].items():
        if f32:
            assert _rel(grads[n], g) < 1e-3, (n, _rel(grads[n], g))
        else:  # bf16 opt-in: per-tensor direction and norm
            a, b = grads[n].flatten().double(), g.flatten().double()
            cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
            assert cos >= 0.99 and abs(a.norm().item() / b.norm().item() - 1) <= 0.05, (n, cos)
    after = dict(m.named_parameters())
    for n, w in gold["dora_after"].items():
        before = gold["dora_A_init"].get(n) if n.endswith("delta_D_A") else gold["dora_B_init"].get(n)
        if before is None or not f32:
            # m (large values), or bf16: AdamW's first step moves each element by ~lr * sign(g), so
            # a bf16 gradient near zero may flip an element's step; bound it against the parameter
            assert _rel(after[n], w) < (1e-5 if f32 else 1e-2), n
        else:  # f32 A, B: compare the update itself
            assert _rel(after[n].detach().cpu() - before, w - before) < 1e-3, n


@pytest.mark.gpu
def test_clip_text_cache_is_exact_and_invalidated(gold):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = _hba(gold, torch.bfloat16).cuda()
    img = gold["image"].cuda()
    with torch.no_grad():
        a = m(img)
        b = m(img)
        assert torch.equal(a, b)
        m.clip_model.cache_frozen_text = False
        c = m(img)
        assert torch.equal(a, c)
        m.clip_model.cache_frozen_text = True
        m.clip_model.transformer.resblocks[0].ln_1.bias.add_(0.5)  # a frozen prefix parameter changes
        d = m(img)
        assert not torch.equal(a, d)


@pytest.mark.gpu
def test_clip_l14_step_runs():
    """Full-size CLIPHBA ViT-L/14 + DoRA (config C3 shapes, bs=4): finite MSE step, only DoRA grads."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vit_amd
    m = vit_amd.CLIPHBA(["x%d" % i for i in range(66)], "ViT-L/14", pos_embedding=True)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    m = m.cuda()
    opt = vit_amd.FusedAdamW(m.parameters(), lr=3e-4)
    x = torch.randn(4, 3, 224, 224, device="cuda")
    y = torch.randn(4, 66, device="cuda")
    for _ in range(2):
        opt.zero_grad()
        pred = m(x)
        loss = vit_amd.mse_loss(pred, y)
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    assert tuple(pred.shape) == (4, 66) and torch.isfinite(pred).all() and torch.isfinite(loss)
    with_grad = [n for n, q in m.named_parameters() if q.grad is not None]
    assert len(with_grad) == 9 and all(n.rsplit(".", 1)[1] in ("m", "delta_D_A", "delta_D_B") for n in with_grad)


@pytest.mark.gpu
def test_sweep_condition_on_cliphba(tmp_path):
    """vit_amd.sweep on the real CLIPHBA(ViT-L/14) + DoRA: a baseline epoch, then one perturbed
    condition resumed from its files; the DoRA checkpoint keys are the reference's (NEWP:666-683)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    import vit_amd
    from vit_amd import sweep as S

    def make():
        torch.manual_seed(0)
        m = vit_amd.CLIPHBA(["c%d" % i for i in range(66)], "ViT-L/14", pos_embedding=True)
        vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
        vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
        m = m.cuda()
        return m, vit_amd.FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=3e-4)

    g = torch.Generator().manual_seed(1)
    dev = "cuda"
    mk = lambda n: (torch.randn(n, 3, 224, 224, generator=g).to(dev), (torch.randn(n, 66, generator=g) + 2).to(dev))
    a = np.random.default_rng(0).random((48, 48))
    ref = (a + a.T) / 2
    np.fill_diagonal(ref, 0)
    data = dict(train=mk(16), test=mk(8), inference=torch.randn(48, 3, 224, 224, generator=g).to(dev),
                reference_rdm=ref)
    m, opt = make()
    base = tmp_path / "base"
    rows = S.train_condition(m, opt, vit_amd.mse_loss, data, epochs=1, training_run=1, perturb_length=0,
                             perturb_type=None, batch_size=8, training_res_path=str(tmp_path / "b.csv"),
                             dora_parameters_path=str(base / "dora"), random_state_path=str(base / "rs"),
                             dataloader_generator=torch.Generator().manual_seed(0))
    assert len(rows) == 1 and np.isfinite(rows[0][1]) and np.isfinite(rows[0][3])
    sd = torch.load(str(base / "dora" / "epoch1_dora_params.pth"), weights_only=True)
    assert sorted(sd) == sorted(f"{p}.{k}" for p in S.DORA_MODULES for k in ("m", "delta_D_A", "delta_D_B"))
    done = S.run_sweep(make, vit_amd.mse_loss, data, [(2, 1)], perturb_type="label_shuffle",
                       out_dir=str(tmp_path / "sw"), baseline_dora_path=str(base / "dora"),
                       baseline_random_state_path=str(base / "rs"), epochs=2, batch_size=8)
    with open(done[0][1]) as fh:
        out = fh.read().splitlines()
    assert out[0].split(",") == S.CSV_HEADERS and out[1].split(",")[0] == "2" and out[1].split(",")[6] == "True"


def _make_fp8_cliphba():
    """CLIPHBA(ViT-L/14) + DoRA with fp8 attention in the frozen blocks (BASELINE configs[4]) and its
    AdamW -- module level so the sweep launcher's worker processes can rebuild it."""
    import vit_amd
    torch.manual_seed(0)
    m = vit_amd.CLIPHBA(["c%d" % i for i in range(66)], "ViT-L/14", pos_embedding=True, attention_fp8=True)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    m = m.cuda()
    return m, vit_amd.FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=3e-4)


@pytest.mark.gpu
def test_c5_sweep_launcher_fp8_on_cliphba(tmp_path):
    """Config C5 end to end at small scale: a baseline run, then the process-per-GPU sweep launcher
    (two worker processes sharing this box's one GPU) over a start x length grid on the real
    CLIPHBA with fp8 attention; every condition once, longer windows resumed from their siblings."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    import vit_amd
    from vit_amd import sweep as S
    g = torch.Generator().manual_seed(1)
    mk = lambda n: (torch.randn(n, 3, 224, 224, generator=g), torch.randn(n, 66, generator=g) + 2)
    a = np.random.default_rng(0).random((48, 48))
    ref = (a + a.T) / 2
    np.fill_diagonal(ref, 0)
    data = dict(train=mk(16), test=mk(8), inference=torch.randn(48, 3, 224, 224, generator=g), reference_rdm=ref)
    m, opt = _make_fp8_cliphba()
    dev = {k: (tuple(t.cuda() for t in v) if isinstance(v, tuple) else (v.cuda() if torch.is_tensor(v) else v))
           for k, v in data.items()}
    base = tmp_path / "base"
    S.train_condition(m, opt, vit_amd.mse_loss, dev, epochs=2, training_run=1, perturb_length=0, perturb_type=None,
                      batch_size=8, training_res_path=str(tmp_path / "b.csv"), dora_parameters_path=str(base / "dora"),
                      random_state_path=str(base / "rs"), dataloader_generator=torch.Generator().manual_seed(0))
    del m, opt, dev
    conds = [(2, 1), (2, 2), (3, 1)]
    res = S.launch_sweep(2, _make_fp8_cliphba, vit_amd.mse_loss, data, conds, gpus=[0], perturb_type="random_target",
                         out_dir=str(tmp_path / "sw"), baseline_dora_path=str(base / "dora"),
                         baseline_random_state_path=str(base / "rs"), epochs=4, batch_size=8, torch_threads=4)
    flat = {c: (p, src) for r in res.values() for c, p, src in r}
    assert sorted(flat) == sorted(conds)
    assert flat[(2, 2)][1] == "sibling l1" and flat[(2, 1)][1] == "baseline"
    for (e, l), (path, _) in flat.items():
        with open(path) as fh:
            rows = [r.split(",") for r in fh.read().splitlines()[1:]]
        assert [int(r[0]) for r in rows] == list(range(e, 5)) and all(np.isfinite(float(r[2])) for r in rows)


# ---------------------------------------------------------------------------- config C3 at the bench's shape

C3_IMAGES = (0, 1, 31, 32, 63)  # straddle the f32 GEMM's 128-row tiles (64 x 257 = 16 448 rows = 128.5 tiles)


@pytest.mark.gpu
def test_c3_bench_shape_matches_oracle():
    """bench.py's ``c3`` leg configuration (NEWP:274 fp32, NEWP:986-1001 step): CLIPHBA ViT-L/14 +
    DoRA r=32 on the last 2 visual blocks and the last text block, f32, bs=64, frozen-text cache on.
    (a) per-image predictions of images {0, 1, 31, 32, 63} against the oracle run on those five
    images alone (the forward is per-image independent; the rows straddle the ragged 128-row f32
    GEMM tiles); (b) the MSE loss and the 9 DoRA gradients of the bs=64 step against the oracle's
    CPU step on the same batch.  Tolerance 1e-3 relative (north_star), max-abs over each row /
    tensor.  Weights: oracle init_params(CLIP_L14) loaded into the product model; DoRA A/B as the
    product's own init drew them, copied into the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vit_amd
    from vit_amd import clip
    cfg, B = CR.CLIP_L14, 64
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    p = CR.init_params(cfg, seed=5)
    prompts = CR.synthetic_prompts(66, cfg, seed=6)
    cm = clip.build_model(p, compute_dtype=torch.float32)
    assert cm.cache_frozen_text
    m = vit_amd.CLIPHBA([f"c{i}" for i in range(66)], "ViT-L/14", pos_embedding=True, clip_model=cm,
                        tokenized_prompts=prompts)
    vit_amd.apply_dora_to_ViT(m, n_vision_layers=2, n_transformer_layers=1, r=32)
    vit_amd.switch_dora_layers(m, freeze_all=True, dora_state=True)
    sd = m.state_dict()
    d = CR.init_dora(p, cfg, r=32, seed=0)
    for k in list(d):
        if not k.endswith(".scaling"):
            if k.endswith(".m") or k.endswith(".D"):
                assert _rel(sd[k], d[k]) < 1e-6, k  # DoRALayer.__init__ (NEWP:416-425) agrees
            d[k] = sd[k].detach().clone().float()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randn(B, 66, generator=g) * 0.5 + 1.0

    m = m.cuda()
    with torch.no_grad():  # fills the frozen-text cache (bench warm-up does the same)
        m(x[:2].cuda())
    opt = vit_amd.FusedAdamW([q for q in m.parameters() if q.requires_grad], lr=3e-4)
    opt.zero_grad(set_to_none=True)
    pred = m(x.cuda())
    loss = vit_amd.mse_loss(pred, y.cuda())
    loss.backward()
    grads = {n: q.grad.detach().cpu().clone() for n, q in m.named_parameters() if q.requires_grad}
    torch.cuda.synchronize()
    pred = pred.detach().cpu()
    assert len(grads) == 9

    with torch.no_grad():
        idx = list(C3_IMAGES)
        pr5 = CR.forward(p, x[idx], prompts, cfg, d, pos_embedding=True)
    for r, i in enumerate(idx):
        assert _rel(pred[i], pr5[r]) < 1e-3, (i, _rel(pred[i], pr5[r]))
    ref_loss, ref_pred, ref_grads = CR.train_step(p, d, {}, x, prompts, y, cfg, lr=3e-4, pos_embedding=True)
    assert _rel(pred, ref_pred) < 1e-3
    assert abs(float(loss.detach()) - ref_loss) <= 1e-3 * abs(ref_loss)
    for k, rg in ref_grads.items():
        assert _rel(grads[k], rg) < 1e-3, (k, _rel(grads[k], rg))
