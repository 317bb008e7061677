"""GPU: the full training step through the C-ABI kernels against the CPU oracle.

Tolerances (north_star: 1e-3 relative fp32 on logits / embeddings / RSA rho):
  * compute_dtype=float32 (parity path): logits, loss, every parameter gradient
    and the post-SGD parameters within 1e-3 relative of the oracle / golden
    fixture (measured ~1e-6).
  * compute_dtype=bfloat16 (performance path): logits within 3e-2 of the logit
    scale and cosine >= 0.999, loss within 2e-2; RSA rho on 48 synthetic images
    within +-0.005 of the fp32 oracle (the north_star RSA bar).
"""
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import vit_ref as R  # noqa: E402

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(cfg, params, dtype):
    import vit_amd
    m = vit_amd.VisionTransformer(img_size=cfg.img_size, patch_size=cfg.patch_size, in_chans=cfg.in_chans,
                                  num_classes=cfg.num_classes, embed_dim=cfg.embed_dim, depth=cfg.depth,
                                  num_heads=cfg.num_heads, mlp_ratio=cfg.mlp_ratio, eps=cfg.eps,
                                  compute_dtype=dtype)
    m.load_state_dict(params)
    return m.to(DEV)


def _inputs(cfg, B, seed):
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, cfg.in_chans, cfg.img_size, cfg.img_size, generator=g)
    y = torch.randint(0, cfg.num_classes, (B,), generator=g)
    return x, y


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)


def _step(model, x, y, lr=0.1):
    import vit_amd
    opt = vit_amd.FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    opt.zero_grad(set_to_none=True)
    logits = model(x.to(DEV))
    loss = vit_amd.cross_entropy(logits, y.to(DEV))
    loss.backward()
    grads = OrderedDict((k, p.grad.detach().clone()) for k, p in model.named_parameters())
    opt.step()
    torch.cuda.synchronize()
    return logits.detach(), loss.detach(), grads


def test_tiny_f32_full_step_matches_golden(golden_dir):
    fx = torch.load(os.path.join(golden_dir, "vit_tiny_golden.pt"), weights_only=True)
    cfg = R.ViTConfig(**fx["cfg"])
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    x, y = _inputs(cfg, fx["B"], fx["seed"])
    m = _model(cfg, p, torch.float32)
    with torch.no_grad():
        f = m.forward_features(x.to(DEV))
    assert _rel(f, fx["features"]) < 1e-3
    logits, loss, grads = _step(m, x, y)
    assert _rel(logits, fx["logits"]) < 1e-3
    assert abs(loss.item() - fx["loss"]) < 1e-3 * abs(fx["loss"])
    for k, g in grads.items():
        assert _rel(g, fx["grads"][k]) < 1e-3, k
    for k, v in m.state_dict().items():
        assert _rel(v, fx["params_after"][k]) < 1e-3, k
    # flat-gradient mode (the data-parallel / bench configuration) gives the same step
    m2 = _model(cfg, p, torch.float32)
    m2.use_flat_grads(True)
    _, _, grads2 = _step(m2, x, y)
    for k, g in grads2.items():
        assert _rel(g, grads[k]) < 1e-6, k
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert _rel(b, a) < 1e-6, k


def test_vit_b16_f32_step_matches_golden(golden_dir):
    fx = torch.load(os.path.join(golden_dir, "vit_b16_golden.pt"), weights_only=True)
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    x, y = _inputs(cfg, fx["B"], fx["seed"])
    m = _model(cfg, p, torch.float32)
    logits, loss, grads = _step(m, x, y)
    assert _rel(logits, fx["hf_logits"]) < 1e-3
    assert abs(loss.item() - fx["hf_loss"]) < 1e-3 * abs(fx["hf_loss"])
    for k, g in grads.items():
        n = g.norm().item()
        assert abs(n - fx["grad_norm"][k]) <= 1e-3 * fx["grad_norm"][k] + 1e-12, k
        sl = g.flatten()[:64].cpu()
        assert (sl - fx["grad_slice"][k]).abs().max().item() <= 1e-3 * max(fx["grad_norm"][k], 1e-12), k
    sd = m.state_dict()
    for k, v in fx["param_after_slice"].items():
        got = sd[k].flatten()[:64].cpu()
        assert (got - v).abs().max().item() <= 1e-3 * v.abs().max().item() + 1e-9, k


def test_vit_b16_bf16_step_close_to_oracle(golden_dir):
    fx = torch.load(os.path.join(golden_dir, "vit_b16_golden.pt"), weights_only=True)
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    x, y = _inputs(cfg, fx["B"], fx["seed"])
    m = _model(cfg, p, torch.bfloat16)
    logits, loss, grads = _step(m, x, y)
    ref = fx["hf_logits"]
    assert _rel(logits, ref) < 3e-2
    cos = torch.nn.functional.cosine_similarity(logits.cpu().flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.999
    assert abs(loss.item() - fx["hf_loss"]) < 2e-2
    # gradients: direction agrees for every parameter tensor
    for k, g in grads.items():
        assert abs(g.norm().item() - fx["grad_norm"][k]) <= 0.1 * fx["grad_norm"][k] + 1e-9, k


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rsa_rho_within_north_star(dtype):
    """RSA rho from forward_features[:,0] on 48 images within +-0.005 of the oracle."""
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
    m = _model(cfg, p, dtype).eval()
    emb = vit_amd.rsa.cls_embeddings(m, imgs.to(DEV))
    rho, _, _ = vit_amd.rsa.rsa(emb, ref)
    assert abs(rho - rho_o) <= 0.005, (rho, rho_o)
    # the MEAS:298 entry point (world 1) gives the same score
    rho2, _ = vit_amd.rsa.compute_rsa_score(m, imgs.to(DEV), ref)
    assert abs(rho2 - rho) <= 1e-6, (rho2, rho)
    if dtype == torch.float32:
        assert np.abs(emb - emb_o).max() <= 1e-3 * np.abs(emb_o).max()


def test_bf16_batch32_matches_oracle_and_graph_replay():
    """Large-grid fast paths (M = 32*197) + HIP-graph capture of fwd+bwd+SGD."""
    import vit_amd
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=3, random_affine=True)
    x, y = _inputs(cfg, 32, 3)
    with torch.no_grad():
        ref = R.forward(p, x[:4], cfg)
    m = _model(cfg, p, torch.bfloat16)
    m.use_flat_grads(True)
    opt = vit_amd.FusedSGD(m.parameters(), lr=0.05)
    xd, yd = x.to(DEV), y.to(DEV)
    with torch.no_grad():
        logits = m(xd)
    assert _rel(logits[:4], ref) < 3e-2
    # second model: same weights, graph-captured steps
    m2 = _model(cfg, p, torch.bfloat16)
    m2.use_flat_grads(True)  # fixed gradient addresses: the optimizer table is built once, outside capture
    opt2 = vit_amd.FusedSGD(m2.parameters(), lr=0.05)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(1):  # warmup builds workspaces / shadows / tables
            l2 = vit_amd.cross_entropy(m2(xd), yd)
            l2.backward()
            opt2.step()
            opt2.zero_grad(set_to_none=True)
    torch.cuda.current_stream().wait_stream(s)
    del l2
    # the warmup took one step on m2: the eager model takes its first here
    logits = m(xd)
    loss = vit_amd.cross_entropy(logits, yd)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gl = vit_amd.cross_entropy(m2(xd), yd)
        gl.backward()
        opt2.step()
    graph.replay()
    logits = m(xd)
    loss = vit_amd.cross_entropy(logits, yd)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(gl).all()
    assert abs(gl.item() - loss.item()) < 1e-3 * abs(loss.item()) + 1e-4
    for (k, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert _rel(b, a) < 1e-5, k


def test_reference_training_loop_unchanged(golden_dir):
    """VIT:132-147 as the reference writes it -- DDP wrapper (VIT:287), autocast, GradScaler,
    torch.optim.SGD (VIT:294-299), torch's F.cross_entropy -- around our model gives the
    golden step (f32 parity path, 1e-3 relative)."""
    import socket
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP
    fx = torch.load(os.path.join(golden_dir, "vit_tiny_golden.pt"), weights_only=True)
    cfg = R.ViTConfig(**fx["cfg"])
    p = R.init_params(cfg, seed=fx["seed"], random_affine=True)
    x, y = _inputs(cfg, fx["B"], fx["seed"])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        model = DDP(_model(cfg, p, torch.float32), device_ids=[0])
        optimizer = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        scaler = torch.amp.GradScaler("cuda")
        model.train()
        images, targets = x.to(DEV, non_blocking=True), y.to(DEV, non_blocking=True)
        optimizer.zero_grad()
        with torch.autocast("cuda"):
            outputs = model(images)
            loss = torch.nn.functional.cross_entropy(outputs, targets)
        scaler.scale(loss).backward()
        scaler.step(optimizer)
        scaler.update()
        torch.cuda.synchronize()
        assert _rel(outputs, fx["logits"]) < 1e-3
        assert abs(loss.item() - fx["loss"]) < 1e-3 * abs(fx["loss"])
        for k, v in model.module.state_dict().items():
            assert _rel(v, fx["params_after"][k]) < 1e-3, k
    finally:
        dist.destroy_process_group()


def _ddp_worker(rank, world, port, q):
    import os as _os
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                       LOCAL_RANK="0")
    import torch.distributed as dist
    import vit_amd
    from vit_amd import parallel
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=5, random_affine=True)
    x, y = _inputs(cfg, 4, 100 + rank)  # different images per rank
    m = _model(cfg, p, torch.bfloat16)
    flat = m.use_flat_grads(True)
    xd, yd = x.to(DEV), y.to(DEV)
    vit_amd.cross_entropy(m(xd), yd).backward()  # local gradients
    torch.cuda.synchronize()
    local = flat.detach().cpu().clone()
    m.zero_grad(set_to_none=True)
    red = parallel.OverlappedGradReduce(m)
    vit_amd.cross_entropy(m(xd), yd).backward()  # block spans all-reduced during the backward
    ncov = len(red.covered)
    red.finish()
    torch.cuda.synchronize()
    # numpy (pickled by value): torch tensors would travel as shared-memory handles that die with this process
    q.put((rank, local.numpy(), flat.detach().cpu().numpy(), ncov))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_overlapped_allreduce_two_ranks():
    """The N>1 bench path: OverlappedGradReduce hooked into the block backward (spans reduced
    from the side stream while the backward continues) gives the rank-average of the local
    flat gradients.  Two processes on the one GPU, gloo over CUDA tensors (RCCL needs one GPU
    per rank); the stream ordering under test is the same."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    mean = (res[0][1] + res[1][1]) / 2
    for rank, local, reduced, ncov in res:
        assert ncov == 12  # one span per block
        assert np.abs(reduced - mean).max() <= 1e-6 * np.abs(mean).max() + 1e-7, rank


@pytest.mark.parametrize("train", [True, False])
def test_two_stream_schedule_is_race_free(train):
    """The bench path leaves side-stream work pending across blocks (forward half-batch chain
    joined after the block stack, weight gradients joined in the patch embedding).  Tensors
    that work reads are freed on the caller's stream before it runs; the allocator must not
    hand them out again (record_stream).  Eager "end" joins must give bit-identical results to
    the per-block-joined schedule, over several steps of allocator churn at bs=128."""
    import vit_amd
    from vit_amd import model as VM
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=21, random_affine=True)
    x, y = _inputs(cfg, 128, 31)
    xd, yd = x.to(DEV), y.to(DEV)
    m = _model(cfg, p, torch.bfloat16)
    if train:
        flat = m.use_flat_grads(True)
    else:
        m.eval()

    def run():
        outs = []
        for _ in range(3):
            if train:
                m.zero_grad(set_to_none=True)
                vit_amd.cross_entropy(m(xd), yd).backward()
                torch.cuda.synchronize()
                outs.append(flat.detach().clone())
            else:
                with torch.no_grad():
                    f = m.forward_features(xd)
                    torch.cuda.synchronize()
                    outs.append(f.float().clone())
        return outs

    saved = (VM._FWD_JOIN[0], VM._BWD_JOIN[0])
    try:
        VM._FWD_JOIN[0], VM._BWD_JOIN[0] = "block", "block"
        ref = run()
        VM._FWD_JOIN[0], VM._BWD_JOIN[0] = "end", "end"
        got = run()
    finally:
        VM._FWD_JOIN[0], VM._BWD_JOIN[0] = saved
    assert all(torch.equal(ref[0], r) for r in ref[1:]), "per-block joined schedule not deterministic"
    for i, g in enumerate(got):
        assert torch.equal(g, ref[0]), (i, (g - ref[0]).abs().max().item())
