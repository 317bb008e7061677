"""Headline benchmark: ViT-B/16 224 training step, bs=256 per GPU, bf16 (BASELINE.json configs[1]).

One step = forward + mean cross-entropy + backward + fused SGD (lr 0.1, momentum
0.9, wd 1e-4) on one synthetic batch already resident in HBM (VIT:132-147 minus
the data loader).  N>1: one process per GPU (torchrun), 256 images per rank
(weak scaling), gradients averaged with bucketed RCCL all-reduces (DDP in the
reference, VIT:287).  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-graph]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FWD_FLOP_PER_IMG = 35.128e9          # SURVEY §8d (oracle.vit_flops_per_image)
STEP_FLOP_PER_IMG = 3 * FWD_FLOP_PER_IMG
# gfx950 dense bf16 MFMA: 256 CU x 4 SIMD x 1024 FLOP/clk (16x16x32: 16384 FLOP / 16 clk) x 2.4 GHz
PEAK_BF16_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--graph", action="store_true",
                    help="replay one captured HIP graph per step (ROCm replays graph branches serially, so the "
                         "two-stream overlap is lost; eager is faster with overlap on)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-overlap", action="store_true", help="weight gradients inline instead of on a side stream")
    return ap.parse_args()


def cpu_baseline(seconds: float):
    """The oracle's fp32 ViT-B/16 train step (bs=4, configs[0]) on the host cores."""
    from oracle import vit_ref as R
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = R.VIT_B16
    p = R.init_params(cfg, seed=0)
    bufs = {}
    g = torch.Generator().manual_seed(0)
    B = 4
    x = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randint(0, 1000, (B,), generator=g)
    R.train_step(p, bufs, x, y, lr=0.1, cfg=cfg)  # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        R.train_step(p, bufs, x, y, lr=0.1, cfg=cfg)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": round(n * B / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} fp32 ViT-B/16 train steps (bs=4, fwd+CE+bwd+SGD) of oracle/vit_ref.py, "
                      f"{el:.1f} s, torch CPU {threads} threads"}


def _pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed counter passes
    (tools/pmc_traffic.py; FETCH_SIZE doubled per the gfx950 correction), or None."""
    f = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01", "pmc_traffic_fc1_fwd_gelu.json")
    try:
        with open(f) as fh:
            return int(json.load(fh)["traffic_bytes_per_launch"])
    except (OSError, KeyError, ValueError):
        return None


def main():
    a = parse()
    import vit_amd
    from vit_amd import parallel, ops
    from vit_amd import _lib as L

    rank, world, local = parallel.init_from_env("nccl")
    if world != a.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    torch.manual_seed(1234 + rank)

    B = a.batch
    model = vit_amd.create_model("vit_base_patch16_224", num_classes=1000, compute_dtype=torch.bfloat16).to(dev)
    flat = model.use_flat_grads(True)
    vit_amd.set_wgrad_overlap(not a.no_overlap)
    opt = vit_amd.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(B, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (B,), device=dev)

    # world > 1: gradients averaged block by block during the backward (RCCL beside compute);
    # VIT_DDP_OVERLAP=0 falls back to bucketed all-reduces after the backward
    reducer = None
    if world > 1 and os.environ.get("VIT_DDP_OVERLAP", "1") != "0":
        reducer = parallel.OverlappedGradReduce(model)

    def step():
        loss = vit_amd.cross_entropy(model(x), y)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        elif world > 1:
            parallel.allreduce_flat(flat, bucket_mb=64.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    use_graph = a.graph and world == 1
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(max(1, a.warmup)):
            loss = step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    warm_loss = float(loss.item())
    del loss
    graph = None
    if use_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            gloss = step()
        graph.replay()  # one untimed replay
        torch.cuda.synchronize(dev)

    def run_steps(k):
        for _ in range(k):
            if graph is not None:
                graph.replay()
            else:
                step()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(a.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    final_loss = float(gloss.item()) if graph is not None else warm_loss

    # --- dominant-kernel roofline: fc1 forward GEMM (M=B*197, N=3072, K=768, bias+GELU epilogue),
    #     timed with HIP events on the stream it is launched on
    blk = model.blocks[0]
    M = B * 197
    h = torch.randn(M, 768, device=dev).to(torch.bfloat16)
    w1 = blk.mlp.fc1.weight._vit_shadow
    b1 = blk.mlp.fc1.bias.detach()
    pre = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
    act = torch.empty_like(pre)
    # 20 warm-up launches: the first ones over the freshly allocated h / pre / act run ~20 % slower
    # (tools/probe_fc1_data.py); the step reuses its buffers, so the steady state is what it sees
    for _ in range(20):
        ops.linear_fwd(h, w1, b1, epi=L.EPI_BIAS_GELU, out=pre, act_out=act)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        ops.linear_fwd(h, w1, b1, epi=L.EPI_BIAS_GELU, out=pre, act_out=act)
    e1.record()
    torch.cuda.synchronize(dev)
    k_ms = e0.elapsed_time(e1) / reps
    k_flop = 2.0 * M * 3072 * 768
    k_tflops = k_flop / (k_ms * 1e-3) / 1e12

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    imgs = world * B * a.steps
    value = imgs / el
    ms = el / a.steps * 1e3
    step_tflops = value / world * STEP_FLOP_PER_IMG / 1e12
    out = {
        "metric": "images/sec ViT-B/16 224 train step bs=256 (whole job)",
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic randn images [256,3,224,224] f32 + randint labels, resident in HBM; random-init ViT-B/16",
        "config": {"workload": "ViT-B/16 224 train step (fwd+CE+bwd+SGD), BASELINE configs[1]",
                   "model": "vit_base_patch16_224", "global_batch": world * B, "per_gpu_batch": B,
                   "seq_len": 197, "parallelism": f"dp{world}", "launch": "hipgraph" if graph is not None else "eager",
                   "final_loss": round(final_loss, 4)},
        "roofline": {"bound": "mfma", "kernel": "big::gemm_kernel<V5,RC,RC,BIAS_GELU> fc1 fwd, M=%d N=3072 K=768" % M,
                     "achieved": round(k_tflops, 1), "peak": round(PEAK_BF16_TFLOPS, 1), "unit": "TFLOP/s",
                     "frac": round(k_tflops / PEAK_BF16_TFLOPS, 4), "traffic": _pmc_traffic(),
                     "traffic_unit": "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 --pmc passes, "
                                     "profiles/r01/pmc_traffic_fc1_fwd_gelu.json)",
                     "algorithmic_bytes": (M * 768 + 3072 * 768 + 2 * M * 3072) * 2 + 3072 * 4,
                     "kernel_ms": round(k_ms, 4), "flop_per_launch": k_flop},
        "step_mfma": {"achieved_tflops": round(step_tflops, 1), "frac": round(step_tflops / PEAK_BF16_TFLOPS, 4),
                      "flop_per_img": STEP_FLOP_PER_IMG},
    }
    if world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
