"""Is the eager bs=256 step host-bound?  Times the host's enqueue of K steps (no sync) against
the wall time of the same K steps, for wgrad/fwd overlap on and off, and a captured-graph replay.

    python tools/host_probe.py [--steps 10] [--batch 256]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import vit_amd
    dev = torch.device("cuda", 0)
    model = vit_amd.create_model("vit_base_patch16_224", compute_dtype=torch.bfloat16).to(dev)
    model.use_flat_grads(True)
    opt = vit_amd.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        loss = vit_amd.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    out = {}
    for overlap in (True, False):
        vit_amd.set_wgrad_overlap(overlap)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"overlap={overlap}"] = {"host_enqueue_ms_per_step": round((t1 - t0) / a.steps * 1e3, 2),
                                     "wall_ms_per_step": round((t2 - t0) / a.steps * 1e3, 2)}
        print(json.dumps(out), flush=True)
    for overlap in (True, False):
        vit_amd.set_wgrad_overlap(overlap)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        out[f"graph overlap={overlap}"] = {"wall_ms_per_step": round((time.perf_counter() - t0) / a.steps * 1e3, 2)}
        print(json.dumps(out), flush=True)
        del g


if __name__ == "__main__":
    main()
