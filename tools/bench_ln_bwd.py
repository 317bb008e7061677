"""LayerNorm backward at the ViT-B/16 bs=256 step shape (M = 50 432 rows x 768, as the block backward
calls it: x f32, dy bf16, residual gradient f32 in; dx f32 + bf16 copy out; dgamma / dbeta / dsum
partials), timed with HIP events; GB/s over the algorithmic bytes.  One JSON line.

    VIT_LN_BWD_ROWS=<rows per workgroup> python tools/bench_ln_bwd.py [--reps 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402

from vit_amd import _lib as L, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rows", type=int, default=256 * 197)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, D = a.rows, 768
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, D, device=dev, generator=g)
    dy = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    dres = torch.randn(M, D, device=dev, generator=g)
    w = torch.rand(D, device=dev, generator=g) + 0.5
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-6)
    dx = torch.empty(M, D, device=dev)
    cp = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    dg, db, ds = (torch.empty(D, device=dev) for _ in range(3))

    def run(cb):
        ops.layer_norm_bwd(x, D, dy, w, mean, rstd, dx, D, M, dres=dres, ldres=D, dx_copy=cp, ld_copy=D,
                           dgamma=dg, dbeta=db, dsum=ds, reduce_on=cb)

    st = torch.cuda.current_stream(dev)
    for _ in range(5):
        cb = ops.ColBatch()
        run(cb)
        cb.launch()
    torch.cuda.synchronize()
    # back-to-back launches between the events (the host enqueues faster than the kernel runs), the
    # per-block partial sums queued in ColBatches and launched after the second event
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    cbs = [ops.ColBatch() for _ in range(a.reps)]
    ev[0].record(st)
    for cb in cbs:
        run(cb)
    ev[1].record(st)
    for cb in cbs:
        cb.launch()
    ev[2].record(st)
    torch.cuda.synchronize()
    t_ln = ev[0].elapsed_time(ev[1]) / a.reps
    t_all = ev[0].elapsed_time(ev[2]) / a.reps
    byts = M * D * (4 + 2 + 4 + 4 + 2)
    nb = L.lib().vit_layer_norm_bwd_blocks(M)
    print(json.dumps({"rows_per_wg": os.environ.get("VIT_LN_BWD_ROWS", "default"), "blocks": nb, "ln_bwd_us": round(t_ln * 1e3, 1),
                      "with_partial_sums_us": round(t_all * 1e3, 1), "algorithmic_MB": round(byts / 1e6, 1),
                      "GBps": round(byts / (t_ln * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
