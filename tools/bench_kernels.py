"""Per-kernel timing of the ViT-B/16 bs=256 step's GEMM / attention / LN shapes.

    python tools/bench_kernels.py [--batch 256] [--reps 20]

Times each launch with HIP events on the launch stream and prints achieved
TFLOP/s (GEMM, attention) or GB/s (LayerNorm) per shape; used to tune kernels.
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

PEAK = 256 * 4 * 1024 * 2.4e9 / 1e12


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sweep", type=str, default="", help="comma list of GEMM variants to sweep (big::V<n>)")
    ap.add_argument("--torch", action="store_true", help="time torch.matmul (hipBLASLt) on the same shapes")
    ap.add_argument("--groups", type=str, default="", help="comma list of tile-walk bands (vit_gemm_group) to time")
    a = ap.parse_args()
    if a.torch:
        return torch_ref(a)
    if a.groups:
        return groups(a, [int(v) for v in a.groups.split(",")])
    if a.sweep:
        return sweep(a, [int(v) for v in a.sweep.split(",")])
    dev = "cuda"
    B, N, D, H, F = a.batch, 197, 768, 12, 3072
    M = B * N
    bf = torch.bfloat16
    r = lambda *s: torch.randn(*s, device=dev).to(bf)
    res = []

    def rec(name, flop, t, extra=None):
        d = {"name": name, "ms": round(t * 1e3, 4), "tflops": round(flop / t / 1e12, 1),
             "frac": round(flop / t / 1e12 / PEAK, 4)}
        if extra:
            d.update(extra)
        res.append(d)
        print(json.dumps(d), flush=True)

    shapes = {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, F), "fc2": (F, D)}
    for nm, (K, Nout) in shapes.items():
        x, w, b = r(M, K), r(Nout, K) * 0.05, torch.randn(Nout, device=dev)
        out = torch.empty(M, Nout, device=dev, dtype=bf)
        act = torch.empty_like(out)
        res32 = torch.randn(M, Nout, device=dev)
        flop = 2.0 * M * Nout * K
        rec(f"fwd_{nm}_store_bf16", flop, timeit(lambda: ops.linear_fwd(x, w, b, out=out), a.reps))
        if nm == "fc1":
            rec("fwd_fc1_gelu", flop, timeit(lambda: ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU, out=out,
                                                                    act_out=act), a.reps))
        if nm in ("proj", "fc2"):
            rec(f"fwd_{nm}_resid", flop, timeit(lambda: ops.linear_fwd(x, w, b, epi=L.EPI_RESID, resid=res32,
                                                                       out=res32), a.reps))
        dy = r(M, Nout)
        dx32 = torch.empty(M, K, device=dev)
        rec(f"dgrad_{nm}_f32", flop, timeit(lambda: ops.linear_dgrad(dy, w, out=dx32), a.reps))
        dxb16 = torch.empty(M, K, device=dev, dtype=bf)
        rec(f"dgrad_{nm}_bf16", flop, timeit(lambda: ops.linear_dgrad(dy, w, out=dxb16), a.reps))
        if nm == "fc2":
            pre = r(M, K)
            dxb = torch.empty(M, K, device=dev, dtype=bf)
            rec("dgrad_fc2_gelubwd", flop, timeit(lambda: ops.linear_dgrad(dy, w, out_dtype=bf, epi=L.EPI_GELU_BWD,
                                                                          pre=pre, out=dxb), a.reps))
        dw = torch.empty(Nout, K, device=dev)
        rec(f"wgrad_{nm}", flop, timeit(lambda: ops.linear_wgrad(dy, x, out=dw), a.reps),
            {"split": ops._wgrad_split(M, Nout, K)})
    qkv = r(M, 3 * D)
    o, lse = ops.sdpa_fwd(qkv, B, H, N)
    aflop = 4.0 * B * H * N * N * 64
    rec("sdpa_fwd", aflop, timeit(lambda: ops.sdpa_fwd(qkv, B, H, N, o=o), a.reps))
    do = r(M, D)
    dq = torch.empty_like(qkv)
    rec("sdpa_bwd", 2.5 * aflop, timeit(lambda: ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq), a.reps))
    x = torch.randn(M, D, device=dev)
    w, bb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    y = torch.empty(M, D, device=dev, dtype=bf)
    t = timeit(lambda: ops.layer_norm_fwd(x, w, bb, 1e-6, bf, out=y), a.reps)
    print(json.dumps({"name": "ln_fwd", "ms": round(t * 1e3, 4), "GBps": round(M * D * 6 / t / 1e9, 1)}))
    # block backward's LayerNorm: x f32, dy bf16, dres f32 in; dx f32 + bf16 copy out; dgamma/dbeta/dsum
    _, mean, rstd = ops.layer_norm_fwd(x, w, bb, 1e-6, bf, out=y)
    dres, dxo = torch.randn(M, D, device=dev), torch.empty(M, D, device=dev)
    dxc = torch.empty(M, D, device=dev, dtype=bf)
    gg, gb, gs = (torch.empty(D, device=dev) for _ in range(3))
    t = timeit(lambda: ops.layer_norm_bwd(x, D, y, w, mean, rstd, dxo, D, M, dres=dres, ldres=D, dx_copy=dxc,
                                          ld_copy=D, dgamma=gg, dbeta=gb, dsum=gs), a.reps)
    print(json.dumps({"name": "ln_bwd", "ms": round(t * 1e3, 4), "GBps": round(M * D * 20 / t / 1e9, 1)}))


def torch_ref(a):
    """Library (hipBLASLt via torch.matmul) timings on the model GEMM shapes, bf16 out."""
    dev, bf = "cuda", torch.bfloat16
    M, D, F = a.batch * 197, 768, 3072
    r = lambda *s: torch.randn(*s, device=dev).to(bf)
    for nm, (K, Nout) in {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, F), "fc2": (F, D)}.items():
        x, w, dy = r(M, K), r(Nout, K), r(M, Nout)
        flop = 2.0 * M * Nout * K
        for kind, fn in (("fwd", lambda: torch.matmul(x, w.t())), ("dgrad", lambda: torch.matmul(dy, w)),
                         ("wgrad", lambda: torch.matmul(dy.t(), x))):
            t = timeit(fn, a.reps)
            print(json.dumps({"lib": "torch.matmul", "name": f"{kind}_{nm}", "ms": round(t * 1e3, 4),
                              "tflops": round(flop / t / 1e12, 1)}), flush=True)


def groups(a, bands):
    """Forward / input-gradient GEMMs (the step's epilogues) under each tile-walk band, interleaved
    rounds in one process; results checked against the row-major walk."""
    dev, bf = "cuda", torch.bfloat16
    M, D, F = a.batch * 197, 768, 3072
    r = lambda *s: torch.randn(*s, device=dev).to(bf)
    cases = []
    for nm, (K, Nout) in {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, F), "fc2": (F, D)}.items():
        x, w, dy = r(M, K), r(Nout, K) * 0.05, r(M, Nout)
        b = torch.randn(Nout, device=dev)
        flop = 2.0 * M * Nout * K
        outb = torch.empty(M, Nout, device=dev, dtype=bf)
        dxb = torch.empty(M, K, device=dev, dtype=bf)
        if nm == "fc1":
            act = torch.empty_like(outb)
            cases.append(("fwd_fc1_gelu", flop, lambda x=x, w=w, o=outb, a_=act, b_=b:
                          ops.linear_fwd(x, w, b_, epi=L.EPI_BIAS_GELU, out=o, act_out=a_), act))
        else:
            cases.append((f"fwd_{nm}", flop, lambda x=x, w=w, o=outb, b_=b: ops.linear_fwd(x, w, b_, out=o), outb))
        if nm == "fc2":
            pre = r(M, K)
            cases.append(("dgrad_fc2_gelubwd", flop, lambda dy=dy, w=w, p_=pre, o=dxb:
                          ops.linear_dgrad(dy, w, out_dtype=bf, epi=L.EPI_GELU_BWD, pre=p_, out=o), dxb))
        else:
            cases.append((f"dgrad_{nm}", flop, lambda dy=dy, w=w, o=dxb: ops.linear_dgrad(dy, w, out=o), dxb))
    lib = L.lib()
    lib.vit_gemm_group(0, 0)  # the row-major walk is the reference
    ref = {}
    for name, flop, fn, out in cases:
        fn(); torch.cuda.synchronize(); ref[name] = out.float().clone()
    table = {}
    for rnd in range(2):
        for g in bands:
            lib.vit_gemm_group(g, g)
            for name, flop, fn, out in cases:
                t = timeit(fn, a.reps)
                err = ((out.float() - ref[name]).abs().max() / ref[name].abs().max()).item()
                table.setdefault(name, {}).setdefault(g, []).append(round(flop / t / 1e12, 1))
                assert err == 0.0, (name, g, err)
    lib.vit_gemm_group(-2, -2)  # the defaults
    print("GROUPS", json.dumps({"batch": a.batch, "tflops": table}))


def sweep(a, variants):
    """Time every model GEMM under each forced configuration; check results against the default choice."""
    dev, bf = "cuda", torch.bfloat16
    M, D, F = a.batch * 197, 768, 3072
    r = lambda *s: torch.randn(*s, device=dev).to(bf)
    cases = []
    for nm, (K, Nout) in {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, F), "fc2": (F, D)}.items():
        x, w, dy = r(M, K), r(Nout, K) * 0.05, r(M, Nout)
        flop = 2.0 * M * Nout * K
        outb = torch.empty(M, Nout, device=dev, dtype=bf)
        dxb = torch.empty(M, K, device=dev, dtype=bf)
        dw = torch.empty(Nout, K, device=dev)
        cases.append((f"fwd_{nm}", flop, lambda x=x, w=w, o=outb: ops.linear_fwd(x, w, None, out=o), outb))
        cases.append((f"dgrad_{nm}", flop, lambda dy=dy, w=w, o=dxb: ops.linear_dgrad(dy, w, out=o), dxb))
        cases.append((f"wgrad_{nm}", flop, lambda dy=dy, x=x, o=dw: ops.linear_wgrad(dy, x, out=o), dw))
        if nm == "fc1":
            act = torch.empty_like(outb)
            b1 = torch.randn(Nout, device=dev)
            cases.append(("fwd_fc1_gelu", flop, lambda x=x, w=w, o=outb, a_=act, b_=b1:
                          ops.linear_fwd(x, w, b_, epi=L.EPI_BIAS_GELU, out=o, act_out=a_), act))
        if nm in ("proj", "fc2"):
            res = torch.randn(M, Nout, device=dev)
            cases.append((f"fwd_{nm}_resid", flop, lambda x=x, w=w, r_=res:
                          ops.linear_fwd(x, w, None, epi=L.EPI_RESID, resid=r_, out=r_), res))
        if nm == "fc2":
            pre = r(M, K)
            dxg = torch.empty(M, K, device=dev, dtype=bf)
            cases.append(("dgrad_fc2_gelubwd", flop, lambda dy=dy, w=w, p_=pre, o=dxg:
                          ops.linear_dgrad(dy, w, out_dtype=bf, epi=L.EPI_GELU_BWD, pre=p_, out=o), dxg))
    lib = L.lib()
    ref = {}
    lib.vit_gemm_variant(-1)
    for name, flop, fn, out in cases:
        fn(); torch.cuda.synchronize(); ref[name] = out.float().clone()
    table = {}
    for v in variants:
        lib.vit_gemm_variant(v)
        for name, flop, fn, out in cases:
            t = timeit(fn, a.reps)
            err = ((out.float() - ref[name]).abs().max() / ref[name].abs().max()).item() if "resid" not in name else 0.0
            table.setdefault(name, {})[v] = round(flop / t / 1e12, 1)
            print(json.dumps({"variant": v, "name": name, "ms": round(t * 1e3, 4), "tflops": round(flop / t / 1e12, 1),
                              "max_rel_vs_default": round(err, 6)}), flush=True)
    lib.vit_gemm_variant(-1)
    print("SUMMARY", json.dumps(table))


if __name__ == "__main__":
    main()
