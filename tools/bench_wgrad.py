"""Weight-gradient kernels on the step's shapes: every forced wgrad configuration (vit_gemm_variant: 8 =
the ping-pong kernel of rounds 1-4, 11 = w4 default, 12-15 = w4 ring / load-placement variants, +400 = no
epilogue, +500 = no loads and no epilogue), at the side stream's split (128 workgroups) and the full GPU
(256), single GEMMs and the MLP / attention pairs as the step launches them (grouped launch + slab sums).
Interleaved rounds, HIP events; results checked bit-for-bit against variant 8.

    python tools/bench_wgrad.py [--variants 8,11,12,13,14,15] [--reps 20] [--rounds 2]
"""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L

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
    ap.add_argument("--variants", default="8,11,12,13,14,15")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    vs = [int(v) for v in a.variants.split(",")]
    lib = L.lib()
    dev, bf = "cuda", torch.bfloat16
    M = a.batch * 197
    r = lambda *s: torch.randn(*s, device=dev).to(bf)
    x768, x3072 = r(M, 768), r(M, 3072)
    dy768, dy2304, dy3072 = r(M, 768), r(M, 2304), r(M, 3072)
    cases = []
    for wgs in (128, 256):
        for nm, dy, x in (("qkv", dy2304, x768), ("proj", dy768, x768), ("fc1", dy3072, x768), ("fc2", dy768, x3072)):
            N, K = dy.shape[1], x.shape[1]
            split = ops._wgrad_split(M, N, K, wgs)
            out = torch.empty(N, K, device=dev)
            cases.append((f"{nm}@{wgs}", 2.0 * M * N * K, lambda dy=dy, x=x, o=out, s=split: ops.linear_wgrad(dy, x, out=o, split=s), out))
    for nm, (dya, xa, dyb, xb) in (("mlp_pair", (dy768, x3072, dy3072, x768)), ("attn_pair", (dy768, x768, dy2304, x768))):
        oa = torch.empty(dya.shape[1], xa.shape[1], device=dev)
        ob = torch.empty(dyb.shape[1], xb.shape[1], device=dev)

        def pair(dya=dya, xa=xa, dyb=dyb, xb=xb, oa=oa, ob=ob):
            cb = ops.ColBatch()
            ops.linear_wgrad_pair((dya, xa, oa), (dyb, xb, ob), cb)
            cb.launch()
        fl = 2.0 * M * (dya.shape[1] * xa.shape[1] + dyb.shape[1] * xb.shape[1])
        cases.append((f"{nm}@128", fl, pair, oa))
    ref = {}
    lib.vit_gemm_variant(8)
    for name, fl, fn, out in cases:
        fn(); torch.cuda.synchronize(); ref[name] = out.clone()
    table = {}
    for rnd in range(a.rounds):
        for v in vs:
            lib.vit_gemm_variant(v)
            for name, fl, fn, out in cases:
                t = timeit(fn, a.reps)
                tf = fl / t / 1e12
                rec = table.setdefault(name, {}).setdefault(str(v), [])
                rec.append(round(tf, 1))
                if rnd == 0 and v < 100:
                    assert torch.equal(out, ref[name]), (name, v)
    lib.vit_gemm_variant(-1)
    for name, d in table.items():
        print(json.dumps({"case": name, "tflops": d, "best": {k: max(x) for k, x in d.items()}}), flush=True)
    print(json.dumps({"summary": "bitwise equal to variant 8 for every variant < 100", "peak": round(PEAK, 1)}))


if __name__ == "__main__":
    main()
