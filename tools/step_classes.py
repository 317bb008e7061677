"""Per-class kernel time of the bench step from a rocprofv3 kernel trace.

    python tools/step_classes.py <run_kernel_trace.csv> [steps] [--json out.json]

Steps are delimited by the optimizer kernel (sgd_kernel, one per step); the last `steps` (default 3)
are used.  Classes: the GEMMs by layout (forward = RC x RC, input gradient = RC x CR, weight
gradient = the split-K ping-pong kernel + its slab reduce), attention forward / backward, LayerNorm
forward / backward, the bias / LN-affine column reductions, SGD, other.  For each class: kernel
ms per step (summed durations; the two streams overlap, so the classes sum to more than the wall
time), share of the summed kernel time, launches per step, and -- for the MFMA classes -- the
algorithmic TFLOP/s over that kernel time (ViT-B/16, bs=256: SURVEY §8d shapes).
"""
import csv
import json
import re
import sys
from collections import defaultdict

PEAK = 256 * 4 * 1024 * 2.4e9 / 1e12
B, N, D, F, H = 256, 197, 768, 3072, 12
M = B * N
# algorithmic FLOP per step by class (12 blocks; + the patch-embedding GEMMs on 50176 rows)
GEMM_BLOCK = 2 * M * D * (3 * D + D + F + F)
PATCH = 2 * B * 196 * D * D
FLOP = {
    "gemm fwd": 12 * GEMM_BLOCK + PATCH,
    "gemm dgrad": 12 * GEMM_BLOCK,
    "gemm wgrad": 12 * GEMM_BLOCK + PATCH,
    "attention fwd": 12 * 4 * B * H * N * N * 64,
    "attention bwd": 12 * 10 * B * H * N * N * 64,
}
_CFG = re.compile(r"gemm_kernelINS_3CfgI(?:L[ib]\d+E)+EELi(\d)ELi(\d)E")
# the wide-wave kernels (csrc/gemm_w4.inc, round 5): the pair launch is always a weight gradient; the
# single launch's layout pair is its 2nd / 3rd template argument (mangled or demangled)
_W4 = re.compile(r"_ZN2w46kernelINS_3CfgI(?:Li\d+E)+EELi(\d)ELi(\d)E|w4::kernel<w4::Cfg<\d+, \d+>, (\d), (\d),")


def classify(name: str) -> str:
    if "pp_kernel" in name or "splitk_reduce" in name or "w47kernel2" in name or "w4::kernel2" in name:
        return "gemm wgrad"
    w = _W4.search(name)
    if w:
        pl, ql = (int(w.group(1)), int(w.group(2))) if w.group(1) else (int(w.group(3)), int(w.group(4)))
        return {(0, 0): "gemm fwd", (0, 1): "gemm dgrad", (1, 1): "gemm wgrad"}.get((pl, ql), "gemm other")
    m = _CFG.search(name)
    if m or "pers" in name and "gemm_kernel" in name:
        pl, ql = (int(m.group(1)), int(m.group(2))) if m else (0, 0)
        return {(0, 0): "gemm fwd", (0, 1): "gemm dgrad", (1, 1): "gemm wgrad"}.get((pl, ql), "gemm other")
    if "_ZN2g46kernelILi0E" in name or "g4::kernel<0," in name:  # the 4-wave plain GEMM (csrc/gemm_g4.hip, round 6)
        return "gemm fwd"
    if "_ZN2g46kernelILi1E" in name or "g4::kernel<1," in name:
        return "gemm dgrad"
    if "Cijk_" in name:  # hipBLASLt (round 5's blaslt.hip): A = W read transposed (Alik) = forward, else dgrad
        return "gemm fwd" if "Cijk_Alik" in name else "gemm dgrad" if "Cijk_Ailk" in name else "gemm other"
    if "gen9gemm_kernel" in name or "gen::gemm_kernel" in name:
        return "head (fp32 generic GEMMs)"
    if "attn_fwd" in name:
        return "attention fwd"
    if "attn_bwd" in name:
        return "attention bwd"
    if "ln_fwd" in name:
        return "layernorm fwd"
    if "ln_bwd" in name:
        return "layernorm bwd"
    if "colreduce" in name or "colsum" in name:
        return "bias / affine column sums"
    if "sgd_kernel" in name:
        return "sgd"
    return "other"


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 3
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ends = [e for s, e, n in ev if n.startswith("sgd_kernel")]
    t0, t1 = ends[-steps - 1], ends[-1]
    wall = (t1 - t0) / steps / 1e6
    tot, cnt = defaultdict(float), defaultdict(int)
    for s, e, n in ev:
        if s >= t0 and e <= t1:
            c = classify(n)
            tot[c] += (e - s) / 1e6 / steps
            cnt[c] += 1
    ksum = sum(tot.values())
    table = []
    for c in sorted(tot, key=lambda k: -tot[k]):
        r = {"class": c, "ms_per_step": round(tot[c], 3), "share": round(tot[c] / ksum, 4),
             "launches_per_step": cnt[c] / steps}
        if c in FLOP:
            tf = FLOP[c] / (tot[c] * 1e-3) / 1e12
            r.update({"tflop_per_step": round(FLOP[c] / 1e12, 3), "tflops_over_kernel_time": round(tf, 1),
                      "frac_of_peak": round(tf / PEAK, 4)})
        table.append(r)
    res = {"trace": path, "steps": steps, "wall_ms_per_step": round(wall, 3),
           "kernel_ms_per_step": round(ksum, 3), "classes": table}
    print(f"wall {wall:.3f} ms/step, summed kernel time {ksum:.3f} ms/step (overlap {ksum / wall:.2f}x)")
    for r in table:
        extra = f"  {r['tflops_over_kernel_time']:7.1f} TF/s ({r['frac_of_peak']:.3f})" if "frac_of_peak" in r else ""
        print(f"  {r['class']:28s} {r['ms_per_step']:8.3f} ms  {100 * r['share']:5.1f} %  "
              f"n={r['launches_per_step']:5.1f}{extra}")
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
