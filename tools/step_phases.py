"""Forward / backward split of a rocprofv3 kernel trace of bench.py steps.

A step runs from the end of one sgd_kernel to the end of the next; its forward ends with ce_fwd_kernel
(loss), the backward starts with ce_bwd_kernel.  For each phase: wall time, the busy union of all
kernels, and kernel time per class (tools/step_classes.py's classes) summed over both streams.

    python tools/step_phases.py <kernel_trace.csv> [steps_to_use] [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from step_classes import classify  # noqa: E402


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if ce is not None else 0)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out in args:
        args.remove(out)
    rows = list(csv.DictReader(open(args[0])))
    use = int(args[1]) if len(args) > 1 else 3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    sgd = [e for s, e, n in ev if n.startswith("sgd_kernel")]
    res = {"steps": use, "phases": {}}
    acc = {"forward": defaultdict(float), "backward": defaultdict(float)}
    wall = {"forward": 0.0, "backward": 0.0}
    busy = {"forward": 0.0, "backward": 0.0}
    for k in range(len(sgd) - use - 1, len(sgd) - 1):
        t0, t1 = sgd[k], sgd[k + 1]
        win = [(s, e, n) for s, e, n in ev if s >= t0 and e <= t1]
        ce_f = [e for s, e, n in win if "ce_fwd_kernel" in n]
        ce_b = [s for s, e, n in win if "ce_bwd_kernel" in n]
        if not ce_f or not ce_b:
            continue
        split = (ce_f[0], ce_b[0])
        for ph, (a, b) in (("forward", (t0, split[0])), ("backward", (split[1], t1))):
            w = [(s, e, n) for s, e, n in win if s >= a and e <= b]
            wall[ph] += (b - a) / 1e6
            busy[ph] += union([(s, e) for s, e, n in w]) / 1e6
            for s, e, n in w:
                acc[ph][classify(n)] += (e - s) / 1e6
    for ph in ("forward", "backward"):
        res["phases"][ph] = {"wall_ms": round(wall[ph] / use, 3), "busy_ms": round(busy[ph] / use, 3),
                             "kernel_ms": round(sum(acc[ph].values()) / use, 3),
                             "classes": {c: round(v / use, 3) for c, v in sorted(acc[ph].items(), key=lambda x: -x[1])}}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
