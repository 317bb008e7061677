"""Step-level view of a rocprofv3 kernel trace: wall time per step, GPU-busy union,
sum of kernel durations (> union means kernels overlapped), per-kernel totals.

    python tools/trace_overlap.py <kernel_trace.csv> [steps_to_use]

Steps are delimited by the optimizer kernel (sgd_kernel), one per step.
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    use = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ends = [e for s, e, n in ev if n.startswith("sgd_kernel")]
    if len(ends) < use + 1:
        print("not enough steps", len(ends))
        return
    t0, t1 = ends[-use - 1], ends[-1]
    win = [(max(s, t0), min(e, t1), n) for s, e, n in ev if e > t0 and s < t1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, n in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(e - s for s, e, n in win)
    wall = t1 - t0
    print(f"wall/step {wall / use / 1e6:.3f} ms  busy-union/step {busy / use / 1e6:.3f} ms  "
          f"sum-of-kernels/step {tot / use / 1e6:.3f} ms  (overlap factor {tot / busy:.3f})")
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        a = agg[n[:100]]
        a[0] += e - s
        a[1] += 1
    for n, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{d / use / 1e6:8.3f} ms/step  n={c / use:5.1f}  avg={d / c / 1e3:8.1f} us  {n}")


if __name__ == "__main__":
    main()
