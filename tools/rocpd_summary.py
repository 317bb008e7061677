"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite, ROCm 7.2 default output).

    python tools/rocpd_summary.py <run_results.db> [steps] [top] [--csv out.csv]

Prints ms/step, share, calls/step and average duration per kernel name, like
rocprofv3's kernel_stats.csv.  Durations of kernels that overlap on two streams
are each counted in full, so the column can sum to more than the step time.
"""
import csv
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
    if out in args:
        args.remove(out)
    db = args[0]
    steps = float(args[1]) if len(args) > 1 else 1.0
    top = int(args[2]) if len(args) > 2 else 30
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    span = c.execute("select min(start), max(end) from kernels").fetchone()
    tot = sum(r[2] for r in rows)
    for name, n, s, avg, mn, mx in rows[:top]:
        print(f"{s / 1e6 / steps:8.2f}ms/step {100 * s / tot:6.2f}% n={n / steps:6.1f}/step avg={avg / 1e3:8.1f}us  "
              f"{name[:110]}")
    print("sum of kernel durations ms/step", round(tot / 1e6 / steps, 3),
          "| trace span ms", round((span[1] - span[0]) / 1e6, 3))
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            for name, n, s, avg, mn, mx in rows:
                w.writerow([name, n, int(s), round(avg, 1), int(mn), int(mx), round(100 * s / tot, 3)])


if __name__ == "__main__":
    main()
