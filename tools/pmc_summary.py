"""Average rocprofv3 counters per dispatch for kernels matching a substring, plus the
kernel duration from the kernel-trace rows of the same passes.

    python tools/pmc_summary.py <dir> <kernel-substring>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, sub = sys.argv[1], sys.argv[2]
    vals = defaultdict(list)
    durs = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if sub in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if sub in row["Kernel_Name"]:
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    for k in sorted(avg):
        print(f"{k:28s} {avg[k]:.4g}")
    if durs:
        t = sorted(durs)[len(durs) // 2]
        print(f"{'duration_us (median)':28s} {t:.1f}")
        if "GRBM_GUI_ACTIVE" in avg:
            print(f"{'clock_GHz (GUI_ACTIVE/dur)':28s} {avg['GRBM_GUI_ACTIVE'] / (t * 1e3):.3f}")
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                print(f"{k + ' / WAVE_CYCLES':28s} {avg[k] / w:.3f}")


if __name__ == "__main__":
    main()
