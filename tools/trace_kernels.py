"""Per-kernel ms/step of the last 3 bench steps of a rocprofv3 kernel trace (steps end at sgd_kernel),
the g4 GEMMs labelled by class and grid, then the per-class table of tools/step_classes.py.

    python tools/trace_kernels.py <run_kernel_trace.csv> [top]
"""
import collections
import csv
import os
import subprocess
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 18
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
sel = rows[idx[-4] + 1: idx[-1] + 1]
agg = collections.defaultdict(list)
for r in sel:
    n = r["Kernel_Name"]
    key = n[:70]
    if "g46kernel" in n or "g4::kernel" in n:
        fwd = "_ZN2g46kernelILi0E" in n or "g4::kernel<0" in n
        key = ("g4 fwd" if fwd else "g4 dgrad") + f" wgs={int(r['Grid_Size_X']) // 256}"
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / 3 / 1e3:7.3f} ms/step n={len(v) / 3:5.1f} avg={sum(v) / len(v):7.1f} us  {k}")
here = os.path.dirname(os.path.abspath(__file__))
subprocess.run([sys.executable, os.path.join(here, "step_classes.py"), path, "3"], check=False)
