"""Per-dispatch HBM traffic of one kernel from rocprofv3 counter CSVs.

    python tools/pmc_traffic.py <dir with *_counter_collection.csv> <kernel-name substring>[,<substring>...] [--out f.json]

With several comma-separated substrings (a kernel and its companion launches, e.g. the split-K
weight gradient and its slab reduce) the per-dispatch averages of each are summed: traffic per
call of the operation.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch.
Correction applied (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  The calibration kernel
(ln_fwd in tools/kernel_probe.py, known byte counts) checks both.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def collect(d, sub):
    vals = defaultdict(list)
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if sub in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
                    names.add(row["Kernel_Name"][:160])
    return vals, names


def main():
    d, subs = sys.argv[1], sys.argv[2].split(",")
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    res = {"kernel_match": subs, "kernels": [], "dispatches": {}}
    for sub in subs:
        vals, names = collect(d, sub)
        res["kernels"] += sorted(names)
        for k, v in vals.items():
            res["dispatches"][sub + ":" + k] = len(v)
            res[k + "_KiB_avg"] = res.get(k + "_KiB_avg", 0.0) + sum(v) / len(v)
    fetch = res.get("FETCH_SIZE_KiB_avg")
    write = res.get("WRITE_SIZE_KiB_avg")
    if fetch is not None:
        res["fetch_bytes_corrected"] = fetch * 1024 * 2
    if write is not None:
        res["write_bytes"] = write * 1024
    if fetch is not None and write is not None:
        res["traffic_bytes_per_launch"] = res["fetch_bytes_corrected"] + res["write_bytes"]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import wgrad_src_sha  # the kernel sources these counters were taken on
    res["src_sha"] = wgrad_src_sha()
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
