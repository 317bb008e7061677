"""Per-kernel MFMA utilisation and HBM traffic of the bench step from rocprofv3 counter passes.

    python tools/pmc_step_classes.py <dir> [--json out.json]

<dir> holds three passes over tools/step_probe.py (tools/gpu_job.sh pmc): sq/ (kernel trace +
SQ_* + GRBM_*), fetch/ (FETCH_SIZE), write/ (WRITE_SIZE).  Under counter collection every
dispatch runs serialized, so these are per-kernel (standalone-in-step) figures, not the
two-stream overlap of the timed step.

Per kernel (grouped by name; `label` names what it computes) and per step class
(tools/step_classes.classify):
  * mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of
    SIMD-cycles the matrix pipe was busy (SQ_VALU_MFMA_BUSY_CYCLES counts busy cycles summed over
    SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md);
  * clock_ghz = GRBM_GUI_ACTIVE / 8 / duration;
  * wait_any / wait_inst_any / active_inst_any: shares of SQ_WAVE_CYCLES;
  * hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (the gfx950 FETCH correction, MI355X_MICROARCH.md HBM)
    and hbm_gbs = hbm_bytes / duration, against 8 TB/s (peak) and 6.3 TB/s (achievable).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_classes import classify  # noqa: E402

LABELS = [  # (regex on the mangled name, label)
    (r"pp_kernel", "wgrad: split-K ping-pong 256x256x32 (every dW)"),
    (r"w47kernel2|w4::kernel2|_ZN2w46kernelINS_3CfgI(?:Li\d+E)+EELi1ELi1E", "wgrad: w4 4-wave 256x256x32 (every dW)"),
    (r"splitk_reduce", "wgrad: split-K slab reduce"),
    (r"CfgILi256ELi256ELi64E.*ELi0ELi0ELi0E", "fwd: V5 256x256x64 plain bf16 (qkv, fc2)"),
    (r"CfgILi256ELi256ELi64E.*ELi0ELi0ELi1E", "fwd: V5 256x256x64 bias+GELU pair (fc1)"),
    (r"CfgILi128ELi128ELi64E.*ELi0ELi0ELi0E", "fwd: V2 128x128x64 plain (proj)"),
    (r"CfgILi128ELi128ELi64E.*ELi0ELi0ELi4E", "fwd: V2 patch embed"),
    (r"CfgILi128ELi256ELi32E.*ELi0ELi1ELi0E", "dgrad: V3 128x256x32 (fc1, qkv)"),
    (r"CfgILi256ELi128ELi32E.*ELi0ELi1ELi3E", "dgrad: V1 256x128x32 GELU' (fc2)"),
    (r"CfgILi256ELi128ELi32E.*ELi0ELi1ELi0E", "dgrad: V1 256x128x32 (proj)"),
    (r"Cijk_Alik", "fwd: hipBLASLt plain + bias (qkv, proj, fc2)"),
    (r"Cijk_Ailk", "dgrad: hipBLASLt plain (qkv, fc1, proj)"),
    (r"attn_fwd", "attention fwd"),
    (r"attn_bwd", "attention bwd"),
    (r"ln_bwd_kernel", "layernorm bwd"),
    (r"add_ln_fwd", "add + layernorm fwd"),
    (r"ln_fwd_kernel", "layernorm fwd"),
    (r"colreduce", "column-sum reduce"),
    (r"sgd_kernel", "fused SGD"),
]
SIMDS = 256 * 4


def label(name):
    for rx, lb in LABELS:
        if re.search(rx, name):
            return lb
    return name[:60]


def load(d, sub):
    """{kernel name: {counter: [values per dispatch]}} and durations (ns) from kernel traces."""
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, sub, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, durs


def avg(v):
    return sum(v) / len(v) if v else None


def summarize(sq, dur, fetch, write):
    out = {"dispatches": len(dur) or len(sq.get("SQ_WAVE_CYCLES", []))}
    t = avg(dur)
    gui = avg(sq.get("GRBM_GUI_ACTIVE", []))
    mb = avg(sq.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
    wc = avg(sq.get("SQ_WAVE_CYCLES", []))
    if t:
        out["avg_us"] = round(t / 1e3, 2)
    if gui and mb is not None:
        out["mfma_busy"] = round(mb / (SIMDS * gui / 8), 4)
    if gui and t:
        out["clock_ghz"] = round(gui / 8 / t, 3)
    if wc:
        for k, n in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_any"), ("SQ_ACTIVE_INST_LDS", "active_inst_lds")):
            if sq.get(k):
                out[n] = round(avg(sq[k]) / wc, 4)
    f, w = avg(fetch), avg(write)
    if f is not None and w is not None:
        b = 2 * f * 1024 + w * 1024
        out["hbm_bytes"] = int(b)
        out["fetch_bytes_corrected"] = int(2 * f * 1024)
        out["write_bytes"] = int(w * 1024)
        if t:
            out["hbm_gbs"] = round(b / t, 1)
            out["hbm_frac_of_8tbs"] = round(b / t / 8000, 4)
    return out


def main():
    d = sys.argv[1]
    outp = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    sq, dsq = load(d, "sq")
    fe, _ = load(d, "fetch")
    wr, _ = load(d, "write")
    names = set(sq) | set(dsq)
    kernels = {}
    for n in names:
        lb = label(n)
        r = summarize(sq.get(n, {}), dsq.get(n, []), fe.get(n, {}).get("FETCH_SIZE", []),
                      wr.get(n, {}).get("WRITE_SIZE", []))
        r["label"], r["class"], r["name"] = lb, classify(n), n[:160]
        kernels[n] = r
    # per step class: dispatch-weighted (time-weighted for the ratios)
    cls = defaultdict(lambda: {"time_us": 0.0, "mfma_cycles": 0.0, "simd_cycles": 0.0, "bytes": 0.0, "n": 0})
    for n, r in kernels.items():
        c = cls[r["class"]]
        k = r.get("dispatches", 0)
        c["n"] += k
        if "avg_us" in r:
            c["time_us"] += r["avg_us"] * k
            if "mfma_busy" in r:
                c["mfma_cycles"] += r["mfma_busy"] * r["avg_us"] * k
                c["simd_cycles"] += r["avg_us"] * k
            if "hbm_bytes" in r:
                c["bytes"] += r["hbm_bytes"] * k
    classes = {}
    for name, c in cls.items():
        e = {"dispatches": c["n"], "time_ms": round(c["time_us"] / 1e3, 3)}
        if c["simd_cycles"]:
            e["mfma_busy"] = round(c["mfma_cycles"] / c["simd_cycles"], 4)
        if c["time_us"] and c["bytes"]:
            e["hbm_gbs"] = round(c["bytes"] / (c["time_us"] * 1e3), 1)
        classes[name] = e
    rows = sorted(kernels.values(), key=lambda r: -(r.get("avg_us", 0) * r.get("dispatches", 0)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import wgrad_src_sha  # the weight-gradient kernel sources these counters were taken on
    res = {"source": d, "program": "tools/step_probe.py (bench step, bs=256 bf16), dispatches serialized by the "
                                   "counter passes", "src_sha": wgrad_src_sha(), "kernels": rows, "classes": classes}
    for r in rows[:24]:
        print(f"{r['label'][:46]:46s} n={r.get('dispatches', 0):4d} {r.get('avg_us', 0):8.1f} us  "
              f"mfma {r.get('mfma_busy', float('nan')):.3f}  clk {r.get('clock_ghz', float('nan')):.2f}  "
              f"{r.get('hbm_gbs', float('nan')):7.0f} GB/s  wait {r.get('wait_any', float('nan')):.2f}")
    if outp:
        with open(outp, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
