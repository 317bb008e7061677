"""Run a command as a child process while sampling the GPU's clocks and power from this (GPU-idle) parent
with amdsmi, so two trees whose bench.py differ can be compared on the same box at the same clocks:

    python tools/telemetry_wrap.py OUT.json -- python bench.py --steps 40 ...

The child's stdout/stderr pass through.  OUT.json gets the means over the busy samples (gfx activity >= 80 %).
Exits with the child's exit code.  This process never touches HIP (amdsmi reads the SMU's metrics table).
"""
import json
import subprocess
import sys
import threading
import time

KEYS = ("current_gfxclk", "current_gfxclks", "current_uclk", "current_socket_power", "temperature_hotspot",
        "average_gfx_activity")


def main():
    out_path = sys.argv[1]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    samples, stop = [], threading.Event()
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        handles = amdsmi.amdsmi_get_processor_handles()
    except Exception as ex:  # noqa: BLE001
        handles, err = [], str(ex)[:120]
    else:
        err = None

    def one(h):
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        r = {}
        for k in KEYS:
            v = m.get(k)
            vals = v if isinstance(v, (list, tuple)) else [v]
            vals = [float(x) for x in vals if isinstance(x, (int, float)) and 0 < x < 65535]
            if vals:
                r[k] = sum(vals) / len(vals)
        return r

    def run():
        while not stop.is_set():
            try:
                # the busiest visible GPU is ours (a 1-GPU box shows one)
                rs = [one(h) for h in handles]
                if rs:
                    r = max(rs, key=lambda d: d.get("average_gfx_activity", 0))
                    r["t"] = time.time()
                    samples.append(r)
            except Exception:  # noqa: BLE001
                return
            stop.wait(0.05)

    th = threading.Thread(target=run, daemon=True)
    th.start()
    rc = subprocess.call(cmd)
    stop.set()
    th.join()
    busy = [s for s in samples if s.get("average_gfx_activity", 0) >= 80]
    res = {"samples": len(samples), "busy": len(busy), "error": err}
    for k in KEYS:
        vals = [s[k] for s in busy if k in s]
        if vals:
            res[k] = round(sum(vals) / len(vals), 1)
    with open(out_path, "w") as f:
        json.dump(res, f)
    sys.exit(rc)


if __name__ == "__main__":
    main()
