"""Config C3 step rate alone: CLIP-HBA ViT-L/14 + DoRA train step (bench.py's ``c3`` leg, which
the default bench line carries in both dtypes).  Prints one JSON line.

    python tools/bench_clip.py [--batch 64] [--steps 10] [--warmup 3] [--dtype f32|bf16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32",
                    help="compute dtype: f32 = the reference's precision (NEWP:274), bf16 opt-in")
    a = ap.parse_args()
    import torch
    r = bench.c3_leg(torch.device("cuda", 0), a.dtype, a.batch, a.steps, a.warmup)
    r["metric"] = "images/sec CLIP-HBA ViT-L/14 + DoRA train step (config C3)"
    print(json.dumps(r))


if __name__ == "__main__":
    main()
