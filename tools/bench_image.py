"""Throughput of the GPU input transforms (csrc/image.hip) vs the reference's per-image CPU work
(Pillow crop + bilinear resize + flip + ToTensor/Normalize in numpy) on synthetic decoded images.

    python tools/bench_image.py [--batch 256] [--h 375] [--w 500] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--h", type=int, default=375)
    ap.add_argument("--w", type=int, default=500)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu-images", type=int, default=256)
    a = ap.parse_args()
    from vit_amd import data
    rng = np.random.default_rng(0)
    imgs = [rng.integers(0, 256, (a.h, a.w, 3), dtype=np.uint8) for _ in range(a.batch)]
    res = {}
    for train in (True, False):
        tr = data.GpuTransform(train=train)
        g = torch.Generator().manual_seed(0)
        shapes = [(a.h, a.w)] * a.batch
        params = tr.draw(shapes, g) if train else None
        # host staging (pack + H2D) and the kernels on a device-resident batch, timed apart
        st = tr.stage(imgs, params=params)
        tr.apply(st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st = tr.stage(imgs, params=params)
        torch.cuda.synchronize()
        stage_s = (time.perf_counter() - t0) / a.reps
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            tr.apply(st)
        e.record()
        torch.cuda.synchronize()
        k = s.elapsed_time(e) / 1e3 / a.reps
        res["train" if train else "val"] = {"kernel_ms_per_batch": round(k * 1e3, 3),
                                            "kernel_images_per_s": round(a.batch / k, 1),
                                            "host_stage_ms_per_batch": round(stage_s * 1e3, 3)}
    # CPU: what each DataLoader worker does per image (one core)
    from PIL import Image
    mean = np.array([0.485, 0.456, 0.406], np.float32)[:, None, None]
    std = np.array([0.229, 0.224, 0.225], np.float32)[:, None, None]
    pil = [Image.fromarray(im) for im in imgs[:a.cpu_images]]
    t0 = time.perf_counter()
    for im in pil:
        r = np.asarray(im.crop((50, 30, 450, 330)).resize((224, 224), Image.BILINEAR))[:, ::-1]
        x = (np.transpose(r, (2, 0, 1)).astype(np.float32) / np.float32(255) - mean) / std
    cpu = (time.perf_counter() - t0) / len(pil)
    res["cpu_pillow_one_core_images_per_s"] = round(1.0 / cpu, 1)
    res["config"] = {"batch": a.batch, "image": [a.h, a.w, 3], "out": [3, 224, 224]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
