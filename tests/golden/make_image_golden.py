"""Generates tests/golden/image_golden.npz: Pillow's Image.resize(BILINEAR) on seeded RGB
uint8 images (the resampling torchvision's RandomResizedCrop / Resize run on PIL images,
VIT:32-46), the pin of oracle/image_ref.py.  Run from the repo root:
python tests/golden/make_image_golden.py"""
import os

import numpy as np
from PIL import Image

CASES = [  # (H, W, out_h, out_w)
    (37, 53, 24, 24), (64, 48, 7, 9), (1, 5, 3, 2), (90, 17, 32, 32), (20, 20, 20, 20), (50, 33, 26, 38),
    (13, 180, 16, 16), (41, 67, 60, 100),
]


def main():
    rng = np.random.default_rng(2024)
    out = {"PIL_version": np.array(Image.__version__)}
    for i, (h, w, oh, ow) in enumerate(CASES):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        out[f"in{i}"] = img
        out[f"out{i}"] = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    np.savez_compressed(os.path.join(os.path.dirname(__file__), "image_golden.npz"), **out)


if __name__ == "__main__":
    main()
