"""Input pipeline for the ImageNet loops: host decode, GPU transforms.

The reference's DataLoader workers run, per image (VIT:29-90, MEAS:141-223)::

    train: RandomResizedCrop(224) -> RandomHorizontalFlip() -> ToTensor() -> Normalize(mean, std)
    val:   Resize(256) -> CenterCrop(224) -> ToTensor() -> Normalize(mean, std)

on PIL images from ``ImageFolder`` -- at ~10k img/s/GPU that host work is the bottleneck
(SURVEY §8f).  Here the host only decodes (``decode``: Pillow, as ImageFolder's loader)
and draws the random parameters; the uint8 images travel to HBM once and one C-ABI call
(``vit_image_transform``, csrc/image.hip) crops, resamples with Pillow's bilinear filter
bit-exactly, flips and normalises the whole batch into the f32 [B, 3, 224, 224] tensor the
model takes.

The random parameters follow torchvision's published ``RandomResizedCrop.get_params`` and
``RandomHorizontalFlip`` (torchvision itself is not installed, SURVEY §8c, so the draw order
is restated, not pinned): per image, up to 10 tries of ``uniform_(scale)``,
``exp(uniform_(log ratio))``, ``randint`` top / left, then the central-crop fallback, then
``rand(1) < 0.5`` for the flip -- from the caller's ``torch.Generator``.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L
from ._lib import call, ptr

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)
_NPARAM = 12


def decode(path) -> np.ndarray:
    """ImageFolder's default loader (``Image.open(f).convert('RGB')``) as an [H, W, 3] uint8 array."""
    from PIL import Image
    with open(path, "rb") as f:
        return np.asarray(Image.open(f).convert("RGB"))


def random_resized_crop_params(height: int, width: int, generator: Optional[torch.Generator] = None,
                               scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0)) -> Tuple[int, int, int, int]:
    """(top, left, h, w) as torchvision ``RandomResizedCrop.get_params``."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=generator).item()
        aspect_ratio = math.exp(torch.empty(1).uniform_(log_ratio[0].item(), log_ratio[1].item(),
                                                        generator=generator).item())
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = int(torch.randint(0, height - h + 1, size=(1,), generator=generator).item())
            j = int(torch.randint(0, width - w + 1, size=(1,), generator=generator).item())
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def resize_shorter(h: int, w: int, size: int = 256) -> Tuple[int, int]:
    """Output (rows, cols) of torchvision ``Resize(size)`` (int size: shorter side -> size)."""
    if w <= h:
        return int(size * h / w), size
    return size, int(size * w / h)


def _taps(in_size: int, out_size: int) -> int:
    """Pillow's ksize for the bilinear filter: ceil(support) * 2 + 1."""
    return int(math.ceil(max(float(in_size) / out_size, 1.0))) * 2 + 1


class GpuTransform:
    """The reference's train / val transform chain for a batch of decoded images, on the GPU.

    ``__call__(images, generator=None, params=None)``: ``images`` is a list of [H, W, 3] uint8
    arrays (or uint8 tensors); returns f32 [B, 3, size, size] on ``device``.  ``params``
    (train only) overrides the random draw with explicit ``(top, left, h, w, flip)`` tuples."""

    def __init__(self, train: bool = True, size: int = 224, resize: int = 256, device="cuda",
                 mean: Sequence[float] = MEAN, std: Sequence[float] = STD):
        self.train, self.size, self.resize = train, size, resize
        self.device = torch.device(device)
        self.norm6 = (torch.tensor(list(mean) + list(std), dtype=torch.float32)).numpy()

    def draw(self, shapes: Sequence[Tuple[int, int]], generator=None) -> List[Tuple[int, int, int, int, bool]]:
        out = []
        for h, w in shapes:
            t, l, ch, cw = random_resized_crop_params(h, w, generator)
            flip = bool(torch.rand(1, generator=generator).item() < 0.5)
            out.append((t, l, ch, cw, flip))
        return out

    def plan(self, shapes, generator=None, params=None) -> np.ndarray:
        """int64 [B][12] kernel parameters (see image.hip) for images of the given (H, W)."""
        S = self.size
        B = len(shapes)
        tab = np.zeros((B, _NPARAM), dtype=np.int64)
        if self.train and params is None:
            params = self.draw(shapes, generator)
        off = tmp = 0
        for b, (H, W) in enumerate(shapes):
            if self.train:
                top, left, h, w, flip = params[b]
                RH = RW = S
                oy0 = ox0 = 0
            else:
                top = left = 0
                h, w, flip = H, W, False
                RH, RW = resize_shorter(H, W, self.resize)
                oy0, ox0 = int(round((RH - S) / 2.0)), int(round((RW - S) / 2.0))
            if not (0 <= top and 0 <= left and 0 < h and 0 < w and top + h <= H and left + w <= W):
                raise ValueError(f"image {b}: crop ({top}, {left}, {h}, {w}) outside {H}x{W}")
            if not (0 <= oy0 and 0 <= ox0 and oy0 + S <= RH and ox0 + S <= RW):
                raise ValueError(f"image {b}: {S}x{S} window at ({oy0}, {ox0}) outside {RH}x{RW} "
                                 "(CenterCrop padding is not supported)")
            tab[b] = (off, W, top, left, h, w, RH, RW, oy0, ox0, int(flip), tmp)
            off += H * W * 3
            tmp += h * S * 3
        return tab

    def stage(self, images, generator=None, params=None):
        """Host half: draw / validate the parameters, pack the uint8 images into one pinned buffer
        and queue one host-to-device copy.  Returns the device-side batch for ``apply``."""
        shapes = [(int(im.shape[0]), int(im.shape[1])) for im in images]
        for im in images:
            if im.ndim != 3 or im.shape[2] != 3 or (im.dtype not in (np.uint8, torch.uint8)):
                raise ValueError("images must be [H, W, 3] uint8")
        tab = self.plan(shapes, generator, params)
        total = int(sum(h * w * 3 for h, w in shapes))
        host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        hv = host.numpy()
        for b, im in enumerate(images):
            a = im.numpy() if isinstance(im, torch.Tensor) else im
            n = a.shape[0] * a.shape[1] * 3
            hv[tab[b, 0]:tab[b, 0] + n] = np.ascontiguousarray(a).reshape(-1)
        staged = {"tab": tab, "host": host}
        if len(images):
            staged["src"] = host.to(self.device, non_blocking=True)
            staged["params"] = torch.from_numpy(tab).to(self.device, non_blocking=True)
        return staged

    def apply(self, staged) -> torch.Tensor:
        """Device half: one ``vit_image_transform`` call over a staged batch -> f32 [B, 3, S, S]."""
        S = self.size
        tab = staged["tab"]
        B = tab.shape[0]
        out = torch.empty(B, 3, S, S, dtype=torch.float32, device=self.device)
        if B == 0:
            return out
        L.require_gpu(out)
        kmax = max(max(_taps(int(t[5]), int(t[7])), _taps(int(t[4]), int(t[6]))) for t in tab)
        max_rows = int(tab[:, 4].max())
        tmp = torch.empty(int((tab[:, 4] * S * 3).sum()), dtype=torch.uint8, device=self.device)
        cws = torch.empty(L.lib().vit_image_coeff_bytes(B, S, kmax), dtype=torch.uint8, device=self.device)
        call("vit_image_transform", B, S, ptr(staged["src"]), ptr(staged["params"]), kmax, max_rows, ptr(cws),
             ptr(tmp), ptr(out), self.norm6.ctypes.data, L.stream_ptr(self.device))
        # the staging buffers are read by the queued kernels: keep them alive until they ran
        ev = torch.cuda.Event()
        ev.record()
        self._inflight = (staged, tmp, cws, ev)
        return out

    def __call__(self, images, generator=None, params=None) -> torch.Tensor:
        return self.apply(self.stage(images, generator, params))


def gaussian_noise(batch: torch.Tensor, epsilon: float = 0.1, generator=None) -> torch.Tensor:
    """MEAS:36-46 GaussianNoiseTransform: the transformed image is replaced by randn * epsilon."""
    return torch.randn(batch.shape, generator=generator, device=batch.device, dtype=batch.dtype) * epsilon


def uniform_gray(batch: torch.Tensor) -> torch.Tensor:
    """MEAS:48-57 UniformGrayTransform: the transformed image is replaced by zeros."""
    return torch.zeros_like(batch)
