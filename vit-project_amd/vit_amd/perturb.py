"""Perturbation windows of the CLIP-HBA sweeps (NEWP = Training/functions/
new_cvpr_train_behavior_things_pipeline.py).

Host-side rules the training loop applies around every step, mirrored so a sweep driver on
this package makes the same decisions as the reference:

  * the window: condition ``training_run`` (1-based start epoch) perturbs the 0-based epochs
    ``[training_run - 1, training_run - 1 + perturb_length - 1]`` (NEWP:843-871, 1043-1046);
  * per-batch seeding ``perturb_seed + training_run * 1000 + batch_idx`` (NEWP:882, 920, 939);
  * ``random_target``: ``randn(targets.shape, generator) [* std + mean]`` (NEWP:918-927);
  * ``label_shuffle``: :func:`shuffle_targets` (NEWP:731-779, called at NEWP:959);
  * ``image_noise``: every image replaced by ``randn * std + mean`` drawn after
    ``torch.manual_seed(seed)`` (NEWP:880-897, replace_with_gaussian_noise NEWP:207-221;
    quirk Q4: the *target* mean/std are used for pixels);
  * ``uniform_images``: ``ones_like(images) * 0.5`` (NEWP:904-906, quirk Q4);
  * perturbation-aware early stopping (NEWP:1048-1063).

These are data-side draws on torch generators, not kernels.  On a ROCm device the Philox
stream differs from CUDA's (SURVEY §7 hard parts), so bit-identical perturbations across
vendors hold for CPU generators only (tests/golden/perturb_golden.pt pins those).
"""
from __future__ import annotations

import random

import numpy as np
import torch

KINDS = ("random_target", "label_shuffle", "image_noise", "uniform_images")


def window(training_run: int, perturb_length: int):
    """0-based (first, last) perturbed epoch of a condition (NEWP:844-845)."""
    start = training_run - 1
    return start, start + perturb_length - 1


def in_window(epoch: int, training_run: int, perturb_length: int) -> bool:
    s, e = window(training_run, perturb_length)
    return s <= epoch <= e


def batch_seed(perturb_seed: int, training_run: int, batch_idx: int) -> int:
    return perturb_seed + training_run * 1000 + batch_idx


def shuffle_targets(targets, perturb_seed=None, generator=None):
    """NEWP:731-779: permute the batch rows of ``targets`` (values kept, pairing broken)."""
    saved = None
    if generator is None and perturb_seed is not None:
        saved = (torch.get_rng_state(), np.random.get_state(), random.getstate())
        torch.manual_seed(perturb_seed)
        np.random.seed(perturb_seed)
        random.seed(perturb_seed)
    out = targets.clone()
    if generator is not None:
        perm = torch.randperm(targets.shape[0], device=targets.device, generator=generator)
    else:
        perm = torch.randperm(targets.shape[0], device=targets.device)
    out = out[perm]
    if saved is not None:
        torch.set_rng_state(saved[0])
        np.random.set_state(saved[1])
        random.setstate(saved[2])
    return out


def random_targets(shape, seed: int, device, distribution="target", mean=0.0, std=1.0):
    """NEWP:918-927: a fresh generator per batch seeded with ``batch_seed``."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    t = torch.randn(shape, device=device, dtype=torch.float32, generator=g)
    if distribution == "target":
        t = t * std + mean
    elif distribution != "normal":
        raise ValueError(f"perturb_distribution {distribution!r}")
    return t


def noise_images(images, seed: int, mean: float, std: float):
    """NEWP:880-897: torch.manual_seed(seed) (+ cuda seed), then each image replaced in order."""
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    for i in range(len(images)):
        C, H, W = images[i].shape
        images[i] = torch.randn((C, H, W), device=images.device) * std + mean
    return images


def uniform_images(images):
    """NEWP:904-906 (quirk Q4: 0.5 in normalised space)."""
    return torch.ones_like(images) * 0.5


def perturb_batch(kind, images, targets, *, epoch, batch_idx, training_run, perturb_length, perturb_seed,
                  mean=0.0, std=1.0, distribution="target"):
    """Apply the condition's perturbation to one batch if ``epoch`` is inside its window;
    returns (images, targets) ready for the step (NEWP:874-959)."""
    if kind is None or not in_window(epoch, training_run, perturb_length):
        return images, targets
    s = batch_seed(perturb_seed, training_run, batch_idx)
    if kind == "image_noise":
        images = noise_images(images, s, mean, std)
    elif kind == "uniform_images":
        images = uniform_images(images)
    elif kind == "random_target":
        targets = random_targets(targets.shape, s, targets.device, distribution, mean, std)
    elif kind == "label_shuffle":
        g = torch.Generator(device=targets.device)
        g.manual_seed(s)
        targets = shuffle_targets(targets, generator=g)
    else:
        raise ValueError(f"perturb_type {kind!r}; known {KINDS}")
    return images, targets


class EarlyStopping:
    """NEWP:1048-1063: the patience counter does not advance inside the perturbation window."""

    def __init__(self, patience: int, training_run: int, perturb_length: int, best=500000.0):
        self.patience, self.run, self.length = patience, training_run, perturb_length
        self.best, self.bad = best, 0

    def step(self, epoch: int, test_loss: float) -> bool:
        """Record one epoch; True when training should stop."""
        if test_loss < self.best:
            self.best, self.bad = test_loss, 0
        elif not in_window(epoch, self.run, self.length):
            self.bad += 1
        return self.bad == self.patience
