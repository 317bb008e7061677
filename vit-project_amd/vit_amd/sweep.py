"""Perturbation-sweep runner for the CLIP-HBA DoRA fine-tuning (config C5).

Mirrors the reference's per-condition training loop and its on-disk formats so sweeps run on
this package resume from, and write, the same files (NEWP = Training/functions/
new_cvpr_train_behavior_things_pipeline.py):

  * ``save_dora_parameters`` / ``load_dora_parameters``: ``epoch{N}_dora_params.pth`` holding
    ``<module path>.m / .delta_D_A / .delta_D_B`` of the three DoRA ``out_proj`` layers
    (NEWP:657-694; loaded with ``load_state_dict(strict=False)`` as NEWP:1168 does);
  * ``save_random_states`` / ``load_random_states``: ``epoch{N}_random_states.pth`` with the
    reference's keys (``epoch, optimizer_state_dict, torch_rng_state, numpy_rng_state,
    python_rng_state, dataloader_generator_state[, cuda_rng_state(_all)]``, NEWP:88-135, 696-729);
  * the training-results CSV with the reference's header row (NEWP:795-797, 1017-1023);
  * ``train_condition``: the epoch loop of ``train_model`` (NEWP:782-1063) -- perturbed batches
    (``perturb.perturb_batch``), MSE step, test loss, behavioural RSA, CSV row, DoRA and RNG
    checkpoints, perturbation-aware early stopping;
  * ``run_sweep``: the conditions of this rank (``parallel.shard_conditions``: start-epoch chains
    stay on one GPU), each resumed from the baseline run's epoch ``training_run - 1`` files.

Data is whatever the caller passes as (images, targets) tensors -- THINGS images and SPOSE
targets are not in the reference tree; the driver's tests use synthetic ones.  The RNG-state
files are pickles holding numpy / Python RNG tuples, exactly as the reference writes them:
``load_random_states`` is meant for files this runner (or the reference) wrote, and reads them
with ``weights_only=False`` for that reason only.
"""
from __future__ import annotations

import csv
import os
import random
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import perturb as P
from . import rsa as RSA
from .parallel import shard_conditions

CSV_HEADERS = ['epoch', 'train_loss', 'test_loss', 'behavioral_rsa_rho', 'behavioral_rsa_p_value',
               'used_random_targets', 'used_shuffled_targets', 'used_uniform_images', 'used_image_noise']

# NEWP:666-670: the DoRA layers of CLIPHBA(ViT-L/14) with n_vision_layers=2, n_transformer_layers=1
DORA_MODULES = ("clip_model.visual.transformer.resblocks.22.attn.out_proj",
                "clip_model.visual.transformer.resblocks.23.attn.out_proj",
                "clip_model.transformer.resblocks.11.attn.out_proj")


def _module(model, path):
    m = model
    for attr in path.split("."):
        m = getattr(m, attr)
    return m


def save_dora_parameters(model, dora_parameters_path, epoch, modules=DORA_MODULES):
    """NEWP:657-694: one file per epoch, keys ``<path>.m``, ``.delta_D_A``, ``.delta_D_B`` (CPU tensors)."""
    params = {}
    for path in modules:
        mod = _module(model, path)
        params[f"{path}.m"] = mod.m.detach().cpu()
        params[f"{path}.delta_D_A"] = mod.delta_D_A.detach().cpu()
        params[f"{path}.delta_D_B"] = mod.delta_D_B.detach().cpu()
    os.makedirs(dora_parameters_path, exist_ok=True)
    f = os.path.join(dora_parameters_path, f"epoch{epoch + 1}_dora_params.pth")
    torch.save(params, f)
    return f


def load_dora_parameters(model, dora_parameters_path, epoch):
    """The resume step of NEWP:1160-1170: ``epoch{epoch}_dora_params.pth`` into the model
    (tensors only: ``weights_only=True``)."""
    f = os.path.join(dora_parameters_path, f"epoch{epoch}_dora_params.pth")
    sd = torch.load(f, map_location="cpu", weights_only=True)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    if unexpected:
        raise KeyError(f"{f}: keys not in the model: {unexpected[:3]}")
    return sd


def save_random_states(optimizer, epoch, random_state_path, dataloader_generator):
    """NEWP:696-729 (same keys, same file name)."""
    ck = {
        'epoch': epoch,
        'optimizer_state_dict': optimizer.state_dict(),
        'torch_rng_state': torch.get_rng_state(),
        'numpy_rng_state': np.random.get_state(),
        'python_rng_state': random.getstate(),
        'dataloader_generator_state': dataloader_generator.get_state(),
    }
    if torch.cuda.is_available():
        ck['cuda_rng_state'] = torch.cuda.get_rng_state()
        ck['cuda_rng_state_all'] = torch.cuda.get_rng_state_all()
    os.makedirs(random_state_path, exist_ok=True)
    f = os.path.join(random_state_path, f"epoch{epoch + 1}_random_states.pth")
    torch.save(ck, f)
    return f


def load_random_states(random_state_path, epoch, optimizer=None, dataloader_generator=None) -> bool:
    """NEWP:88-135; False when the file does not exist (the reference's behaviour)."""
    f = os.path.join(random_state_path, f"epoch{epoch}_random_states.pth")
    if not os.path.exists(f):
        return False
    ck = torch.load(f, weights_only=False)  # numpy / Python RNG tuples (see module docstring)
    torch.set_rng_state(ck['torch_rng_state'])
    np.random.set_state(ck['numpy_rng_state'])
    random.setstate(ck['python_rng_state'])
    if torch.cuda.is_available() and 'cuda_rng_state' in ck:
        torch.cuda.set_rng_state(ck['cuda_rng_state'])
        if 'cuda_rng_state_all' in ck:
            torch.cuda.set_rng_state_all(ck['cuda_rng_state_all'])
    if optimizer is not None and 'optimizer_state_dict' in ck:
        optimizer.load_state_dict(ck['optimizer_state_dict'])
    if dataloader_generator is not None and 'dataloader_generator_state' in ck:
        dataloader_generator.set_state(ck['dataloader_generator_state'])
    return True


def _batches(images, targets, batch_size, generator, shuffle=True):
    """torch DataLoader(shuffle=True, generator=g) order over in-memory tensors."""
    n = images.shape[0]
    order = torch.randperm(n, generator=generator) if shuffle else torch.arange(n)
    for i in range(0, n, batch_size):
        idx = order[i:i + batch_size]
        yield images[idx], targets[idx]


def evaluate(model, images, targets, batch_size, criterion):
    """NEWP:584-602: mean criterion over the test set (no grad)."""
    model.eval()
    tot, n = 0.0, 0
    with torch.no_grad():
        for x, y in _batches(images, targets, batch_size, None, shuffle=False):
            pred = model(x)
            tot += float(criterion(pred, y)) * x.shape[0]
            n += x.shape[0]
    model.train()
    return tot / max(n, 1)


def behavioral_rsa(model, inference_images, reference_rdm, batch_size=16):
    """NEWP:605-654: 66-D predictions of the 48 inference images -> RDM -> Spearman vs the
    reference RDM (vit_amd.rsa restates the reference's float64 corrcoef / upper triangle)."""
    model.eval()
    with torch.no_grad():
        preds = torch.cat([model(inference_images[i:i + batch_size]).float().cpu()
                           for i in range(0, inference_images.shape[0], batch_size)])
    model.train()
    rho, p, _ = RSA.rsa(preds.numpy().astype(np.float64), reference_rdm)
    return rho, p


def train_condition(model, optimizer, criterion, data, *, epochs, training_run, perturb_length, perturb_type,
                    perturb_seed=42, perturb_distribution="target", batch_size=64, early_stopping_patience=5,
                    training_res_path, dora_parameters_path, random_state_path, dataloader_generator,
                    resume_from_epoch=0, modules=DORA_MODULES):
    """The epoch loop of NEWP:train_model for one (training_run, perturb_length) condition.

    ``data`` = dict(train=(images, targets), test=(images, targets), inference=images,
    reference_rdm=ndarray[48, 48]).  Target mean / std for the perturbations are the scalar
    mean / std over all training targets (NEWP:1098-1105, quirk Q4)."""
    tr_x, tr_y = data["train"]
    te_x, te_y = data["test"]
    mean, std = float(tr_y.mean()), float(tr_y.std())
    if resume_from_epoch == 0 or not os.path.exists(training_res_path):
        with open(training_res_path, "w", newline="") as fh:
            csv.writer(fh).writerow(CSV_HEADERS)
    stopper = P.EarlyStopping(early_stopping_patience, training_run, perturb_length)
    rows = []
    model.train()
    for epoch in range(resume_from_epoch, epochs):
        used = dict(random_target=False, label_shuffle=False, uniform_images=False, image_noise=False)
        total = 0.0
        for batch_idx, (x, y) in enumerate(_batches(tr_x, tr_y, batch_size, dataloader_generator)):
            if P.in_window(epoch, training_run, perturb_length) and perturb_type is not None:
                x, y = P.perturb_batch(perturb_type, x.clone(), y, epoch=epoch, batch_idx=batch_idx,
                                       training_run=training_run, perturb_length=perturb_length,
                                       perturb_seed=perturb_seed, mean=mean, std=std,
                                       distribution=perturb_distribution)
                used[perturb_type] = True
            optimizer.zero_grad()
            loss = criterion(model(x), y)
            loss.backward()
            optimizer.step()
            total += float(loss.detach()) * x.shape[0]
        train_loss = total / tr_x.shape[0]
        test_loss = evaluate(model, te_x, te_y, batch_size, criterion)
        rho, p = behavioral_rsa(model, data["inference"], data["reference_rdm"])
        row = [epoch + 1, train_loss, test_loss, rho, p, used["random_target"], used["label_shuffle"],
               used["uniform_images"], used["image_noise"]]
        with open(training_res_path, "a", newline="") as fh:
            csv.writer(fh).writerow(row)
        rows.append(row)
        save_dora_parameters(model, dora_parameters_path, epoch, modules)
        save_random_states(optimizer, epoch, random_state_path, dataloader_generator)
        if stopper.step(epoch, test_loss):
            break
    return rows


def run_sweep(make_model_and_optimizer, criterion, data, conditions: Sequence[Tuple[int, int]], *, rank=0,
              world=1, perturb_type, out_dir, baseline_dora_path, baseline_random_state_path, epochs,
              **train_kw) -> List[Tuple[Tuple[int, int], str]]:
    """Run this rank's share of ``conditions`` ((training_run, perturb_length) pairs, LEN:42-83).

    Each condition resumes from the baseline run at epoch ``training_run - 1`` (its DoRA file and
    RNG / optimizer state, NEWP:1157-1201), trains to ``epochs`` with the perturbation window,
    and writes its CSV / DoRA / RNG files under ``out_dir/run{start}_len{length}``.  No
    collective: conditions are independent."""
    done = []
    for start, length in shard_conditions(conditions, world, rank):
        model, optimizer = make_model_and_optimizer()
        gen = torch.Generator()
        resume = start - 1
        if resume > 0:
            load_dora_parameters(model, baseline_dora_path, resume)
            load_random_states(baseline_random_state_path, resume, optimizer, gen)
        d = os.path.join(out_dir, f"run{start}_len{length}")
        os.makedirs(d, exist_ok=True)
        res = os.path.join(d, "training_res.csv")
        train_condition(model, optimizer, criterion, data, epochs=epochs, training_run=start, perturb_length=length,
                        perturb_type=perturb_type, training_res_path=res, dora_parameters_path=os.path.join(d, "dora"),
                        random_state_path=os.path.join(d, "random_states"), dataloader_generator=gen,
                        resume_from_epoch=resume, **train_kw)
        done.append(((start, length), res))
    return done
