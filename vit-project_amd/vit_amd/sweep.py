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
files are pickles holding numpy / Python RNG tuples, exactly as the reference writes them.
``load_random_states`` reads them with ``torch.load(weights_only=True)`` and an allow-list of
exactly the globals such a file needs (numpy's ndarray / dtype reconstruction, in both the
numpy 1.x and 2.x module paths); a file naming any other global is refused, so a resume never
executes code from the checkpoint.
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


def _rng_state_globals():
    """The globals a reference RNG-state file references (numpy's MT19937 state is an ndarray
    inside a tuple): ndarray / dtype reconstruction under numpy 2.x (``numpy._core``) and 1.x
    (``numpy.core``), plus the per-dtype classes numpy >= 1.25 pickles dtypes with."""
    import numpy.dtypes as npd
    g = [np.ndarray, np.dtype]
    g += [getattr(npd, n) for n in ("UInt32DType", "Int64DType", "Float64DType") if hasattr(npd, n)]
    for mod in ("numpy._core.multiarray", "numpy.core.multiarray"):
        try:
            m = __import__(mod, fromlist=["_reconstruct"])
        except ImportError:
            continue
        g.append((m._reconstruct, f"{mod}._reconstruct"))
    return g


def load_random_states(random_state_path, epoch, optimizer=None, dataloader_generator=None) -> bool:
    """NEWP:88-135; False when the file does not exist (the reference's behaviour).
    Weights-only load: the allow-list is ``_rng_state_globals``; anything else in the pickle
    raises ``pickle.UnpicklingError`` before any of it runs."""
    f = os.path.join(random_state_path, f"epoch{epoch}_random_states.pth")
    if not os.path.exists(f):
        return False
    with torch.serialization.safe_globals(_rng_state_globals()):
        ck = torch.load(f, map_location="cpu", weights_only=True)
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
                    resume_from_epoch=0, previous_training_res_path=None, modules=DORA_MODULES):
    """The epoch loop of NEWP:train_model for one (training_run, perturb_length) condition.

    ``data`` = dict(train=(images, targets), test=(images, targets), inference=images,
    reference_rdm=ndarray[48, 48]).  Target mean / std for the perturbations are the scalar
    mean / std over all training targets (NEWP:1098-1105, quirk Q4).

    CSV start (NEWP:797-834): resuming in place (``previous_training_res_path`` is this CSV)
    appends; otherwise the file is rewritten with the header and, when resuming from another
    run (a shorter sibling, LEN:246-253), that run's rows for epochs <= ``resume_from_epoch``."""
    tr_x, tr_y = data["train"]
    te_x, te_y = data["test"]
    mean, std = float(tr_y.mean()), float(tr_y.std())
    in_place = (previous_training_res_path == training_res_path and os.path.exists(training_res_path)
                and resume_from_epoch > 0)
    if not in_place:
        with open(training_res_path, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(CSV_HEADERS)
            if previous_training_res_path and resume_from_epoch > 0 and os.path.exists(previous_training_res_path):
                with open(previous_training_res_path, newline="") as prev:
                    r = csv.reader(prev)
                    next(r, None)
                    for row in r:
                        try:
                            if int(row[0]) <= resume_from_epoch:
                                w.writerow(row)
                        except (ValueError, IndexError):
                            continue
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


# The 136 (start epoch, length) conditions of the reference's length sweep, as they are on disk
# under Data/clip_results/perturb_length_experiments_baselineseed1_perturbseed0/random_target_e{E}_l{L}
# (README:47-48): 21 start epochs x lengths {2, 5, 10, 20, 30, 40, 50}, less the 11 that were
# not run (length 2 at starts 13, 16, 19, 58, 94; start 22 only at length 5).
REFERENCE_LENGTHS = (2, 5, 10, 20, 30, 40, 50)
_REFERENCE_STARTS = {1: REFERENCE_LENGTHS, 2: REFERENCE_LENGTHS, 3: REFERENCE_LENGTHS, 6: REFERENCE_LENGTHS,
                     7: REFERENCE_LENGTHS, 8: REFERENCE_LENGTHS, 10: REFERENCE_LENGTHS, 13: REFERENCE_LENGTHS[1:],
                     16: REFERENCE_LENGTHS[1:], 19: REFERENCE_LENGTHS[1:], 20: REFERENCE_LENGTHS, 22: (5,),
                     30: REFERENCE_LENGTHS, 40: REFERENCE_LENGTHS, 50: REFERENCE_LENGTHS,
                     58: REFERENCE_LENGTHS[1:], 60: REFERENCE_LENGTHS, 70: REFERENCE_LENGTHS,
                     80: REFERENCE_LENGTHS, 90: REFERENCE_LENGTHS, 94: REFERENCE_LENGTHS[1:]}


def reference_length_grid() -> List[Tuple[int, int]]:
    """The reference's 136-condition start x duration grid (sorted by start, then length)."""
    return [(e, l) for e in sorted(_REFERENCE_STARTS) for l in _REFERENCE_STARTS[e]]


def condition_dir(out_dir, perturb_type, start, length):
    """LEN's per-condition output directory name (``--output_dir random_target_e2_l2``)."""
    return os.path.join(out_dir, f"{perturb_type}_e{start}_l{length}")


def last_completed_epoch(csv_path) -> int:
    """LEN:137-160: the largest (1-based) epoch in an existing results CSV, 0 if none."""
    last = 0
    if not os.path.exists(csv_path):
        return 0
    with open(csv_path, newline="") as fh:
        r = csv.reader(fh)
        next(r, None)
        for row in r:
            try:
                last = max(last, int(row[0]))
            except (ValueError, IndexError):
                continue
    return last


def find_previous_run_dir(base_dir, perturb_type, start_epoch, current_length):
    """LEN:188-218: the run directory with the same start epoch (token ``e{start}_``, and the
    perturbation type as the name prefix) and the longest length below ``current_length``;
    returns (dir, length) or (None, None).  Candidates longest first (see ``resume_plan``)."""
    c = _sibling_candidates(base_dir, perturb_type, start_epoch, current_length)
    return c[0] if c else (None, None)


def _sibling_candidates(base_dir, perturb_type, start_epoch, current_length):
    out = []
    if not os.path.isdir(base_dir):
        return out
    for name in os.listdir(base_dir):
        full = os.path.join(base_dir, name)
        if not os.path.isdir(full) or f"e{start_epoch}_" not in name:
            continue
        if perturb_type in ("random_target", "label_shuffle") and not name.startswith(perturb_type):
            continue
        length = next((int(p[1:]) for p in name.split("_") if p.startswith("l") and p[1:].isdigit()), None)
        if length is not None and length < current_length:
            out.append((full, length))
    return sorted(out, key=lambda t: -t[1])


def resume_plan(out_dir, perturb_type, start, length, baseline_dora_path, baseline_random_state_path):
    """Where condition (start, length) resumes from, by LEN:137-256 / NEWP:1156-1201:

    1. its own results CSV has epochs: continue in place from the last one (its own
       ``dora_params_{E}`` / ``random_states_{E}``);
    2. else the longest shorter sibling with the same start (same trajectory through the end of
       the sibling's window, since the per-batch perturbation seeds depend only on the start
       epoch and batch): resume at epoch ``start - 1 + sibling_length`` from the sibling's files,
       with its CSV rows up to there.  A sibling whose files for that epoch are missing (it
       stopped early) is passed over for the next shorter one -- the reference would fall back
       to the freshly initialised DoRA parameters there (NEWP:1166-1171);
    3. else the baseline run at epoch ``start - 1``.

    Returns dict(resume_from_epoch, dora_dir, random_state_dir, previous_csv, source)."""
    d = condition_dir(out_dir, perturb_type, start, length)
    own_csv = os.path.join(d, "training_res.csv")
    own_dora, own_rs = os.path.join(d, f"dora_params_{start}"), os.path.join(d, f"random_states_{start}")
    last = last_completed_epoch(own_csv)
    if last > 0:
        return dict(resume_from_epoch=last, dora_dir=own_dora, random_state_dir=own_rs, previous_csv=own_csv,
                    source="self")
    for sib, sib_len in _sibling_candidates(out_dir, perturb_type, start, length):
        ep = max(0, start - 1) + sib_len
        sd, sr = os.path.join(sib, f"dora_params_{start}"), os.path.join(sib, f"random_states_{start}")
        if (os.path.exists(os.path.join(sd, f"epoch{ep}_dora_params.pth"))
                and os.path.exists(os.path.join(sr, f"epoch{ep}_random_states.pth"))):
            return dict(resume_from_epoch=ep, dora_dir=sd, random_state_dir=sr,
                        previous_csv=os.path.join(sib, "training_res.csv"), source=f"sibling l{sib_len}")
    return dict(resume_from_epoch=max(0, start - 1), dora_dir=baseline_dora_path,
                random_state_dir=baseline_random_state_path, previous_csv=None, source="baseline")


def run_sweep(make_model_and_optimizer, criterion, data, conditions: Sequence[Tuple[int, int]], *, rank=0,
              world=1, perturb_type, out_dir, baseline_dora_path, baseline_random_state_path, epochs,
              **train_kw) -> List[Tuple[Tuple[int, int], str]]:
    """Run this rank's share of ``conditions`` ((training_run, perturb_length) pairs, LEN:42-83).

    ``parallel.shard_conditions`` keeps each start epoch's chain on one rank, and a chain runs in
    increasing length, so each condition finds its shorter sibling finished (``resume_plan``).
    Each condition writes LEN's layout: ``out_dir/{perturb_type}_e{E}_l{L}/training_res.csv``,
    ``dora_params_{E}/``, ``random_states_{E}/``.  No collective: conditions are independent
    (SURVEY §8e).  Returns [((start, length), csv path, resume source)]."""
    done = []
    for start, length in shard_conditions(conditions, world, rank):
        plan = resume_plan(out_dir, perturb_type, start, length, baseline_dora_path, baseline_random_state_path)
        d = condition_dir(out_dir, perturb_type, start, length)
        res = os.path.join(d, "training_res.csv")
        if last_completed_epoch(res) >= epochs:
            done.append(((start, length), res, "complete"))
            continue
        model, optimizer = make_model_and_optimizer()
        gen = torch.Generator()
        resume = plan["resume_from_epoch"]
        if resume > 0 and start >= 1:
            load_dora_parameters(model, plan["dora_dir"], resume)
            load_random_states(plan["random_state_dir"], resume, optimizer, gen)
        os.makedirs(d, exist_ok=True)
        train_condition(model, optimizer, criterion, data, epochs=epochs, training_run=start, perturb_length=length,
                        perturb_type=perturb_type, training_res_path=res,
                        dora_parameters_path=os.path.join(d, f"dora_params_{start}"),
                        random_state_path=os.path.join(d, f"random_states_{start}"), dataloader_generator=gen,
                        resume_from_epoch=resume, previous_training_res_path=plan["previous_csv"], **train_kw)
        done.append(((start, length), res, plan["source"]))
    return done


def _sweep_worker(rank, world, make_model_and_optimizer, criterion, data, conditions, kw, results, devices):
    threads = kw.pop("torch_threads", None)
    if threads:
        torch.set_num_threads(threads)
    if devices:
        dev = torch.device("cuda", devices[rank % len(devices)])
        torch.cuda.set_device(dev)
        mv = lambda t: t.to(dev) if torch.is_tensor(t) else t
        data = {k: (tuple(mv(t) for t in v) if isinstance(v, tuple) else mv(v)) for k, v in data.items()}
    out = run_sweep(make_model_and_optimizer, criterion, data, conditions, rank=rank, world=world, **kw)
    results.put((rank, out))


def launch_sweep(nprocs, make_model_and_optimizer, criterion, data, conditions, *, gpus=None, **kw):
    """One process per GPU (or per CPU worker when ``gpus`` is None), each running its
    ``shard_conditions`` share of ``conditions`` through :func:`run_sweep` -- the 8-way sharded
    C5 sweep with no collective.  ``make_model_and_optimizer`` and ``criterion``
    must be picklable (module-level).  Returns {rank: [((start, length), csv, source)]}."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    devices = list(gpus) if gpus else []
    procs = [ctx.Process(target=_sweep_worker,
                         args=(r, nprocs, make_model_and_optimizer, criterion, data, conditions, kw, q, devices))
             for r in range(nprocs)]
    for p in procs:
        p.start()
    import queue as _queue
    out = {}
    try:
        while len(out) < nprocs:
            try:
                r, res = q.get(timeout=1.0)
                out[r] = res
            except _queue.Empty:
                dead = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode not in (None, 0) and i not in out]
                if dead:
                    raise RuntimeError(f"sweep workers failed (rank, exit code): {dead}")
    finally:
        for p in procs:
            if p.exitcode is None and len(out) < nprocs:
                p.terminate()
            p.join()
    return out
