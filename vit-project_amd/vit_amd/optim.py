"""Fused optimizers and the reference LR schedule.

``FusedSGD`` is ``torch.optim.SGD(params, lr, momentum, weight_decay)`` (VIT:294-299,
dampening 0, nesterov off) as ONE multi-tensor HIP launch over every parameter:
``d = g + wd*p; buf = momentum*buf + d; p -= lr*buf`` (zero-initialised ``buf``
makes the first step identical to torch's ``buf = d.clone()``), writing the bf16
GEMM shadow of each weight in the same pass.  ``lr`` lives in a device scalar so
a captured HIP graph follows the schedule (call :meth:`sync_lr` outside the graph).

``FusedAdamW`` is ``torch.optim.AdamW`` (NEWP:1181; amsgrad off) the same way; its per-step
bias corrections travel in a separate device array, so its tensor table is fixed too.
``CosineAnnealingLRWithWarmup`` restates VIT:206-244 (stepped once per epoch
after training, so epoch 0 runs at the base LR: quirk Q1).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib as L
from ._lib import call


def _table(entries, struct_fields):
    """Pack a list of tuples into a device table matching the C struct layout
    {ptr, ptr, ptr, ptr, int64} (5 x 8 bytes)."""
    arr = np.zeros((len(entries), struct_fields), dtype=np.int64)
    for i, e in enumerate(entries):
        arr[i] = [0 if v is None else int(v) for v in e]
    return arr


class _MultiTensor:
    CHUNK = 4096

    def __init__(self, device, fields=5):
        self.device = device
        self.fields = fields
        self._key = None
        self._tdev = None
        self._cdev = None
        self._pinned = None
        self.nchunks = 0

    def build(self, entries, sizes):
        key = tuple(tuple(0 if v is None else int(v) for v in e) for e in entries)
        if key == self._key:
            return
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("optimizer tensor table changed during HIP-graph capture: enable "
                               "model.use_flat_grads() so gradient addresses are fixed, and warm up once "
                               "before capturing")
        t = _table(entries, self.fields)
        chunks = []
        for i, n in enumerate(sizes):
            for s in range(0, n, self.CHUNK):
                chunks.append((i, s))
        c = np.zeros((len(chunks), 2), dtype=np.int64)
        for k, (i, s) in enumerate(chunks):
            c[k, 0] = i  # {int tensor; int pad} packed little-endian in one int64
            c[k, 1] = s
        tb = torch.from_numpy(t.reshape(-1).view(np.uint8).copy())
        cb = torch.from_numpy(c.reshape(-1).view(np.uint8).copy())
        host = torch.cat([tb, cb]).pin_memory() if torch.cuda.is_available() else torch.cat([tb, cb])
        dev = torch.empty(host.numel(), dtype=torch.uint8, device=self.device)
        dev.copy_(host, non_blocking=True)
        self._pinned = host  # keep alive for async copy / graph replay
        self._tdev = dev[: tb.numel()]
        self._cdev = dev[tb.numel():]
        self.nchunks = len(chunks)
        self._key = key


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=0.1, momentum=0.9, weight_decay=1e-4, dampening=0.0, nesterov=False):
        if dampening != 0 or nesterov:
            raise ValueError("FusedSGD implements the reference configuration: dampening 0, nesterov False")
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, dampening=0.0,
                                      nesterov=False))
        self._mt = None
        self._lr_dev = None
        self._lr_host = None

    def _device(self):
        for g in self.param_groups:
            for p in g["params"]:
                return p.device
        return None

    def sync_lr(self):
        """Copy param_groups[0]['lr'] into the device scalar the kernel reads."""
        lrs = {g["lr"] for g in self.param_groups}
        if len(lrs) != 1:
            raise ValueError("FusedSGD supports one LR across param groups")
        lr = lrs.pop()
        dev = self._device()
        if self._lr_dev is None:
            self._lr_dev = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
            self._lr_host = lr
        elif lr != self._lr_host:
            self._lr_dev.fill_(float(lr))
            self._lr_host = lr

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        dev = self._device()
        L.require_gpu(torch.empty(0, device=dev))
        if self._mt is None:
            self._mt = _MultiTensor(dev)
        if self._lr_dev is None or not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        g0 = self.param_groups[0]
        mom, wd = g0["momentum"], g0["weight_decay"]
        for g in self.param_groups:
            if g["momentum"] != mom or g["weight_decay"] != wd:
                raise ValueError("FusedSGD supports one (momentum, weight_decay) across groups")
        entries, sizes = [], []
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    p.grad = p.grad.float().contiguous()
                st = self.state[p]
                if "momentum_buffer" not in st:
                    st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                sh = getattr(p, "_vit_shadow", None)
                entries.append((p.data_ptr(), p.grad.data_ptr(), st["momentum_buffer"].data_ptr(),
                                None if sh is None else sh.data_ptr(), p.numel()))
                sizes.append(p.numel())
        if not entries:
            return loss
        self._mt.build(entries, sizes)
        call("vit_sgd_step", self._mt._tdev.data_ptr(), self._mt._cdev.data_ptr(), self._mt.nchunks,
             self._lr_dev.data_ptr(), float(mom), float(wd), L.stream_ptr(dev))
        # raw-pointer update: bump versions; the shadows the kernel wrote stay fresh
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    _mark_updated(p)
        return loss


def _mark_updated(p: torch.Tensor):
    """A parameter was rewritten through a raw pointer: bump its version counter (what an
    in-place torch op would do), so version-keyed caches (the bf16 GEMM shadow, the CLIP
    frozen-prefix cache) see the change; a shadow the kernel itself rewrote stays fresh."""
    torch.autograd.graph.increment_version(p)
    if getattr(p, "_vit_shadow", None) is not None:
        p._vit_shadow_version = p._version


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (NEWP:1181; amsgrad off, maximize off) as one launch per group.

    Per-parameter state matches torch's (``step`` a float32 scalar tensor, ``exp_avg``,
    ``exp_avg_sq``), so ``state_dict()`` / ``load_state_dict()`` round-trip with
    ``torch.optim.AdamW`` and a resumed optimizer (NEWP:1189-1195) continues each tensor's
    bias correction from its saved ``step``.  Bias corrections are computed in double on the
    host per tensor, as torch's single-tensor path does, into a small device array (one
    host-to-device copy per step from a pinned ring); the tensor table the kernel reads holds
    only pointers and sizes, so it is built once and stays fixed.  The kernel also refreshes
    the bf16 GEMM shadow of shadowed weights.

    HIP-graph capture: after one eager step (which builds the table), ``step()`` under capture
    records the update kernel only; call :meth:`prepare_replay` outside the graph before each
    replay -- it advances every ``state['step']`` and uploads that step's coefficients."""

    RING = 4  # pinned coefficient buffers in flight (the host waits only when it is RING steps ahead)

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._mt = {}
        self._coef = {}   # group index -> device float32 [4 * ntensors]
        self._ring = {}   # group index -> [pinned host buffer, event or None] * RING
        self._ring_pos = {}
        self._captured = {}  # group index -> the parameter list a capture recorded

    def _group_params(self, group):
        return [p for p in group["params"] if p.grad is not None]

    def _advance(self, group, params):
        """state['step'] += 1 for each tensor; the (lr / bc1, sqrt(bc2), 1 - lr * wd, 0) rows of the
        new step (the decay is per step too, so a replay follows a changed lr in both terms)."""
        lr, (b1, b2) = float(group["lr"]), group["betas"]
        decay = 1.0 - lr * float(group["weight_decay"])
        coef = np.zeros(4 * len(params), dtype=np.float32)
        for i, p in enumerate(params):
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["step"] += 1
            step = float(st["step"].item())
            coef[4 * i] = lr / (1.0 - b1 ** step)
            coef[4 * i + 1] = math.sqrt(1.0 - b2 ** step)
            coef[4 * i + 2] = decay
        return coef

    def _upload(self, gi, coef, dev, replay=False):
        """One async copy of this step's coefficients into the group's device array, through a
        ring of pinned buffers (a buffer is rewritten only after its previous copy finished).
        ``replay``: the array is the one a captured graph reads, so it must not be reallocated."""
        cd = self._coef.get(gi)
        if replay and (cd is None or cd.numel() != coef.size or cd.device != dev):
            raise RuntimeError("FusedAdamW.prepare_replay: the captured coefficient array does not match "
                               "the captured parameter list; re-capture the graph")
        if cd is None or cd.numel() != coef.size or cd.device != dev:
            cd = self._coef[gi] = torch.empty(coef.size, dtype=torch.float32, device=dev)
            self._ring[gi] = [[torch.empty(coef.size, dtype=torch.float32).pin_memory(), None]
                              for _ in range(self.RING)]
            self._ring_pos[gi] = 0
        k = self._ring_pos[gi]
        slot = self._ring[gi][k]
        if slot[1] is not None:
            slot[1].synchronize()
        slot[0].numpy()[:] = coef
        cd.copy_(slot[0], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slot[1] = ev
        self._ring_pos[gi] = (k + 1) % self.RING
        return cd

    @torch.no_grad()
    def prepare_replay(self):
        """Before each replay of a graph that captured ``step()``: advance the steps and upload
        the coefficients the captured kernel will read (eager mode never needs this)."""
        for gi, group in enumerate(self.param_groups):
            params = self._captured.get(gi)
            if params:
                self._upload(gi, self._advance(group, params), params[0].device, replay=True)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        for gi, group in enumerate(self.param_groups):
            params = self._group_params(group)
            if not params:
                continue
            dev = params[0].device
            L.require_gpu(torch.empty(0, device=dev))
            (b1, b2), eps = group["betas"], float(group["eps"])
            if capturing:
                if self._coef.get(gi) is None:
                    raise RuntimeError("FusedAdamW: run one eager step() before capturing (it builds the tensor "
                                       "table and the coefficient buffer); then call prepare_replay() before "
                                       "each replay")
                cd = self._coef[gi]
                if cd.numel() != 4 * len(params):
                    raise RuntimeError(f"FusedAdamW: capturing {len(params)} tensors with gradients in group {gi}, "
                                       f"but the last eager step() built the table for {cd.numel() // 4}; run an "
                                       "eager step with the same parameters first")
                self._captured[gi] = params
            else:
                coef = self._advance(group, params)
                for p in params:
                    st = self.state[p]
                    if not p.grad.is_contiguous() or p.grad.dtype != torch.float32:
                        p.grad = p.grad.float().contiguous()
                    for k in ("exp_avg", "exp_avg_sq"):
                        if st[k].device != p.device or not st[k].is_contiguous():
                            st[k] = st[k].to(p.device).contiguous()
                cd = self._upload(gi, coef, dev)
            entries, sizes = [], []
            base = cd.data_ptr()
            for i, p in enumerate(params):
                st = self.state[p]
                sh = getattr(p, "_vit_shadow", None)
                entries.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                                None if sh is None else sh.data_ptr(), p.numel(), base + 16 * i))
                sizes.append(p.numel())
            mt = self._mt.get(gi)
            if mt is None:
                mt = self._mt[gi] = _MultiTensor(dev, fields=7)
            mt.build(entries, sizes)
            call("vit_adamw_step", mt._tdev.data_ptr(), mt._cdev.data_ptr(), mt.nchunks,
                 float(b1), float(b2), eps, L.stream_ptr(dev))
            for p in params:
                _mark_updated(p)
        return loss


class CosineAnnealingLRWithWarmup:
    """Linear warmup then cosine, stepped once per epoch (VIT:206-244)."""

    def __init__(self, optimizer, warmup_epochs, max_epochs, eta_min=0):
        self.optimizer = optimizer
        self.warmup_epochs = warmup_epochs
        self.max_epochs = max_epochs
        self.eta_min = eta_min
        self.base_lrs = [g["lr"] for g in optimizer.param_groups]
        self.current_epoch = 0

    def lr_at(self, c: int, base_lr: float) -> float:
        if c < self.warmup_epochs:
            return base_lr * ((c + 1) / self.warmup_epochs)
        progress = (c - self.warmup_epochs) / (self.max_epochs - self.warmup_epochs)
        return self.eta_min + (base_lr - self.eta_min) * 0.5 * (1 + math.cos(math.pi * progress))

    def step(self):
        for g, base in zip(self.optimizer.param_groups, self.base_lrs):
            g["lr"] = self.lr_at(self.current_epoch, base)
        self.current_epoch += 1

    def state_dict(self):
        return {"current_epoch": self.current_epoch, "base_lrs": self.base_lrs,
                "warmup_epochs": self.warmup_epochs, "max_epochs": self.max_epochs, "eta_min": self.eta_min}

    def load_state_dict(self, sd):
        self.current_epoch = sd["current_epoch"]
        self.base_lrs = sd["base_lrs"]
        self.warmup_epochs = sd["warmup_epochs"]
        self.max_epochs = sd["max_epochs"]
        self.eta_min = sd["eta_min"]
