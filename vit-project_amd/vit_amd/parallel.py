"""Multi-GPU plumbing for the two parallel shapes in SURVEY §8(e).

* ViT-B/16 data parallel (config 4, DDP in the reference: VIT:287): one process
  per GPU, gradients written into one flat fp32 buffer by the backward
  (``VisionTransformer.use_flat_grads``) and averaged with a handful of large
  RCCL all-reduces over xGMI (``allreduce_flat``) -- 346 MB per step, bucketed so
  each collective is tens of MB (per-link-bound ring on point-to-point xGMI).
* Perturbation sweeps (config 5): conditions are independent once the baseline
  epoch-(E-1) state exists, so they shard across ranks with no collective at all
  (``shard_conditions``).  Conditions with the same start epoch stay on one rank
  because the length sweep resumes from its shorter sibling (LEN:188-256).
"""
from __future__ import annotations

import os
from typing import Iterable, List, Sequence, Tuple

import torch
import torch.distributed as dist


def init_from_env(backend: str = "nccl"):
    """torchrun-style rendezvous (VIT:13-27).  Returns (rank, world, local_rank)."""
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        return 0, 1, 0
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, init_method="env://")
    return rank, world, local


def bucket_bounds(n: int, bucket_elems: int) -> List[Tuple[int, int]]:
    out, s = [], 0
    while s < n:
        e = min(n, s + bucket_elems)
        out.append((s, e))
        s = e
    return out


def allreduce_flat(flat: torch.Tensor, bucket_mb: float = 64.0, group=None, average: bool = True):
    """Average a flat gradient buffer across the group in fixed-size buckets."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return flat
    world = dist.get_world_size(group)
    elems = max(1, int(bucket_mb * 1024 * 1024 // flat.element_size()))
    use_avg = average and dist.get_backend(group) == "nccl"
    for s, e in bucket_bounds(flat.numel(), elems):
        seg = flat[s:e]
        if use_avg:
            dist.all_reduce(seg, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=group)
            if average:
                seg.div_(world)
    return flat


class OverlappedGradReduce:
    """Data-parallel gradient averaging overlapped with the backward (what DDP's bucket hooks do
    for the reference, VIT:287), for a model with flat gradients (``use_flat_grads``).

    When a transformer block's backward has enqueued its weight / bias gradients, the block's
    contiguous slice of the flat buffer (~28 MB for ViT-B/16) is all-reduced asynchronously: the
    collective is issued from the stream that produced the gradients, so RCCL's stream waits for
    exactly that work and the reduction runs beside the rest of the backward.  ``finish()``
    reduces the ranges no block covered (final norm / head first in the buffer, the patch
    embedding last) and makes the caller's stream wait for every collective -- call it after
    ``loss.backward()`` and before the optimizer step."""

    def __init__(self, model, group=None):
        self.model, self.group = model, group
        self.flat = model.flat_grad
        assert self.flat is not None, "use_flat_grads(True) first"
        self.world = dist.get_world_size(group)
        self.use_avg = dist.get_backend(group) == "nccl"  # gloo has no AVG: SUM, then divide
        self.pending, self.covered = [], []
        model.set_grad_ready_hook(self._span_ready)
        if hasattr(model, "set_deferred_grad_join"):
            model.set_deferred_grad_join(True)  # gradients are read only in finish()

    def _reduce(self, lo, hi):
        seg = self.flat[lo:hi]
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        self.pending.append((dist.all_reduce(seg, op=op, group=self.group, async_op=True), seg))
        self.covered.append((lo, hi))

    def _span_ready(self, lo, hi):
        if self.world > 1:
            self._reduce(lo, hi)

    def finish(self):
        if self.world > 1:
            pos = 0
            for lo, hi in sorted(self.covered):
                if lo > pos:
                    self._reduce(pos, lo)
                pos = max(pos, hi)
            if pos < self.flat.numel():
                self._reduce(pos, self.flat.numel())
            for work, seg in self.pending:
                work.wait()
                if not self.use_avg:
                    seg.div_(self.world)
        self.pending, self.covered = [], []
        return self.flat


def shard_conditions(conditions: Sequence[Tuple[int, int]], world: int, rank: int,
                     cost=lambda c: c[1]) -> List[Tuple[int, int]]:
    """Deterministic assignment of (start_epoch, length) conditions to ranks.

    Conditions sharing a start epoch form one chain (a longer run resumes from the
    longest shorter sibling, LEN:188-256) and go to the same rank; chains are
    placed largest-cost first on the least-loaded rank (LPT greedy)."""
    chains = {}
    for c in conditions:
        chains.setdefault(c[0], []).append(c)
    items = sorted(chains.items(), key=lambda kv: (-sum(cost(c) for c in kv[1]), kv[0]))
    load = [0.0] * world
    owner = {}
    for start, cs in items:
        r = min(range(world), key=lambda i: (load[i], i))
        load[r] += sum(cost(c) for c in cs)
        owner[start] = r
    mine = [c for c in conditions if owner[c[0]] == rank]
    return sorted(mine, key=lambda c: (c[0], c[1]))


def length_sweep_conditions(starts=None, lengths=None):
    """The start x duration conditions of the length sweep (LEN:42-83).  Default: the reference's
    own 136-condition grid (``sweep.reference_length_grid``, README:47-48); with ``starts`` /
    ``lengths`` the full product of the two."""
    if starts is None and lengths is None:
        from .sweep import reference_length_grid
        return reference_length_grid()
    from .sweep import REFERENCE_LENGTHS
    return [(e, l) for e in (starts or range(1, 17)) for l in (lengths or REFERENCE_LENGTHS)]
