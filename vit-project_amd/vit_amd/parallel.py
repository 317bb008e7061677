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


def length_sweep_conditions(max_epoch: int = 16, lengths: Iterable[int] = (1, 2, 4, 8, 16, 32, 64, 100)):
    """A start x duration grid in the shape of the reference's 136-condition sweep
    (README:47-48); the exact grid is a driver argument (LEN:42-83)."""
    return [(e, l) for e in range(1, max_epoch + 1) for l in lengths if l <= 100]
