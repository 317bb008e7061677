"""Representational similarity analysis (host side).

behavioral_RSA (NEWP:605-654) and compute_rsa_score (MEAS:298-355) both do:
``1 - np.corrcoef(emb)`` (float64), zero diagonal, upper triangle (k=1) against
the reference RDM, Spearman rho with average ranks on ties.  48 x 48 -> 1128
pairs: a few microseconds of host work, deliberately not a kernel.
"""
from __future__ import annotations

import numpy as np


def model_rdm(emb) -> np.ndarray:
    e = np.asarray(emb, dtype=np.float64)
    r = 1.0 - np.corrcoef(e)
    np.fill_diagonal(r, 0.0)
    return r


def _rankdata(a: np.ndarray) -> np.ndarray:
    """Average ranks (1-based) with ties shared, as scipy.stats.rankdata(method='average')."""
    order = np.argsort(a, kind="mergesort")
    s = a[order]
    ranks = np.empty(len(a), dtype=np.float64)
    i = 0
    n = len(a)
    while i < n:
        j = i
        while j + 1 < n and s[j + 1] == s[i]:
            j += 1
        ranks[order[i:j + 1]] = 0.5 * (i + j) + 1.0
        i = j + 1
    return ranks


def spearman(x, y):
    """(rho, two-sided p) as scipy.stats.spearmanr for 1-D inputs."""
    from math import erfc, sqrt
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    rx, ry = _rankdata(x), _rankdata(y)
    rx -= rx.mean()
    ry -= ry.mean()
    rho = float((rx * ry).sum() / np.sqrt((rx * rx).sum() * (ry * ry).sum()))
    n = len(x)
    # scipy: t = rho*sqrt((n-2)/((rho+1)(1-rho))), p = 2*sf(|t|, n-2) (Student t)
    dof = n - 2
    if abs(rho) >= 1.0:
        return rho, 0.0
    t = rho * np.sqrt(dof / ((rho + 1.0) * (1.0 - rho)))
    try:
        from scipy.stats import t as student_t
        p = float(2 * student_t.sf(abs(t), dof))
    except Exception:  # pragma: no cover - scipy is present in the image
        p = float(erfc(abs(t) / sqrt(2.0)))
    return rho, p


def rsa(emb, ref_rdm):
    """(rho, p, model_rdm) exactly as behavioral_RSA computes them."""
    rdm = model_rdm(emb)
    ref = np.asarray(ref_rdm, dtype=np.float64)
    iu = np.triu_indices_from(ref, k=1)
    rho, p = spearman(ref[iu], rdm[iu])
    return rho, p, rdm


def cls_embeddings(model, images, batch_size=8):
    """compute_rsa_score's embedding: forward_features(x)[:, 0] (global_pool 'token'),
    or the mean of the patch tokens when ``global_pool == 'avg'`` (MEAS:313-322)."""
    import torch
    outs = []
    with torch.no_grad():
        for i in range(0, images.shape[0], batch_size):
            f = model.forward_features(images[i:i + batch_size])
            if getattr(model, "global_pool", "token") == "avg":
                outs.append(f[:, 1:].mean(dim=1).float().cpu())
            else:
                outs.append(f[:, 0].float().cpu())
    return torch.cat(outs).numpy()


def sampler_indices(n: int, world: int, rank: int):
    """Indices rank ``rank`` sees under DistributedSampler(shuffle=False, drop_last=False)
    (torch/utils/data/distributed.py: pad to a multiple of ``world`` by repeating the head of
    the index list, then take every ``world``-th index from ``rank``) -- the THINGS loader
    of MEAS:298 at world > 1."""
    idx = list(range(n))
    total = -(-n // world) * world
    pad = total - n
    if pad:
        idx += (idx * (-(-pad // n)))[:pad]
    return idx[rank:total:world]


def compute_rsa_score(model, images, reference_rdm, world: int = 1, rank: int = 0, batch_size: int = 8,
                      order: str = "image", group=None):
    """compute_rsa_score (MEAS:298-355) over ``world`` ranks: each rank embeds its
    DistributedSampler share of the 48 images (``cls_embeddings``: forward_features[:, 0]),
    the shares are all-gathered, and rank 0 returns (rho, p) of the model RDM against
    ``reference_rdm``; other ranks return (None, None).

    ``order`` settles SURVEY Appendix B Q3.  The reference concatenates the gathered shares
    rank by rank and keeps the first 48 rows (MEAS:327-334), so at world > 1 its RDM rows are
    [0, w, 2w, ..., 1, w+1, ...] against a reference RDM in image order.  ``"image"`` (default)
    puts every row back at its image's index before the RDM; ``"reference"`` reproduces the
    reference's concatenation order.  At world == 1 both are the reference's result."""
    import torch
    if order not in ("image", "reference"):
        raise ValueError(f"order must be 'image' or 'reference', not {order!r}")
    n = images.shape[0]
    idx = sampler_indices(n, world, rank)
    was_training = getattr(model, "training", False)
    if hasattr(model, "eval"):
        model.eval()
    emb = cls_embeddings(model, images[idx], batch_size=batch_size)
    if was_training:
        model.train()
    if world > 1:
        import torch.distributed as dist
        dev = images.device if images.device.type == "cuda" else torch.device("cpu")
        t = torch.from_numpy(emb).to(dev)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        if rank != 0:
            return None, None
        rows = torch.cat(parts).cpu().numpy()
        if order == "reference":
            emb = rows[:n]
        else:
            where = [i for r in range(world) for i in sampler_indices(n, world, r)]
            emb = np.empty((n, rows.shape[1]), dtype=rows.dtype)
            for row, i in zip(rows, where):  # padded repeats carry the same image's row
                emb[i] = row
    rho, p, _ = rsa(emb, reference_rdm)
    return rho, p
