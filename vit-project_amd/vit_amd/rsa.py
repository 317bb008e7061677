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
