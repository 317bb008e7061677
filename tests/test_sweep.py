"""Sweep runner (vit_amd.sweep): the reference's per-condition loop and on-disk formats
(NEWP:657-729 file names / keys, NEWP:795-797 CSV header, NEWP:843-871 windows, NEWP:1048-1063
early stopping), exercised on CPU with a stand-in model that has the DoRA parameter layout at
the reference's module paths (the real CLIPHBA needs the GPU kernels: tests/test_clip.py)."""
import csv
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn as nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vit-project_amd"))

from vit_amd import sweep as S  # noqa: E402
from vit_amd import perturb as P  # noqa: E402


class _DoRAStandIn(nn.Module):
    def __init__(self, d, r=4):
        super().__init__()
        self.m = nn.Parameter(torch.ones(d))
        self.delta_D_A = nn.Parameter(torch.randn(r, d) * 0.1)
        self.delta_D_B = nn.Parameter(torch.zeros(d, r))

    def weight(self):
        return torch.diag(self.m) + self.delta_D_B @ self.delta_D_A


class _Attn(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.out_proj = _DoRAStandIn(d)


class _Block(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.attn = _Attn(d)


class _Tower(nn.Module):
    def __init__(self, n, d):
        super().__init__()
        self.resblocks = nn.ModuleList([_Block(d) for _ in range(n)])


class _Clip(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.visual = nn.Module()
        self.visual.transformer = _Tower(24, d)
        self.transformer = _Tower(12, d)


class TinyHBA(nn.Module):
    """images [B, 3, 4, 4] -> 66-D predictions through the three DoRA stand-ins."""

    def __init__(self, d=48):
        super().__init__()
        self.clip_model = _Clip(d)
        self.inp = nn.Linear(48, d)
        self.out = nn.Linear(d, 66)
        for p in list(self.inp.parameters()) + list(self.out.parameters()):
            p.requires_grad_(False)

    def forward(self, x):
        h = self.inp(x.reshape(x.shape[0], -1))
        for path in S.DORA_MODULES:
            h = torch.tanh(h @ S._module(self, path).weight())
        return self.out(h)


def _data(seed=0, n_train=96, n_test=32):
    g = torch.Generator().manual_seed(seed)
    mk = lambda n: (torch.randn(n, 3, 4, 4, generator=g), torch.randn(n, 66, generator=g) * 0.5 + 2.0)
    inf = torch.randn(48, 3, 4, 4, generator=g)
    a = np.random.default_rng(seed).random((48, 48))
    ref = (a + a.T) / 2
    np.fill_diagonal(ref, 0)
    return dict(train=mk(n_train), test=mk(n_test), inference=inf, reference_rdm=ref)


def _make():
    torch.manual_seed(123)
    m = TinyHBA()
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=3e-4)
    return m, opt


def test_dora_and_random_state_files_match_reference_format(tmp_path):
    m, opt = _make()
    f = S.save_dora_parameters(m, str(tmp_path / "dora"), epoch=4)
    assert os.path.basename(f) == "epoch5_dora_params.pth"
    sd = torch.load(f, weights_only=True)
    assert sorted(sd) == sorted(f"{p}.{k}" for p in S.DORA_MODULES for k in ("m", "delta_D_A", "delta_D_B"))
    m2, _ = _make()
    with torch.no_grad():
        for p in m2.parameters():
            p.add_(1.0)
    S.load_dora_parameters(m2, str(tmp_path / "dora"), 5)
    for k, v in sd.items():
        assert torch.equal(m2.state_dict()[k], v)
    g = torch.Generator().manual_seed(7)
    rf = S.save_random_states(opt, 4, str(tmp_path / "rs"), g)
    assert os.path.basename(rf) == "epoch5_random_states.pth"
    ck = torch.load(rf, weights_only=False)
    assert {'epoch', 'optimizer_state_dict', 'torch_rng_state', 'numpy_rng_state', 'python_rng_state',
            'dataloader_generator_state'} <= set(ck)
    a = torch.rand(3)
    g2 = torch.Generator()
    assert S.load_random_states(str(tmp_path / "rs"), 5, opt, g2)
    assert torch.equal(torch.rand(3), a)  # torch RNG restored to the saved point
    assert torch.equal(g2.get_state(), ck['dataloader_generator_state'])
    assert not S.load_random_states(str(tmp_path / "rs"), 99)


def test_train_condition_window_csv_and_resume(tmp_path):
    data = _data()
    crit = nn.MSELoss()
    m, opt = _make()
    g = torch.Generator().manual_seed(0)
    rows = S.train_condition(m, opt, crit, data, epochs=4, training_run=2, perturb_length=2,
                             perturb_type="random_target", batch_size=32, training_res_path=str(tmp_path / "r.csv"),
                             dora_parameters_path=str(tmp_path / "d"), random_state_path=str(tmp_path / "s"),
                             dataloader_generator=g, early_stopping_patience=10)
    with open(tmp_path / "r.csv") as fh:
        got = list(csv.reader(fh))
    assert got[0] == S.CSV_HEADERS and len(got) == 5
    # 0-based epochs 1 and 2 are perturbed (window of training_run 2, length 2: NEWP:844-845)
    assert [r[5] for r in rows] == [False, True, True, False]
    assert all(np.isfinite(r[1]) and np.isfinite(r[2]) and -1 <= r[3] <= 1 for r in rows)
    assert sorted(os.listdir(tmp_path / "d")) == [f"epoch{i}_dora_params.pth" for i in range(1, 5)]


def test_run_sweep_shards_and_resumes_from_baseline(tmp_path):
    data = _data(1)
    crit = nn.MSELoss()
    m, opt = _make()
    g = torch.Generator().manual_seed(0)
    base = tmp_path / "baseline"
    S.train_condition(m, opt, crit, data, epochs=3, training_run=1, perturb_length=0, perturb_type=None,
                      batch_size=32, training_res_path=str(tmp_path / "base.csv"),
                      dora_parameters_path=str(base / "dora"), random_state_path=str(base / "rs"),
                      dataloader_generator=g)
    conds = [(1, 1), (2, 1), (2, 2), (3, 1)]
    done = []
    for rank in range(2):
        done += S.run_sweep(_make, crit, data, conds, rank=rank, world=2, perturb_type="label_shuffle",
                            out_dir=str(tmp_path / "sweep"), baseline_dora_path=str(base / "dora"),
                            baseline_random_state_path=str(base / "rs"), epochs=4, batch_size=32)
    assert sorted(c for c, _ in done) == sorted(conds)  # every condition exactly once over the ranks
    for (start, length), res in done:
        with open(res) as fh:
            rows = list(csv.reader(fh))[1:]
        # resumed at epoch start-1: rows for epochs start..4, shuffles flagged inside the window only
        assert [int(r[0]) for r in rows] == list(range(start, 5))
        flags = [r[6] == "True" for r in rows]
        assert flags == [P.in_window(int(r[0]) - 1, start, length) for r in rows]
