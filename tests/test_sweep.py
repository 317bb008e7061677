"""Sweep runner (vit_amd.sweep): the reference's per-condition loop and on-disk formats
(NEWP:657-729 file names / keys, NEWP:795-797 CSV header, NEWP:843-871 windows, NEWP:1048-1063
early stopping), exercised on CPU with a stand-in model that has the DoRA parameter layout at
the reference's module paths (the real CLIPHBA needs the GPU kernels: tests/test_clip.py)."""
import csv
import os
import random
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
    with torch.serialization.safe_globals(S._rng_state_globals()):
        ck = torch.load(rf, weights_only=True)
    assert {'epoch', 'optimizer_state_dict', 'torch_rng_state', 'numpy_rng_state', 'python_rng_state',
            'dataloader_generator_state'} <= set(ck)
    a = torch.rand(3)
    g2 = torch.Generator()
    assert S.load_random_states(str(tmp_path / "rs"), 5, opt, g2)
    assert torch.equal(torch.rand(3), a)  # torch RNG restored to the saved point
    assert torch.equal(g2.get_state(), ck['dataloader_generator_state'])
    assert not S.load_random_states(str(tmp_path / "rs"), 99)


class _Payload:
    """A pickled object whose reconstruction would run code (os.system here)."""

    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


def test_load_random_states_refuses_non_allowlisted_globals(tmp_path):
    import pickle
    d = tmp_path / "rs"
    d.mkdir()
    ck = {'epoch': 3, 'torch_rng_state': torch.get_rng_state(), 'numpy_rng_state': np.random.get_state(),
          'python_rng_state': random.getstate(), 'evil': _Payload()}
    torch.save(ck, str(d / "epoch4_random_states.pth"))
    before = torch.get_rng_state()
    with pytest.raises(pickle.UnpicklingError):
        S.load_random_states(str(d), 4)
    assert torch.equal(torch.get_rng_state(), before)  # nothing was applied
    # the same file without the payload resumes
    del ck['evil']
    torch.save(ck, str(d / "epoch4_random_states.pth"))
    assert S.load_random_states(str(d), 4)


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
    assert sorted(c for c, _, _ in done) == sorted(conds)  # every condition exactly once over the ranks
    for (start, length), res, _ in done:
        with open(res) as fh:
            rows = list(csv.reader(fh))[1:]
        # resumed at epoch start-1: rows for epochs start..4, shuffles flagged inside the window only
        assert [int(r[0]) for r in rows] == list(range(start, 5))
        flags = [r[6] == "True" for r in rows]
        assert flags == [P.in_window(int(r[0]) - 1, start, length) for r in rows]


def test_reference_grid_is_the_136_conditions_on_disk():
    grid = S.reference_length_grid()
    assert len(grid) == 136 and len(set(grid)) == 136
    starts = sorted({e for e, _ in grid})
    assert starts == [1, 2, 3, 6, 7, 8, 10, 13, 16, 19, 20, 22, 30, 40, 50, 58, 60, 70, 80, 90, 94]
    assert {l for _, l in grid} == {2, 5, 10, 20, 30, 40, 50}
    assert (22, 5) in grid and (22, 2) not in grid and (13, 2) not in grid and (94, 50) in grid
    from vit_amd import parallel
    assert parallel.length_sweep_conditions() == grid
    ref = "/root/reference/Data/clip_results/perturb_length_experiments_baselineseed1_perturbseed0"
    if os.path.isdir(ref):  # build container only: the directory names themselves
        names = sorted(os.listdir(ref))
        assert sorted(os.path.basename(S.condition_dir("", "random_target", e, l)) for e, l in grid) == names
    # 8-way shards: every condition exactly once, start-epoch chains never split
    seen = []
    for r in range(8):
        mine = parallel.shard_conditions(grid, 8, r)
        seen += mine
        for e in {e for e, _ in mine}:
            assert sorted(c for c in mine if c[0] == e) == sorted(c for c in grid if c[0] == e)
    assert sorted(seen) == grid


def _baseline(tmp_path, data, epochs):
    m, opt = _make()
    base = tmp_path / "baseline"
    S.train_condition(m, opt, nn.MSELoss(), data, epochs=epochs, training_run=1, perturb_length=0, perturb_type=None,
                      batch_size=32, training_res_path=str(tmp_path / "base.csv"),
                      dora_parameters_path=str(base / "dora"), random_state_path=str(base / "rs"),
                      dataloader_generator=torch.Generator().manual_seed(0))
    return str(base / "dora"), str(base / "rs")


def _rows(path):
    with open(path) as fh:
        return list(csv.reader(fh))


def test_sibling_resume_is_exact(tmp_path):
    """LEN:188-256: a longer window resumes from the longest shorter sibling at epoch
    start-1+sibling_length -- and gives exactly the rows a run from the baseline gives."""
    data = _data(2)
    bd, br = _baseline(tmp_path, data, 4)
    kw = dict(perturb_type="random_target", baseline_dora_path=bd, baseline_random_state_path=br, epochs=9,
              batch_size=32, early_stopping_patience=50)
    chained = S.run_sweep(_make, nn.MSELoss(), data, [(3, 2), (3, 5)], out_dir=str(tmp_path / "a"), **kw)
    assert [src for _, _, src in chained] == ["baseline", "sibling l2"]
    alone = S.run_sweep(_make, nn.MSELoss(), data, [(3, 5)], out_dir=str(tmp_path / "b"), **kw)
    assert alone[0][2] == "baseline"
    got, ref = _rows(chained[1][1]), _rows(alone[0][1])
    assert got[0] == S.CSV_HEADERS and [int(r[0]) for r in got[1:]] == list(range(3, 10))
    assert got == ref  # bit-identical losses / rho: the resume restored model, optimizer, RNG and loader state
    sib = _rows(chained[0][1])
    assert got[1:3] == sib[1:3]  # epochs 3..4 (through the sibling's window end) copied from the sibling
    # own-CSV resume: a finished condition is skipped, a truncated one continues in place
    again = S.run_sweep(_make, nn.MSELoss(), data, [(3, 5)], out_dir=str(tmp_path / "a"), **kw)
    assert again[0][2] == "complete"


def test_launch_sweep_world8_covers_every_condition_once(tmp_path):
    """The 8-process launcher (one process per GPU on the box; CPU workers here) over a
    scaled-down grid with the reference grid's structure: chains per start epoch stay on one
    rank, every condition runs exactly once, longer windows resume from their siblings."""
    data = _data(3, n_train=64, n_test=16)
    bd, br = _baseline(tmp_path, data, 15)
    starts = [1, 2, 3, 6, 7, 8, 10, 13, 16]
    conds = [(e, l) for e in starts for l in (2, 5)]
    res = S.launch_sweep(8, _make, nn.MSELoss(), data, conds, perturb_type="random_target",
                         out_dir=str(tmp_path / "sw"), baseline_dora_path=bd, baseline_random_state_path=br,
                         epochs=20, batch_size=32, early_stopping_patience=50, torch_threads=1)
    assert sorted(res) == list(range(8))
    flat = [c for r in res.values() for c, _, _ in r]
    assert sorted(flat) == sorted(conds)
    src = {c: s for r in res.values() for c, _, s in r}
    assert all(src[(e, 2)] == "baseline" and src[(e, 5)] == "sibling l2" for e in starts)
    for r, items in res.items():
        assert {c for c, _, _ in items} == set(parallel_shard(conds, r))
    for (e, l), path, _ in (x for r in res.values() for x in r):
        rows = _rows(path)
        assert [int(v[0]) for v in rows[1:]] == list(range(e, 21))
        assert [v[5] == "True" for v in rows[1:]] == [P.in_window(int(v[0]) - 1, e, l) for v in rows[1:]]


def parallel_shard(conds, r):
    from vit_amd import parallel
    return parallel.shard_conditions(conds, 8, r)
