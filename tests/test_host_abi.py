"""CPU: the C-ABI library loads and exports what include/vit_hip.h declares; host logic."""
import os
import re

import numpy as np
import pytest
import torch

from oracle import vit_ref as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "vit_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\bint\s+(vit_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import ctypes
    from vit_amd import _lib
    lib = _lib.load()
    declared = _header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} missing from the ctypes signature table"
    for name in _lib.SIGNATURES:
        assert name in declared, f"{name} bound in Python but not declared in include/vit_hip.h"
    assert lib.vit_abi_version() == 10
    assert lib.vit_sgd_tensor_bytes() == 40 and lib.vit_sgd_chunk_bytes() == 16
    assert lib.vit_sgd_chunk_size() == 4096


def test_gemm_32bit_offset_plan():
    """The bf16 MFMA GEMM stages row-contiguous operands through 32-bit byte offsets (gemm.hip
    gemm_tile): operands past 4 GiB are split into row chunks (multiples of 256 rows) so the
    offsets never wrap.  Host-only query, no GPU call."""
    from vit_amd import _lib
    lib = _lib.load()
    rows = lib.vit_gemm_rc_chunk_rows
    M = 256 * 197
    assert rows(M, 3072) == M and rows(M, 768) == M  # the bench shapes: one launch
    for m, ld in ((3600 * 197, 3072), (2100 * 257, 4096), (1 << 21, 1024), (5000 * 197, 768)):
        r = rows(m, ld)
        fits = (m - 1) * ld * 2 + 128 < (1 << 32)
        if fits:
            assert r == m
        else:
            assert 0 < r < m and r % 256 == 0, (m, ld, r)
            assert (r - 1) * ld * 2 + 128 < (1 << 32) <= (r + 255) * ld * 2 + 128, (m, ld, r)
    assert rows(3600 * 197, 3072) < 3600 * 197  # fc1 activations at bs 3600 (ADVICE example)
    assert rows(1000, 1 << 25) == 0  # 64 MiB rows: no 256-row chunk fits, the fast path is refused


def test_library_links_no_vendor_blas():
    """Every GEMM of the path is hand-written since ABI 10 (round 6): the library's dynamic section names no
    hipBLASLt / rocBLAS / hipBLAS, and no exported symbol mentions them."""
    import subprocess
    so = os.path.join(ROOT, "vit-project_amd", "vit_amd", "lib", "libvit_hip.so")
    dyn = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-d", "--dyn-syms", so], capture_output=True,
                         text=True, check=True).stdout.lower()
    for name in ("hipblaslt", "rocblas", "hipblas"):
        assert name not in dyn, f"libvit_hip.so references {name}"


def test_library_is_gfx950_code_object(tmp_path):
    import shutil
    import subprocess
    so = os.path.join(ROOT, "vit-project_amd", "vit_amd", "lib", "libvit_hip.so")
    # --offloading extracts the device images next to its input: run it on a copy in tmp
    cp = shutil.copy(so, tmp_path / "libvit_hip.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(cp)], capture_output=True,
                         text=True)
    assert "gfx950" in (out.stdout + out.stderr)


def test_timm_surface_on_cpu_module():
    import vit_amd
    m = vit_amd.create_model("vit_base_patch16_224", pretrained=False, num_classes=1000)
    sd = m.state_dict()
    shapes = R.param_shapes(R.VIT_B16)
    assert list(sd.keys()) == list(shapes.keys())
    for k, s in shapes.items():
        assert tuple(sd[k].shape) == tuple(s), k
    assert sum(p.numel() for p in m.parameters()) == 86_567_656
    assert m.global_pool == "token"
    with pytest.raises(KeyError):
        vit_amd.create_model("resnet50")
    with pytest.raises(ValueError):
        vit_amd.create_model("vit_base_patch16_224", pretrained=True)


def test_product_path_fails_loudly_without_gpu():
    import vit_amd
    m = vit_amd.create_model("vit_base_patch16_224")
    with pytest.raises(vit_amd._lib.HipError):
        m(torch.zeros(1, 3, 224, 224))
    with pytest.raises(vit_amd._lib.HipError):
        vit_amd.cross_entropy(torch.zeros(2, 10), torch.zeros(2, dtype=torch.long))


def test_oracle_state_dict_loads_into_model():
    import vit_amd
    m = vit_amd.VisionTransformer(img_size=32, patch_size=16, embed_dim=128, depth=2, num_heads=2, num_classes=10)
    cfg = R.ViTConfig(img_size=32, patch_size=16, embed_dim=128, depth=2, num_heads=2, num_classes=10)
    p = R.init_params(cfg, seed=1)
    m.load_oracle_params(p)
    for k, v in m.state_dict().items():
        assert torch.equal(v, p[k])


def test_lr_scheduler_class_matches_reference_fixture(golden_dir):
    import json
    import vit_amd
    with open(os.path.join(golden_dir, "lr_golden.json")) as f:
        fx = json.load(f)
    net = torch.nn.Linear(2, 2)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
    sch = vit_amd.CosineAnnealingLRWithWarmup(opt, warmup_epochs=5, max_epochs=100)
    got = []
    for _ in range(100):
        got.append(opt.param_groups[0]["lr"])
        sch.step()
    assert got == fx["lr_per_epoch"]
    sd = sch.state_dict()
    sch2 = vit_amd.CosineAnnealingLRWithWarmup(opt, warmup_epochs=1, max_epochs=2)
    sch2.load_state_dict(sd)
    assert sch2.state_dict() == sd


def test_multitensor_table_layout():
    from vit_amd.optim import _MultiTensor
    mt = _MultiTensor(torch.device("cpu"))
    mt.build([(16, 32, 48, None, 5000), (64, 80, 96, 112, 10)], [5000, 10])
    assert mt.nchunks == 3
    raw = mt._tdev.numpy().view(np.int64).reshape(-1, 5)
    assert raw[0].tolist() == [16, 32, 48, 0, 5000]
    ch = mt._cdev.numpy().view(np.int64).reshape(-1, 2)
    assert ch.tolist() == [[0, 0], [0, 4096], [1, 0]]
