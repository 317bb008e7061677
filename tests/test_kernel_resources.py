"""CPU: register / scratch audit of the built code objects (no GPU needed).

- the inline-asm wide-wave GEMM kernels (csrc/gemm_w4.inc): no scratch, and no instruction touches an asm
  LDS read's destination before the next lgkmcnt(0) wait (tools/w4_audit.py);
- every instantiation of the fused attention backward (its phase-1 query loop is fully
  unrolled): no VGPR spill, no scratch.

Skipped when the objects are not built (``make -C vit-project_amd/csrc``).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "vit-project_amd", "csrc", "build")
LLVM = "/opt/rocm/lib/llvm/bin"


def _need(obj):
    path = os.path.join(BUILD, obj)
    if not os.path.exists(path) or not os.path.exists(f"{LLVM}/llvm-readelf"):
        pytest.skip(f"{obj} not built / no ROCm LLVM tools")
    return path


def test_w4_kernels_pass_the_asm_audit():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import w4_audit
    text = w4_audit.disassemble(_need("gemm.o"))
    assert w4_audit.audit(text, r"w4") == 0


def test_attention_backward_has_no_spills():
    out = subprocess.run(["bash", os.path.join(ROOT, "tools", "kres.sh"), _need("attention.o"), "attn_bwd"],
                         capture_output=True, text=True, check=True).stdout.splitlines()
    assert out, "no attn_bwd kernels found"
    bad = [l for l in out if " spill 0 " not in l or " priv 0 " not in l]
    assert not bad, bad[:5]
