"""Loader for the C-ABI HIP library ``libvit_hip.so`` (include/vit_hip.h).

The library is the only compute path.  There is no CPU or PyTorch fallback:
if the shared object is missing, or the process has no ROCm GPU, every op
raises.  ``torch`` is imported first so that the HIP runtime torch ships
(SONAME libamdhip64.so.7) is the one our library binds to -- one runtime, one
set of streams, graph capture works across both.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VIT_HIP_LIB", os.path.join(_HERE, "lib", "libvit_hip.so"))

F32, BF16 = 0, 1
LAY_RC, LAY_CR = 0, 1
EPI_STORE, EPI_BIAS_GELU, EPI_RESID, EPI_GELU_BWD, EPI_PATCH, EPI_BIAS_QGELU, EPI_QGELU_BWD = range(7)

i32, i64, f32, vp = C.c_int, C.c_int64, C.c_float, C.c_void_p

# name -> argtypes (all return int = hipError_t)
SIGNATURES = {
    "vit_abi_version": [],
    "vit_gemm_variant": [i32],
    "vit_gemm_group": [i32, i32],
    "vit_gemm_g4_config": [i32, i32, i32, i32],
    "vit_gemm_g4_count": [i32],
    "vit_gemm_g4_gelu": [i32],
    "vit_gemm_streamk_workspace": [vp, vp, i64, vp, i32],
    "vit_gemm_rc_chunk_rows": [i32, i64],
    "vit_gemm": [i32, i32, i32, i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, i32, vp],
    "vit_linear_fwd": [i32, i32, i32, i32, i32, i32, vp, i64, vp, vp, vp, i64, vp, vp, vp],
    "vit_linear_dgrad": [i32, i32, i32, i32, i32, i32, vp, i64, vp, vp, i64, vp, vp, vp, i64, i32, vp],
    "vit_linear_dgrad_partial_floats": [i32, i32],
    "vit_colreduce": [vp, i32, i32, vp, i32, vp, vp],
    "vit_colreduce_multi": [vp, i32, i32, i32, vp, vp, vp, i32, vp, vp],
    "vit_colreduce_batch_sizes": [vp, i32, vp, vp],
    "vit_colreduce_batch": [vp, i32, vp, i64, vp, i32, vp],
    "vit_linear_wgrad": [i32, i32, i32, i32, vp, i64, vp, i64, vp, i32, vp, i64, vp],
    "vit_linear_wgrad_nslabs": [i32, i32, i32, i32, i32],
    "vit_linear_wgrad_partials": [i32, i32, i32, i32, vp, i64, vp, i64, i32, vp, i64, vp],
    "vit_linear_wgrad_partials2": [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, i32, i32, vp, i64, vp, i64, vp,
                                   i64, vp],
    "vit_colsum": [i32, i32, i32, vp, i64, vp, vp, i64, i32, vp],
    "vit_patch_embed_fwd": [i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp],
    "vit_patch_embed_fwd_ld": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp],
    "vit_layer_norm_fwd": [i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp, f32, vp],
    "vit_add_layer_norm_fwd": [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp, f32, vp],
    "vit_layer_norm_bwd": [i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, i64, i32,
                           i32, vp, vp, vp, vp, i64, i32, vp],
    "vit_layer_norm_bwd_partial_floats": [i32, i32],
    "vit_layer_norm_bwd_blocks": [i32],
    "vit_layer_norm_bwd_variant": [i32],
    "vit_sdpa_fwd": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, f32, i32, vp],
    "vit_sdpa_fwd_fp8": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, f32, i32, vp],
    "vit_sdpa_bwd_variant": [i32],
    "vit_sdpa_bwd": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, vp, i64, vp, f32, i32, vp, vp, i64, vp],
    "vit_sdpa_bwd_partial_floats": [i32, i32, i32],
    "vit_patch_unfold": [i32, i32, i32, i32, i32, i32, vp, vp, vp],
    "vit_patch_unfold_ld": [i32, i32, i32, i32, i32, i32, i32, vp, vp, vp],
    "vit_copy_rows_padded": [i32, i32, i32, vp, i64, vp, i64, vp],
    "vit_cls_pos_fill": [i32, i32, i32, vp, vp, vp, vp],
    "vit_pos_grad": [i32, i32, i32, vp, vp, vp, vp],
    "vit_cross_entropy_fwd": [i32, i32, vp, i64, vp, vp, vp, vp, vp],
    "vit_cross_entropy_bwd": [i32, i32, i32, vp, i64, vp, vp, vp, vp, i64, vp],
    "vit_sgd_step": [vp, vp, i32, vp, f32, f32, vp],
    "vit_sgd_chunk_size": [],
    "vit_sgd_tensor_bytes": [],
    "vit_sgd_chunk_bytes": [],
    "vit_cast_f32_bf16": [vp, vp, i64, vp],
    "vit_zero": [vp, i64, vp],
    "vit_dora_weight_fwd": [i32, i32, i32, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp],
    "vit_dora_weight_bwd": [i32, i32, i32, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp],
    "vit_dora_weight_bwd_ws": [i32, i32, i32, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, i64, vp, vp],
    "vit_gemm_splitk": [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, i64, vp],
    "vit_adamw_step": [vp, vp, i32, f32, f32, f32, vp],
    "vit_adamw_tensor_bytes": [],
    "vit_token_embed": [i32, i32, i32, i32, vp, vp, vp, vp, vp],
    "vit_gather_rows": [i32, i32, vp, i64, vp, vp, i64, vp],
    "vit_scatter_rows": [i32, i32, vp, i64, vp, vp, i64, vp],
    "vit_rownorm_fwd": [i32, i32, vp, vp, vp, vp, vp],
    "vit_rownorm_bwd": [i32, i32, vp, vp, vp, vp, vp, vp],
    "vit_mse_fwd": [i32, vp, vp, vp, vp],
    "vit_mse_bwd": [i32, vp, vp, vp, vp, vp],
    "vit_image_coeff_bytes": [i32, i32, i32],
    "vit_image_transform": [i32, i32, vp, vp, i32, i32, vp, vp, vp, vp, vp],
}

_lib = None


class HipError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the ctypes library; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise HipError(f"libvit_hip.so not found at {p}: build it with `python __graft_entry__.py` "
                       f"or `make -C vit-project_amd/csrc` (no CPU fallback exists)")
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = i32
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def check(rc: int, what: str):
    if rc != 0:
        raise HipError(f"{what} failed with hipError {rc}")


def call(name: str, *args):
    check(getattr(lib(), name)(*args), name)


def require_gpu(t: torch.Tensor):
    if not t.is_cuda:
        raise HipError("vit_amd ops run only on a ROCm GPU tensor (no CPU fallback); got device "
                       f"{t.device}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise HipError(f"unsupported dtype {t.dtype}")


def exported_symbols():
    return list(SIGNATURES)
