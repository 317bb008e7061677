"""vit_amd: MI355X-native (gfx950) ViT training step behind the timm / DoRA surface.

Compute runs only in ``lib/libvit_hip.so`` (C-ABI, include/vit_hip.h); this
package is the host-side mirror of the reference's module/optimizer interface.
"""
from . import _lib
from .model import VisionTransformer, create_model, cross_entropy, set_wgrad_overlap
from .optim import FusedSGD, FusedAdamW, CosineAnnealingLRWithWarmup
from .dora import DoRALayer, dora_weight
from . import rsa
from . import clip
from . import sweep
from . import data
from .clip import CLIPHBA, MSELoss, mse_loss, apply_dora_to_ViT, switch_dora_layers, count_trainable_parameters

__all__ = ["VisionTransformer", "create_model", "cross_entropy", "set_wgrad_overlap", "FusedSGD", "FusedAdamW",
           "CosineAnnealingLRWithWarmup", "DoRALayer", "dora_weight", "rsa", "clip", "data", "CLIPHBA", "MSELoss",
           "mse_loss", "apply_dora_to_ViT", "switch_dora_layers", "count_trainable_parameters"]


def load_library(path=None):
    return _lib.load(path)
