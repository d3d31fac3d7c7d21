"""vmatting — MI355X-native per-frame alpha-matting path of tangih/video-matting.

Host code (this package) mirrors the reference's model-builder / flow / reader API;
all numeric work runs in libvmatting.so (hand-written gfx950 HIP kernels behind the
C ABI in include/vmatting.h).  No CPU fallback: a missing library or GPU raises.
"""

from . import _lib, ops, weights  # noqa: F401
from .params import VGG_MEAN  # noqa: F401

__all__ = ["unet", "unet_simple", "small", "refine", "flow", "reader", "tps", "augmentation", "loader", "parallel", "ops",
           "weights"]
