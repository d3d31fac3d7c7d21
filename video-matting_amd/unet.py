"""Reference-named entry point: `import unet` as the reference's train.py / small_train.py do.

Re-exports vmatting.unet (gfx950 implementation of the reference's unet.py API).
"""
from vmatting.unet import *  # noqa: F401,F403
