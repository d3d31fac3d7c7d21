"""Reference-named entry point: `import unet_simple` as the reference's train.py / small_train.py do.

Re-exports vmatting.unet_simple (gfx950 implementation of the reference's unet_simple.py API).
"""
from vmatting.unet_simple import *  # noqa: F401,F403
