"""Reference-named entry point: `import augmentation` as the reference does.

Re-exports vmatting.augmentation (gfx950 implementation of the reference's augmentation.py API).
"""
from vmatting.augmentation import *  # noqa: F401,F403
