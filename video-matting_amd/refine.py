"""Reference-named entry point: `import refine` as the reference's train.py / small_train.py do.

Re-exports vmatting.refine (gfx950 implementation of the reference's refine.py API).
"""
from vmatting.refine import *  # noqa: F401,F403
