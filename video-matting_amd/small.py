"""Reference-named entry point: `import small` as the reference's train.py / small_train.py do.

Re-exports vmatting.small (gfx950 implementation of the reference's small.py API).
"""
from vmatting.small import *  # noqa: F401,F403
