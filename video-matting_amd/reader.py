"""Reference-named entry point: `import reader` as the reference's train.py / small_train.py do.

Re-exports vmatting.reader (gfx950 implementation of the reference's reader.py API).
"""
from vmatting.reader import *  # noqa: F401,F403
