"""Reference-named entry point: `import data` as the reference does.

Re-exports vmatting.data (gfx950 implementation of data.trimap_from_matte).
"""
from vmatting.data import *  # noqa: F401,F403
