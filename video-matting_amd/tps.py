"""Reference-named entry point: `import tps` as the reference does.

Re-exports vmatting.tps (gfx950 implementation of the reference's tps.py API).
"""
from vmatting.tps import *  # noqa: F401,F403
