"""Reference-named entry point: `import params` as the reference's train.py / small_train.py do.

Re-exports vmatting.params (gfx950 implementation of the reference's params.py API).
"""
from vmatting.params import *  # noqa: F401,F403
