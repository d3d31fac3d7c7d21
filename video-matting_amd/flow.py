"""Reference-named entry point: `import flow` as the reference's train.py / small_train.py do.

Re-exports vmatting.flow (gfx950 implementation of the reference's flow.py API).
"""
from vmatting.flow import *  # noqa: F401,F403
