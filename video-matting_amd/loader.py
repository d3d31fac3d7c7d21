"""Reference-named entry point: `import loader` as the reference's train.py / small_train.py do.

Re-exports vmatting.loader (training-sample loader with the per-pixel work on gfx950).
"""
from vmatting.loader import *  # noqa: F401,F403
from vmatting.loader import get_padded_img, plan_crop  # noqa: F401
