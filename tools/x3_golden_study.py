"""Which part of the f16x3 forward holds its error on a golden case (study tool, GPU): the alpha / logit error
against the golden (float64 reference output) under kernel and layout variants, next to fp32 and bf16x6.

    python tools/x3_golden_study.py [case ...]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "video-matting_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import golden  # noqa: E402
from oracle import models as om  # noqa: E402
from vmatting import _lib, split3, unet  # noqa: E402


def run(case, dtype, opts=(), first_slab=32):
    g = golden(case)
    cls = unet.UNetVideo if int(g["video"]) else unet.UNetImage
    for k, v in opts:
        _lib.set_option(k, v)
    split3.Split3Forward.first_slab = first_slab
    try:
        np.random.seed(int(g["weight_seed"]))
        m = cls(om.synthetic_vgg16(0), dtype=dtype)
        m.build(g["x"])
        torch.cuda.synchronize()
        a = m.output.float().cpu().numpy()
        lg = m.conv1_3.float().cpu().numpy()
    finally:
        split3.Split3Forward.first_slab = 32
    da = np.abs(a - g["output"])
    dl = np.abs(lg - g["logits"])
    i = np.unravel_index(np.argmax(da), da.shape)
    return da.max(), dl.max() / np.abs(g["logits"]).max(), float(g["logits"][i]), float(dl[i])


def main():
    cases = sys.argv[1:] or ["unet_video_64x96", "unet_image_70x90"]
    variants = [("fp32", "fp32", (), 32), ("bf16x6", "bf16x6", (), 32), ("f16x3", "f16x3", (), 32),
                ("f16x3 rows off", "f16x3", (("rows_kernel", 0),), 32),
                ("f16x3 slab8", "f16x3", (), 8),
                ("f16x3 rows off slab8", "f16x3", (("rows_kernel", 0),), 8)]
    for case in cases:
        for name, dt, opts, fs in variants:
            try:
                ea, el, z, dz = run(case, dt, opts, fs)
            finally:
                _lib.set_option("rows_kernel", 1)
            print("%-18s %-24s alpha %.3e  logits rel %.3e  worst pixel: logit %.4g, its error %.3e" % (
                case, name, ea, el, z, dz), flush=True)


if __name__ == "__main__":
    main()
