"""Same-box A/B of UNetVideo forward variants (graph replay, 1080p bf16): python tools/ab_unet.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-matting_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmatting import _lib, unet, video  # noqa: E402
from vmatting.weights import synthetic_vgg16  # noqa: E402

VARIANTS = {
    "default": {},
    "fold_up2": {"fold_upconv": ("upconv_2", "upconv_3", "upconv_4")},
    "fold3": {"fold_upconv": ("upconv_3", "upconv_4")},  # round-3 default before upconv_2 was folded
    "nosplit": {"split_head": False},
    "noskip": {"_opt": {"up_skip": 0}},  # folded upconvs without the zero-tap skipping
    "fold_up2_noskip": {"fold_upconv": ("upconv_2", "upconv_3", "upconv_4"), "_opt": {"up_skip": 0}},
    # r06: grouped patch tile order (ConvArgs::ngroup) for filters >= cband_bytes
    "ng2": {"_opt": {"ngroup": 2}},
    "ng4": {"_opt": {"ngroup": 4}},
    "ng8": {"_opt": {"ngroup": 8}},
    "ng4_1m": {"_opt": {"ngroup": 4, "cband_bytes": 1 << 20}},
}
DEFAULT_OPT = {"up_skip": 1, "cband_bytes": 4 << 20}


def run(name, steps=100):
    np.random.seed(0)
    m = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device="cuda")
    opts = VARIANTS[name].get("_opt", {})
    for k, v in VARIANTS[name].items():
        if k != "_opt":
            setattr(m, k, v)
    for k, v in opts.items():
        _lib.set_option(k, v)
    m.prepare()
    x = video.synthetic_frames(1, 1080, 1920, first=0, device="cuda")
    g = m.capture(x)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / steps
    for k in opts:
        _lib.set_option(k, DEFAULT_OPT.get(k, 0))
    return ms


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for rep in range(3):
        for n in names:
            print("%-10s %.4f ms/frame" % (n, run(n)), flush=True)
