"""Microbenchmark of the fused first pair (conv1_1 -> conv1_2 -> pool1) at 1080p, for rocprofv3 --pmc runs.

    python tools/pairbench.py [--pair-kernel 0|1] [--pair-strip 0|1] [--head 0|1] [--iters N] [--xdtype fp32|bf16]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmatting import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pair-kernel", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--xdtype", default="fp32")
    ap.add_argument("--hw", default="1080x1920")
    ap.add_argument("--xin-wide", type=int, default=1)
    ap.add_argument("--pair-strip", type=int, default=1)
    ap.add_argument("--abl", type=int, default=0)
    ap.add_argument("--pin", type=int, default=1)
    ap.add_argument("--head", type=int, default=1, help="head split partials + no conv1_2 store (the UNetVideo path)")
    a = ap.parse_args()
    _lib.set_option("pair_xin_wide", a.xin_wide)
    h, w = (int(v) for v in a.hw.split("x"))
    _lib.set_option("pair_kernel", a.pair_kernel)
    _lib.set_option("pair_strip", a.pair_strip)
    if a.pin != 1:
        _lib.set_option("pair_strip_pin", a.pin)
    if a.abl:  # timing-only ablations: the study build (VM_LIB_PATH=video-matting_amd/study/libvmatting_study.so)
        _lib.set_option("pair_strip_abl", a.abl)
    rs = np.random.RandomState(0)
    xf = (torch.rand(1, h, w, 7, device="cuda") * 255 - 120)
    x = xf if a.xdtype == "fp32" else ops.convert(xf, torch.empty(1, h, w, 8, dtype=torch.bfloat16, device="cuda"))[..., :7]
    pc1 = ops.PackedConv((rs.normal(size=(3, 3, 7, 64)) * 0.17).astype(np.float32), np.zeros(64, np.float32), torch.bfloat16)
    pc2 = ops.PackedConv((rs.normal(size=(3, 3, 64, 64)) * 0.06).astype(np.float32), np.zeros(64, np.float32), torch.bfloat16)
    y = torch.empty(1, h, w, 64, dtype=torch.bfloat16, device="cuda")
    p = torch.empty(1, (h + 1) // 2, (w + 1) // 2, 64, dtype=torch.bfloat16, device="cuda")
    whd = torch.from_numpy((rs.normal(size=(3, 3, 128, 1)) * 0.04).astype(np.float32)).cuda()
    part = torch.empty(1, h, w, 12, dtype=torch.float32, device="cuda")

    def run():
        if a.head:
            ops.conv_pair_first_head(x, pc1, pc2, whd, 64, part, "relu", out=y, pool_out=p, store_y=False)
        else:
            ops.conv_pair_first(x, pc1, pc2, "relu", out=y, pool_out=p)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = 2.0 * h * w * 9 * (7 * 64 + 64 * 64)
    print("pair %s %s: %.4f ms %.1f TFLOP/s" % (a.hw, _lib.last_conv_kernel(), ms, fl / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
