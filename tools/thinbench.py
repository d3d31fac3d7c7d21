"""The narrow select conv (conv3x3_thin, unet_simple.py:136-138 select1_2 / select1_3 shape) alone, for timing and PMC
passes:  python tools/thinbench.py [n h w cin cout] [--option KEY=VALUE ...]

Prints HIP-event ms per launch and the algorithmic rate (input + filter read once, f32 output written once).
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
    ap.add_argument("shape", nargs="*", type=int, default=[8, 320, 320, 192, 8])
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    n, h, w, cin, cout = args.shape
    for kv in args.option:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    rs = np.random.RandomState(0)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to("cuda", torch.bfloat16)
    pc = ops.PackedConv(rs.normal(size=(3, 3, cin, cout)).astype(np.float32) / 40, None, "bf16", "cuda")
    out = torch.empty((n, h, w, cout), dtype=torch.float32, device="cuda")
    fn = lambda: ops.conv3x3(x, pc, "none", out=out, affine=False, splitk=True)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    nbytes = n * h * w * (cin * 2 + cout * 4) + 9 * cin * cout * 2
    print("%s %dx%dx%dx%d -> %d: %.4f ms, %.2f TB/s algorithmic (%.1f MB)" % (
        _lib.last_conv_kernel(), n, h, w, cin, cout, ms, nbytes / ms / 1e9, nbytes / 1e6), flush=True)
    # the same input bytes read by a plain streaming reduction (what the input read alone can reach here)
    xv = x.view(-1, 8)
    for _ in range(3):
        torch.amax(xv, dim=0)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(args.iters):
        torch.amax(xv, dim=0)
    e1.record()
    torch.cuda.synchronize()
    ms2 = e0.elapsed_time(e1) / args.iters
    print("reference stream read (torch.amax over the input): %.4f ms, %.2f TB/s" % (
        ms2, x.numel() * 2 / ms2 / 1e9), flush=True)


if __name__ == "__main__":
    main()
