"""Time the narrow-cout convs of the training step (the select convs, unet_simple.py:153-168) on the thin kernel
vs the generic kernels:  python tools/thinbench.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-matting_amd"))
from vmatting import _lib, ops  # noqa: E402

SHAPES = [  # (name, n, h, w, per-source channels, sources, cout)
    ("select1_2", 8, 320, 320, 64, 3, 8), ("select1_1", 8, 320, 320, 32, 1, 8), ("select2", 8, 160, 160, 128, 3, 8),
    ("select3", 8, 80, 80, 256, 3, 8), ("select4", 8, 40, 40, 512, 3, 16)]


def bench(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = "cuda"
    for name, n, h, w, c, ns, cout in SHAPES:
        base = torch.randn((ns * n, h, w, c), device=dev).to(torch.bfloat16)
        x = ops.SourceConcat(base, ns) if ns > 1 else base
        pc = ops.PackedConv(torch.randn(3, 3, ns * c, cout) * 0.05, torch.zeros(cout), "bf16", dev)
        y = torch.empty((n, h, w, cout), device=dev)
        run = lambda: ops.conv3x3(x, pc, "none", out=y, affine=False, splitk=True)  # noqa: E731
        extra = []
        for nb in (256, 1024, 2048):
            _lib.set_option("thin_blocks", nb)
            extra.append("blk%d %.1f" % (nb, bench(run, reps)))
        _lib.set_option("thin_blocks", 512)
        t1 = bench(run, reps)
        k1 = _lib.last_conv_kernel()
        _lib.set_option("thin_kernel", 0)
        t0 = bench(run, reps)
        k0 = _lib.last_conv_kernel()
        _lib.set_option("thin_kernel", 1)
        gb = base.numel() * 2 / 1e9
        print("%-10s %7.1f us (%5.2f TB/s) %-24s | %s | generic %7.1f us %s" % (name, t1, gb / t1 * 1e3, k1,
                                                                              " ".join(extra), t0, k0), flush=True)


if __name__ == "__main__":
    main()
