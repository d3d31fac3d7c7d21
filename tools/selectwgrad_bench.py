"""The select convs' weight gradients at the config-5 training shapes (8 x 320^2 batch; tower-major 3-source x,
unet_simple.py:120-139), standalone: HIP-event ms per call and the x stream rate (bytes of x / time) for each
wgrad_dma / wgrad_dma_cfg setting given.   python tools/selectwgrad_bench.py [iters] [dma:cfg ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

from vmatting import _lib, ops  # noqa: E402

# (name, side, channels per tower source, cout) — x = 3 sources of c channels at side^2, batch 8
SHAPES = [("select1_2", 320, 64, 2), ("select2_1", 160, 128, 4), ("select3_1", 80, 256, 8), ("select4_1", 40, 512, 16)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfgs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[2:]] or [(0, 0), (1, 0)]
    n = 8
    tot = {c: 0.0 for c in cfgs}
    flush = None if os.environ.get("NO_FLUSH") else torch.empty(256 << 20, device="cuda")  # 1 GiB
    for name, s, c, cout in SHAPES:
        base = torch.randn(3 * n, s, s, c, device="cuda").to(torch.bfloat16)
        x = ops.SourceConcat(base, 3)
        dy = torch.randn(n, s, s, cout, device="cuda")
        dw = torch.zeros((3, 3, 3 * c, cout), device="cuda")
        line = []
        for cfg in cfgs:
            _lib.set_option("wgrad_dma", cfg[0])
            _lib.set_option("wgrad_dma_cfg", cfg[1])
            for _ in range(3):
                ops.conv_wgrad(x, dy, dw, mfma=True)
            ev = []
            for _ in range(iters):
                if flush is not None:  # evict L2 / MALL: x streams from HBM, as inside the training step
                    flush.fill_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.conv_wgrad(x, dy, dw, mfma=True)
                e1.record()
                ev.append((e0, e1))
            torch.cuda.synchronize()
            ms = sum(a.elapsed_time(b) for a, b in ev) / iters
            tot[cfg] += ms
            line.append("dma%d:cfg%d %.4f ms %6.0f GB/s" % (cfg[0], cfg[1], ms, base.numel() * 2 / ms / 1e6))
        print("%-10s %3d^2 %4d->%-2d  %s" % (name, s, 3 * c, cout, " | ".join(line)), flush=True)
    print("total " + " | ".join("dma%d:cfg%d %.3f ms" % (c[0], c[1], t) for c, t in tot.items()))


if __name__ == "__main__":
    main()
