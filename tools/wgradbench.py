"""Weight-gradient microbenchmark on the config-5 shapes (8 x 320x320, unet_simple's trainable convs):
the exact-f32 FMA kernel vs the bf16 MFMA kernel.   python tools/wgradbench.py [iters]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

from vmatting import ops  # noqa: E402

# (name, level side, cin (x buffer width), cout) at 8 x 320^2
SHAPES = [("select4", 40, 1536, 16), ("upconv4", 40, 1536, 48), ("conv4", 40, 96, 48), ("select3", 80, 768, 8),
          ("upconv3", 80, 48, 24), ("conv3", 80, 48, 24), ("select2", 160, 384, 4), ("upconv2", 160, 24, 24),
          ("conv2", 160, 32, 32), ("select1_1", 320, 9, 2), ("select1_2", 320, 192, 2), ("upconv1", 320, 32, 24),
          ("conv1", 320, 30, 32), ("output", 320, 32, 1)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    if os.environ.get("WGRAD_VARIANT"):
        from vmatting import _lib
        _lib.set_option("wgrad_variant", int(os.environ["WGRAD_VARIANT"]))
    tot = [0.0, 0.0]
    for name, s, cin, cout in SHAPES:
        cs = (cin + 15) // 16 * 16
        x = (torch.randn(8, s, s, cs, device="cuda")).to(torch.bfloat16)[..., :cin]
        dy = torch.randn(8, s, s, cout, device="cuda")
        dw = torch.zeros((3, 3, cin, cout), device="cuda")
        res = []
        for mf in (False, True):
            for _ in range(2):
                ops.conv_wgrad(x, dy, dw, mfma=mf)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ops.conv_wgrad(x, dy, dw, mfma=mf)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / iters)
        fl = 2.0 * 8 * s * s * 9 * cin * cout
        tot[0] += res[0]
        tot[1] += res[1]
        print("%-10s %3d^2 %5d->%-3d  fma %.4f ms  mfma %.4f ms  (%.1f / %.1f TFLOP/s)" %
              (name, s, cin, cout, res[0], res[1], fl / res[0] / 1e9, fl / res[1] / 1e9), flush=True)
    print("total fma %.3f ms  mfma %.3f ms" % tuple(tot))


if __name__ == "__main__":
    main()
