"""The wide weight gradients of the UNetImage training step (8 x 320^2, bf16 x and bf16 dy, every conv but conv1_5):
per-layer ms / TFLOP/s and the total.   python tools/wgradwide_bench.py [iters] [key=value ...]   (vm_set_option
A/B knobs, e.g. wgrad_wide_pipe=0; VM_LIB_PATH for an A/B build)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

from vmatting import _lib, ops  # noqa: E402

# (name, side, cin, cout) at 8 x 320^2 (unet.py:96-143)
SHAPES = [("upconv_4", 320, 128, 64), ("conv2_3", 160, 256, 128), ("upconv_3", 160, 256, 128),
          ("conv3_4", 80, 512, 256), ("upconv_2", 80, 512, 256), ("conv4_4", 40, 1024, 512),
          ("upconv_1", 40, 512, 512), ("conv5_2", 20, 512, 512), ("conv5_1", 20, 512, 512),
          ("conv4_3", 40, 512, 512), ("conv4_2", 40, 512, 512), ("conv4_1", 40, 256, 512),
          ("conv3_3", 80, 256, 256), ("conv3_2", 80, 256, 256), ("conv3_1", 80, 128, 256),
          ("conv2_2", 160, 128, 128), ("conv2_1", 160, 64, 128), ("conv1_2", 320, 64, 64), ("conv1_1", 320, 6, 64)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    tot_ms, tot_fl = 0.0, 0.0
    for name, s, cin, cout in SHAPES:
        cs = (cin + 7) // 8 * 8
        x = torch.randn(8, s, s, cs, device="cuda").to(torch.bfloat16)[..., :cin]
        dy = torch.randn(8, s, s, cout, device="cuda").to(torch.bfloat16)
        dw = torch.zeros((3, 3, cin, cout), device="cuda")
        for _ in range(2):
            ops.conv_wgrad(x, dy, dw, mfma=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.conv_wgrad(x, dy, dw, mfma=True)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / iters
        fl = 2.0 * 8 * s * s * 9 * cin * cout
        tot_ms += t
        tot_fl += fl
        print("%-9s %3d^2 %5d->%-4d %.4f ms %7.1f TFLOP/s" % (name, s, cin, cout, t, fl / t / 1e9), flush=True)
    print("total %.3f ms, %.1f TFLOP/s" % (tot_ms, tot_fl / tot_ms / 1e9))


if __name__ == "__main__":
    main()
