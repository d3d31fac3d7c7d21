"""Refine conv4 + softmax (refine.py:27-32) at 1080p, bf16 and fp32: vm softmax_kernel variants side by side.

0 = generic conv kernel + LDS softmax epilogue, 1 = conv3x3_first_softmax, 2 = its nontemporal-store form,
4 = + per-wave LDS transpose (default), 5 = weights in LDS, 6 = wave-private strips (conv3x3_first_softmax_strip);
fp32: 0 = generic f32 kernel, else conv3x3_first_softmax_f32.
Algorithmic bytes: 16 B/px bf16 input chunk (8 channels) + 256 B/px f32 softmax out.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/video-matting_amd")
from vmatting import _lib, ops  # noqa: E402

h, w = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (1080, 1920)))
rs = np.random.RandomState(0)
xf = torch.from_numpy(rs.uniform(-1, 1, size=(1, h, w, 8)).astype(np.float32)).cuda()
wt, bias = (rs.normal(size=(3, 3, 5, 64)) * 0.3).astype(np.float32), rs.normal(size=64).astype(np.float32)
pcs = {"bf16": ops.PackedConv(wt, bias, "bf16"), "fp32": ops.PackedConv(wt, bias, "fp32")}
xs = {"bf16": xf.to(torch.bfloat16), "fp32": xf}
out = torch.empty((1, h, w, 64), dtype=torch.float32, device="cuda")
CFGS = [("bf16", 6, 2048, 0), ("fp32", 0, 1024, 0)] + [("fp32", 6, b, 0) for b in (1024, 2048, 4096)] + \
    [("fp32", 6, 2048, p) for p in (1, 2, 3, 4, 5, 6, 4, 6)]  # pipelined f32 kernel: one resident round whatever softmax_blocks
if len(sys.argv) > 3 and sys.argv[3] == "fp32":
    CFGS = CFGS[2:]
for dt, k, blocks, f32p in CFGS:
    _lib.set_option("softmax_kernel", k)
    _lib.set_option("softmax_blocks", blocks)
    _lib.set_option("softmax_f32p", f32p)
    x, pc = xs[dt], pcs[dt]
    nbytes = h * w * ((16 if dt == "bf16" else 32) + 256)
    fn = lambda: ops.conv3x3(x[..., :5], pc, "softmax", out=out)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 50
    print("%s softmax_kernel %d blocks %5d  %-42s %.1f us  %.2f TB/s algorithmic" % (
        dt, k, blocks, _lib.last_conv_kernel(), ms * 1e3, nbytes / ms / 1e9), flush=True)
_lib.set_option("softmax_kernel", 6)
_lib.set_option("softmax_blocks", 2048)
_lib.set_option("softmax_f32p", 4)
