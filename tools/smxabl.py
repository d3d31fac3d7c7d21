"""f32 refine conv4 + softmax (refine.py:27-32) at 1080p: timing ablations of conv3x3_first_softmax_f32 (study build:
VM_LIB_PATH=video-matting_amd/study/libvmatting_study.so).  0 = full kernel, 1 = no softmax / store, 2 = no MFMA,
3 = neither (staging + loads only).  The pipelined kernel (default; first argument "old" for the r03 kernel): bit 1 =
no stores, 2 = no MFMA, 4 = no softmax arithmetic."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/video-matting_amd")
from vmatting import _lib, ops  # noqa: E402

h, w = 1080, 1920
rs = np.random.RandomState(0)
xf = torch.from_numpy(rs.uniform(-1, 1, size=(1, h, w, 8)).astype(np.float32)).cuda()
wt, bias = (rs.normal(size=(3, 3, 5, 64)) * 0.3).astype(np.float32), rs.normal(size=64).astype(np.float32)
pc = ops.PackedConv(wt, bias, "fp32")
out = torch.empty((1, h, w, 64), dtype=torch.float32, device="cuda")
args = sys.argv[1:]
if args and args[0] == "old":
    _lib.set_option("softmax_f32p", 0)
    args = args[1:]
for abl in [int(v) for v in (args or ["0", "1", "2", "3", "4", "5", "6", "7", "0"])]:
    _lib.set_option("softmax_abl", abl)
    fn = lambda: ops.conv3x3(xf[..., :5], pc, "softmax", out=out)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print("abl %d %s: %.4f ms" % (abl, _lib.last_conv_kernel(), e0.elapsed_time(e1) / 50), flush=True)
_lib.set_option("softmax_abl", 0)
