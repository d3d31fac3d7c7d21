"""Diagnostic: per-tensor relative L2 error of the bf16 training step's gradients vs the f64 autograd restatement,
with the MFMA and the exact-f32 weight-gradient kernels.   python tools/bf16_grad_diag.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import models as om  # noqa: E402
from oracle import train_ref as tr  # noqa: E402
from test_gpu_train import _batch  # noqa: E402
from vmatting.train import VideoTrainer  # noqa: E402
from vmatting.weights import synthetic_vgg16  # noqa: E402


def main():
    params = om.unet_simple_params(np.random.RandomState(1))
    cmp, bg, warped, gt, fg = _batch(2, 64, 80)
    vgg = synthetic_vgg16(0)
    _, _, grads = tr.train_step_grads(cmp, bg, warped, gt, fg, vgg, params)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    res = {}
    for dt, mf in (("bf16", True), ("bf16", False), ("fp32", False)):
        trn = VideoTrainer(vgg, dt, "cuda", params=params)
        trn._mfma_wgrad = mf
        trn.forward(cmp, bg, warped)
        trn.grad.zero_()
        trn.backward(T(gt), T(fg), T(bg), T(cmp))
        torch.cuda.synchronize()
        res[(dt, mf)] = {k: trn.G[k].cpu().numpy().astype(np.float64) for k in grads}
        a = trn.output.cpu().numpy()
        print(dt, "mfma" if mf else "fma", "alpha range", a.min(), a.max())
    print("%-22s %10s %10s %10s" % ("tensor", "bf16-mfma", "bf16-fma", "fp32"))
    for k, g in grads.items():
        if k[1] == "b":
            continue
        e = [np.linalg.norm(res[c][k] - g) / max(np.linalg.norm(g), 1e-30) for c in res]
        print("%-22s %10.3e %10.3e %10.3e" % (k, *e))


if __name__ == "__main__":
    main()
