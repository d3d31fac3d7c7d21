"""Conv + batch-norm building blocks shared by unet_simple.py and small.py.

tf.contrib.layers.batch_norm(center=True, scale=True, is_training=phase) (unet_simple.py:25,41;
small.py:22,32): with phase False the moving statistics are used — never updated by the reference
(UPDATE_OPS is not wired: train.py:180,304; small_train.py:48), so they stay mean 0 / var 1 and BN
is the affine x*gamma/sqrt(1+eps)+beta, folded into the conv epilogue.  With phase True, batch
statistics over N,H,W (biased variance) come from the wave-reduction kernels, then one apply pass.
"""

import numpy as np
import torch

from . import ops
from .weights import bn_inference_affine

EPS = 1e-3


class BatchNorm:
    """Per-scope BN variables: gamma (ones), beta (zeros), moving mean (zeros), moving var (ones)."""

    def __init__(self, c, device):
        self.c = c
        self.device = device
        self.set(np.ones(c, np.float32), np.zeros(c, np.float32))

    def set(self, gamma, beta, moving_mean=None, moving_var=None):
        self.gamma_np = np.asarray(gamma, np.float32)
        self.beta_np = np.asarray(beta, np.float32)
        self.mm_np = np.zeros(self.c, np.float32) if moving_mean is None else np.asarray(moving_mean, np.float32)
        self.mv_np = np.ones(self.c, np.float32) if moving_var is None else np.asarray(moving_var, np.float32)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
        self.gamma, self.beta = dev(self.gamma_np), dev(self.beta_np)
        self.mm, self.mv = dev(self.mm_np), dev(self.mv_np)
        s, t = bn_inference_affine(self.gamma_np, self.beta_np, self.mm_np, self.mv_np, EPS)
        self.inf_scale, self.inf_shift = dev(s), dev(t)
        return self

    def __call__(self, x, phase, act="none", out=None):
        """BN (+ activation) of an NHWC view, into ``out`` (default: in place)."""
        if phase:
            mean, var = ops.bn_stats(x)
            return ops.bn_apply(x, mean, var, self.gamma, self.beta, EPS, act, out=out)
        return ops.bn_apply(x, self.mm, self.mv, self.gamma, self.beta, EPS, act, out=out)


def conv_bn(x, pc, bn, phase, act, out):
    """new_conv (conv + bias -> BN) followed by ``act`` (unet_simple.py:19-27 + the relu at the call site)."""
    if not phase:  # inference: no split-K, so a frame's result does not depend on its batch (ops.conv3x3)
        return ops.conv3x3(x, pc, act, out=out, affine=(bn.inf_scale, bn.inf_shift))
    ops.conv3x3(x, pc, "none", out=out, affine=False, splitk=True)
    return bn(out, True, act)
