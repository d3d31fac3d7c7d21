"""Matte refinement net (reference refine.py) on gfx950 kernels.

``RefineNet().build(input)`` sets ``.output`` = ``.conv4`` = softmax over 64 channels of a
3x3 conv of ``input`` (refine.py:27-32); the softmax is fused into the conv epilogue (one
tile holds all 64 channels of a pixel).  conv1..conv3 are three more independent relu
convs of the same input that the reference wires but never consumes; they are computed
lazily on first attribute access so the output path pays nothing for them.
"""

import numpy as np
import torch

from . import ops
from .weights import init_conv


class RefineNet:
    def __init__(self, dtype="bf16", device="cuda"):
        self.dtype = ops.TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.device = torch.device(device)
        self.params = None
        self.convs = None
        self._x = None
        self._lazy = {}

    def build(self, input):
        x = input if isinstance(input, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(input, np.float32))
        x = x.to(self.device, torch.float32)
        if self.params is None:  # refine.py:28-31: conv1..conv4 drawn in order, each with its bias
            cin = int(x.shape[-1])
            self.params = {k: init_conv(cin, 64) for k in ("conv1", "conv2", "conv3", "conv4")}
        if self.convs is None:
            self.convs = {k: ops.PackedConv(w, b, self.dtype, self.device) for k, (w, b) in self.params.items()}
        return self.forward(x)

    def forward(self, input):
        x = input.to(self.device, torch.float32) if isinstance(input, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(input, np.float32)).to(self.device)
        n, h, w, c = x.shape
        cpad = (c + 7) // 8 * 8
        xin = torch.empty((n, h, w, cpad), dtype=self.dtype, device=self.device)
        ops.convert(x, xin)
        return self.forward_prepared(xin[..., :c])

    def prepare(self, cin):
        """Draw (refine.py:28-31 order) and pack the four filters for a ``cin``-channel input without a frame."""
        if self.params is None:
            self.params = {k: init_conv(cin, 64) for k in ("conv1", "conv2", "conv3", "conv4")}
        if self.convs is None:
            self.convs = {k: ops.PackedConv(w, b, self.dtype, self.device) for k, (w, b) in self.params.items()}
        return self

    def forward_prepared(self, x, out=None):
        """Forward on an input already in the compute dtype with channels padded to 8 (a channel view such as
        the one vm_temporal_refine_input writes); ``out`` optionally receives the f32 [N,H,W,64] softmax."""
        self._x = x
        self._lazy = {}
        self.conv4 = ops.conv3x3(x, self.convs["conv4"], "softmax", out=out, out_dtype=torch.float32)
        self.output = self.conv4
        return self.output

    def __getattr__(self, name):
        if name in ("conv1", "conv2", "conv3"):
            lazy = self.__dict__.get("_lazy", {})
            if name not in lazy:
                if self.__dict__.get("_x") is None:
                    raise AttributeError(name)
                lazy[name] = ops.conv3x3(self._x, self.convs[name], "relu", out_dtype=torch.float32)
            return lazy[name]
        raise AttributeError(name)
