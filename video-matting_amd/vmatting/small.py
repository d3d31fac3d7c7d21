"""Small 3-level U-Net (reference small.py; imported as ``unet`` by small_train.py:3).

``UNetSmall(input, phase)`` evaluates on construction and exposes ``.output`` ('probs') and the
reference's attributes (small.py:38-50).  Concat order is [skip, up] (small.py:20), realised as
channel-slice writes into one buffer per level.
"""

import numpy as np
import torch

from . import ops
from .layers import BatchNorm, conv_bn
from .weights import init_conv

# small.py:39-49 build order; conv1_1's cin is the caller's input width (6 in small_train.py:95)
NEW_CONVS = (("conv1_1", None, 8), ("conv2_1", 8, 16), ("conv3_1", 16, 32), ("conv3_2", 32, 32),
             ("upconv1", 32, 16), ("conv2_2", 32, 16), ("upconv2", 16, 8), ("conv1_2", 16, 8),
             ("conv1_3", 8, 1))


class UNetSmall:
    def __init__(self, input, phase, dtype="bf16", device="cuda", params=None):
        x = input if isinstance(input, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(input, np.float32))
        self.dtype = ops.TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.device = torch.device(device)
        self.phase = bool(phase)
        cin = int(x.shape[-1])
        self.cin = cin
        if params is None:
            params = {}
            for name, ci, co in NEW_CONVS:
                w, b = init_conv(cin if ci is None else ci, co)
                params[name] = (w, None if name.startswith("upconv") else b)
        self.params = params
        self.convs = {k: ops.PackedConv(w, b, self.dtype, self.device) for k, (w, b) in params.items()}
        self.bn = {k: BatchNorm(co, self.device) for k, _, co in NEW_CONVS if not k.startswith("upconv")}
        self.bn["upconv1"] = BatchNorm(32, self.device)
        self.bn["upconv2"] = BatchNorm(16, self.device)
        self._ws, self._key = None, None
        self.forward(x)

    def _buffers(self, n, h, w):
        if self._key == (n, h, w):
            return self._ws
        h2, w2 = (h + 1) // 2, (w + 1) // 2
        h3, w3 = (h2 + 1) // 2, (w2 + 1) // 2
        T, dev = self.dtype, self.device
        Z = lambda hh, ww, c, dt=T: torch.zeros((n, hh, ww, c), dtype=dt, device=dev)  # noqa: E731
        cpad = (self.cin + 7) // 8 * 8
        b = dict(inp=Z(h, w, cpad), up2=Z(h, w, 16), up2n=Z(h, w, 16), r2=Z(h, w, 16), c12=Z(h, w, 8),
                 p1=Z(h2, w2, 8), up1=Z(h2, w2, 32), up1n=Z(h2, w2, 32), r1=Z(h2, w2, 32), c22=Z(h2, w2, 16),
                 p2=Z(h3, w3, 16), c31=Z(h3, w3, 32), c32=Z(h3, w3, 32),
                 logits=Z(h, w, 1, torch.float32), out=Z(h, w, 1, torch.float32))
        self._ws, self._key = b, (n, h, w)
        return b

    def forward(self, input, phase=None):
        ph = self.phase if phase is None else bool(phase)
        x = input if isinstance(input, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(input, np.float32))
        x = x.to(self.device, torch.float32)
        n, h, w, c = x.shape
        b = self._buffers(n, h, w)
        C, B = self.convs, self.bn
        R = lambda t, k, out: conv_bn(t, C[k], B[k], ph, "relu", out)  # noqa: E731
        ops.convert(x, b["inp"])
        R(b["inp"][..., :c], "conv1_1", b["up2"][..., :8])        # conv1_1 lives in the [skip, up] buffer
        ops.maxpool2x2(b["up2"][..., :8], out=b["p1"])
        R(b["p1"], "conv2_1", b["up1"][..., :16])
        ops.maxpool2x2(b["up1"][..., :16], out=b["p2"])
        R(b["p2"], "conv3_1", b["c31"])
        R(b["c31"], "conv3_2", b["c32"])
        self._upconv(b["c32"], b["up1"], b["up1n"], "upconv1", b["r1"], 16, ph)
        R(b["up1n"], "conv2_2", b["c22"])
        self._upconv(b["c22"], b["up2"], b["up2n"], "upconv2", b["r2"], 8, ph)
        R(b["up2n"], "conv1_2", b["c12"])
        conv_bn(b["c12"], C["conv1_3"], B["conv1_3"], ph, "none", b["logits"])
        ops.convert(b["logits"], b["out"], act="sigmoid")
        self.conv1_1, self.pool1 = b["up2"][..., :8], b["p1"]
        self.conv2_1, self.pool2 = b["up1"][..., :16], b["p2"]
        self.conv3_1, self.conv3_2 = b["c31"], b["c32"]
        self.upconv1, self.conv2_2 = b["up1n"], b["c22"]
        self.upconv2, self.conv1_2 = b["up2n"], b["c12"]
        self.conv1_3, self.output = b["logits"], b["out"]
        return self.output

    def _upconv(self, down, cat, catn, scope, rbuf, skip_c, phase):
        """small.upconv_concat (small.py:13-23): resize -> conv (no bias) -> relu -> concat [skip, up] -> BN."""
        ops.resize_bilinear(down, cat.shape[1:3], out=rbuf)
        ops.conv3x3(rbuf, self.convs[scope], "relu", out=cat[..., skip_c:], affine=False)
        self.bn[scope](cat, phase, out=catn)
