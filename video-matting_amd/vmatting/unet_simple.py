"""Three-tower "simple" U-Net (reference unet_simple.py) on gfx950 kernels.

``create_model(cmp, bg, diff, phase)`` returns a ``UNetSimple`` whose ``.output`` is the
sigmoid alpha ('probs', unet_simple.py:142) — the call shape of train.py:251-252,356-357.
The three frozen VGG16 towers (unet_simple.py:45-113) share one set of weights; each tower
writes its feature maps straight into channel slices of the per-level concat buffers
(``layers['convK'][i]``, unet_simple.py:153-168), so no tf.concat is ever materialised.

Inputs: NHWC float32 [N,H,W,3] BGR, mean-subtracted (loader.py:76-77); ``diff`` is cmp-bg
(train.py:245) or the warped previous alpha (train.py:356).  ``phase``: BN mode (bool).
"""

import numpy as np
import torch

from . import ops
from .layers import BatchNorm, conv_bn
from .weights import init_conv, load_vgg16

TOWER = ("conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3",
         "conv4_1", "conv4_2", "conv4_3", "conv5_1", "conv5_2", "conv5_3")

# UNetSimple.__init__ build order (unet_simple.py:119-142): scope, cin, cout
NEW_CONVS = (("select4_1", 1536, 16), ("select4_2", 1536, 16), ("select4_3", 1536, 16),
             ("upconv4", 1536, 48), ("conv4", 96, 48),
             ("select3_1", 768, 8), ("select3_2", 768, 8), ("select3_3", 768, 8),
             ("upconv3", 48, 24), ("conv3", 48, 24),
             ("select2_1", 384, 4), ("select2_2", 384, 4),
             ("upconv2", 24, 24), ("conv2", 32, 32),
             ("select1_1", 9, 2), ("select1_2", 192, 2), ("select1_3", 192, 2),
             ("upconv1", 32, 24), ("conv1", 30, 32),
             ("output", 32, 1))
BN_SCOPES = {"upconv4": 96, "upconv3": 48, "upconv2": 32, "upconv1": 30}
# bf16: convs whose input width is not a multiple of 32 read a zero-padded buffer through a channel-padded pack,
# so they run on the patch-reuse MFMA kernel (cin % 32 == 0) instead of the generic one
CIN_PAD = {"select1_1": 32, "upconv2": 32, "upconv3": 64, "conv3": 64}


def _levels(h, w):
    lv = [(h, w)]
    for _ in range(4):
        lv.append(((lv[-1][0] + 1) // 2, (lv[-1][1] + 1) // 2))
    return lv


class Vgg16:
    """unet_simple.Vgg16 (unet_simple.py:45-113): frozen VGG16 conv1_1..conv5_3 (tf.constant weights)."""

    def __init__(self, vgg16_npy_path=None, dtype="bf16", device="cuda"):
        self.data_dict = load_vgg16(vgg16_npy_path)
        self.dtype = ops.TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.device = torch.device(device)
        self.convs = {n: ops.PackedConv(self.data_dict[n][0], self.data_dict[n][1], self.dtype, self.device)
                      for n in TOWER}


class UNetSimple:
    """unet_simple.UNetSimple + create_model on device.  Build once, evaluate with forward()."""

    def __init__(self, vgg, phase, dtype="bf16", device="cuda", params=None):
        self.vgg = vgg
        self.phase = bool(phase)
        self.dtype = vgg.dtype
        self.device = vgg.device
        if params is None:
            params = {}
            for name, cin, cout in NEW_CONVS:
                w, b = init_conv(cin, cout)
                params[name] = (w, None if name.startswith("upconv") else b)
        self.params = params
        self.convs = {k: ops.PackedConv(w, b, self.dtype, self.device) for k, (w, b) in params.items()}
        self.padded = {}
        if self.dtype == torch.bfloat16:
            self.padded = {k: ops.PackedConv.from_source(self.convs[k], c, self.convs[k].cout, self.dtype,
                                                         bias=self.convs[k].bias) for k, c in CIN_PAD.items()}
        self.bn = {k: BatchNorm(c, self.device) for k, _, c in NEW_CONVS if not k.startswith("upconv")}
        self.bn.update({k: BatchNorm(c, self.device) for k, c in BN_SCOPES.items()})
        self._ws, self._key = None, None

    def _buffers(self, n, h, w):
        """Activation buffers for an [n,h,w] batch.  The three towers run as ONE batch of 3n frames (tower t =
        frames t*n .. t*n+n-1 of every t_* buffer); the per-level concats of create_model (unet_simple.py:153-168)
        are ops.SourceConcat views of those tower-major buffers, read as three sources by the select convs."""
        if self._key == (n, h, w):
            return self._ws
        L = _levels(h, w)
        T, dev = self.dtype, self.device
        Z = lambda lv, c, dt=T, k=1: torch.zeros((k * n, L[lv][0], L[lv][1], c), dtype=dt, device=dev)  # noqa: E731
        b = {"tin": Z(0, 8, k=3), "in9": Z(0, 32)}
        widths = {"conv1_1": (0, 64), "conv1_2": (0, 64), "conv2_1": (1, 128), "conv2_2": (1, 128),
                  "conv3_1": (2, 256), "conv3_2": (2, 256), "conv3_3": (2, 256), "conv4_1": (3, 512),
                  "conv4_2": (3, 512), "conv4_3": (3, 512), "conv5_1": (4, 512), "conv5_2": (4, 512),
                  "conv5_3": (4, 512)}
        for k, (lv, c) in widths.items():
            b["t_" + k] = Z(lv, c, k=3)
            b["cat_" + k] = ops.SourceConcat(b["t_" + k], 3)
        for i, c in enumerate((64, 128, 256, 512)):
            b["tpool%d" % (i + 1)] = Z(i + 1, c, k=3)
        # the upconv_concat buffers (select outputs + upconv relu, the input of the upconv BN) are f32: with batch
        # statistics, bf16 rounding of them feeds the BN backward's x-hat projection and costs the select gammas'
        # gradients 4-14x their f64 sensitivity (tests/test_gpu_train.py::test_train_step_bf16_gradients)
        F = torch.float32
        b.update(up4=Z(3, 96, F), up4n=Z(3, 96), r4=ops.SourceConcat(Z(3, 512, k=3), 3), c4=Z(3, 48),
                 up3=Z(2, 48, F), up3n=Z(2, 64)[..., :48], r3=Z(2, 64)[..., :48], c3=Z(2, 24),
                 up2=Z(1, 32, F), up2n=Z(1, 32), r2=Z(1, 32)[..., :24], c2=Z(1, 32),
                 up1=Z(0, 32, F), up1n=Z(0, 32), r1=Z(0, 32), c1=Z(0, 32),
                 logits=Z(0, 1, torch.float32), out=Z(0, 1, torch.float32))
        self._ws, self._key = b, (n, h, w)
        return b

    def conv(self, scope, x):
        """(pack, input) for conv ``scope`` on the logical view x: the channel-padded pack on x widened to its
        buffer's zero pad channels (bf16, CIN_PAD), else the conv itself on x."""
        pc = self.padded.get(scope)
        if pc is None:
            return self.convs[scope], x
        return pc, ops.widen(x, pc.cin)

    def relink_padded(self):
        """Point the padded packs' biases at their convs' (after VideoTrainer aliases them onto its flat buffer)."""
        for k, pc in self.padded.items():
            pc.bias = self.convs[k].bias

    def _towers(self, b, splitk=True):
        """The three frozen towers of create_model (vgg1/2/3 on cmp/bg/diff, unet_simple.py:57-89, 148-152) as one
        batch-3n VGG16 pass over b['tin'] (the towers share weights); 2x2 pools fused into the conv epilogue.
        ``splitk``: split-K on the small L4/L5 grids (training); inference leaves it off so frames are
        batch-invariant."""
        V = self.vgg.convs
        t = lambda k: b["t_" + k]  # noqa: E731
        # conv1_1 -> conv1_2 -> pool1 as one strip-walking kernel that also writes conv1_1 (select1_2 reads it)
        ops.conv_pair_first(b["tin"][..., :3], V["conv1_1"], V["conv1_2"], "relu", out=t("conv1_2"),
                            pool_out=b["tpool1"], mid=t("conv1_1"), keep_mid=True)
        ops.conv3x3(b["tpool1"], V["conv2_1"], "relu", out=t("conv2_1"))
        ops.conv3x3(t("conv2_1"), V["conv2_2"], "relu", out=t("conv2_2"), pool_out=b["tpool2"])
        ops.conv3x3(b["tpool2"], V["conv3_1"], "relu", out=t("conv3_1"))
        ops.conv3x3(t("conv3_1"), V["conv3_2"], "relu", out=t("conv3_2"))
        ops.conv3x3(t("conv3_2"), V["conv3_3"], "relu", out=t("conv3_3"), pool_out=b["tpool3"])
        ops.conv3x3(b["tpool3"], V["conv4_1"], "relu", out=t("conv4_1"), splitk=splitk)
        ops.conv3x3(t("conv4_1"), V["conv4_2"], "relu", out=t("conv4_2"), splitk=splitk)
        ops.conv3x3(t("conv4_2"), V["conv4_3"], "relu", out=t("conv4_3"), pool_out=b["tpool4"])
        ops.conv3x3(b["tpool4"], V["conv5_1"], "relu", out=t("conv5_1"), splitk=splitk)
        ops.conv3x3(t("conv5_1"), V["conv5_2"], "relu", out=t("conv5_2"), splitk=splitk)
        ops.conv3x3(t("conv5_2"), V["conv5_3"], "relu", out=t("conv5_3"), splitk=splitk)

    def load_inputs(self, b, xs):
        """cmp / bg / diff (f32 device tensors) into the towers' batch (tower t = frames t*n..) and into the 9-channel
        layers['conv1'][0] = concat(cmp, bg, diff) (unet_simple.py:148-152)."""
        self.load_towers(b, xs)
        self.load_in9(b, xs)

    def load_towers(self, b, xs):
        """cmp / bg / diff into the towers' batch only."""
        n = xs[0].shape[0]
        for t in range(3):
            ops.convert(xs[t], b["tin"][t * n:(t + 1) * n])

    def load_in9(self, b, xs):
        """cmp / bg / diff into the 9-channel concat only (read first by the level-0 select convs)."""
        for t in range(3):
            ops.convert(xs[t], b["in9"][..., 3 * t:3 * t + 3])

    def forward(self, cmp, bg, diff, phase=None):
        ph = self.phase if phase is None else bool(phase)
        xs = [t if isinstance(t, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(t, np.float32))
              for t in (cmp, bg, diff)]
        xs = [t.to(self.device, torch.float32) for t in xs]
        n, h, w, _ = xs[0].shape
        b = self._buffers(n, h, w)
        L = _levels(h, w)
        C, B = self.convs, self.bn
        self.load_inputs(b, xs)
        self._towers(b, splitk=ph)
        R = lambda x, k, out: conv_bn(*self.conv(k, x)[::-1], B[k], ph, "relu", out)  # noqa: E731
        # level 4
        for i in range(3):
            R(b["cat_conv4_%d" % (i + 1)], "select4_%d" % (i + 1), b["up4"][..., 16 * i:16 * (i + 1)])
        self._upconv(b["cat_conv5_3"], L[3], "upconv4", b["r4"], b["up4"][..., 48:96], b["up4"], b["up4n"], ph)
        R(b["up4n"], "conv4", b["c4"])
        # level 3
        for i in range(3):
            R(b["cat_conv3_%d" % (i + 1)], "select3_%d" % (i + 1), b["up3"][..., 8 * i:8 * (i + 1)])
        self._upconv(b["c4"], L[2], "upconv3", b["r3"], b["up3"][..., 24:48], b["up3"], b["up3n"], ph)
        R(b["up3n"], "conv3", b["c3"])
        # level 2
        for i in range(2):
            R(b["cat_conv2_%d" % (i + 1)], "select2_%d" % (i + 1), b["up2"][..., 4 * i:4 * (i + 1)])
        self._upconv(b["c3"], L[1], "upconv2", b["r2"], b["up2"][..., 8:32], b["up2"], b["up2n"], ph)
        R(b["up2n"], "conv2", b["c2"])
        # level 1
        R(b["in9"][..., :9], "select1_1", b["up1"][..., 0:2])
        R(b["cat_conv1_1"], "select1_2", b["up1"][..., 2:4])
        R(b["cat_conv1_2"], "select1_3", b["up1"][..., 4:6])
        self._upconv(b["c2"], L[0], "upconv1", b["r1"], b["up1"][..., 6:30], b["up1"][..., :30],
                     b["up1n"][..., :30], ph)
        R(b["up1n"][..., :30], "conv1", b["c1"])
        conv_bn(b["c1"], C["output"], B["output"], ph, "none", b["logits"])
        ops.convert(b["logits"], b["out"], act="sigmoid")
        self._publish(b)
        return self.output

    def _upconv(self, prev, size, scope, rbuf, up_slice, cat, catn, phase):
        """upconv_concat (unet_simple.py:30-42): resize -> conv (no bias) -> relu -> concat -> BN."""
        if isinstance(prev, ops.SourceConcat):  # upconv4 on the towers' conv5_3: resize the tower-major batch
            ops.resize_bilinear(prev.base, size, out=rbuf.base)
        else:
            ops.resize_bilinear(prev, size, out=rbuf)
        pc, x = self.conv(scope, rbuf)
        ops.conv3x3(x, pc, "relu", out=up_slice, affine=False, splitk=bool(phase))
        self.bn[scope](cat, phase, out=catn)

    def _publish(self, b):
        for k in ("select4_1", "select4_2", "select4_3"):
            i = int(k[-1]) - 1
            setattr(self, k, b["up4"][..., 16 * i:16 * (i + 1)])
        for k in ("select3_1", "select3_2", "select3_3"):
            i = int(k[-1]) - 1
            setattr(self, k, b["up3"][..., 8 * i:8 * (i + 1)])
        self.select2_1, self.select2_2 = b["up2"][..., 0:4], b["up2"][..., 4:8]
        self.select1_1, self.select1_2, self.select1_3 = b["up1"][..., 0:2], b["up1"][..., 2:4], b["up1"][..., 4:6]
        self.upconv4, self.conv4 = b["up4n"], b["c4"]
        self.upconv3, self.conv3 = b["up3n"], b["c3"]
        self.upconv2, self.conv2 = b["up2n"], b["c2"]
        self.upconv1, self.conv1 = b["up1n"][..., :30], b["c1"]
        self.logits = b["logits"]
        self.output = b["out"]


def create_model(cmp, bg, diff, phase, vgg16_npy_path=None, dtype="bf16", device="cuda", params=None):
    """unet_simple.create_model (unet_simple.py:145-171): builds and evaluates once; returns the model."""
    vgg = Vgg16(vgg16_npy_path, dtype, device)
    model = UNetSimple(vgg, phase, dtype, device, params)
    model.forward(cmp, bg, diff)
    return model
