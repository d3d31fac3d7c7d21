"""unet.py's forward at f32 accuracy on the bf16 MFMA kernels: the split-bf16 x6 conv (``UNetVideo(dtype="bf16x6")``).

north_star asks for alpha within 1e-4 of the reference's CPU forward (unet.py:161-205).  The bf16 path misses it
(20 bf16-rounded layers; alpha 0.45 max-abs on the timed frame's steep-sigmoid pixels) and the exact-f32 MFMA
(v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16 rate.  Here every conv input and filter is carried as three bf16
parts (x = h + m + l, csrc/elementwise.hip vm_split6_nhwc; 24 significant bits) and each conv is ONE bf16 MFMA conv
over 6 stacked channel slabs,

    y = l*Wh + m*Wm + h*Wl + m*Wh + h*Wm + h*Wh       (all cross products down to 2^-16 of h*Wh)

with exact bf16 x bf16 products and f32 accumulation, smallest terms first along K.  A float64 emulation of the
whole 1080p forward puts the representation error at 3.6e-8 of max |logit| (alpha 4e-7): what remains is the f32
accumulation order, as in the f32 path.  Cost: 6x the MFMA work of the bf16 forward plus one split pass per
activation; no kernel changes — the convs run on the same patch / row kernels with f32 epilogues.

Per layer: conv (bias + relu in the f32 epilogue) -> f32 scratch -> vm_split6_nhwc into the next conv's split input
(and, fused, the split of its 2x2 SAME max-pool); the [up, skip] concats are channel ranges of one split buffer
(slab p of channel c at p*S + c, S = the concat's width), so each producer writes its own range; the upconvs resize
the f32 conv output (TF-1 legacy bilinear) before splitting.  conv1_5 (cout 1) runs with its output channels padded
to 8 and the sigmoid from the logits in a second pass.
"""

import numpy as np
import torch

from . import ops

# slab order of the activations and of the filter parts they meet (vm_split6_nhwc): l*h, m*m, h*l, m*h, h*m, h*h
W_PARTS = (0, 1, 2, 0, 1, 0)  # index into (wh, wm, wl)

# (conv scope, input channels of its split input (the concat width), output channels)
LAYERS = (("conv1_1", 16, 64), ("conv1_2", 64, 64), ("conv2_1", 64, 128), ("conv2_2", 128, 128),
          ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256), ("conv4_1", 256, 512),
          ("conv4_2", 512, 512), ("conv4_3", 512, 512), ("conv5_1", 512, 512), ("conv5_2", 512, 512),
          ("upconv_1", 512, 512), ("conv4_4", 1024, 512), ("upconv_2", 512, 256), ("conv3_4", 512, 256),
          ("upconv_3", 256, 128), ("conv2_3", 256, 128), ("upconv_4", 128, 64), ("conv1_5", 128, 8))


def split3(w):
    """f32 -> (h, m, l): h = bf16(w), m = bf16(w - h), l = bf16(w - h - m) (RNE), each returned as f32 holding a
    bf16 value exactly (the pack's bf16 rounding then keeps it)."""
    w = torch.as_tensor(w, dtype=torch.float32)
    h = w.bfloat16().float()
    r = w - h
    m = r.bfloat16().float()
    lo = (r - m).bfloat16().float()
    return h, m, lo


def split6_filter(w_hwio, cin, cout):
    """[3,3,ci,co] f32 filter -> the [3,3,6*cin,cout] stack of its parts in slab order (zero rows past ci, zero
    columns past co)."""
    w = torch.as_tensor(np.asarray(w_hwio, np.float32) if not isinstance(w_hwio, torch.Tensor) else w_hwio,
                        dtype=torch.float32).cpu()
    ci, co = int(w.shape[2]), int(w.shape[3])
    parts = split3(w)
    out = torch.zeros((3, 3, 6 * cin, cout), dtype=torch.float32)
    for p, k in enumerate(W_PARTS):
        out[:, :, p * cin:p * cin + ci, :co] = parts[k]
    return out


def split6(x, y, pool=None):
    """vm_split6_nhwc: f32 view x -> its split slabs in the bf16 view y (a channel range of a 6*S-wide buffer, S =
    y's concat width), and optionally the split of its 2x2 SAME max-pool into ``pool``."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    pv = ops.nhwc(pool) if pool is not None else None
    ref = (lambda v: None if v is None else ops.ctypes.byref(v))
    ops.check(ops.lib().vm_split6_nhwc(ref(xv), ref(yv), ref(pv), ops.stream_handle()), "split6")
    return y


def whole(buf):
    """The split-layout view of all channels of a 6*S-wide split buffer."""
    return buf[..., :buf.shape[-1] // 6]


def seg(buf, off, c):
    """The split-layout view of channels [off, off + c) of a 6*S-wide split buffer: a [n,h,w,c] view starting at
    channel off whose rows are 6*S wide (split6 writes the 6 slabs at p*S + off)."""
    return buf[..., off:off + c]


class Split6Forward:
    """The split-bf16 x6 forward of a UNet (unet.UNetVideo / UNetImage) with its parameters."""

    def __init__(self, model):
        self.m = model
        self.dev = model.device
        self.convs = {}
        self.bias8 = None
        for name, cin, cout in LAYERS:
            w, b = model.params[name]
            if name == "conv1_1":
                cin = 16  # 6 slabs of 16 (8 live): 96 channels, whole 32-channel granules for the patch kernel
            if name == "conv1_5":
                # the cout-1 head over 6 x 128 channels as three 256-channel MFMA-head chunks [l m | h m | h h],
                # the smallest first, each adding the previous chunk's logits (vm_conv3x3_head_acc_nhwc)
                wf = split6_filter(w, cin, 1)
                self.head = [ops.PackedConv(wf[:, :, 256 * k:256 * (k + 1)].contiguous(), b if k == 0 else None,
                                            "bf16", self.dev) for k in range(3)]
                self.convs[name] = self.head[0]
                continue
            pc = ops.PackedConv(split6_filter(w, cin, cout), b, "bf16", self.dev)
            self.convs[name] = pc
        self._b, self._key = None, None

    def weights_flat(self):
        out = []
        for pc in [self.convs[k] for k in sorted(self.convs) if k != "conv1_5"] + self.head:
            out.append(pc.packed)
            if pc.bias is not None:
                out.append(pc.bias)
        return out

    def _buffers(self, n, h, w):
        if self._key == (n, h, w):
            return self._b
        from .unet import _levels
        L = _levels(h, w)
        dev = self.dev
        S = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], 6 * c), dtype=torch.bfloat16, device=dev)  # noqa
        F = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], c), dtype=torch.float32, device=dev)  # noqa
        b = {"x": torch.zeros((n, L[0][0], L[0][1], 6 * 16), dtype=torch.bfloat16, device=dev), "s11": S(0, 64), "cat1": S(0, 128), "r4": S(0, 128),
             "p1": S(1, 64), "s21": S(1, 128), "cat2": S(1, 256), "r3": S(1, 256),
             "p2": S(2, 128), "s31": S(2, 256), "s32": S(2, 256), "cat3": S(2, 512), "r2": S(2, 512),
             "p3": S(3, 256), "s41": S(3, 512), "s42": S(3, 512), "cat4": S(3, 1024), "r1": S(3, 512),
             "p4": S(4, 512), "s51": S(4, 512),
             "f0": F(0, 128), "f1": F(1, 256), "f2": F(2, 512), "f3": F(3, 512), "f4": F(4, 512),
             "rr0": F(0, 128), "rr1": F(1, 256), "rr2": F(2, 512), "rr3": F(3, 512),
             "lg0": F(0, 1), "lg1": F(0, 1), "lg2": F(0, 1), "zero": torch.zeros((n, L[0][0], L[0][1], 1), device=dev),
             "out": F(0, 1)}
        self._b, self._key = b, (n, h, w)
        return b

    def forward(self, x, out=None):
        """x: [N,H,W,C] f32 frames (C = 7 video / 6 image) -> alpha [N,H,W,1] f32 (``out`` if given)."""
        from .unet import _levels
        n, h, w, c = x.shape
        b = self._buffers(n, h, w)
        L = _levels(h, w)
        C = self.convs
        split6(x, b["x"][..., :8])  # 6 slabs of 16 channels, 8 written (the rest stay zero)

        def conv(src, name, dst_f32, act="relu"):
            return ops.conv3x3(src, C[name], act, out=dst_f32, affine=False, splitk=True)

        def resize_split(f_src, lv, rr_f32, r_split):
            ops.resize_bilinear(f_src, L[lv], out=rr_f32)
            split6(rr_f32, r_split)

        f0, f1, f2, f3, f4 = b["f0"], b["f1"], b["f2"], b["f3"], b["f4"]
        # encoder (unet.py:170-189)
        split6(conv(b["x"], "conv1_1", f0[..., :64]), whole(b["s11"]))
        split6(conv(b["s11"], "conv1_2", f0[..., :64]), seg(b["cat1"], 64, 64), pool=whole(b["p1"]))
        split6(conv(b["p1"], "conv2_1", f1[..., :128]), whole(b["s21"]))
        split6(conv(b["s21"], "conv2_2", f1[..., :128]), seg(b["cat2"], 128, 128), pool=whole(b["p2"]))
        split6(conv(b["p2"], "conv3_1", f2[..., :256]), whole(b["s31"]))
        split6(conv(b["s31"], "conv3_2", f2[..., :256]), whole(b["s32"]))
        split6(conv(b["s32"], "conv3_3", f2[..., :256]), seg(b["cat3"], 256, 256), pool=whole(b["p3"]))
        split6(conv(b["p3"], "conv4_1", f3), whole(b["s41"]))
        split6(conv(b["s41"], "conv4_2", f3), whole(b["s42"]))
        split6(conv(b["s42"], "conv4_3", f3), seg(b["cat4"], 512, 512), pool=whole(b["p4"]))
        split6(conv(b["p4"], "conv5_1", f4), whole(b["s51"]))
        y52 = conv(b["s51"], "conv5_2", f4)
        # decoder: resize (f32) -> split -> conv (no bias, no relu) into the concat's up range (unet.py:191-200)
        resize_split(y52, 3, b["rr3"], whole(b["r1"]))
        split6(conv(b["r1"], "upconv_1", f3, act="none"), seg(b["cat4"], 0, 512))
        y44 = conv(b["cat4"], "conv4_4", f3)
        resize_split(y44, 2, b["rr2"], whole(b["r2"]))
        split6(conv(b["r2"], "upconv_2", f2[..., :256], act="none"), seg(b["cat3"], 0, 256))
        y34 = conv(b["cat3"], "conv3_4", f2[..., :256])
        resize_split(y34, 1, b["rr1"], whole(b["r3"]))
        split6(conv(b["r3"], "upconv_3", f1[..., :128], act="none"), seg(b["cat2"], 0, 128))
        y23 = conv(b["cat2"], "conv2_3", f1[..., :128])
        resize_split(y23, 0, b["rr0"], whole(b["r4"]))
        split6(conv(b["r4"], "upconv_4", f0[..., :64], act="none"), seg(b["cat1"], 0, 64))
        # conv1_5 + sigmoid (unet.py:203-205): three 256-channel chunks of the split cat1, logits accumulated,
        # the sigmoid from the last
        alpha = b["out"] if out is None else out
        lg = [b["lg0"], b["lg1"], b["lg2"]]
        for k in range(3):
            xv, yv = ops.nhwc(b["cat1"][..., 256 * k:256 * (k + 1)]), ops.nhwc(lg[k])
            pc = self.head[k]
            ops.check(ops.lib().vm_conv3x3_head_acc_nhwc(
                ops.ctypes.byref(xv), ops._ptr(pc.packed), 256, ops._ptr(pc.bias),
                ops._ptr(lg[k - 1] if k else b["zero"]), ops.ctypes.byref(yv),
                ops._ptr(alpha if k == 2 else None), ops.stream_handle()), "conv3x3_head_acc")
        self.logits = lg[2]
        return alpha
