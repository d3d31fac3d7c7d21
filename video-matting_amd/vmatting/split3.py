"""unet.py's forward at f32 accuracy in three fp16 MFMA products per conv: the split-fp16 x3 path
(``UNetVideo(dtype="f16x3")``).

north_star asks for alpha within 1e-4 of the reference's CPU forward (unet.py:161-205).  The split-bf16 x6 path
(split6.py) gets there with SIX bf16 products per conv, because a bf16 part holds 8 significant bits and two parts
(16 bits; x3 = hh + hl + lh) leave alpha 7.3e-4 off on the timed frame.  An fp16 part holds 11 bits, so two parts
hold 22:

    x = h + l,  h = fp16(x), l = fp16(x - h)          (the difference is exact in f32)
    W * 2^t = Wh + Wl                                  (t per filter: max |W * 2^t| just under 2^12)
    y = (l*Wh + h*Wl + h*Wh) * 2^-t                    (exact fp16 x fp16 products, f32 accumulation)

The dropped l*Wl term and the parts' residuals are ~2^-22 of h*Wh, 64x below bf16 x3's.  A float64 emulation of the
whole 1080p forward on the bench's frame and weights (tools/split_emulate.py) puts alpha 1.9e-5 from the exact
forward (logits 4.0e-7 relative), bf16 x3 7.3e-4.  The filter scale keeps the small parts Wl in fp16's normal range
(He-normal filters are ~0.01-0.1, so their unscaled low parts would be subnormal); it is a power of two, so the
epilogue's ``* 2^-t`` is exact (the conv's per-channel scale; the bias rides in the shift).  Activations stay
unscaled: |x| on this network is ~2e3 against fp16's 65504; a split that meets |x| >= 65520 sets an overflow flag
(``overflowed()``), and ``UNet.build`` then re-runs the frames on the bf16x6 path.

Cost: 3x the MFMA work of the bf16 forward (x6: 6x) on the same patch kernels (their fp16 MFMA form,
v_mfma_f32_16x16x32_f16); the conv's epilogue writes its output split (vm_conv3x3_split3_nhwc, and the split of the
fused 2x2 pool), so activations never round-trip through f32 except where a resize follows (conv5_2, conv4_4,
conv3_4, conv2_3 feed the TF-1 resizes, which run in f32).  Layout: a split buffer holds slabs [l, h] of its S
channels at p*S + c (S = the concat width, so the [up, skip] concats are channel ranges written by their own
producers, as in split6.py); the convs read it as [l, h, h] (the kernel re-reads slab h for the third K range,
ConvArgs::xalias), so h is stored once.  conv1_1's 7-channel frame is split into two stored slabs [l, h] of 32 channels, read as
[l, h, h] (Split3Forward.first_slab).  conv1_5 (cout 1) is one MFMA-head call over cat1's [l, h] read as [l, h, h] (12 k-steps, the third
range's fragments reused), undoing the filter scale before the sigmoid (Split3Forward.head_fused).
"""

import numpy as np
import torch

from . import ops

# slab order of the activations and the filter parts they meet: l*Wh, h*Wl, h*Wh
W_PARTS = (0, 1, 0)  # index into (Wh, Wl)
WTOP = 12  # filter scale: max |W * 2^t| in (2^11, 2^12]

# (conv scope, channels of its split input (the concat width), output channels)
LAYERS = (("conv1_1", 8, 64), ("conv1_2", 64, 64), ("conv2_1", 64, 128), ("conv2_2", 128, 128),
          ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256), ("conv4_1", 256, 512),
          ("conv4_2", 512, 512), ("conv4_3", 512, 512), ("conv5_1", 512, 512), ("conv5_2", 512, 512),
          ("upconv_1", 512, 512), ("conv4_4", 1024, 512), ("upconv_2", 512, 256), ("conv3_4", 512, 256),
          ("upconv_3", 256, 128), ("conv2_3", 256, 128), ("upconv_4", 128, 64), ("conv1_5", 128, 1))


def filter_scale(w):
    """2^t putting max |w * 2^t| in (2^(WTOP-1), 2^WTOP] (1 for an all-zero filter)."""
    m = float(np.abs(np.asarray(w, np.float64)).max())
    if m == 0.0:
        return 1.0
    return 2.0 ** (WTOP - int(np.ceil(np.log2(m))))


def split2h(w):
    """f32 -> (h, l): h = fp16(w), l = fp16(w - h) (RNE), returned as f32 holding fp16 values exactly."""
    w = torch.as_tensor(w, dtype=torch.float32)
    h = w.half().float()
    lo = (w - h).half().float()
    return h, lo


def split3_filter(w_hwio, cin, cout, t):
    """[3,3,ci,co] filter (f32, or f64 for a folded one), scale 2^t -> the [3,3,3*cin,cout] f32 stack of the fp16 parts
    of w * 2^t in slab order (zero rows past ci, zero columns past co).  Split in float64: h = fp16(w * 2^t), l =
    fp16(w * 2^t - h) (for an f32 w the same parts as in f32, whose difference is exact)."""
    w = torch.from_numpy(np.asarray(w_hwio, np.float64) * float(t))  # exact: a power of two
    ci, co = int(w.shape[2]), int(w.shape[3])
    h = w.half().double()
    parts = (h.float(), (w - h).half().float())
    out = torch.zeros((3, 3, 3 * cin, cout), dtype=torch.float32)
    for p, k in enumerate(W_PARTS):
        out[:, :, p * cin:p * cin + ci, :co] = parts[k]
    return out


# TF-1 legacy bilinear 2x (scale 0.5) as a phase filter: resized row 2i + a blends low-res rows by R[a] (rows: the
# low-res tap u = offset u - 1, columns: the 3x3 kernel row kh), the same table as csrc/conv3x3.hip fold_up2x_weights
_R = np.array([[[.5, 0., 0.], [.5, 1., .5], [0., 0., .5]], [[0., 0., 0.], [1., .5, 0.], [0., .5, 1.]]])


def fold_up2x(w_hwio):
    """conv3x3(resize2x(x), w) = conv3x3(x, W') away from the frame border: W' [3,3,cin,4*cout] (channel p*cout + co =
    phase p = 2a + b of output channel co, pixel (2i + a, 2j + b)), in float64 (vm_conv3x3_fold_up2x_weights rounds it
    to f32; here the fp16 parts are cut from the exact sum)."""
    w = np.asarray(w_hwio, np.float64)
    co = w.shape[3]
    out = np.zeros((3, 3, w.shape[2], 4 * co))
    for p in range(4):
        out[..., p * co:(p + 1) * co] = np.einsum("uk,vl,klio->uvio", _R[p >> 1], _R[p & 1], w)
    return out


# upconvs whose resize is an exact 2x (unet.py:191-200 at 1080p: upconv_2..4; upconv_1's 68 -> 135 is not): with
# Split3Forward.fold_up the resize is folded into the filter (vm_conv3x3_up2x_split3_nhwc), zero phase taps skipped
# (25 of 36), no resized tensor
FOLD = ("upconv_2", "upconv_3", "upconv_4")


def split3h(x, y, pool=None, slab=0, overflow=None):
    """vm_split3h_nhwc: f32 view x -> its [l, h, h] slabs in the fp16 view y (a channel range of a 3*S-wide buffer,
    S = ``slab`` or y's concat width), optionally the split of its 2x2 SAME max-pool into ``pool``; ``overflow`` (a
    device int32) is set to 1 where |x| >= 65520."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    pv = ops.nhwc(pool) if pool is not None else None
    ref = (lambda v: None if v is None else ops.ctypes.byref(v))
    ops.check(ops.lib().vm_split3h_nhwc(ref(xv), ref(yv), ref(pv), int(slab), ops._ptr(overflow),
                                        ops.stream_handle()), "split3h")
    return y


def resize_split3h(x, y, slab=0, overflow=None):
    """vm_resize_split3h_nhwc: TF-1 legacy bilinear resize (unet.py:58) of the f32 view x to y's size, written split
    into the fp16 view y (bit-identical to ops.resize_bilinear + split3h)."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    ops.check(ops.lib().vm_resize_split3h_nhwc(ops.ctypes.byref(xv), ops.ctypes.byref(yv), int(slab),
                                               ops._ptr(overflow), ops.stream_handle()), "resize_split3h")
    return y


def _prof_begin():
    prof = ops._CONV_PROFILE
    if prof is None:
        return None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    return prof, ev0, ev1


def _prof_end(p, x, pc):
    if p is not None:
        prof, ev0, ev1 = p
        ev1.record()
        n, h, w, _ = x.shape
        prof.append((2 * n * h * w * 9 * pc.cin * pc.cout, ops._lib.last_conv_kernel(), ev0, ev1,
                     (n, h, w, pc.cin, pc.cout)))


def conv_f32(x, pc, y, act="relu", splitk=True):
    """The fp16 conv of split input x (a two-slab [l, h] view read as [l, h, h], or a plain fp16 view of pc.cin
    channels) into the f32 view y (vm_conv3x3_ex_nhwc; split-K on small grids)."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    wsz = ops.lib().vm_conv3x3_workspace_bytes(ops.ctypes.byref(xv), pc.cin, pc.cout) if splitk else 0
    ws = ops._workspace(wsz, x.device) if wsz else None
    p = _prof_begin()
    ops.check(ops.lib().vm_conv3x3_ex_nhwc(ops.ctypes.byref(xv), 1, 0, ops._ptr(pc.packed), pc.cin, pc.cout,
                                           ops._ptr(pc.bias), ops._ptr(pc.scale), ops._ptr(pc.shift), ops._lib.ACT[act],
                                           ops.ctypes.byref(yv), ops._ptr(ws), wsz, ops.stream_handle()), "conv3x3(f16)")
    _prof_end(p, x, pc)
    return y


def conv_split(x, pc, y, act="relu", pool=None, overflow=None, y_slab=0, pool_slab=0, splitk=True):
    """vm_conv3x3_split3_nhwc: the fp16 conv of split input x with its output written split into the fp16 view y
    (and the split of its 2x2 SAME max-pool into ``pool``) from the conv's epilogue — no f32 round trip."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    pv = ops.nhwc(pool) if pool is not None else None
    wsz = ops.lib().vm_conv3x3_workspace_bytes(ops.ctypes.byref(xv), pc.cin, pc.cout) if (splitk and pool is None) else 0
    ws = ops._workspace(wsz, x.device) if wsz else None
    ref = (lambda v: None if v is None else ops.ctypes.byref(v))
    p = _prof_begin()
    ops.check(ops.lib().vm_conv3x3_split3_nhwc(
        ref(xv), ops._ptr(pc.packed), pc.cin, pc.cout, ops._ptr(pc.bias), ops._ptr(pc.scale), ops._ptr(pc.shift),
        ops._lib.ACT[act], ref(yv), int(y_slab), ref(pv), int(pool_slab), ops._ptr(overflow), ops._ptr(ws), wsz,
        ops.stream_handle()), "conv3x3_split3")
    _prof_end(p, x, pc)
    return y


def up_split(x, pc_up, pc, y, overflow=None, act="none", y_slab=0):
    """vm_conv3x3_up2x_split3_nhwc: the folded 2x upconv of the low-res split input x ([l, h]) into the full-res split
    view y (pc_up: the folded filter's parts, pc: the plain filter's, for the border pass; same scale)."""
    xv, yv = ops.nhwc(x), ops.nhwc(y)
    p = _prof_begin()
    ops.check(ops.lib().vm_conv3x3_up2x_split3_nhwc(
        ops.ctypes.byref(xv), ops._ptr(pc_up.packed), ops._ptr(pc.packed), pc.cin, pc.cout, ops._ptr(pc.bias),
        ops._ptr(pc.scale), ops._ptr(pc.shift), ops._lib.ACT[act], ops.ctypes.byref(yv), int(y_slab),
        ops._ptr(overflow), ops.stream_handle()), "conv3x3_up2x_split3")
    if p is not None:  # FLOPs of the unfolded conv it stands for (its output pixels)
        prof, ev0, ev1 = p
        ev1.record()
        n, h, w, _ = y.shape
        prof.append((2 * n * h * w * 9 * pc.cin * pc.cout, ops._lib.last_conv_kernel(), ev0, ev1,
                     (n, h, w, pc.cin, pc.cout)))
    return y


def whole(buf):
    """The split-layout view of all channels of a 2*S-wide split buffer [l, h]."""
    return buf[..., :buf.shape[-1] // 2]


def seg(buf, off, c):
    """Channels [off, off + c) of a 2*S-wide split buffer (the writers put the slabs at p*S + off)."""
    return buf[..., off:off + c]


class Split3Forward:
    """The split-fp16 x3 forward of a UNet (unet.UNetVideo / UNetImage) with its parameters."""

    # conv -> split in the conv's epilogue (vm_conv3x3_split3_nhwc); False: f32 output + vm_split3h_nhwc (A/B)
    fuse_split = True
    # the exact-2x upconvs on the folded filter (fuse_split only) — measured slower here (1080p: upconv_2 / _3 / _4
    # 1.49 / 1.06 / 0.92 ms folded with their split border pass, against 0.75 / 0.82 / 0.85 resized; the 12-step split
    # border pass is latency-bound) and ~2x the f32 accumulation error (the 64x96 golden 1.4e-4): off, kept for A/B
    fold_up = False
    # conv1_1's input slab width: 32 (three granules: the l*Wh and h*Wl sums run before h*Wh joins them) or 8 (three
    # slabs + a zero 4th in ONE granule, 0.03 ms faster at 1080p, but every MFMA mixes the small and the large products:
    # the 64x96 golden's alpha 1.01e-4 against 7.8e-5 with 32, fp32 4.1e-5 — tools/x3_golden_study.py)
    first_slab = 32
    # conv1_5 in one MFMA-head call over cat1's [l, h] read as [l, h, h] (12 k-steps, the third range's fragments
    # reused); False: two calls, [l | h] x [Wh | Wl] then [h] x [Wh] adding the first's logits (A/B)
    head_fused = True

    def __init__(self, model):
        self.m = model
        self.dev = model.device
        self.convs = {}
        self.scales = {}
        self.up = {}  # folded upconv filters (FOLD)
        for name, cin, cout in LAYERS:
            w, b = model.params[name]
            t = filter_scale(w)
            self.scales[name] = t
            if name == "conv1_5":
                wf = split3_filter(w, cin, 1, t)
                if self.head_fused:  # [l, h, h] x [Wh, Wl, Wh], descaled + bias in the epilogue
                    self.head = [ops.PackedConv(wf, None, "f16", self.dev, scale=np.full(1, 1.0 / t, np.float32),
                                                shift=np.zeros(1, np.float32) if b is None else b)]
                    self.convs[name] = self.head[0]
                    continue
                # [l | h] against [Wh | Wl] (256 channels), then [h] against [Wh] adding the first chunk's logits
                self.head = [ops.PackedConv(wf[:, :, :256].contiguous(), None, "f16", self.dev),
                             ops.PackedConv(wf[:, :, 256:].contiguous(), None, "f16", self.dev,
                                            scale=np.full(1, 1.0 / t, np.float32),
                                            shift=np.zeros(1, np.float32) if b is None else b)]
                self.convs[name] = self.head[1]
                continue
            cp = cin
            if name == "conv1_1":
                cp = self.first_slab  # slab width (7 or 6 live channels): see first_slab
            if name in FOLD:  # one scale for the folded filter and the plain one (its border pass)
                wu = fold_up2x(w)
                t = min(t, filter_scale(wu))  # max |W' * 2^t| and max |W * 2^t| both <= 2^12
                self.scales[name] = t
                self.up[name] = ops.PackedConv(split3_filter(wu, cin, 4 * cout, t), None, "f16", self.dev,
                                               scale=np.full(cout, 1.0 / t, np.float32),
                                               shift=np.zeros(cout, np.float32))
            wf = split3_filter(w, cp, cout, t)
            if name == "conv1_1" and cp == 8:
                wf = torch.cat([wf, torch.zeros((3, 3, 8, cout))], 2)
            # epilogue (acc * 2^-t) + b: exact descale, then the bias (unet.py:41,73)
            self.convs[name] = ops.PackedConv(wf, None, "f16", self.dev, scale=np.full(cout, 1.0 / t, np.float32),
                                              shift=np.zeros(cout, np.float32) if b is None else b)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._b, self._key = None, None
        self.logits = None

    def weights_flat(self):
        out = []
        for pc in [self.convs[k] for k in sorted(self.convs) if k != "conv1_5"] + self.head + [self.up[k] for k in
                                                                                             sorted(self.up)]:
            out.append(pc.packed)
            for t in (pc.bias, pc.scale, pc.shift):
                if t is not None:
                    out.append(t)
        return out

    def _buffers(self, n, h, w):
        if self._key == (n, h, w):
            return self._b
        from .unet import _levels
        L = _levels(h, w)
        dev = self.dev
        S = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], 2 * c), dtype=torch.float16, device=dev)  # noqa
        F = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], c), dtype=torch.float32, device=dev)  # noqa
        fs = self.first_slab
        # (slab 8: [l, h, h] + a zero 4th slab in one granule; wider: the two stored slabs [l, h], read as [l, h, h])
        b = {"x": torch.zeros((n, L[0][0], L[0][1], 32 if fs == 8 else 2 * fs), dtype=torch.float16, device=dev),
             "s11": S(0, 64), "cat1": S(0, 128), "r4": S(0, 128),
             "p1": S(1, 64), "s21": S(1, 128), "cat2": S(1, 256), "r3": S(1, 256),
             "p2": S(2, 128), "s31": S(2, 256), "s32": S(2, 256), "cat3": S(2, 512), "r2": S(2, 512),
             "p3": S(3, 256), "s41": S(3, 512), "s42": S(3, 512), "cat4": S(3, 1024), "r1": S(3, 512),
             "p4": S(4, 512), "s51": S(4, 512),
             "c44s": S(3, 512), "c34s": S(2, 256), "c23s": S(1, 128),  # the folded upconvs' low-res inputs
             "f0": F(0, 128), "f1": F(1, 256), "f2": F(2, 512), "f3": F(3, 512), "f4": F(4, 512),
             "lg0": F(0, 1), "out": F(0, 1)}
        self._b, self._key = b, (n, h, w)
        return b

    def overflowed(self):
        """True when a split of the last forward(s) since reset met |x| >= 65520 (synchronises)."""
        return bool(self.overflow.item())

    def forward(self, x, out=None):
        """x: [N,H,W,C] f32 frames (C = 7 video / 6 image) -> alpha [N,H,W,1] f32 (``out`` if given)."""
        from .unet import _levels
        n, h, w, c = x.shape
        b = self._buffers(n, h, w)
        L = _levels(h, w)
        C = self.convs
        ovf = self.overflow
        ovf.zero_()
        fs = self.first_slab
        # channels 0..7 of each slab (the frame's 7 or 6 and zeros); the rest of the slabs stay zero from allocation
        split3h(x, b["x"][..., :8], slab=fs, overflow=ovf)

        def conv(src, name, dst_f32, act="relu", splitk=True):
            return conv_f32(src, C[name], dst_f32, act, splitk)

        def sp(f, y, pool=None):
            return split3h(f, y, pool, overflow=ovf)

        def cs(src, name, dst_f32, y, pool=None, act="relu"):
            """conv -> split (-> pool split): fused, or the f32 round trip"""
            if self.fuse_split:
                return conv_split(src, C[name], y, act, pool, ovf)
            # (no split-K under a pool, as the fused form: the same sums, bit for bit)
            return sp(conv(src, name, dst_f32, act, splitk=pool is None), y, pool)

        def resize_split(f_src, lv, r_split):
            if self.fuse_split:  # the resize written split, no f32 resized tensor
                return resize_split3h(f_src, r_split, overflow=ovf)
            rr = torch.empty((n, L[lv][0], L[lv][1], f_src.shape[-1]), dtype=torch.float32, device=x.device)
            ops.resize_bilinear(f_src, L[lv], out=rr)
            sp(rr, r_split)

        f0, f1, f2, f3, f4 = b["f0"], b["f1"], b["f2"], b["f3"], b["f4"]
        # encoder (unet.py:170-189)
        cs(b["x"], "conv1_1", f0[..., :64], whole(b["s11"]))
        cs(b["s11"], "conv1_2", f0[..., :64], seg(b["cat1"], 64, 64), pool=whole(b["p1"]))
        cs(b["p1"], "conv2_1", f1[..., :128], whole(b["s21"]))
        cs(b["s21"], "conv2_2", f1[..., :128], seg(b["cat2"], 128, 128), pool=whole(b["p2"]))
        cs(b["p2"], "conv3_1", f2[..., :256], whole(b["s31"]))
        cs(b["s31"], "conv3_2", f2[..., :256], whole(b["s32"]))
        cs(b["s32"], "conv3_3", f2[..., :256], seg(b["cat3"], 256, 256), pool=whole(b["p3"]))
        cs(b["p3"], "conv4_1", f3, whole(b["s41"]))
        cs(b["s41"], "conv4_2", f3, whole(b["s42"]))
        cs(b["s42"], "conv4_3", f3, seg(b["cat4"], 512, 512), pool=whole(b["p4"]))
        cs(b["p4"], "conv5_1", f4, whole(b["s51"]))
        y52 = conv(b["s51"], "conv5_2", f4)
        # decoder: resize (f32) -> split -> conv (no bias, no relu) into the concat's up range (unet.py:191-200)
        resize_split(y52, 3, whole(b["r1"]))
        cs(b["r1"], "upconv_1", f3, seg(b["cat4"], 0, 512), act="none")
        fold = self.fold_up and self.fuse_split

        def level(src_cat, conv_name, f_dst, s_name, lv, r_name, up_name, up_f32, y):
            """conv (relu) over the concat -> upconv (no bias, no relu) into the next concat's up range: the folded
            2x upconv on its split low-res output where the resize is an exact 2x, else f32 -> resize -> split ->
            conv (unet.py:192-200)"""
            if fold and L[lv] == (2 * L[lv + 1][0], 2 * L[lv + 1][1]):
                cs(b[src_cat], conv_name, f_dst, whole(b[s_name]))
                up_split(b[s_name], self.up[up_name], C[up_name], y, ovf)
            else:
                f = conv(b[src_cat], conv_name, f_dst)
                resize_split(f, lv, whole(b[r_name]))
                cs(b[r_name], up_name, up_f32, y, act="none")

        level("cat4", "conv4_4", f3, "c44s", 2, "r2", "upconv_2", f2[..., :256], seg(b["cat3"], 0, 256))
        level("cat3", "conv3_4", f2[..., :256], "c34s", 1, "r3", "upconv_3", f1[..., :128], seg(b["cat2"], 0, 128))
        level("cat2", "conv2_3", f1[..., :128], "c23s", 0, "r4", "upconv_4", f0[..., :64], seg(b["cat1"], 0, 64))
        # conv1_5 + sigmoid (unet.py:203-205): [l | h] x [Wh | Wl], then [h] x [Wh] + those logits, * 2^-t + bias
        alpha = b["out"] if out is None else out
        lg0 = b["lg0"]
        logits = f0[..., :1]
        chunks = (((b["cat1"], logits, None),) if self.head_fused else
                  ((b["cat1"], lg0, None), (b["cat1"][..., 128:], logits, lg0)))
        for k, (xs, yv, acc) in enumerate(chunks):
            pc = self.head[k]
            xv, yvv = ops.nhwc(xs), ops.nhwc(yv)
            ops.check(ops.lib().vm_conv3x3_head_acc_ex_nhwc(
                ops.ctypes.byref(xv), ops._ptr(pc.packed), pc.cin, None, ops._ptr(pc.scale),
                ops._ptr(pc.shift), ops._ptr(acc), ops.ctypes.byref(yvv),
                ops._ptr(alpha if k == len(chunks) - 1 else None), ops.stream_handle()), "conv3x3_head_acc_ex")
        self.logits = logits
        return alpha
