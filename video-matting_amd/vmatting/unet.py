"""U-Net encoder-decoder (reference unet.py) on gfx950 kernels.

Same construction API as the reference: ``UNetVideo(vgg16_npy_path).build(input)``
sets ``.output`` (sigmoid alpha) and every intermediate attribute the reference
sets (conv1_1 ... conv5_2, pool1..4, upconv1..4, conv4_4, conv3_4, conv2_3,
conv1_3) — unet.py:86-217.  ``input`` is an NHWC [N,H,W,7] (video) / [N,H,W,6]
(image) float32 frame batch (cmp-VGG_MEAN, bg-VGG_MEAN[, trimap-0.5]); numpy
arrays are uploaded.  Because the reference's build() only wires a graph that
sess.run evaluates later, the GPU version also offers ``forward(x)`` to evaluate
the built network again on new frames with the same weights and buffers.

Data layout in HBM (compute dtype T = bf16 or f32, NHWC, channels innermost):
  in8   [N,H,W,8]      the 7-ch frame padded to 8 channels (16-byte pixel rows)
  cat1  [N,H,W,128]    [upconv_4 conv | conv1_2]  = the reference's upconv4 concat
  cat2  [N,H/2,W/2,256], cat3 [..,512], cat4 [..,1024]: the same for levels 2..4
so every tf.concat (unet.py:62) is a pair of channel-slice writes, never a copy.
"""

import weakref

import numpy as np
import torch

from . import ops
from .weights import init_conv, load_vgg16

# fresh convs in graph-build order (unet.py:191-203): scope, cin, cout, keeps bias
NEW_CONVS = (("upconv_1", 512, 512, False), ("conv4_4", 1024, 512, True),
             ("upconv_2", 512, 256, False), ("conv3_4", 512, 256, True),
             ("upconv_3", 256, 128, False), ("conv2_3", 256, 128, True),
             ("upconv_4", 128, 64, False), ("conv1_5", 128, 1, True))

VGG_USED = ("conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3",
            "conv4_1", "conv4_2", "conv4_3", "conv5_1", "conv5_2")


def _levels(h, w):
    lv = [(h, w)]
    for _ in range(4):
        lv.append(((lv[-1][0] + 1) // 2, (lv[-1][1] + 1) // 2))  # SAME 2x2/2 pool: ceil
    return lv


class _LazyBuffers(dict):
    """Buffer dict whose listed entries are allocated on first access."""

    def __init__(self, lazy, make):
        super().__init__()
        self._lazy, self._make = lazy, make

    def __missing__(self, key):
        if key not in self._lazy:
            raise KeyError(key)
        t = self._make(*self._lazy[key])
        self[key] = t
        return t


class UNet:
    """Base class (unet.py:20-83)."""

    IN_CH = None
    # upconvs whose exact-2x resize is folded into the conv (ops.upconv3x3; bf16 only, others resize + conv)
    # conv1_1 -> conv1_2 as one kernel (ops.conv_pair_first; bf16 only, others run them separately)
    fuse_first = True
    # head split (bf16 + fuse_first): the pair kernel takes conv1_5's share of the skip half of cat1 in its epilogue
    # (vm_conv3x3_pair_first_head_nhwc), so conv1_2's 64-channel output never reaches HBM and the head reads only
    # the upconv_4 half; .conv1_2 / .upconv4 are then evaluated on first access
    split_head = True
    # upconv_2 too since its odd phases skip their zero taps (same-box A/B: -0.5 % on the whole forward vs resize +
    # conv on the rows kernel; without the skip, folding it was slower)
    fold_upconv = ("upconv_2", "upconv_3", "upconv_4")
    # with the head split, upconv_4 takes conv1_5's shares of its own half of cat1 in its epilogue too
    # (vm_conv3x3_up2x_head_nhwc): cat1 never reaches HBM and the head only sums the two partial sets
    fuse_up_head = True

    def __init__(self, vgg16_npy_path=None, dtype="bf16", device="cuda"):
        self.data_dict = load_vgg16(vgg16_npy_path)
        # split-operand paths at f32 accuracy on the 16-bit MFMA kernels: "bf16x6" (vmatting/split6.py, six bf16
        # products per conv) and "f16x3" (vmatting/split3.py, three fp16 products per conv)
        self.split_mode = dtype if dtype in ("bf16x6", "f16x3") else None
        self.x6mode = self.split_mode is not None
        self._x6 = None
        self.dtype = ({"bf16x6": torch.bfloat16, "f16x3": torch.float16}[dtype] if self.x6mode else
                      (ops.TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype))
        self.device = torch.device(device)
        self.params = None       # name -> (w_hwio f32 np, bias f32 np | None)
        self.convs = None        # name -> ops.PackedConv
        self._ws = None
        self._ws_key = None
        self._ws_all = weakref.WeakValueDictionary()  # (n,h,w) -> buffer set, while something holds it
        self._c11 = None
        self._x = None
        self._in8_valid = False
        self._skip_valid = True
        self._head_up = None     # split head: (conv1_5 HWIO f32 on the device, PackedConv of its upconv_4 half)
        self._up_valid = True    # cat1's upconv_4 half holds this forward's values (False: head split kept it on chip)

    # ------------------------------------------------------------------ weights
    def get_conv_filter(self, name):
        raise NotImplementedError

    def _make_params(self):
        """VGG filters from data_dict (unet.py:65-77, 150-157/210-217) and init_conv draws in build order."""
        p = {}
        for name in VGG_USED:
            p[name] = (self.get_conv_filter(name), np.asarray(self.data_dict[name][1], np.float32))
        for name, cin, cout, keep_bias in NEW_CONVS:
            w, b = init_conv(cin, cout)
            p[name] = (w, b if keep_bias else None)
        return p

    def load_params(self, params):
        """Install explicit weights {scope: (w_hwio, bias|None)} (e.g. from a checkpoint)."""
        self.params = {k: (np.asarray(w, np.float32), None if b is None else np.asarray(b, np.float32))
                       for k, (w, b) in params.items()}
        self.convs = None
        return self

    def prepare(self):
        """Create (first call) and pack the weights without running a frame, e.g. before an RCCL broadcast."""
        if self.params is None:
            self.params = self._make_params()
        if self.convs is None:
            self._pack()
        return self

    def _pack(self):
        if self.x6mode:
            if self.split_mode == "f16x3":
                from .split3 import Split3Forward
                self._x6 = Split3Forward(self)
            else:
                from .split6 import Split6Forward
                self._x6 = Split6Forward(self)
            self.convs = self._x6.convs
            self._head_up = None
            return
        self.convs = {k: ops.PackedConv(w, b, self.dtype, self.device) for k, (w, b) in self.params.items()}
        self._head_up = None
        if self._lean():
            w, b = self.params["conv1_5"]
            self._head_up = (torch.as_tensor(np.ascontiguousarray(w, np.float32)).to(self.device),
                             ops.PackedConv(np.ascontiguousarray(w[:, :, :64, :]), b, self.dtype, self.device))

    def _lean(self):
        return not self.x6mode and self.split_head and self.fuse_first and self.dtype == torch.bfloat16

    def weights_flat(self):
        """All packed weights as one list of tensors (for an RCCL broadcast from rank 0)."""
        if self._x6 is not None:
            return self._x6.weights_flat()
        out = []
        for k in sorted(self.convs):
            pc = self.convs[k]
            out.append(pc.packed)
            if k in self.fold_upconv and pc.up2x() is not None:
                out.append(pc.up2x())
            if pc.bias is not None:
                out.append(pc.bias)
        if self._head_up is not None:
            out += [self._head_up[0], self._head_up[1].packed, self._head_up[1].bias]
        return out

    # ------------------------------------------------------------------ buffers
    def _buffers(self, n, h, w):
        """Activation buffers for an [n,h,w] batch.  The model holds the current shape's set; a HIP graph captured
        on a set holds that one (GraphedForward), e.g. video.py's full chunks and its shorter last chunk.  A set
        nobody holds any more is freed, so a model that sees many frame sizes does not accumulate buffers."""
        key = (n, h, w)
        if self._ws_key == key:
            return self._ws
        if key in self._ws_all:
            self._ws, self._ws_key = self._ws_all[key], key
            return self._ws
        T, dev = self.dtype, self.device
        L = _levels(h, w)
        E = lambda lv, c, dt=T: torch.empty((n, L[lv][0], L[lv][1], c), dtype=dt, device=dev)  # noqa: E731
        # in8 / c11 (unfused first pair, the lazily evaluated .conv1_1) and the resize targets r1..r4 (unfolded
        # upconvs) are allocated on first use only: the bf16 fused/folded forward never touches in8, c11, r3, r4
        ws = _LazyBuffers(dict(in8=(0, 8), c11=(0, 64), r4=(0, 128), r3=(1, 256), r2=(2, 512), r1=(3, 512),
                               hpart=(0, 12, torch.float32), upart=(0, 12, torch.float32)), E)
        ws.update(
            cat1=E(0, 128),
            p1=E(1, 64), c21=E(1, 128), cat2=E(1, 256), c23=E(1, 128),
            p2=E(2, 128), c31=E(2, 256), c32=E(2, 256), cat3=E(2, 512), c34=E(2, 256),
            p3=E(3, 256), c41=E(3, 512), c42=E(3, 512), cat4=E(3, 1024), c44=E(3, 512),
            p4=E(4, 512), c51=E(4, 512), c52=E(4, 512),
            logits=E(0, 1, torch.float32), out=E(0, 1, torch.float32))
        self._ws, self._ws_key = ws, key
        self._ws_all[key] = ws
        return ws

    # ------------------------------------------------------------------ graph
    def build(self, input):
        """unet.UNet*.build (unet.py:87-148 / 161-208): create weights (first call), run, set attributes."""
        x = self._as_input(input)
        self.prepare()
        self.forward(x)
        if self.split_mode == "f16x3" and self._x6.overflowed():
            # an activation left fp16's range (|x| >= 65520): these frames take the bf16x6 path (f32 range)
            from .split6 import Split6Forward
            self.split_mode, self.dtype = "bf16x6", torch.bfloat16
            self._x6 = Split6Forward(self)
            self.convs = self._x6.convs
            self.forward(x)
        self.data_dict = None  # unet.py:147,207
        return self.output

    def overflowed(self):
        """f16x3: whether a split since the last forward began met |x| >= 65520 (its alpha is then invalid and the
        frames belong on the bf16x6 path); synchronises.  False on the other paths."""
        return self.split_mode == "f16x3" and self._x6 is not None and self._x6.overflowed()

    def _as_input(self, input):
        x = input if isinstance(input, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(input, np.float32))
        x = x.to(self.device, torch.float32)
        if x.dim() != 4 or x.shape[-1] != self.IN_CH:
            raise ValueError("%s.build expects [N,H,W,%d] input, got %s" % (type(self).__name__, self.IN_CH,
                                                                            tuple(x.shape)))
        return x

    def forward(self, input, out=None):
        """Evaluate the built network on new frames; returns .output (f32 [N,H,W,1]).  ``out`` (contiguous f32
        [N,H,W,1] on the device) receives the alpha instead of the model's own buffer (video.py writes each chunk
        of frames straight into its slice of the result)."""
        x = self._as_input(input) if not (isinstance(input, torch.Tensor) and input.is_cuda and
                                          input.dtype == torch.float32) else input
        if self.convs is None:
            raise RuntimeError("call build() first")
        if self._x6 is not None:  # split paths (bf16x6 / f16x3): only .output and .conv1_3 (the logits) are kept
            alpha = self._x6.forward(x, out)
            self._x, self._ws, self._ws_key = x, self._x6._b, self._x6._key
            self.conv1_3, self.output = self._x6.logits, alpha
            return alpha
        n, h, w, c = x.shape
        b = self._buffers(n, h, w)
        L = _levels(h, w)
        C = self.convs
        lean = self._lean() and self._head_up is not None
        # conv1_1 and conv1_2 stay on chip: only pool1 and the head's per-tap shares of conv1_2 leave the kernel
        lean = lean and ops.conv_pair_first_head(x, C["conv1_1"], C["conv1_2"], self._head_up[0], 64, b["hpart"],
                                                 "relu", out=b["cat1"][..., 64:], pool_out=b["p1"], store_y=False,
                                                 fallback=True) is not None
        self._skip_valid = not lean
        if lean:
            self._c11 = None
            self._in8_valid = False
        elif self.fuse_first and self.dtype == torch.bfloat16:
            # conv1_1 stays on chip and reads the f32 frame itself (bf16 rounding on load); .conv1_1 is evaluated
            # on first access
            ops.conv_pair_first(x, C["conv1_1"], C["conv1_2"], "relu", out=b["cat1"][..., 64:], pool_out=b["p1"])
            self._c11 = None
            self._in8_valid = False
        else:
            ops.convert(x, b["in8"])
            xin = b["in8"][..., :c]
            self._in8_valid = True
            self._c11 = ops.conv3x3(xin, C["conv1_1"], "relu", out=b["c11"])
            ops.conv3x3(b["c11"], C["conv1_2"], "relu", out=b["cat1"][..., 64:], pool_out=b["p1"])
        self._x = x
        ops.conv3x3(b["p1"], C["conv2_1"], "relu", out=b["c21"])
        ops.conv3x3(b["c21"], C["conv2_2"], "relu", out=b["cat2"][..., 128:], pool_out=b["p2"])
        ops.conv3x3(b["p2"], C["conv3_1"], "relu", out=b["c31"])
        ops.conv3x3(b["c31"], C["conv3_2"], "relu", out=b["c32"])
        ops.conv3x3(b["c32"], C["conv3_3"], "relu", out=b["cat3"][..., 256:], pool_out=b["p3"])
        ops.conv3x3(b["p3"], C["conv4_1"], "relu", out=b["c41"])
        ops.conv3x3(b["c41"], C["conv4_2"], "relu", out=b["c42"])
        ops.conv3x3(b["c42"], C["conv4_3"], "relu", out=b["cat4"][..., 512:], pool_out=b["p4"])
        ops.conv3x3(b["p4"], C["conv5_1"], "relu", out=b["c51"])
        ops.conv3x3(b["c51"], C["conv5_2"], "relu", out=b["c52"])
        # decoder: upconv_concat = resize -> conv (no bias, no relu) -> [up, skip] (unet.py:44-63)
        up = lambda src, scope, lv, out, rkey: ops.upconv3x3(  # noqa: E731
            src, C[scope], "none", out=out, size=L[lv], rbuf=b[rkey], fold=scope in self.fold_upconv)
        up(b["c52"], "upconv_1", 3, b["cat4"][..., :512], "r1")
        ops.conv3x3(b["cat4"], C["conv4_4"], "relu", out=b["c44"])
        up(b["c44"], "upconv_2", 2, b["cat3"][..., :256], "r2")
        ops.conv3x3(b["cat3"], C["conv3_4"], "relu", out=b["c34"])
        up(b["c34"], "upconv_3", 1, b["cat2"][..., :128], "r3")
        ops.conv3x3(b["cat2"], C["conv2_3"], "relu", out=b["c23"])
        alpha = b["out"] if out is None else out
        # lean: upconv_4 takes conv1_5's shares of its own half of cat1 in its epilogue too, so neither half of cat1
        # reaches HBM and the head only sums the two partial sets (.upconv4 is evaluated on first access)
        self._up_valid = not (lean and self.fuse_up_head and "upconv_4" in self.fold_upconv and ops.upconv3x3_head(
            b["c23"], C["upconv_4"], self._head_up[0], 0, b["upart"], "none", out=b["cat1"][..., :64],
            store_y=False) is not None)
        if self._up_valid:
            up(b["c23"], "upconv_4", 0, b["cat1"][..., :64], "r4")
        if lean and not self._up_valid:
            ops.head_from_partials(b["upart"], b["hpart"], self._head_up[1].bias, logits=b["logits"], alpha=alpha)
        elif lean:  # conv1_5 + sigmoid over the upconv_4 half + the pair kernel's shares of the conv1_2 half
            ops.conv_head(b["cat1"][..., :64], self._head_up[1], "none", out=b["logits"], alpha=alpha,
                          partial=b["hpart"])
        else:
            ops.conv_head(b["cat1"], C["conv1_5"], "none", out=b["logits"], alpha=alpha)  # conv1_5 + sigmoid
        self._publish(b)
        self.output = alpha
        return self.output

    def capture(self, x, static=False, out=None):
        """Record one forward over frames shaped like ``x`` into a HIP graph (torch.cuda.CUDAGraph over the same
        C-ABI launches) and return a GraphedForward: replaying it re-runs the whole forward with one host call, so
        throughput no longer depends on the host's per-launch cost.  New frames are copied into ``.input``;
        ``static=True`` records ``x`` itself as the input (no copy; x must stay allocated and in place) and ``out``
        the alpha destination."""
        return GraphedForward(self, x, static, out)

    @property
    def conv1_1(self):
        """unet.py:170 conv1_1 — with fuse_first the forward never writes it to HBM, so it is evaluated here."""
        if self._c11 is None and self._ws is not None:
            if not self._in8_valid:
                ops.convert(self._x, self._ws["in8"])
                self._in8_valid = True
            xin = self._ws["in8"][..., :self.IN_CH]
            self._c11 = ops.conv3x3(xin, self.convs["conv1_1"], "relu", out=self._ws["c11"])
        return self._c11

    @property
    def conv1_2(self):
        """unet.py:171 conv1_2 — with the head split the forward never writes it to HBM, so it is evaluated here
        (conv1_1 -> conv1_2 unfused: bit-identical to the pair kernel's values)."""
        if self._ws is None:
            return None
        if not self._skip_valid:
            ops.conv3x3(self.conv1_1, self.convs["conv1_2"], "relu", out=self._ws["cat1"][..., 64:])
            self._skip_valid = True
        return self._ws["cat1"][..., 64:]

    @property
    def upconv4(self):
        """unet.py:200 upconv4 = concat([upconv_4, conv1_2]) (either half evaluated on first access when the head
        split kept it on chip; bit-identical to the forward's values)."""
        if self.conv1_2 is None:
            return None
        if not self._up_valid:
            L = _levels(self._ws_key[1], self._ws_key[2])
            ops.upconv3x3(self._ws["c23"], self.convs["upconv_4"], "none", out=self._ws["cat1"][..., :64], size=L[0],
                          rbuf=self._ws["r4"], fold="upconv_4" in self.fold_upconv)
            self._up_valid = True
        return self._ws["cat1"]

    def _publish(self, b):
        self.pool1 = b["p1"]
        self.conv2_1 = b["c21"]
        self.conv2_2 = b["cat2"][..., 128:]
        self.pool2 = b["p2"]
        self.conv3_1, self.conv3_2 = b["c31"], b["c32"]
        self.conv3_3 = b["cat3"][..., 256:]
        self.pool3 = b["p3"]
        self.conv4_1, self.conv4_2 = b["c41"], b["c42"]
        self.conv4_3 = b["cat4"][..., 512:]
        self.pool4 = b["p4"]
        self.conv5_1, self.conv5_2 = b["c51"], b["c52"]
        self.upconv1, self.conv4_4 = b["cat4"], b["c44"]
        self.upconv2, self.conv3_4 = b["cat3"], b["c34"]
        self.upconv3, self.conv2_3 = b["cat2"], b["c23"]
        self.conv1_3 = b["logits"]  # scope 'conv1_5' (unet.py:143/203)
        self.output = b["out"]

    # FLOPs of the 20 convs for an [n,h,w] batch (2 * sum H*W*9*Cin*Cout) — the roofline numerator
    def conv_flops(self, n, h, w):
        L = _levels(h, w)
        lv = {"conv1_1": 0, "conv1_2": 0, "conv2_1": 1, "conv2_2": 1, "conv3_1": 2, "conv3_2": 2, "conv3_3": 2,
              "conv4_1": 3, "conv4_2": 3, "conv4_3": 3, "conv5_1": 4, "conv5_2": 4, "upconv_1": 3, "conv4_4": 3,
              "upconv_2": 2, "conv3_4": 2, "upconv_3": 1, "conv2_3": 1, "upconv_4": 0, "conv1_5": 0}
        tot = 0
        for k, (wt, _) in self.params.items():
            hh, ww = L[lv[k]]
            cin = self.IN_CH if k == "conv1_1" else wt.shape[2]
            tot += 2 * n * hh * ww * 9 * cin * wt.shape[3]
        return tot


class UNetImage(UNet):
    """unet.UNetImage (unet.py:86-157): 6-channel input, conv1_1 = [VGG/2, VGG/2]."""

    IN_CH = 6

    def get_conv_filter(self, name):
        w = np.asarray(self.data_dict[name][0], np.float32)
        if name == "conv1_1":
            t = np.zeros((3, 3, 6, 64), dtype=np.float32)
            t[:, :, :3, :] = w / 2.0
            t[:, :, 3:6, :] = w / 2.0
            return t
        return w


class UNetVideo(UNet):
    """unet.UNetVideo (unet.py:160-217): 7-channel input (cmp, bg, trimap), conv1_1 = [VGG, VGG, 0]."""

    IN_CH = 7

    def get_conv_filter(self, name):
        w = np.asarray(self.data_dict[name][0], np.float32)
        if name == "conv1_1":
            t = np.zeros((3, 3, 7, 64), dtype=np.float32)
            t[:, :, :3, :] = w
            t[:, :, 3:6, :] = w
            return t
        return w


class GraphedForward:
    """A UNet forward captured once into a HIP graph (see UNet.capture).

    ``input`` is the static frame buffer the graph reads ([N,H,W,C] f32 on the device) and ``output`` the static
    alpha buffer it writes; ``replay()`` launches the graph on the current stream, ``__call__(frames)`` copies frames
    in first.  The model's weights and activation buffers are the ones captured: do not change the model's shape or
    weights afterwards (capture again instead)."""

    def __init__(self, model, x, static=False, out=None):
        x = model._as_input(x)
        self.model = model
        if static:
            self.input = x
        else:
            self.input = torch.empty_like(x)
            self.input.copy_(x)
        side = torch.cuda.Stream(device=self.input.device)
        side.wait_stream(torch.cuda.current_stream(self.input.device))
        with torch.cuda.stream(side):  # lazily built kernels/weights (folded filters, attributes) before capture
            model.forward(self.input, out)
        main = torch.cuda.current_stream(self.input.device)
        main.wait_stream(side)
        torch.cuda.synchronize(self.input.device)
        # the buffer set (and any lazily allocated entry) was allocated on the side stream but the graph replays on
        # the caller's: tell the caching allocator, so a set freed later (the model moved to another shape and this
        # graph was dropped) is not handed out again while replays queued on that stream may still use it
        for t in model._ws.values():
            t.record_stream(main)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.output = model.forward(self.input, out)
        # the buffer set the graph writes stays alive with the graph; so does the forward's host-side state
        self._ws, self._ws_key = model._ws, model._ws_key
        self._skip_valid = model._skip_valid
        self._up_valid = model._up_valid
        self._logits = model.conv1_3 if model._x6 is not None else None

    def replay(self):
        self.graph.replay()
        m = self.model
        if m._ws is not self._ws:  # the model ran another shape since: its attributes follow this replay
            m._ws, m._ws_key = self._ws, self._ws_key
            if m._x6 is None:
                m._publish(self._ws)
        if m._x6 is not None:
            m.conv1_3 = self._logits
        m._x, m._c11, m._in8_valid, m._skip_valid = self.input, None, False, self._skip_valid
        m._up_valid = self._up_valid
        m.output = self.output
        return self.output

    def __call__(self, frames):
        self.input.copy_(self.model._as_input(frames))
        return self.replay()
