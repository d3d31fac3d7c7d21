"""small_train.py's training step on gfx950 kernels: one iteration of ``small_training`` (small_train.py:34-88).

``SmallTrainer.step(cmp, bg, gt, raw_fg)`` is one ``sess.run([train_merged, train_op], feed_dict)`` of the reference
(small_train.py:72-74) with the graph ``train(learning_rate=1e-5)`` builds (small_train.py:91-112):

  input     concat(cmp, bg) (small_train.py:95), 6 channels
  forward   small.UNetSmall(input, phase=True) (small.py:37-50): conv + bias -> batch_norm(is_training) -> relu,
            SAME 2x2 max-pools, upconv_concat's resize -> conv (no bias) -> relu -> concat [skip, up] -> BN
  loss      mean(0.5*regular_l1(pred, gt) + 0.5*regular_l1(composite(raw_fg, bg, pred), cmp))
            (small_train.py:39-44; the summary scalars [loss, alpha_loss, cmp_loss] are returned)
  backward  through EVERY variable (small_train.py:47-48: AdamOptimizer.minimize with the default var_list — no frozen
            towers here): BN backward with the relu masks, the max-pool adjoint (the window's gradient to its first
            maximum, TF's MaxPoolGrad), the skip concat's gradient added to the pool path's, the TF-1 resize adjoint,
            conv weight gradients down to the 6-channel first layer and data gradients down to its output.  The
            upconvs' drawn biases (small.py:18) feed nothing and get no gradient, so Adam skips them; here they are
            not parameters
  exchange  DDP: one all-reduce of the flat gradient buffer; optional SyncBN (the reference's single-device batch)
  update    tf.train.AdamOptimizer(lr, 0.9, 0.999, 1e-8) over the flat buffer in one launch, then re-packs

The moving BN statistics are never updated, as in the reference (UPDATE_OPS is not wired, small_train.py:48).
"""

import numpy as np
import torch

from . import ops, parallel
from .layers import EPS
from .small import NEW_CONVS
from .train import TrainerBase
from .weights import init_conv

# batch-norm width per scope: new_conv's cout, upconv_concat's concat (small.py:20-22)
BN_WIDTH = {"upconv1": 32, "upconv2": 16}
# convs whose input carries a gradient (all but conv1_1, whose input is the network input)
DGRAD = ("conv1_3", "conv1_2", "upconv2", "conv2_2", "upconv1", "conv3_2", "conv3_1", "conv2_1")


def _levels(h, w):
    h2, w2 = (h + 1) // 2, (w + 1) // 2
    return [(h, w), (h2, w2), ((h2 + 1) // 2, (w2 + 1) // 2)]


def param_layout(cin=6):
    """Flat f32 layout of UNetSmall's trainable variables in TF creation order (small.py:39-49): per scope the
    filter, the bias (new_conv only), bn/beta, bn/gamma.  -> ([(scope, kind, offset, shape)], total)"""
    out, off = [], 0
    for name, ci, co in NEW_CONVS:
        ents = [("w", (3, 3, cin if ci is None else ci, co))]
        if not name.startswith("upconv"):
            ents.append(("b", (co,)))
        c = BN_WIDTH.get(name, co)
        ents += [("beta", (c,)), ("gamma", (c,))]
        for kind, shape in ents:
            out.append((name, kind, off, shape))
            off += int(np.prod(shape))
    return out, off


class SmallTrainer(TrainerBase):
    """small_train.small_training's iteration on device (small.UNetSmall, all variables trainable)."""

    def __init__(self, cin=6, dtype="fp32", device="cuda", params=None, bn=None, lr=1e-5, beta1=0.9, beta2=0.999,
                 epsilon=1e-8, sync_bn=False):
        self.dtype = ops.TORCH_DTYPE[dtype] if isinstance(dtype, str) else dtype
        self.device = torch.device(device)
        self.cin = int(cin)
        layout, n = param_layout(self.cin)
        self._init_flat(layout, n, lr, beta1, beta2, epsilon, sync_bn)
        if params is None:  # init_conv draws in build order from the global numpy RNG (small.py:5-10)
            params = {}
            for name, ci, co in NEW_CONVS:
                w, b = init_conv(self.cin if ci is None else ci, co)
                params[name] = (w, None if name.startswith("upconv") else b)
        f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32))  # noqa: E731
        for name, _, co in NEW_CONVS:
            w, b = params[name]
            self.P[name, "w"].copy_(f(w))
            if (name, "b") in self.P:
                self.P[name, "b"].copy_(f(b))
            c = BN_WIDTH.get(name, co)
            g, be = (np.ones(c), np.zeros(c)) if bn is None or name not in bn else bn[name]
            self.P[name, "gamma"].copy_(f(g))
            self.P[name, "beta"].copy_(f(be))
        if parallel.world_size() > 1:  # every replica starts from rank 0's draws
            parallel.broadcast_tensors([self.flat], src=0)
        bf16 = self.dtype == torch.bfloat16
        # forward packs, aliased onto the flat buffer (PackedConv.from_source re-reads it at every re-pack); bf16:
        # the cout-1 head on an 8-channel zero-padded pack (the MFMA kernels' f32 epilogue writes >= 8 channels)
        self.convs, self._pad = {}, {}
        for name, ci, co in NEW_CONVS:
            w = self.P[name, "w"]
            bias = self.P.get((name, "b"))
            if bf16 and co % 8:
                bp = torch.zeros(8, dtype=torch.float32, device=self.device)
                self.convs[name] = ops.PackedConv.from_source(w, w.shape[2], 8, self.dtype, bias=bp)
                self._pad[name] = (bp, co)
            else:
                self.convs[name] = ops.PackedConv.from_source(w, w.shape[2], co, self.dtype, bias=bias)
        self._refresh_bias()
        # data-gradient convs: flipped / transposed filters; bf16 packs take the gradient's bf16 copy with its
        # channels zero-padded to 8 or 16 (conv3x3_narrowin's tap-major pieces), wider ones to 32 (the granule)
        self.dconv = {}
        for name in DGRAD:
            w = self.P[name, "w"]
            ci, co = int(w.shape[2]), int(w.shape[3])
            if bf16:
                cg = (co + 7) // 8 * 8 if co <= 16 else (co + 31) // 32 * 32
                self.dconv[name] = ops.PackedConv.from_source(w, cg, (ci + 3) // 4 * 4, "bf16", flip=True)
            else:
                self.dconv[name] = ops.PackedConv.from_source(w, co, ci, "fp32", flip=True)
        self._repack = ops.PackBatch(list(self.convs.values()) + list(self.dconv.values()))
        self._mfma_wgrad = bf16
        self._b, self._key = None, None

    def _refresh_bias(self):
        for name, (bp, co) in self._pad.items():
            bp[:co].copy_(self.P[name, "b"])

    def _refresh_packs(self):
        self._repack()
        self._refresh_bias()

    # ------------------------------------------------------------------------------------------- buffers
    def _buffers(self, n, h, w):
        if self._key == (n, h, w):
            return self._b
        L = _levels(h, w)
        T, dev = self.dtype, self.device
        A = lambda lv, c, dt=T: torch.zeros((n, L[lv][0], L[lv][1], c), dtype=dt, device=dev)  # noqa: E731
        F = lambda lv, c: A(lv, c, torch.float32)  # noqa: E731
        st = lambda c: (torch.empty(c, dtype=torch.float32, device=dev),  # noqa: E731
                        torch.empty(c, dtype=torch.float32, device=dev))
        b = {"in6": F(0, 6), "inp": A(0, 8),
             # activations (compute dtype); cat2 = [conv1_1 | up2], cat1 = [conv2_1 | up1] (small.py:20)
             "cat2": A(0, 16), "cat2n": A(0, 16), "p1": A(1, 8), "cat1": A(1, 32), "cat1n": A(1, 32),
             "p2": A(2, 16), "a31": A(2, 32), "a32": A(2, 32), "r1": A(1, 32), "a22": A(1, 16), "r2": A(0, 16),
             "a12": A(0, 8), "alpha": F(0, 1), "loss": torch.zeros(3, dtype=torch.float32, device=dev),
             # gradients (f32)
             "dlogit": F(0, 1), "da12": F(0, 8), "dcat2n": F(0, 16), "dcat2": F(0, 16), "gskip2": F(0, 8),
             "du2": F(0, 8), "dr2": F(0, 16), "da22": F(1, 16), "dcat1n": F(1, 32), "dcat1": F(1, 32),
             "gskip1": F(1, 16), "du1": F(1, 16), "dr1": F(1, 32), "da32": F(2, 32), "da31": F(2, 32),
             "dp2": F(2, 16), "da21": F(1, 16), "dp1": F(1, 8), "da11": F(0, 8)}
        lv = {"conv1_1": 0, "conv2_1": 1, "conv3_1": 2, "conv3_2": 2, "upconv1": 1, "conv2_2": 1, "upconv2": 0,
              "conv1_2": 0, "conv1_3": 0}
        for name, _, co in NEW_CONVS:
            b["st_" + name] = st(BN_WIDTH.get(name, co))
            if name.startswith("upconv"):
                continue
            if name in self._pad:  # pre-BN output of the padded pack (8 channels), the live one first
                b["zfull_" + name] = F(lv[name], 8)
                b["z_" + name] = b["zfull_" + name][..., :co]
            else:
                b["z_" + name] = F(lv[name], co)
            # (the fp32 data-gradient conv reads dz: a narrow one keeps an 8-channel row, zero padded)
            b["dz_" + name] = F(lv[name], co) if co % 8 == 0 else F(lv[name], 8)[..., :co]
        # bf16 copies of the gradients the data-gradient convs read, channels zero-padded to 32
        if self.dtype == torch.bfloat16:
            for name in DGRAD:
                pc = self.dconv[name]
                b["g16_" + name] = A(lv[name], pc.cin, torch.bfloat16)
        self._b, self._key = b, (n, h, w)
        return b

    # ------------------------------------------------------------------------------------------- forward
    def _new_conv(self, x, name, act, out):
        """new_conv (small.py:26-34) with batch statistics, then ``act``; keeps the pre-BN z and (mean, var)."""
        b = self._b
        z, (mean, var) = b["z_" + name], b["st_" + name]
        ops.conv3x3(x, self.convs[name], "none", out=b.get("zfull_" + name, z), affine=False, splitk=True)
        self._stats(z, mean, var)
        ops.bn_apply(z, mean, var, self.P[name, "gamma"], self.P[name, "beta"], EPS, act, out=out)

    def _upconv(self, down, cat, catn, name, rbuf, skip_c):
        """upconv_concat (small.py:13-23): resize -> conv (no bias) -> relu -> concat [skip, up] -> BN."""
        ops.resize_bilinear(down, cat.shape[1:3], out=rbuf)
        ops.conv3x3(rbuf, self.convs[name], "relu", out=cat[..., skip_c:], affine=False, splitk=True)
        mean, var = self._b["st_" + name]
        self._stats(cat, mean, var)
        ops.bn_apply(cat, mean, var, self.P[name, "gamma"], self.P[name, "beta"], EPS, "none", out=catn)

    def forward(self, cmp, bg):
        """UNetSmall(concat(cmp, bg), phase=True).output (small.py:37-50) -> alpha [N,H,W,1] f32."""
        dev = lambda t: (t if isinstance(t, torch.Tensor) else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(t, np.float32))).to(self.device, torch.float32)
        cmp, bg = dev(cmp), dev(bg)
        n, h, w, c = cmp.shape
        if self.cin != 2 * c or tuple(bg.shape) != (n, h, w, c):
            raise ValueError("SmallTrainer(cin=%d) expects cmp, bg of %d channels each" % (self.cin, self.cin // 2))
        b = self._buffers(n, h, w)
        b["in6"][..., :c].copy_(cmp)  # small_train.py:95 input = concat([in_cmp, in_bg], -1)
        b["in6"][..., c:].copy_(bg)
        ops.convert(b["in6"], b["inp"])
        self._new_conv(b["inp"][..., :self.cin], "conv1_1", "relu", b["cat2"][..., :8])
        ops.maxpool2x2(b["cat2"][..., :8], out=b["p1"])
        self._new_conv(b["p1"], "conv2_1", "relu", b["cat1"][..., :16])
        ops.maxpool2x2(b["cat1"][..., :16], out=b["p2"])
        self._new_conv(b["p2"], "conv3_1", "relu", b["a31"])
        self._new_conv(b["a31"], "conv3_2", "relu", b["a32"])
        self._upconv(b["a32"], b["cat1"], b["cat1n"], "upconv1", b["r1"], 16)
        self._new_conv(b["cat1n"], "conv2_2", "relu", b["a22"])
        self._upconv(b["a22"], b["cat2"], b["cat2n"], "upconv2", b["r2"], 8)
        self._new_conv(b["cat2n"], "conv1_2", "relu", b["a12"])
        self._new_conv(b["a12"], "conv1_3", "sigmoid", b["alpha"])  # BN output -> tf.nn.sigmoid 'probs'
        self.output = b["alpha"]
        return self.output

    # ------------------------------------------------------------------------------------------- backward
    def _dgrad(self, name, dz, out):
        """Data gradient of conv ``name`` from its pre-BN gradient (bf16: from the bf16 copy the BN backward wrote)."""
        pc = self.dconv[name]
        if self.dtype == torch.bfloat16:
            ops.conv3x3(self._b["g16_" + name], pc, "none", out=ops.widen(out, pc.cout), affine=False)
        else:
            ops.conv3x3(dz, pc, "none", out=out, affine=False)

    def _conv_backward(self, name, x_in, dy, mask, dgrad_out=None):
        """BN(+relu) backward into dz (with the conv-bias gradient), the filter gradient, optionally x_in's gradient."""
        b = self._b
        dz, (mean, var) = b["dz_" + name], b["st_" + name]
        g16 = b.get("g16_" + name) if dgrad_out is not None else None
        self._bn_backward(b["z_" + name], dy, mask, mean, var, name, dz,
                          dx2=None if g16 is None else g16[..., :dz.shape[-1]], dbias=self.G[name, "b"])
        ops.conv_wgrad(x_in, dz, self.G[name, "w"], mfma=self._mfma_wgrad)
        if dgrad_out is not None:
            self._dgrad(name, dz, dgrad_out)

    def _upconv_backward(self, name, cat, dcatn, dcat, gskip, du, rbuf, dr, skip_c):
        """BN over the concat, then the split relu backward: the skip half's gradient to ``gskip`` (masked by the skip
        activation, which its own BN backward masks again: idempotent), the upconv half's to ``du``; filter gradient
        and the data gradient through the conv into the resized tensor."""
        b = self._b
        mean, var = b["st_" + name]
        self._bn_backward(cat, dcatn, None, mean, var, name, dcat)
        g16 = b.get("g16_" + name)
        ops.relu_backward(dcat, cat, du, dx2=None if g16 is None else g16[..., :du.shape[-1]], dx_lo=gskip)
        ops.conv_wgrad(rbuf, du, self.G[name, "w"], mfma=self._mfma_wgrad)
        self._dgrad(name, du, dr)

    def backward(self, gt, raw_fg, bg, cmp):
        b = self._b
        ops.matting_loss_backward(b["alpha"], gt, raw_fg, bg, cmp, out=b["dlogit"])
        self._conv_backward("conv1_3", b["a12"], b["dlogit"], None, b["da12"])
        self._conv_backward("conv1_2", b["cat2n"], b["da12"], b["a12"], b["dcat2n"])
        self._upconv_backward("upconv2", b["cat2"], b["dcat2n"], b["dcat2"], b["gskip2"], b["du2"], b["r2"], b["dr2"], 8)
        ops.resize_backward(b["dr2"], b["da22"])
        self._conv_backward("conv2_2", b["cat1n"], b["da22"], b["a22"], b["dcat1n"])
        self._upconv_backward("upconv1", b["cat1"], b["dcat1n"], b["dcat1"], b["gskip1"], b["du1"], b["r1"], b["dr1"],
                              16)
        ops.resize_backward(b["dr1"], b["da32"])
        self._conv_backward("conv3_2", b["a31"], b["da32"], b["a32"], b["da31"])
        self._conv_backward("conv3_1", b["p2"], b["da31"], b["a31"], b["dp2"])
        # conv2_1's output feeds pool2 and the upconv1 concat: the pool adjoint plus the skip gradient
        ops.maxpool_backward(b["cat1"][..., :16], b["dp2"], b["da21"], add=b["gskip1"])
        self._conv_backward("conv2_1", b["p1"], b["da21"], b["cat1"][..., :16], b["dp1"])
        ops.maxpool_backward(b["cat2"][..., :8], b["dp1"], b["da11"], add=b["gskip2"])
        self._conv_backward("conv1_1", b["inp"][..., :self.cin], b["da11"], b["cat2"][..., :8])

    # ------------------------------------------------------------------------------------------- step
    def step(self, cmp, bg, gt, raw_fg):
        """One training iteration; returns a new device tensor [loss, alpha_loss, compositional_loss] (pre-update)."""
        self.forward(cmp, bg)
        dev = lambda t: (t if isinstance(t, torch.Tensor) else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(t, np.float32))).to(self.device, torch.float32).contiguous()
        gt, raw_fg, bg_d, cmp_d = dev(gt), dev(raw_fg), dev(bg), dev(cmp)
        b = self._b
        b["loss"].copy_(ops.matting_loss(b["alpha"], gt, raw_fg, bg_d, cmp_d))
        self.grad.zero_()
        self.backward(gt, raw_fg, bg_d, cmp_d)
        self.apply_gradients()
        return b["loss"].clone()

    def capture(self, cmp, bg, gt, raw_fg):
        """Record one step's forward + loss and its backward as two HIP graphs (torch.cuda.CUDAGraph over the same
        C-ABI launches) -> SmallTrainGraph; its step() replays both and runs the DDP exchange + Adam + re-pack eagerly
        (TF's bias correction changes every step).  The graphs read the trainer's parameters, packs and buffers in
        place.  A tiny UNetSmall step is ~110 launches of a few microseconds each: replay removes their host cost."""
        return SmallTrainGraph(self, cmp, bg, gt, raw_fg)

    def params_numpy(self):
        """{scope: (w, b|None)} and {scope: (gamma, beta)} on the host (checkpoint / small.UNetSmall hand-off)."""
        conv = {s: (self.P[s, "w"].cpu().numpy(), self.P[s, "b"].cpu().numpy() if (s, "b") in self.P else None)
                for s, _, _ in NEW_CONVS}
        bn = {s: (self.P[s, "gamma"].cpu().numpy(), self.P[s, "beta"].cpu().numpy()) for s, _, _ in NEW_CONVS}
        return conv, bn


class SmallTrainGraph:
    """SmallTrainer.capture's result: ``step(cmp, bg, gt, raw_fg)`` = SmallTrainer.step on graph replays."""

    def __init__(self, trn, *batch):
        if trn.sync_bn and torch.distributed.get_backend() != "nccl":
            raise NotImplementedError("capture with sync_bn needs the nccl (RCCL) backend")
        dev = trn.device
        self.trn = trn
        self.inputs = [(t if isinstance(t, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(t, np.float32)))
                       .to(dev, torch.float32).contiguous().clone() for t in batch]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # buffers, workspaces and the SyncBN batch count before capture
            self._forward()
            self._backward()
        main = torch.cuda.current_stream(dev)
        main.wait_stream(side)
        torch.cuda.synchronize(dev)
        for t in trn._b.values():  # allocated on the side stream, replayed on this one
            for u in (t if isinstance(t, tuple) else (t,)):
                u.record_stream(main)
        self.g_fwd, self.g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fwd):
            self._forward()
        with torch.cuda.graph(self.g_bwd):
            self._backward()

    def _forward(self):
        cmp, bg, gt, fg = self.inputs
        t = self.trn
        t.forward(cmp, bg)
        t._b["loss"].copy_(ops.matting_loss(t._b["alpha"], gt, fg, bg, cmp))

    def _backward(self):
        cmp, bg, gt, fg = self.inputs
        self.trn.grad.zero_()
        self.trn.backward(gt, fg, bg, cmp)

    def load(self, *batch):
        for dst, src in zip(self.inputs, batch):
            dst.copy_(src if isinstance(src, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(src, np.float32)))

    def step(self, *batch):
        if batch:
            self.load(*batch)
        self.g_fwd.replay()
        self.g_bwd.replay()
        self.trn.apply_gradients()
        return self.trn._b["loss"].clone()
