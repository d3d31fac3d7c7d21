"""train.py's UNetImage training step on gfx950 kernels: one iteration of ``training_procedure`` (train.py:37-109).

``ImageTrainer.step(cmp, bg, gt, raw_fg)`` is one ``sess.run([train_merged, train_op], feed_dict)`` of the reference
(train.py:79-81) with the graph ``train()`` builds (train.py:112-135):

  input     x = [cmp, bg] (train.py:116: one 6-channel placeholder; training_procedure splits it back,
            train.py:41)
  forward   unet.UNetImage.build(x) (unet.py:86-148): the 12 VGG convs (conv1_1 = [VGG/2, VGG/2] over 6 channels,
            unet.py:150-157) + relu, 4 SAME 2x2 max-pools, 4 upconv_concat (TF-1 resize -> conv, no bias, no relu ->
            concat [up, skip], unet.py:44-63), conv4_4 / conv3_4 / conv2_3 + relu, conv1_5 -> sigmoid.  Every
            activation the backward reads stays in HBM (no fused first pair, no folded upconvs, no head split)
  loss      mean(0.5*regular_l1(pred, gt) + 0.5*regular_l1(composite(raw_fg, in_bg, pred), in_cmp))
            (train.py:42-47; [loss, alpha_loss, cmp_loss] returned)
  backward  through EVERY variable (train.py:51-52: minimize() with the default var_list): the VGG filters and
            biases (tf.Variable, unet.py:76-77,157), the fresh convs' weights and biases; the upconvs' drawn biases
            (unet.py:59) feed nothing and get no gradient, so Adam skips them — here they are not parameters.
            Per relu conv one pass (vm_relu_backward_bias_nhwc) gives the masked gradient as the bf16 operand of
            the filter gradient (ops.conv_wgrad: the wide MFMA kernel for cout >= 64) and of the data gradient
            (forward conv kernels on the flipped filter) plus the bias gradient; the [up, skip] concat gradient
            splits by channel view: the skip conv's pass also takes its max-pool's adjoint (TF MaxPoolGrad's
            first-maximum rule) and adds the concat half; the upconv half goes through its conv's data gradient and
            the TF-1 resize adjoint
  exchange  DDP: one all-reduce of the flat gradient buffer (UNetImage has no BN, so nothing else is exchanged)
  update    tf.train.AdamOptimizer(1e-5, 0.9, 0.999, 1e-8) over the flat buffer in one launch, then re-packs
"""

import numpy as np
import torch

from . import ops, parallel
from .train import TrainerBase
from .unet import UNetImage, _levels

# build order of unet.py:96-143 (the TF variable creation order): scope, keeps a bias
LAYERS = (("conv1_1", True), ("conv1_2", True), ("conv2_1", True), ("conv2_2", True), ("conv3_1", True),
          ("conv3_2", True), ("conv3_3", True), ("conv4_1", True), ("conv4_2", True), ("conv4_3", True),
          ("conv5_1", True), ("conv5_2", True), ("upconv_1", False), ("conv4_4", True), ("upconv_2", False),
          ("conv3_4", True), ("upconv_3", False), ("conv2_3", True), ("upconv_4", False), ("conv1_5", True))


def param_layout(shapes):
    """Flat f32 layout of UNetImage's trainable variables in build order: per scope the filter, then the bias.
    shapes: {scope: (3, 3, cin, cout)} -> ([(scope, kind, offset, shape)], total)"""
    out, off = [], 0
    for name, has_b in LAYERS:
        ents = [("w", tuple(shapes[name]))] + ([("b", (shapes[name][3],))] if has_b else [])
        for kind, shape in ents:
            out.append((name, kind, off, shape))
            off += int(np.prod(shape))
    return out, off


class ImageTrainer(TrainerBase):
    """train.training_procedure's iteration on device (unet.UNetImage, all variables trainable).

    ``streams=1`` runs the filter gradients on a side stream (``_side``) beside the data-gradient chain.  capture()
    (ImageTrainGraph) clears ``_side`` for the duration of the capture, so the graph is recorded on one stream, and
    restores it afterwards (also when the capture raises).  A trainer is not thread-safe: another thread's eager
    step during a capture would run single-stream."""

    bf16_dgrad = True  # bf16 path: data gradients held in bf16 (see _grad_buffers); False = f32 as the fp32 path
    # filter gradients kept on the caller's stream: conv1_1's is the backward's last work and the data-gradient chain
    # (no dgrad for conv1_1) is idle by then, while the side stream still has the earlier layers' queued
    main_wgrad = ("conv1_1",)
    # the side stream: "probe" (ops.concurrent_stream: a pooled stream checked to run beside the caller's; a plain one
    # landed on the caller's hardware queue for 2 of 9 trainers, backward 4.8 ms instead of 4.1), or for A/B "pool"
    # (the r05 form), "high" (high priority: 8.3 ms when it gets the high-priority queue), "masked" (a CU-masked
    # stream: its own queue, 8.3 ms) — kernel traces in profiles/r06o_imgtrace_queues.txt
    side_kind = "probe"

    def __init__(self, vgg16_npy_path=None, dtype="fp32", device="cuda", params=None, lr=1e-5, beta1=0.9,
                 beta2=0.999, epsilon=1e-8, streams=1):
        m = UNetImage(vgg16_npy_path, dtype, device)
        # the backward reads every activation: keep them all in HBM
        m.fuse_first, m.split_head, m.fuse_up_head, m.fold_upconv = False, False, False, ()
        if params is not None:
            m.load_params(params)
        m.prepare()  # init_conv draws in build order from the global numpy RNG (unet.py:11-17) when params is None
        self.model = m
        self.dtype = m.dtype
        self.device = m.device
        layout, n = param_layout({k: v[0].shape for k, v in m.params.items()})
        self._init_flat(layout, n, lr, beta1, beta2, epsilon, False)
        f = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32))  # noqa: E731
        for name, has_b in LAYERS:
            w, b = m.params[name]
            self.P[name, "w"].copy_(f(w))
            pc = m.convs[name]
            pc.w_hwio = self.P[name, "w"]
            if has_b:
                self.P[name, "b"].copy_(f(b))
                pc.bias = self.P[name, "b"]
        if parallel.world_size() > 1:  # every replica starts from rank 0's variables
            parallel.broadcast_tensors([self.flat], src=0)
        bf16 = self.dtype == torch.bfloat16
        # data-gradient convs (every conv but conv1_1, whose input is the network input): flipped / transposed
        # filters; bf16: from the bf16 copy of the gradient, conv1_5's single channel padded to 32
        self.dconv = {}
        for name, _ in LAYERS[1:]:
            w = self.P[name, "w"]
            ci, co = int(w.shape[2]), int(w.shape[3])
            if bf16:
                self.dconv[name] = ops.PackedConv.from_source(w, (co + 31) // 32 * 32, ci, "bf16", flip=True)
            else:
                self.dconv[name] = ops.PackedConv.from_source(w, co, ci, "fp32", flip=True)
        self._repack = ops.PackBatch(list(m.convs.values()) + list(self.dconv.values()))
        if parallel.world_size() > 1:
            self._refresh_packs()
        self._mfma_wgrad = bf16
        self._g, self._key = None, None
        # the filter gradients are leaves of the backward graph: each reads its layer's dz (and the forward input)
        # and only Adam reads its result, so with a side stream they run beside the data-gradient chain (relu
        # backward -> dgrad conv -> next layer), joined before the update.  Same kernels, same arithmetic; per-stream
        # workspaces (ops._workspace)
        dev_ = torch.device(device)
        self._side = None
        if streams and dev_.type == "cuda":
            if self.side_kind == "probe":  # a pooled stream probed to run beside the caller's (ops.concurrent_stream)
                self._side = ops.concurrent_stream(dev_)
            elif self.side_kind == "masked":  # (A/B) a CU-masked stream (ops.side_stream)
                self._side = ops.side_stream(dev_)
            else:  # (A/B) "pool": a torch pool stream (the r05 form); "high": a high-priority one
                self._side = torch.cuda.Stream(device=dev_, priority=-1 if self.side_kind == "high" else 0)
        self._main = None

    def _refresh_packs(self):
        self._repack()

    # ------------------------------------------------------------------------------------------- buffers
    def _grad_buffers(self, n, h, w):
        """f32 gradients per level, and (bf16 path) the bf16 copies the filter / data-gradient convs read."""
        if self._key == (n, h, w):
            return self._g
        L = _levels(h, w)
        dev = self.device
        F = lambda lv, c: torch.zeros((n, L[lv][0], L[lv][1], c), dtype=torch.float32, device=dev)  # noqa: E731
        bf16 = self.dtype == torch.bfloat16
        B = lambda lv, c: torch.zeros((n, L[lv][0], L[lv][1], c), dtype=torch.bfloat16, device=dev)  # noqa: E731
        Z = (lambda lv, c: None) if bf16 else F  # noqa: E731  (f32 dz: the fp32 path only)
        # D: the data gradients the dgrad convs write.  The bf16 path keeps them bf16 (bf16_dgrad): their only
        # readers round to bf16 anyway (the MFMA convs' operands) or widen exactly (the relu / resize adjoints), so
        # the convs write half the bytes and the upconv gradient needs no f32 -> bf16 convert.  The resize adjoint's
        # outputs (dc23, dc34, dc44, dc52) too: it sums in f32 and rounds once, and their only reader is a relu
        # backward with no `add`, whose bf16 dz = mask * bf16(dy) is then the same value either way.
        D = B if bf16 and self.bf16_dgrad else F
        g = {"dlogit": F(0, 1), "dlog8": F(0, 8), "loss": torch.zeros(3, dtype=torch.float32, device=dev),
             "in6": torch.empty((n, h, w, 6), dtype=torch.float32, device=dev),
             "dcat1": D(0, 128), "dr4": D(0, 128), "dz12": Z(0, 64), "dc11": D(0, 64), "dz11": Z(0, 64),
             "dcat2": D(1, 256), "dc23": D(1, 128), "dz23": Z(1, 128), "dr3": D(1, 256), "dz22": Z(1, 128),
             "dc21": D(1, 128), "dz21": Z(1, 128), "dp1": D(1, 64),
             "dcat3": D(2, 512), "dc34": D(2, 256), "dz34": Z(2, 256), "dr2": D(2, 512), "dz33": Z(2, 256),
             "dc32": D(2, 256), "dz32": Z(2, 256), "dc31": D(2, 256), "dz31": Z(2, 256), "dp2": D(2, 128),
             "dcat4": D(3, 1024), "dc44": D(3, 512), "dz44": Z(3, 512), "dr1": D(3, 512), "dz43": Z(3, 512),
             "dc42": D(3, 512), "dz42": Z(3, 512), "dc41": D(3, 512), "dz41": Z(3, 512), "dp3": D(3, 256),
             "dc52": D(4, 512), "dz52": Z(4, 512), "dc51": D(4, 512), "dz51": Z(4, 512), "dp4": D(4, 512)}
        if bf16:
            hb = {"dlog16": (0, 32), "dz12": (0, 64), "dz11": (0, 64),
                  "dz23": (1, 128), "dz22": (1, 128), "dz21": (1, 128),
                  "dz34": (2, 256), "dz33": (2, 256), "dz32": (2, 256), "dz31": (2, 256),
                  "dz44": (3, 512), "dz43": (3, 512), "dz42": (3, 512), "dz41": (3, 512),
                  "dz52": (4, 512), "dz51": (4, 512)}
            if not self.bf16_dgrad:  # dense bf16 copies of the upconv gradients
                hb.update({"du4": (0, 64), "du3": (1, 128), "du2": (2, 256), "du1": (3, 512)})
            for k, (lv, c) in hb.items():
                g["h_" + k] = B(lv, c)
        g = {k: v for k, v in g.items() if v is not None}
        self._g, self._key = g, (n, h, w)
        return g

    # ------------------------------------------------------------------------------------------- forward
    def forward(self, cmp, bg):
        """UNetImage(x = concat(cmp, bg)).output (unet.py:86-145) -> alpha [N,H,W,1] f32."""
        dev = lambda t: (t if isinstance(t, torch.Tensor) else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(t, np.float32))).to(self.device, torch.float32)
        cmp, bg = dev(cmp), dev(bg)
        n, h, w, c = cmp.shape
        if c != 3 or tuple(bg.shape) != (n, h, w, 3):
            raise ValueError("ImageTrainer expects cmp, bg of 3 channels each (train.py:116: x = [cmp, bg])")
        g = self._grad_buffers(n, h, w)
        g["in6"][..., :3].copy_(cmp)
        g["in6"][..., 3:].copy_(bg)
        self.output = self.model.forward(g["in6"])
        return self.output

    # ------------------------------------------------------------------------------------------- backward
    def _bf16(self):
        return self.dtype == torch.bfloat16

    def _relu_conv_backward(self, name, dy, y, x_in, dz_key, dx_out=None, add=None):
        """y = relu(conv(x_in) + b): dz = (y > 0) * (dy (+ add)) — or, when dy is the 2x2 pool's gradient, the pool
        adjoint of dy plus ``add`` — and the bias gradient from ONE pass (vm_relu_backward_bias_nhwc; the bf16 path
        writes only the bf16 dz its MFMA convs read), then the filter gradient and optionally x_in's gradient."""
        g = self._g
        h16 = g.get("h_" + dz_key)
        dz = h16 if h16 is not None else g[dz_key]
        ops.relu_backward_bias(dy, y, dz, self.G[name, "b"], add=add)
        self._wgrad_dgrad(name, x_in, dz, h16, dx_out)

    def _wgrad(self, x_in, dz, dw, mfma, main=False):
        if self._main is None or main:
            ops.conv_wgrad(x_in, dz, dw, mfma=mfma)
            return
        self._side.wait_stream(self._main)
        with torch.cuda.stream(self._side):
            ops.conv_wgrad(x_in, dz, dw, mfma=mfma)

    def _wgrad_dgrad(self, name, x_in, dz, h16, dx_out):
        if h16 is not None:  # bf16 path: the bf16 copy feeds both MFMA convs
            self._wgrad(x_in, h16, self.G[name, "w"], True, name in self.main_wgrad)
            if dx_out is not None:
                ops.conv3x3(h16, self.dconv[name], "none", out=dx_out, affine=False, splitk=True)
        else:
            self._wgrad(x_in, dz, self.G[name, "w"], False, name in self.main_wgrad)
            if dx_out is not None:
                ops.conv3x3(dz, self.dconv[name], "none", out=dx_out, affine=False, splitk=True)

    def _upconv_backward(self, name, dup, rbuf, up_key, dr, dprev):
        """upconv_concat's conv (no bias, no relu) on the resized input: filter gradient, data gradient into the
        resized tensor, then the TF-1 resize adjoint into the low-resolution input's gradient."""
        h16 = self._g.get("h_" + up_key)
        if h16 is not None:
            ops.convert(dup, h16)
        elif dup.dtype == torch.bfloat16:  # bf16_dgrad: the bf16 slice of dcat is the MFMA operand itself
            h16 = dup
        self._wgrad_dgrad(name, rbuf, dup, h16, dr)
        ops.resize_backward(dr, dprev)

    def backward(self, gt, raw_fg, bg, cmp):
        self._main = torch.cuda.current_stream(self.device) if self._side is not None else None
        try:
            self._backward(gt, raw_fg, bg, cmp)
        finally:
            if self._main is not None:  # every filter gradient in place before the all-reduce / Adam
                self._main.wait_stream(self._side)
            self._main = None

    def _backward(self, gt, raw_fg, bg, cmp):
        m, g = self.model, self._g
        b = m._ws
        ops.matting_loss_backward(m.output, gt, raw_fg, bg, cmp, out=g["dlogit"])
        # conv1_5 (cout 1, bias, no relu) over cat1 = [upconv_4, conv1_2] (unet.py:140-145)
        ops.bn_backward(None, g["dlogit"], None, None, None, None, dbeta=self.G["conv1_5", "b"])
        if self._bf16():
            ops.convert(g["dlogit"], g["h_dlog16"][..., :1])
            self._wgrad(b["cat1"], g["dlogit"], self.G["conv1_5", "w"], True)
            ops.conv3x3(g["h_dlog16"], self.dconv["conv1_5"], "none", out=g["dcat1"], affine=False, splitk=True)
        else:
            ops.convert(g["dlogit"], g["dlog8"][..., :1])
            self._wgrad(b["cat1"], g["dlogit"], self.G["conv1_5", "w"], False)
            ops.conv3x3(g["dlog8"][..., :1], self.dconv["conv1_5"], "none", out=g["dcat1"], affine=False,
                        splitk=True)
        # decoder, top down: [up, skip] halves of each concat
        self._upconv_backward("upconv_4", g["dcat1"][..., :64], b["r4"], "du4", g["dr4"], g["dc23"])
        self._relu_conv_backward("conv2_3", g["dc23"], b["c23"], b["cat2"], "dz23", g["dcat2"])
        self._upconv_backward("upconv_3", g["dcat2"][..., :128], b["r3"], "du3", g["dr3"], g["dc34"])
        self._relu_conv_backward("conv3_4", g["dc34"], b["c34"], b["cat3"], "dz34", g["dcat3"])
        self._upconv_backward("upconv_2", g["dcat3"][..., :256], b["r2"], "du2", g["dr2"], g["dc44"])
        self._relu_conv_backward("conv4_4", g["dc44"], b["c44"], b["cat4"], "dz44", g["dcat4"])
        self._upconv_backward("upconv_1", g["dcat4"][..., :512], b["r1"], "du1", g["dr1"], g["dc52"])
        # encoder, bottom up; each skip conv's gradient = its concat half + its pool's adjoint, in the same pass
        self._relu_conv_backward("conv5_2", g["dc52"], b["c52"], b["c51"], "dz52", g["dc51"])
        self._relu_conv_backward("conv5_1", g["dc51"], b["c51"], b["p4"], "dz51", g["dp4"])
        self._relu_conv_backward("conv4_3", g["dp4"], b["cat4"][..., 512:], b["c42"], "dz43", g["dc42"],
                                 add=g["dcat4"][..., 512:])
        self._relu_conv_backward("conv4_2", g["dc42"], b["c42"], b["c41"], "dz42", g["dc41"])
        self._relu_conv_backward("conv4_1", g["dc41"], b["c41"], b["p3"], "dz41", g["dp3"])
        self._relu_conv_backward("conv3_3", g["dp3"], b["cat3"][..., 256:], b["c32"], "dz33", g["dc32"],
                                 add=g["dcat3"][..., 256:])
        self._relu_conv_backward("conv3_2", g["dc32"], b["c32"], b["c31"], "dz32", g["dc31"])
        self._relu_conv_backward("conv3_1", g["dc31"], b["c31"], b["p2"], "dz31", g["dp2"])
        self._relu_conv_backward("conv2_2", g["dp2"], b["cat2"][..., 128:], b["c21"], "dz22", g["dc21"],
                                 add=g["dcat2"][..., 128:])
        self._relu_conv_backward("conv2_1", g["dc21"], b["c21"], b["p1"], "dz21", g["dp1"])
        self._relu_conv_backward("conv1_2", g["dp1"], b["cat1"][..., 64:], b["c11"], "dz12", g["dc11"],
                                 add=g["dcat1"][..., 64:])
        self._relu_conv_backward("conv1_1", g["dc11"], b["c11"], b["in8"][..., :6], "dz11")

    # ------------------------------------------------------------------------------------------- step
    def step(self, cmp, bg, gt, raw_fg):
        """One training iteration; returns a new device tensor [loss, alpha_loss, compositional_loss] (pre-update)."""
        self.forward(cmp, bg)
        dev = lambda t: (t if isinstance(t, torch.Tensor) else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(t, np.float32))).to(self.device, torch.float32).contiguous()
        gt, raw_fg, bg_d, cmp_d = dev(gt), dev(raw_fg), dev(bg), dev(cmp)
        g = self._g
        g["loss"].copy_(ops.matting_loss(self.model.output, gt, raw_fg, bg_d, cmp_d))
        self.grad.zero_()
        self.backward(gt, raw_fg, bg_d, cmp_d)
        self.apply_gradients()
        return g["loss"].clone()

    def capture(self, cmp, bg, gt, raw_fg):
        """Record one step's forward + loss and its backward as two HIP graphs -> ImageTrainGraph (DDP exchange +
        Adam + re-pack eager: TF's bias correction changes every step)."""
        return ImageTrainGraph(self, cmp, bg, gt, raw_fg)

    def params_numpy(self):
        """{scope: (w, b|None)} on the host (checkpoint / unet.UNetImage.load_params hand-off)."""
        return {s: (self.P[s, "w"].cpu().numpy(), self.P[s, "b"].cpu().numpy() if hb else None) for s, hb in LAYERS}

    def conv_flops(self, n, h, w):
        """Algorithmic FLOPs of one step: the forward's 20 convs, the filter gradient of each (the same count) and
        the data gradient of every conv but conv1_1."""
        fwd = self.model.conv_flops(n, h, w)
        c11 = 2.0 * n * h * w * 9 * 6 * 64
        return fwd, fwd + (fwd - c11)


class ImageTrainGraph:
    """ImageTrainer.capture's result: ``step(cmp, bg, gt, raw_fg)`` = ImageTrainer.step on graph replays."""

    def __init__(self, trn, *batch):
        dev = trn.device
        self.trn = trn
        self.inputs = [(t if isinstance(t, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(t, np.float32)))
                       .to(dev, torch.float32).contiguous().clone() for t in batch]
        # captured without the trainer's side stream: a HIP-graph replay on ROCm 7 ran the fork's branches one after
        # the other and the fork cost time (6.7 ms against 6.5 on one stream; eager with the side stream 6.0)
        self._side, trn._side = trn._side, None
        try:
            self._capture(trn, dev)
        finally:
            trn._side = self._side

    def _capture(self, trn, dev):
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # buffers and workspaces before capture
            self._forward()
            self._backward()
        main = torch.cuda.current_stream(dev)
        main.wait_stream(side)
        torch.cuda.synchronize(dev)
        for d in (trn._g, trn.model._ws):  # allocated on the side stream, replayed on this one
            for t in d.values():
                t.record_stream(main)
        for t in ops._ws_cache.values():
            t.record_stream(main)
        self.g_fwd, self.g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fwd):
            self._forward()
        with torch.cuda.graph(self.g_bwd):
            self._backward()

    def _forward(self):
        cmp, bg, gt, fg = self.inputs
        t = self.trn
        t.forward(cmp, bg)
        t._g["loss"].copy_(ops.matting_loss(t.model.output, gt, fg, bg, cmp))

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
        return self.trn._g["loss"].clone()
