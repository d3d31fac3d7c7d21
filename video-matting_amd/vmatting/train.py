"""Config-5 training step on gfx950 kernels: train.py's video_procedure / simple_procedure iteration.

One ``VideoTrainer.step(cmp, bg, warped, gt, raw_fg)`` is one ``sess.run([train_merged, train_op], feed_dict)``
of the reference (train.py:325-327; simple_procedure train.py:205-208 feeds ``diff = cmp - bg`` instead of the
warped previous alpha, train.py:245):

  forward   unet_simple.create_model(cmp, bg, warped, phase=True) (unet_simple.py:145-171) — the frozen VGG16
            towers, then UNetSimple with batch-statistics BN (is_training=True); pre-BN tensors and batch
            statistics are kept for the backward pass
  loss      loss = mean(0.5*regular_l1(pred, gt) + 0.5*regular_l1(composite(raw_fg, bg, pred), cmp))
            (train.py:294-298; the summary scalars [loss, alpha_loss, cmp_loss] are returned)
  backward  through the trainable 'model/simple_unet' variables only (train.py:289: TRAINABLE_VARIABLES of that
            scope — conv weights and biases, BN gamma/beta); hand-written kernels (csrc/train.hip): BN backward
            with the relu mask, conv weight gradient, conv data gradient (forward kernels on flipped weights),
            TF-1 resize adjoint.  The upconv biases (unet_simple.py:34, drawn but unused) get no gradient, so
            TF's apply_gradients skips them; here they are simply not parameters
  exchange  DDP: one RCCL all-reduce of the flat gradient buffer (parallel.allreduce_grads); BN statistics stay
            per replica by default (each rank normalises over its own batch of 8); ``sync_bn=True`` normalises
            over the global batch instead (one small all-reduce of per-channel moments per BN layer, forward and
            backward), the single-device reference's semantics for a batch split over replicas
  update    tf.train.AdamOptimizer(lr, beta1=0.9, beta2=0.999, epsilon=1e-8) (train.py:300-304) over the flat
            parameter buffer in one launch, then the forward / data-gradient filters are re-packed

The moving BN statistics are never updated, as in the reference (UPDATE_OPS is not wired, train.py:304).
"""

import numpy as np
import torch

from . import ops, parallel
from .layers import EPS
from .unet_simple import CIN_PAD, NEW_CONVS, UNetSimple, Vgg16, _levels

# UNetSimple levels from the bottom up (unet_simple.py:119-141):
# (level, concat buffer, width, [(select scope, source)], upconv scope, upconv input, conv scope, conv output)
LEVELS = (
    (3, "up4", 96, (("select4_1", "cat_conv4_1"), ("select4_2", "cat_conv4_2"), ("select4_3", "cat_conv4_3")),
     "upconv4", "cat_conv5_3", "conv4", "c4"),
    (2, "up3", 48, (("select3_1", "cat_conv3_1"), ("select3_2", "cat_conv3_2"), ("select3_3", "cat_conv3_3")),
     "upconv3", "c4", "conv3", "c3"),
    (1, "up2", 32, (("select2_1", "cat_conv2_1"), ("select2_2", "cat_conv2_2")), "upconv2", "c3", "conv2", "c2"),
    (0, "up1", 30, (("select1_1", "in9"), ("select1_2", "cat_conv1_1"), ("select1_3", "cat_conv1_2")),
     "upconv1", "c2", "conv1", "c1"),
)
RBUF = {"upconv4": "r4", "upconv3": "r3", "upconv2": "r2", "upconv1": "r1"}
# convs whose input is itself trainable: they need a data gradient (the select convs and upconv4 read frozen
# VGG features / the network input)
DGRAD = ("output", "conv1", "conv2", "conv3", "conv4", "upconv1", "upconv2", "upconv3")
BN_WIDTH = {lv[4]: lv[2] for lv in LEVELS}


def param_layout():
    """Flat f32 layout of the trainable variables in TF creation order (unet_simple.py:119-142): per scope the
    filter [3,3,cin,cout], the bias (new_conv only), then bn/beta and bn/gamma.  -> [(scope, kind, offset, shape)]"""
    out, off = [], 0
    for name, cin, cout in NEW_CONVS:
        ents = [("w", (3, 3, cin, cout))]
        if not name.startswith("upconv"):
            ents.append(("b", (cout,)))
        c = BN_WIDTH.get(name, cout)
        ents += [("beta", (c,)), ("gamma", (c,))]
        for kind, shape in ents:
            out.append((name, kind, off, shape))
            off += int(np.prod(shape))
    return out, off


class TrainerBase:
    """What the training steps of train.py (video_procedure / simple_procedure) and small_train.py
    (small_training) share: the flat f32 parameter / gradient / Adam-slot buffers, batch statistics with optional
    SyncBN, the BN backward, the DDP exchange and tf.train.AdamOptimizer's update."""

    def _init_flat(self, layout, n, lr, beta1, beta2, epsilon, sync_bn):
        self.lr, self.beta1, self.beta2, self.epsilon = lr, beta1, beta2, epsilon
        # SyncBN: batch statistics (and their gradient sums) over every replica's batch, as the single-device
        # reference normalises its whole batch; one small all-reduce per BN layer in the forward and one in the
        # backward.  Off: per-replica statistics (plain DDP)
        self.sync_bn = bool(sync_bn) and parallel.world_size() > 1
        self.layout = layout
        dev = self.device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.P, self.G = {}, {}
        for scope, kind, off, shape in layout:
            self.P[scope, kind] = self.flat[off:off + int(np.prod(shape))].view(shape)
            self.G[scope, kind] = self.grad[off:off + int(np.prod(shape))].view(shape)
        self.t = 0
        self._b1p = np.float32(1.0)
        self._b2p = np.float32(1.0)
        # SyncBN: every BN layer's global pixel count from its forward all-reduce (device f64), by mean buffer
        self._gcount = {}

    def _stats(self, x, mean, var):
        """Batch mean / biased variance of x's channels; SyncBN: over every replica's pixels (count-weighted, the
        second moment combined in float64 so the per-replica variances do not cancel)."""
        ops.bn_stats(x, mean, var)
        if self.sync_bn:
            m = float(x.shape[0] * x.shape[1] * x.shape[2])
            md = mean.double()
            t = torch.stack([md * m, (var.double() + md * md) * m, torch.full_like(md, m)])
            parallel.allreduce_sum(t)
            gm = t[0] / t[2]
            mean.copy_(gm)
            var.copy_((t[1] / t[2] - gm * gm).clamp_min(0.0))
            # every replica's pixels, summed by the same collective: the count the backward divides by.  Taken per
            # step and per layer from this all-reduce (never cached on a local key: replicas may change their batch
            # independently, e.g. an uneven last shard), and kept on the device (no host sync, capturable)
            self._gcount[mean.data_ptr()] = t[2, :1]

    def _bn_backward(self, x, dy, mask, mean, var, scope, dx, dx2=None, dbias=None):
        """BN(+relu mask) backward: dx, dgamma / dbeta (local sums, DDP averages them) and optionally the conv-bias
        gradient.  SyncBN: the local channel sums are all-reduced and the input gradient uses the global ones over
        the global pixel count — the count the forward's statistics all-reduce summed for this layer (replicas may
        hold different batch sizes or frame sizes, e.g. an uneven last shard)."""
        gamma, dgamma, dbeta = self.P[scope, "gamma"], self.G[scope, "gamma"], self.G[scope, "beta"]
        if not self.sync_bn:
            return ops.bn_backward(x, dy, mask, mean, var, gamma, EPS, dx=dx, dgamma=dgamma, dbeta=dbeta, dx2=dx2,
                                   dbias=dbias)
        ops.bn_backward(x, dy, mask, mean, var, gamma, EPS, dgamma=dgamma, dbeta=dbeta)
        sums = torch.cat([dbeta, dgamma])
        parallel.allreduce_sum(sums)
        c = dbeta.numel()
        # the global sums as means over the global count (device division: the kernel then divides by 1)
        means = (sums.double() / self._gcount[mean.data_ptr()]).float()
        ops.bn_backward_apply(x, dy, mask, mean, var, gamma, means[:c], means[c:], 1, dx, EPS, dx2=dx2)
        if dbias is not None:  # the conv bias's gradient = channel sum of this replica's dx
            ops.bn_backward(None, dx, None, None, None, None, EPS, dbeta=dbias)
        return dx

    def apply_gradients(self):
        """DDP gradient all-reduce + tf.train.AdamOptimizer step over the flat buffer, then re-pack the filters."""
        scale = parallel.allreduce_grads(self.grad)
        self.t += 1
        # TF keeps beta1_power / beta2_power as f32 variables multiplied once per step (adam.py _finish)
        self._b1p = np.float32(self._b1p * np.float32(self.beta1))
        self._b2p = np.float32(self._b2p * np.float32(self.beta2))
        one = np.float32(1.0)
        lr_t = np.float32(np.float32(self.lr) * np.sqrt(one - self._b2p) / (one - self._b1p))
        ops.adam_tf(self.flat, self.m, self.v, self.grad, lr_t, self.beta1, self.beta2, self.epsilon, scale)
        self._refresh_packs()


class VideoTrainer(TrainerBase):
    """train.video_procedure's iteration on device (also simple_procedure's: pass diff = cmp - bg as ``warped``)."""

    # the side streams: "pool" (torch pool streams, whatever hardware queue HIP gives them) or "probe" (pool streams
    # checked to run beside the caller's stream, ops.concurrent_streams; A/B)
    side_kind = "pool"

    def __init__(self, vgg16_npy_path=None, dtype="fp32", device="cuda", params=None, bn=None, lr=1e-3,
                 beta1=0.9, beta2=0.999, epsilon=1e-8, sync_bn=False, streams=3, stream_priority=0,
                 wgrad_stream=True):
        self.vgg = vgg16_npy_path if isinstance(vgg16_npy_path, Vgg16) else Vgg16(vgg16_npy_path, dtype, device)
        self.model = UNetSimple(self.vgg, True, dtype, device, params)
        self.device = self.model.device
        layout, n = param_layout()
        # (SyncBN = the single-device reference's statistics over its whole batch: unet_simple.py:25,41; params.py:8)
        self._init_flat(layout, n, lr, beta1, beta2, epsilon, sync_bn)
        # the select convs (unet_simple.py:120-139) read only the frozen towers' features and feed only their
        # level's concat: their chains (conv -> BN forward; BN backward -> filter gradient) run on `streams` side
        # streams beside the decoder chain, whose small deep-level kernels leave most of the chip idle.  Same
        # kernels, same arithmetic (bit-identical); events order them, also inside a captured graph.  SyncBN keeps
        # one stream (its collectives stay in one issue order)
        dev_ = torch.device(device)
        probe = self.side_kind == "probe" and stream_priority == 0
        nside = 0 if self.sync_bn or streams < 1 or dev_.type != "cuda" else int(streams)
        pool = ops.concurrent_streams(dev_, nside + (1 if nside and wgrad_stream else 0)) if probe and nside else None
        self._side = pool[:nside] if pool else \
            [torch.cuda.Stream(device=dev_, priority=stream_priority) for _ in range(nside)]
        # the decoder chain's own filter gradients (output, conv*, upconv*) are leaves too: with side streams they run
        # on one more, beside the chain's BN backward -> data-gradient convs, joined before the update
        self._wside = None
        if self._side and wgrad_stream:
            self._wside = pool[nside] if pool else torch.cuda.Stream(device=dev_, priority=stream_priority)
        self._capture_origin = None  # the stream a TrainGraph capture began on (see _check_capture_fork)
        dev = self.device
        # move the freshly drawn variables into the flat buffer and alias every consumer onto it
        for scope, pc in self.model.convs.items():
            self.P[scope, "w"].copy_(pc.w_hwio)
            pc.w_hwio = self.P[scope, "w"]
            if (scope, "b") in self.P:
                self.P[scope, "b"].copy_(pc.bias)
                pc.bias = self.P[scope, "b"]
        for scope, bnl in self.model.bn.items():
            if bn is not None and scope in bn:
                bnl.set(*bn[scope])
            self.P[scope, "gamma"].copy_(bnl.gamma)
            self.P[scope, "beta"].copy_(bnl.beta)
            bnl.gamma, bnl.beta = self.P[scope, "gamma"], self.P[scope, "beta"]
        self.model.relink_padded()
        # DDP: every replica starts from rank 0's variables.  init_conv draws from each process's global numpy RNG
        # (unet_simple.py:10-16), so without this the ranks would apply the averaged gradient to different models.
        # Every pack below is made from the broadcast buffer; the model's own packs (convs and the channel-padded
        # bf16 packs of UNetSimple.padded, drawn in UNetSimple.__init__) are re-made from it by _refresh_packs()
        if parallel.world_size() > 1:
            parallel.broadcast_tensors([self.flat], src=0)
        # data-gradient filters: flipped / transposed packs of the forward filters (fp32 path); the bf16 path packs
        # them bf16 with the gradient channels padded to 32, so the data-gradient convs run on the patch-reuse MFMA
        # kernel from bf16 copies of the gradients (bn_backward / relu_backward write them)
        self.dconv, self.dconv16 = {}, {}
        bf16 = self.model.dtype == torch.bfloat16
        for scope in DGRAD:
            pc = self.model.convs[scope]
            if bf16:  # f32 outputs of a multiple of 4 channels (the patch kernel's f32 epilogue): conv1's 30 -> 32
                cp = (pc.cout + 31) // 32 * 32
                self.dconv16[scope] = ops.PackedConv.from_source(pc.w_hwio, cp, (pc.cin + 3) // 4 * 4, "bf16",
                                                                 flip=True)
            else:
                self.dconv[scope] = ops.PackedConv.from_source(pc.w_hwio, pc.cout, pc.cin, "fp32", flip=True)
        # bf16: the patch-reuse conv kernel needs cout % 8 == 0, so the narrow new_convs (select2_* cout 4,
        # select1_* cout 2, output cout 1) run on zero-padded packs of their filters into 8-channel buffers
        self._padconv = {}
        if self.model.dtype == torch.bfloat16:
            for scope, cin, cout in NEW_CONVS:
                if cout % 8 and not scope.startswith("upconv"):
                    bp = torch.zeros((cout + 7) // 8 * 8, dtype=torch.float32, device=dev)
                    bp[:cout].copy_(self.P[scope, "b"])
                    pc = ops.PackedConv.from_source(self.P[scope, "w"], CIN_PAD.get(scope, cin), bp.numel(),
                                                    self.model.dtype, bias=bp)
                    self._padconv[scope] = (pc, bp, cout)
        # every filter re-pack of the optimizer step in one launch
        self._repack = ops.PackBatch(list(self.model.convs.values()) + list(self.dconv16.values()) +
                                     list(self.dconv.values()) + [v[0] for v in self._padconv.values()] +
                                     list(self.model.padded.values()))
        if parallel.world_size() > 1:
            self._refresh_packs()
        # filter gradients: bf16 operands on MFMA in the bf16 path, the exact-f32 kernel in the fp32 (parity) path
        self._mfma_wgrad = self.model.dtype == torch.bfloat16
        self._tb, self._key = None, None

    # ------------------------------------------------------------------------------------------- buffers
    def _train_buffers(self, n, h, w):
        if self._key == (n, h, w):
            return self._tb
        L = _levels(h, w)
        dev = self.device
        F = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], c), dtype=torch.float32, device=dev)  # noqa: E731
        tb = {"alpha": F(0, 1), "dlogit": F(0, 1), "loss": torch.zeros(3, dtype=torch.float32, device=dev)}
        st = lambda c: (torch.empty(c, dtype=torch.float32, device=dev),  # noqa: E731
                        torch.empty(c, dtype=torch.float32, device=dev))
        # pre-BN conv outputs stay f32 in both modes (the patch-reuse kernel writes f32 views): BN's x-hat = (z -
        # mean) * rstd loses most of bf16's 8 bits when a channel's mean is large against its spread, and the
        # gamma gradients (sum g * x-hat) with it (measured: 40-90 % error on the select1_* gammas with bf16 z)
        Z = lambda lv, c: torch.empty((n, L[lv][0], L[lv][1], c), dtype=torch.float32, device=dev)  # noqa: E731
        for lv, cat, width, sels, up, prev, conv, cout_key in LEVELS:
            for s, _ in sels + ((conv, None),):
                c = self.model.convs[s].cout
                if s in self._padconv:
                    tb["zfull_" + s] = Z(lv, (c + 7) // 8 * 8)
                    tb["z_" + s] = tb["zfull_" + s][..., :c]
                else:
                    tb["z_" + s] = Z(lv, c)
                tb["dz_" + s], tb["st_" + s] = F(lv, c), st(c)
            tb["st_" + up] = st(width)
            tb["dcatn_" + up] = F(lv, (width + 3) // 4 * 4)[..., :width]  # conv1's dgrad writes 32 (padded)
            tb["dcat_" + up] = F(lv, width)
            tb["du_" + up] = F(lv, self.model.convs[up].cout)
            # the select convs' masked gradients, split off the concat's in the same relu-backward pass
            tb["gsel_" + up] = F(lv, sum(self.model.convs[s].cout for s, _ in sels))
            if up in DGRAD:
                tb["dr_" + up] = F(lv, self.model.convs[up].cin)
                tb["dprev_" + up] = F(lv + 1, self.model.convs[up].cin)
            tb["dout_" + conv] = F(lv, self.model.convs[conv].cout)
        # the output conv's dz feeds the data-gradient conv, whose input views need channels padded to 8
        if "output" in self._padconv:
            tb["zfull_output"] = Z(0, 8)
            tb["z_output"] = tb["zfull_output"][..., :1]
        else:
            tb["z_output"] = F(0, 1)
        tb["st_output"] = st(1)
        tb["dz_output"] = torch.zeros((n, h, w, 8), dtype=torch.float32, device=dev)[..., :1]
        # bf16 copies of the gradients the data-gradient convs read, channels zero-padded to 32
        for scope, pc16 in self.dconv16.items():
            lv = 0 if scope == "output" else {"conv1": 0, "conv2": 1, "conv3": 2, "conv4": 3, "upconv1": 0,
                                              "upconv2": 1, "upconv3": 2}[scope]
            tb["g16_" + scope] = torch.zeros((n, L[lv][0], L[lv][1], pc16.cin), dtype=torch.bfloat16, device=dev)
        self._tb, self._key = tb, (n, h, w)
        return tb

    @staticmethod
    def _src(b, key):
        return b["in9"][..., :9] if key == "in9" else b[key]

    # ------------------------------------------------------------------------------------------- forward
    def _new_conv(self, x, scope, act, out, tb):
        """new_conv (unet_simple.py:19-27) with batch statistics, then ``act``; keeps z and (mean, var)."""
        z, (mean, var) = tb["z_" + scope], tb["st_" + scope]
        if scope in self._padconv:
            pc = self._padconv[scope][0]
            ops.conv3x3(ops.widen(x, pc.cin), pc, "none", out=tb["zfull_" + scope], affine=False, splitk=True)
        else:
            pc, x = self.model.conv(scope, x)
            ops.conv3x3(x, pc, "none", out=z, affine=False, splitk=True)
        self._stats(z, mean, var)
        bnl = self.model.bn[scope]
        ops.bn_apply(z, mean, var, bnl.gamma, bnl.beta, EPS, act, out=out)

    in9_side = True  # the 9-channel input concat converted on a side stream beside the towers (A/B: False)
    interleave_issue = True  # forward: queue level k+1's select chains after level k's upconv (A/B: False)

    def _check_capture_fork(self):
        """The side-stream fork of forward / backward is legal inside a HIP graph capture only from the stream the
        capture began on.  Forking from a stream that was itself forked inside the capture (e.g. a pass moved onto
        its own high-priority stream) is a nested fork, and ROCm 7's hipStreamEndCapture segfaults on a captured
        nested fork (tools/capture_probe.py: capture -> s1 -> s2 -> joined back dies in capture_end with SIGSEGV,
        with or without stream priorities; a single-level fork is fine).  That was the r04 segfault under
        test_train_graph_step_equals_eager.  Refused here with an exception instead: capture through
        VideoTrainer.capture() (which records the origin), or build the trainer with streams=0."""
        if not self._side or not torch.cuda.is_current_stream_capturing():
            return
        if self._capture_origin is None or torch.cuda.current_stream(self.device) != self._capture_origin:
            raise RuntimeError("VideoTrainer: side-stream fork inside a HIP graph capture from a stream other than "
                               "the capture's origin (a nested fork, which segfaults hipStreamEndCapture on ROCm); "
                               "capture with VideoTrainer.capture() on the caller's stream, or use streams=0")

    def forward(self, cmp, bg, warped):
        self._check_capture_fork()
        m = self.model
        xs = [t if isinstance(t, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(t, np.float32))
              for t in (cmp, bg, warped)]
        xs = [t.to(self.device, torch.float32) for t in xs]
        n, h, w, _ = xs[0].shape
        b = m._buffers(n, h, w)
        tb = self._train_buffers(n, h, w)
        L = _levels(h, w)
        main = torch.cuda.current_stream(self.device) if self._side else None
        ev_in9 = None
        if self._side and self.in9_side:
            # the 9-channel concat is first read by the level-0 select convs, after the towers: its three converts
            # (~85 us of strided 3-channel writes) run on a side stream beside the towers instead of ahead of them
            self._side[0].wait_stream(main)
            with torch.cuda.stream(self._side[0]):
                m.load_in9(b, xs)
            ev_in9 = torch.cuda.Event()
            ev_in9.record(self._side[0])
            m.load_towers(b, xs)
        else:
            m.load_inputs(b, xs)
        m._towers(b)
        if ev_in9 is not None:
            main.wait_event(ev_in9)
        done = {}

        def queue_selects(lv, cat, width, sels):  # one level's select chains on the side streams
            c, off, done[lv] = b[cat][..., :width], 0, []
            for i, (s, src) in enumerate(sels):
                co = m.convs[s].cout
                st = self._side[i % len(self._side)]
                with torch.cuda.stream(st):
                    self._new_conv(self._src(b, src), s, "relu", c[..., off:off + co], tb)
                ev = torch.cuda.Event()
                ev.record(st)
                done[lv].append(ev)
                off += co

        # the select chains go on the side streams right after the towers.  interleave_issue: the host queues level
        # k+1's chains after the decoder's level-k resize + upconv instead of all levels' chains first, so the main
        # stream has work queued while the host issues the ~40 side launches (~0.4 ms of host time after the towers
        # with the decoder idle)
        ahead = self._side and self.interleave_issue
        if self._side:
            for st in self._side:
                st.wait_stream(main)
            for k, (lv, cat, width, sels, *_rest) in enumerate(LEVELS):
                if not ahead or k == 0:
                    queue_selects(lv, cat, width, sels)
        for k, (lv, cat, width, sels, up, prev, conv, out_key) in enumerate(LEVELS):
            c, off = b[cat][..., :width], 0
            for s, src in sels:
                co = m.convs[s].cout
                if not self._side:
                    self._new_conv(self._src(b, src), s, "relu", c[..., off:off + co], tb)
                off += co
            # upconv_concat (unet_simple.py:30-42): resize -> conv (no bias) -> relu -> concat -> BN
            r = b[RBUF[up]]
            if isinstance(r, ops.SourceConcat):  # upconv4 on the towers' conv5_3 (tower-major)
                ops.resize_bilinear(b[prev].base, L[lv], out=r.base)
            else:
                ops.resize_bilinear(b[prev], L[lv], out=r)
            pc, rx = m.conv(up, r)
            ops.conv3x3(rx, pc, "relu", out=c[..., off:width], affine=False, splitk=True)
            if ahead and k + 1 < len(LEVELS):
                nlv, ncat, nwidth, nsels = LEVELS[k + 1][:4]
                queue_selects(nlv, ncat, nwidth, nsels)
            for ev in done.get(lv, ()):
                main.wait_event(ev)
            mean, var = tb["st_" + up]
            self._stats(c, mean, var)
            ops.bn_apply(c, mean, var, m.bn[up].gamma, m.bn[up].beta, EPS, "none", out=b[cat + "n"][..., :width])
            self._new_conv(b[cat + "n"][..., :width], conv, "relu", b[out_key], tb)
        self._new_conv(b["c1"], "output", "sigmoid", tb["alpha"], tb)
        self.output = tb["alpha"]
        return self.output


    # ------------------------------------------------------------------------------------------- backward
    def _chain_wgrad(self, x_in, dz, dw):
        if self._wside is None:
            ops.conv_wgrad(x_in, dz, dw, mfma=self._mfma_wgrad)
            return
        self._wside.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._wside):
            ops.conv_wgrad(x_in, dz, dw, mfma=self._mfma_wgrad)

    def _conv_backward(self, scope, x_in, dy, mask, tb, dgrad_out=None):
        """BN(+relu) backward into dz, then bias / filter gradients, optionally the data gradient of x_in."""
        z, dz, (mean, var) = tb["z_" + scope], tb["dz_" + scope], tb["st_" + scope]
        g16 = tb["g16_" + scope] if dgrad_out is not None and scope in self.dconv16 else None
        self._bn_backward(z, dy, mask, mean, var, scope, dz, dx2=None if g16 is None else g16[..., :dz.shape[-1]],
                          dbias=self.G[scope, "b"])
        if dgrad_out is not None:  # the decoder chain (the select chains, on their side streams, pass None)
            self._chain_wgrad(x_in, dz, self.G[scope, "w"])
        else:
            ops.conv_wgrad(x_in, dz, self.G[scope, "w"], mfma=self._mfma_wgrad)
        if dgrad_out is not None:
            if g16 is not None:
                pc = self.dconv16[scope]
                ops.conv3x3(g16, pc, "none", out=ops.widen(dgrad_out, pc.cout), affine=False)
            else:
                ops.conv3x3(dz, self.dconv[scope], "none", out=dgrad_out, affine=False)
        return dz

    def backward(self, gt, raw_fg, bg, cmp):
        self._check_capture_fork()
        m, tb = self.model, self._tb
        b = m._ws
        main = torch.cuda.current_stream(self.device) if self._side else None
        ops.matting_loss_backward(tb["alpha"], gt, raw_fg, bg, cmp, out=tb["dlogit"])
        dout = tb["dout_conv1"]
        self._conv_backward("output", b["c1"], tb["dlogit"], None, tb, dgrad_out=dout)
        for lv, cat, width, sels, up, prev, conv, out_key in reversed(LEVELS):
            c, cn = b[cat][..., :width], b[cat + "n"][..., :width]
            self._conv_backward(conv, cn, dout, b[out_key], tb, dgrad_out=tb["dcatn_" + up])
            mean, var = tb["st_" + up]
            self._bn_backward(c, tb["dcatn_" + up], None, mean, var, up, tb["dcat_" + up])
            # one relu-backward pass over the concat: the select channels to gsel (dense, so each select's BN
            # backward reads its 2-16 channels without dragging the whole concat row through), the upconv's to du
            gsel, off = tb["gsel_" + up], 0
            g16 = tb.get("g16_" + up)
            nsel = gsel.shape[-1]
            du = ops.relu_backward(tb["dcat_" + up], c, tb["du_" + up],
                                   dx2=None if g16 is None else g16[..., :width - nsel], dx_lo=gsel)
            split = None
            if self._side:
                split = torch.cuda.Event()
                split.record(main)

            def chain_next(up=up, du=du, g16=g16):  # the decoder chain's next step: the upconv's data gradient
                if g16 is not None:
                    ops.conv3x3(g16, self.dconv16[up], "none", out=tb["dr_" + up], affine=False)
                else:
                    ops.conv3x3(du, self.dconv[up], "none", out=tb["dr_" + up], affine=False)
                return ops.resize_backward(tb["dr_" + up], tb["dprev_" + up])

            # interleave_issue: the host queues the upconv's filter gradient (its own stream) and the decoder chain's
            # next step before the select chains, so neither waits behind the ~15 select launches' host time
            first = self._wside is not None and self.interleave_issue
            if first:
                self._chain_wgrad(b[RBUF[up]], du, self.G[up, "w"])
                if up in DGRAD:
                    dout = chain_next()
            for i, (s, src) in enumerate(sels):
                co = m.convs[s].cout
                if self._side:  # leaves of the backward graph: beside the decoder chain, joined before the update
                    st = self._side[i % len(self._side)]
                    st.wait_event(split)
                    with torch.cuda.stream(st):
                        self._conv_backward(s, self._src(b, src), gsel[..., off:off + co], None, tb)
                else:
                    self._conv_backward(s, self._src(b, src), gsel[..., off:off + co], None, tb)
                off += co
            if not first:
                self._chain_wgrad(b[RBUF[up]], du, self.G[up, "w"])
                if up in DGRAD:
                    dout = chain_next()
        for st in self._side + ([self._wside] if self._wside is not None else []):
            main.wait_stream(st)  # every gradient is in place before the all-reduce / Adam that read them

    # ------------------------------------------------------------------------------------------- update

    def _refresh_packs(self):
        """Re-make every kernel-layout copy of the flat parameters (forward, data-gradient and channel-padded packs,
        the padded biases) after the flat buffer changed: the optimizer step, or rank 0's DDP broadcast."""
        self._repack()
        if self._padconv:  # the padded biases: one multi-tensor copy launch instead of one copy per conv
            torch._foreach_copy_([bp[:cout] for _, bp, cout in self._padconv.values()],
                                 [self.P[scope, "b"] for scope in self._padconv])

    def step(self, cmp, bg, warped, gt, raw_fg):
        """One training iteration; returns a new device tensor [loss, alpha_loss, compositional_loss] (pre-update),
        not aliased to the trainer's buffers."""
        self.forward(cmp, bg, warped)
        dev = lambda t: (t if isinstance(t, torch.Tensor) else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(t, np.float32))).to(self.device, torch.float32).contiguous()
        gt, raw_fg, bg_d, cmp_d = dev(gt), dev(raw_fg), dev(bg), dev(cmp)
        tb = self._tb
        loss = ops.matting_loss(tb["alpha"], gt, raw_fg, bg_d, cmp_d)
        tb["loss"].copy_(loss)
        self.grad.zero_()
        self.backward(gt, raw_fg, bg_d, cmp_d)
        self.apply_gradients()
        return tb["loss"].clone()

    def capture(self, cmp, bg, warped, gt, raw_fg):
        """Record one step's forward + loss and its backward over batches shaped like these as two HIP graphs
        (torch.cuda.CUDAGraph over the same C-ABI launches) -> a TrainGraph.  Its step() copies a batch in, replays
        both and runs the DDP exchange + Adam + re-pack eagerly (their host-side bias correction changes every
        step), so the ~300 launches of a step cost one host call each way.  The graphs read the trainer's
        parameters, packs and buffers in place, so updates made by apply_gradients are seen by the next replay."""
        return TrainGraph(self, cmp, bg, warped, gt, raw_fg)

    def params_numpy(self):
        """{scope: (w, b|None)} and {scope: (gamma, beta)} on the host (checkpointing / inference hand-off)."""
        conv = {s: (self.P[s, "w"].cpu().numpy(), self.P[s, "b"].cpu().numpy() if (s, "b") in self.P else None)
                for s, _, _ in NEW_CONVS}
        bn = {s: (self.P[s, "gamma"].cpu().numpy(), self.P[s, "beta"].cpu().numpy()) for s in self.model.bn}
        return conv, bn


class TrainGraph:
    """VideoTrainer.capture's result: ``step(cmp, bg, warped, gt, raw_fg)`` = VideoTrainer.step on graph replays;
    ``inputs`` are the static batch buffers the graphs read."""

    def __init__(self, trn, *batch):
        if trn.sync_bn and torch.distributed.get_backend() != "nccl":
            raise NotImplementedError("capture with sync_bn needs the nccl (RCCL) backend: gloo collectives are not "
                                      "graph-capturable")
        dev = trn.device
        self.trn = trn
        self.inputs = [(t if isinstance(t, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(t, np.float32)))
                       .to(dev, torch.float32).contiguous().clone() for t in batch]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # lazily built buffers / workspaces, no parameter update
            self._forward()
            self._backward()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        for t in trn._tb.values():  # allocated on the side stream, replayed on the caller's
            for u in (t if isinstance(t, tuple) else (t,)):
                if isinstance(u, torch.Tensor):
                    u.record_stream(torch.cuda.current_stream(dev))
        self.g_fwd, self.g_bwd = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.g_fwd):
                trn._capture_origin = torch.cuda.current_stream(dev)
                self._forward()
            with torch.cuda.graph(self.g_bwd):
                trn._capture_origin = torch.cuda.current_stream(dev)
                self._backward()
        finally:
            trn._capture_origin = None

    def _forward(self):
        cmp, bg, warped, gt, fg = self.inputs
        t = self.trn
        t.forward(cmp, bg, warped)
        t._tb["loss"].copy_(ops.matting_loss(t._tb["alpha"], gt, fg, bg, cmp))

    def _backward(self):
        cmp, bg, warped, gt, fg = self.inputs
        self.trn.grad.zero_()
        self.trn.backward(gt, fg, bg, cmp)

    def load(self, *batch):
        for dst, src in zip(self.inputs, batch):
            dst.copy_(src if isinstance(src, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(src, np.float32)))

    def step(self, *batch):
        """One training iteration on graph replays; returns [loss, alpha_loss, compositional_loss] (pre-update)."""
        if batch:
            self.load(*batch)
        self.g_fwd.replay()
        self.g_bwd.replay()
        self.trn.apply_gradients()
        return self.trn._tb["loss"].clone()

