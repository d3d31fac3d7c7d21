"""BASELINE config 3 — the two-frame temporal path: flow warp + occlusion check + matte refinement.

The reference's pieces are flow.warp_img (flow.py:9-18), flow.correct_alpha (flow.py:36-65, chained after the
warp in flow.py's own demo, flow.py:69-77) and refine.RefineNet.build (refine.py:27-32); it never wires them
together (refine.py has no caller), so the chain is the build-defined one of SURVEY.md 8(a) a14: the refine
input is [composite B,G,R - VGG_MEAN, alpha_t, occlusion-corrected warped alpha_{t-1}] (Cin = 5).

gfx950 plan: ONE pass per pixel (vm_temporal_refine_input) does the warp, the forward/backward consistency
gather and writes the refine net's padded NHWC input row, so neither the warped alpha nor the concat exists as
a separate HBM round trip; then the refine conv with its 64-channel softmax fused into the epilogue.  The
separate-op API (flow.warp_img / correct_alpha / RefineNet.build) stays available and gives bit-identical
intermediate values (tests/test_gpu_temporal.py).
"""

import ctypes

import torch

from . import ops
from ._lib import check, lib, stream_handle
from .refine import RefineNet


def _f32c(t, shape, what):
    ops._require_gpu(t)
    t = t.contiguous().float()
    if tuple(t.shape) != tuple(shape):
        raise ValueError("%s must be %s, got %s" % (what, tuple(shape), tuple(t.shape)))
    return t


class TemporalRefiner:
    """``refiner(prev_alpha, alpha, cmp, backward, forward)`` -> RefineNet output [1, H, W, 64] f32 (softmax).

    prev_alpha, alpha: [H,W] f32 mattes of frames t-1 and t; cmp: [H,W,3] composite BGR - VGG_MEAN of frame t;
    backward / forward: [H,W,2] flows (reader.read_flow layout).  Attributes after a call: ``warped`` (the
    corrected warped alpha, [H,W]) and ``refine`` (the RefineNet, its ``conv4``/``output``)."""

    CIN = 5

    def __init__(self, refine=None, dtype="bf16", device="cuda", promote="numpy1", thresh=15.0):
        self.refine = refine if refine is not None else RefineNet(dtype, device)
        self.refine.prepare(self.CIN)
        self.dtype = self.refine.dtype
        self.device = self.refine.device
        self.promote = 0 if promote == "numpy1" else 1
        self.thresh = float(thresh)
        self._bufs = {}
        # the IndexError flag is zeroed when allocated and after a raised error; a call that does not read it
        # (check_index=False) leaves it unknown, and the next checked call zeroes it first (no fill launch per call)
        self._err_dirty = set()

    def _buffers(self, h, w):
        b = self._bufs.get((h, w))
        if b is None:
            dev = self.device
            b = {"xin": torch.empty((1, h, w, 8), dtype=self.dtype, device=dev),
                 "warped": torch.empty((h, w), dtype=torch.float32, device=dev),
                 "out": torch.empty((1, h, w, 64), dtype=torch.float32, device=dev),
                 "err": torch.zeros(1, dtype=torch.int32, device=dev)}
            self._bufs[(h, w)] = b
        return b

    def prepare_input(self, prev_alpha, alpha, cmp, backward, forward, check_index=True):
        """The fused warp + occlusion + concat pass alone; returns the [1,H,W,5] input view."""
        h, w = alpha.shape[-2:]
        prev_alpha = _f32c(prev_alpha, (h, w), "prev_alpha")
        alpha = _f32c(alpha, (h, w), "alpha")
        cmp = _f32c(cmp, (h, w, 3), "cmp")
        backward = _f32c(backward, (h, w, 2), "backward")
        forward = _f32c(forward, (h, w, 2), "forward")
        b = self._buffers(h, w)
        if check_index and (h, w) in self._err_dirty:
            b["err"].zero_()
            self._err_dirty.discard((h, w))
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        check(lib().vm_temporal_refine_input(P(prev_alpha), P(backward), P(forward), P(cmp), P(alpha), h, w,
                                             self.thresh, self.promote, P(b["xin"]), ops._DT[self.dtype],
                                             P(b["warped"]), P(b["err"]), stream_handle()), "temporal_refine_input")
        if not check_index:
            self._err_dirty.add((h, w))
        elif int(b["err"].item()) != 0:
            b["err"].zero_()
            raise IndexError("correct_alpha: a backward-flow target lies more than one frame outside the image "
                             "(the reference's numpy IndexError, flow.py:46)")
        self.warped = b["warped"]
        return b["xin"][..., :self.CIN]

    def __call__(self, prev_alpha, alpha, cmp, backward, forward, check_index=True):
        x = self.prepare_input(prev_alpha, alpha, cmp, backward, forward, check_index)
        b = self._bufs[tuple(x.shape[1:3])]
        return self.refine.forward_prepared(x, out=b["out"])

