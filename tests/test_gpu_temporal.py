"""BASELINE config 3 on the GPU: the fused warp + occlusion + refine-input pass (temporal.TemporalRefiner) against
the separate-op API and the CPU oracle.

* the fused pass's warped / corrected alpha is bit-identical to flow.warp_img -> flow.correct_alpha on the GPU,
  which the golden tests pin to the reference's own flow.py outputs (test_gpu_parity.py);
* the refine input channels are exactly [cmp, alpha, warped] (f32) or their bf16 rounding;
* 500x1200 (the flow.py demo size) and 1080p: the fp32 refine output (64-ch softmax) within 1e-4 max-abs of the
  numpy oracle (oracle.models.refine_forward on the same input) — the chain's size-independent properties
  (softmax rows sum to 1, occluded pixels carry warped alpha 0) at full size.
"""

import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"


def _case(h, w, seed=7):
    from oracle.flow import smooth_flow
    rs = np.random.RandomState(seed)
    bw = smooth_flow(h, w, seed=seed)
    fw = -smooth_flow(h, w, seed=seed)  # round trip closes ...
    yy, xx = np.mgrid[0:h, 0:w]
    occ = ((yy - 0.4 * h) ** 2 + (xx - 0.6 * w) ** 2) < (0.15 * min(h, w)) ** 2
    fw[occ] += 40.0  # ... except inside a disk: occluded (err > 15 px)
    yy, xx = np.mgrid[0:h, 0:w]
    prev = np.clip(1.3 - np.hypot((yy - h / 2) / (h / 3), (xx - w / 2) / (w / 4)), 0, 1).astype(np.float32)
    cur = np.clip(prev + rs.normal(0, 0.02, prev.shape), 0, 1).astype(np.float32)
    cmp = (rs.uniform(0, 255, (h, w, 3)) - np.array([103.939, 116.779, 123.68])).astype(np.float32)
    return prev, cur, cmp, bw.astype(np.float32), fw.astype(np.float32), occ


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("h,w", [(64, 96), (500, 1200)])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_input_equals_separate_ops(h, w, dtype):
    from vmatting import flow, temporal
    prev, cur, cmp, bw, fw, _ = _case(h, w)
    np.random.seed(3)
    tp = temporal.TemporalRefiner(dtype=dtype)
    x = tp.prepare_input(T(prev), T(cur), T(cmp), T(bw), T(fw))
    warped = flow.warp_img(T(prev), T(bw))
    flow.correct_alpha(T(bw), T(fw), warped)
    assert torch.equal(tp.warped, warped)
    want = torch.cat([T(cmp), T(cur)[..., None], warped[..., None]], -1)[None]
    want = want.to(x.dtype)
    assert torch.equal(x, want)
    pad = tp._bufs[(h, w)]["xin"][..., 5:]
    assert torch.count_nonzero(pad) == 0


@pytest.mark.parametrize("h,w", [(500, 1200), (1080, 1920)])
def test_temporal_refine_fp32_vs_oracle(h, w):
    from oracle import flow as oflow
    from oracle import models as om
    from vmatting import temporal
    prev, cur, cmp, bw, fw, occ = _case(h, w)
    np.random.seed(3)
    tp = temporal.TemporalRefiner(dtype="fp32")
    out = tp(T(prev), T(cur), T(cmp), T(bw), T(fw))
    torch.cuda.synchronize()
    warped = oflow.correct_alpha(bw, fw, oflow.warp_img(prev, bw), promote="numpy1").astype(np.float32)
    gw = tp.warped.cpu().numpy()
    assert np.abs(gw - warped).max() <= 1e-6  # the remap golden bound (test_gpu_parity.py)
    # occluded where the backward target lands in the disk where forward flow was perturbed
    assert np.array_equal(gw == 0, warped == 0) and (gw == 0).sum() > (occ.sum() // 2)
    x = np.concatenate([cmp, cur[..., None], warped[..., None]], -1)[None]
    ref = om.refine_forward(x, tp.refine.params, dtype=np.float32)["output"]
    got = out.cpu().numpy()
    err = float(np.abs(got - ref).max())
    print("config 3 %dx%d: fp32 refine softmax max-abs err vs oracle %.2e" % (h, w, err))
    assert err <= 1e-4  # north_star's fp32 bound (f32 summation order in a saturated 64-way softmax: ~2e-5)
    np.testing.assert_allclose(got.sum(-1), 1.0, atol=1e-5)


def test_temporal_refine_bf16_close_to_fp32():
    from vmatting import temporal
    prev, cur, cmp, bw, fw, _ = _case(540, 960)
    np.random.seed(3)
    tb = temporal.TemporalRefiner(dtype="bf16")
    ob = tb(T(prev), T(cur), T(cmp), T(bw), T(fw)).clone()
    np.random.seed(3)
    tf = temporal.TemporalRefiner(dtype="fp32")
    of = tf(T(prev), T(cur), T(cmp), T(bw), T(fw))
    # the refine logits are O(100) (mean-subtracted 0..255 inputs, He weights): bf16's ~0.4 % relative rounding moves
    # near-tied channels of the 64-way softmax a lot, so compare distributions, not a max-abs bound
    d = (ob - of).abs()
    agree = float((ob.argmax(-1) == of.argmax(-1)).float().mean())
    print("config 3 bf16 vs fp32 softmax: max-abs %.2e, mean-abs %.2e, argmax agreement %.4f"
          % (float(d.max()), float(d.mean()), agree))
    assert float(d.mean()) < 1e-2 and agree > 0.95
    np.testing.assert_allclose(ob.sum(-1).cpu().numpy(), 1.0, atol=1e-3)
    assert torch.equal(tb.warped, tf.warped)


@pytest.mark.parametrize("h,w", [(500, 1200), (1080, 1920)])
def test_temporal_refine_bf16_kernel_vs_oracle(h, w):
    """The TIMED bf16 config-3 refine (conv3x3_first_softmax_strip: refine conv4 + the 64-way softmax fused)
    against the oracle's conv + softmax in float64 on the same bf16-rounded input row and bf16-rounded filter (f32
    bias): only the f32 summation order and the device exp differ, so the probabilities stay within 1e-4 max-abs
    (north_star's bound) at full size; rows sum to 1."""
    from oracle import ops as oops
    from vmatting import _lib, temporal
    prev, cur, cmp, bw, fw, _ = _case(h, w)
    np.random.seed(3)
    tp = temporal.TemporalRefiner(dtype="bf16")
    out = tp(T(prev), T(cur), T(cmp), T(bw), T(fw))
    torch.cuda.synchronize()
    assert _lib.last_conv_kernel() == "vm::conv3x3_first_softmax_strip", _lib.last_conv_kernel()
    x = tp._bufs[(h, w)]["xin"][..., :5].float().cpu().numpy().astype(np.float64)  # the bf16 input row
    w4, b4 = tp.refine.params["conv4"]
    w4 = torch.from_numpy(np.ascontiguousarray(w4, np.float32)).to(torch.bfloat16).double().numpy()
    ref = oops.softmax_lastdim(oops.conv3x3_same(x, w4, np.asarray(b4, np.float64)))
    got = out.cpu().numpy()
    err = float(np.abs(got - ref).max())
    print("config 3 %dx%d: bf16 refine kernel max-abs err vs oracle (bf16 operands) %.2e" % (h, w, err))
    assert err <= 1e-4
    np.testing.assert_allclose(got.sum(-1), 1.0, atol=1e-5)


def test_temporal_index_error():
    from vmatting import temporal
    prev, cur, cmp, bw, fw, _ = _case(16, 20)
    bw[3, 4, 1] = -40.0  # i0 = 3 - 40 < -h: the reference's IndexError (flow.py:46)
    tp = temporal.TemporalRefiner(dtype="fp32")
    with pytest.raises(IndexError):
        tp(T(prev), T(cur), T(cmp), T(bw), T(fw))
    # the error flag is not re-zeroed per call: after the raise, an unchecked call over the bad flow and a checked
    # call over a good one must not report it; a checked call over the bad flow raises again
    _, _, _, bw_ok, _, _ = _case(16, 20)
    tp(T(prev), T(cur), T(cmp), T(bw_ok), T(fw))
    tp(T(prev), T(cur), T(cmp), T(bw), T(fw), check_index=False)
    tp(T(prev), T(cur), T(cmp), T(bw_ok), T(fw))
    with pytest.raises(IndexError):
        tp(T(prev), T(cur), T(cmp), T(bw), T(fw))


@pytest.mark.parametrize("n,h,w", [(1, 37, 70), (2, 8, 32), (1, 1, 1), (1, 135, 240), (1, 17, 33)])
def test_refine_softmax_kernel_matches_generic_epilogue(n, h, w):
    """conv3x3_first_softmax (register softmax over the 4 lanes holding a pixel's 64 logits, plain and
    nontemporal stores) against the generic conv kernel's LDS softmax epilogue on the same bf16 refine input:
    same bf16 products, f32 sums in another order -> probabilities within 1e-5, rows sum to 1, ragged tiles."""
    from vmatting import _lib, ops
    rs = np.random.RandomState(h * 131 + w)
    x = rs.uniform(-1, 1, size=(n, h, w, 8)).astype(np.float32)
    x[..., 5:] = 0.0
    pc = ops.PackedConv((rs.normal(size=(3, 3, 5, 64)) * 0.3).astype(np.float32),
                        rs.normal(size=64).astype(np.float32), "bf16")
    xb = T(x).to(torch.bfloat16)[..., :5]  # 5 channels in an 8-channel buffer, as the temporal input
    outs = {}
    try:
        for k in (0, 1, 2):
            _lib.set_option("softmax_kernel", k)
            outs[k] = ops.conv3x3(xb, pc, "softmax", out_dtype=torch.float32)
            name = _lib.last_conv_kernel()
            assert ("first_softmax" in name) == (k != 0), name
        for k in (3, 4, 5):  # the per-wave LDS transpose store forms (5: weights in LDS): same values
            _lib.set_option("softmax_kernel", k)
            assert torch.equal(ops.conv3x3(xb, pc, "softmax", out_dtype=torch.float32), outs[1]), k
        _lib.set_option("softmax_kernel", 6)  # wave strips (the default): bias-initialised sums, v_exp_f32
        outs[6] = ops.conv3x3(xb, pc, "softmax", out_dtype=torch.float32)
        assert _lib.last_conv_kernel() == "vm::conv3x3_first_softmax_strip"
        for blocks in (1, 3, 7):
            _lib.set_option("softmax_blocks", blocks)
            assert torch.equal(ops.conv3x3(xb, pc, "softmax", out_dtype=torch.float32), outs[6]), blocks
        _lib.set_option("softmax_blocks", 2048)
        _lib.set_option("softmax_kernel", 2)
        for blocks in (1, 3, 7):  # persistent walks with partial last rounds
            _lib.set_option("softmax_blocks", blocks)
            assert torch.equal(ops.conv3x3(xb, pc, "softmax", out_dtype=torch.float32), outs[2]), blocks
    finally:
        _lib.set_option("softmax_kernel", 6)
        _lib.set_option("softmax_blocks", 2048)
    ref = outs[0].cpu().numpy()
    for k in (1, 2, 6):
        got = outs[k].cpu().numpy()
        assert np.abs(got - ref).max() <= 1e-5, (k, np.abs(got - ref).max())
        np.testing.assert_allclose(got.sum(-1), 1.0, atol=1e-5)
    assert torch.equal(outs[1], outs[2])


@pytest.mark.parametrize("cin", [1, 3, 5, 8])
@pytest.mark.parametrize("n,h,w", [(1, 37, 70), (2, 8, 32), (1, 1, 1), (1, 135, 240)])
def test_refine_softmax_f32_kernel(n, h, w, cin):
    """conv3x3_first_softmax_f32 (compact-K exact-f32 MFMA conv + register softmax, the fp32 config-3 refine) against
    the generic f32 kernel's softmax epilogue and the float64 oracle: exact f32 products, f32 sums in another order
    -> within 5e-5 of the generic kernel and 1e-4 (north_star's bound) of float64; rows sum to 1; ragged tiles and
    partial persistent rounds."""
    from oracle import ops as oops
    from vmatting import _lib, ops
    rs = np.random.RandomState(h * 7 + w + cin)
    x = np.zeros((n, h, w, 8), np.float32)
    x[..., :cin] = rs.uniform(-30, 30, size=(n, h, w, cin))
    wt = (rs.normal(size=(3, 3, cin, 64)) * 0.3).astype(np.float32)
    b = rs.normal(size=64).astype(np.float32)
    pc = ops.PackedConv(wt, b, "fp32")
    xd = T(x)[..., :cin]
    try:
        got = ops.conv3x3(xd, pc, "softmax").clone()
        want = "vm::conv3x3_first_softmax_f32p<%d, 2, false, 0, 18>" % cin
        assert _lib.last_conv_kernel() == want, _lib.last_conv_kernel()
        _lib.set_option("softmax_blocks", 3)
        assert torch.equal(ops.conv3x3(xd, pc, "softmax"), got)  # persistent walk, partial last round
        # the pipelined kernel (next strip's MFMAs under this strip's softmax, direct stores) computes every output
        # exactly as the r03 one (same K order, same softmax expression); also its 4-waves-per-SIMD build
        _lib.set_option("softmax_blocks", 2048)
        for v in (0, 1, 2, 3, 5, 6):  # 0: the r03 kernel; 1..5 the pipelined one (3..5: store variants, cin 5);
            _lib.set_option("softmax_f32p", v)  # 6: its row-ring form
            assert torch.equal(ops.conv3x3(xd, pc, "softmax"), got), (v, _lib.last_conv_kernel())
            k = _lib.last_conv_kernel()
            assert ("softmax_f32p" in k) == (0 < v < 6) and ("softmax_f32r" in k) == (v == 6), (v, k)
        _lib.set_option("softmax_f32p", 4)
        _lib.set_option("softmax_kernel", 0)
        gen = ops.conv3x3(xd, pc, "softmax").clone()
        assert "first_softmax" not in _lib.last_conv_kernel()
    finally:
        _lib.set_option("softmax_kernel", 6)
        _lib.set_option("softmax_blocks", 2048)
        _lib.set_option("softmax_f32p", 4)
    ref = oops.softmax_lastdim(oops.conv3x3_same(x[..., :cin].astype(np.float64), wt.astype(np.float64),
                                                 b.astype(np.float64)))
    g = got.cpu().numpy()
    # logits reach |100| here (inputs +-30, 9*cin taps): f32 sums of either order sit ~1e-5 from the f64 softmax
    assert np.abs(g - gen.cpu().numpy()).max() <= 5e-5
    assert np.abs(g - ref).max() <= 1e-4, np.abs(g - ref).max()
    np.testing.assert_allclose(g.sum(-1), 1.0, atol=1e-5)


@pytest.mark.parametrize("cin", [1, 3, 5])
@pytest.mark.parametrize("n,h,w", [(1, 37, 70), (2, 8, 32), (1, 1, 1), (1, 135, 240)])
def test_refine_softmax_x6_kernel(n, h, w, cin):
    """The split-bf16 x6 form of the fp32 refine kernel (softmax_f32p 7: each f32 input / filter value split exactly
    into three bf16 parts, six products per term on the bf16 MFMA, f32 sums) at f32 accuracy: within 5e-5 of the
    exact-f32 MFMA kernel and 1e-4 (north_star's bound) of float64, rows sum to 1; ragged tiles, partial rounds."""
    from oracle import ops as oops
    from vmatting import _lib, ops
    rs = np.random.RandomState(h * 11 + w + cin)
    x = np.zeros((n, h, w, 8), np.float32)
    x[..., :cin] = rs.uniform(-30, 30, size=(n, h, w, cin))
    wt = (rs.normal(size=(3, 3, cin, 64)) * 0.3).astype(np.float32)
    b = rs.normal(size=64).astype(np.float32)
    pc = ops.PackedConv(wt, b, "fp32")
    xd = T(x)[..., :cin]
    try:
        f32 = ops.conv3x3(xd, pc, "softmax").clone()
        _lib.set_option("softmax_f32p", 7)
        got = ops.conv3x3(xd, pc, "softmax").clone()
        assert _lib.last_conv_kernel() == "vm::conv3x3_first_softmax_f32p<%d, 2, false, 0, 18, true>" % cin
        _lib.set_option("softmax_blocks", 3)
        assert torch.equal(ops.conv3x3(xd, pc, "softmax"), got)  # persistent walk, partial last round
    finally:
        _lib.set_option("softmax_blocks", 2048)
        _lib.set_option("softmax_f32p", 4)
    ref = oops.softmax_lastdim(oops.conv3x3_same(x[..., :cin].astype(np.float64), wt.astype(np.float64),
                                                 b.astype(np.float64)))
    g = got.cpu().numpy()
    assert np.abs(g - f32.cpu().numpy()).max() <= 5e-5, np.abs(g - f32.cpu().numpy()).max()
    assert np.abs(g - ref).max() <= 1e-4, np.abs(g - ref).max()
    np.testing.assert_allclose(g.sum(-1), 1.0, atol=1e-5)
