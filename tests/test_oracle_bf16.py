"""CPU checks of oracle/bf16.py, the bf16-operand restatements the 1080p layer test (test_gpu_layers_1080p.py) uses."""

import numpy as np
import pytest
import torch

from bf16check import check_bf16, ulp_bf16
from oracle import bf16 as ob
from oracle import ops as oops


def test_bf16_round_matches_torch():
    rs = np.random.RandomState(0)
    a = np.concatenate([rs.normal(size=10000) * 10.0 ** rs.uniform(-30, 30, 10000),
                        [0.0, -0.0, 1.0, 1.00390625, 1.01171875, 2.0 ** -130, 3e38]])
    want = torch.from_numpy(a.astype(np.float32)).to(torch.bfloat16).double().numpy()
    assert np.array_equal(ob.bf16_round(a), want)


@pytest.mark.parametrize("shape", [(1, 5, 7, 3, 2), (2, 4, 4, 8, 5), (1, 1, 1, 4, 3), (1, 9, 2, 6, 4)])
def test_folded_upconv_is_resize_then_conv(shape):
    """unet.py:44-63's resize (TF1 legacy, exact 2x) -> conv3x3 SAME equals the folded phase-filter form with the
    replicate-clamped low-res frame and the unfused border, exactly (float64)."""
    n, h, w, cin, cout = shape
    rs = np.random.RandomState(h * w + cin)
    x = rs.normal(size=(n, h, w, cin))
    wt = rs.normal(size=(3, 3, cin, cout))
    ref = oops.conv3x3_same(oops.resize_bilinear_tf1(x, 2 * h, 2 * w), wt)
    got = ob.upconv2x_folded(x, wt, round_w=False)
    assert np.abs(got - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())


def test_folded_upconv_bf16_form_close():
    """The bf16 form (rounded folded filter, bf16 border resize) stays within bf16 precision of the exact value."""
    rs = np.random.RandomState(3)
    x = ob.bf16_round(np.abs(rs.normal(size=(1, 6, 9, 32))))
    wt = rs.normal(size=(3, 3, 32, 8)).astype(np.float32) * 0.1
    ref = oops.conv3x3_same(oops.resize_bilinear_tf1(x, 12, 18), wt.astype(np.float64))
    got = ob.upconv2x_folded(x, wt, round_w=True)
    assert np.abs(got - ref).max() <= 2e-2 * np.abs(ref).max()


def test_head_shares_sum_to_head_conv():
    rs = np.random.RandomState(4)
    y = rs.normal(size=(2, 7, 9, 16))
    hw = rs.normal(size=(3, 3, 16, 1))
    z = np.zeros_like(y)
    got = ob.head_from_shares(ob.head_shares(y, hw), ob.head_shares(z, hw), 0.25)
    want = oops.conv3x3_same(y, hw, np.array([0.25]))
    assert np.abs(got - want).max() <= 1e-12


def test_check_bf16_accepts_rounded_and_rejects_off_by_two():
    rs = np.random.RandomState(5)
    e = rs.normal(size=100000)
    g = ob.bf16_round(e)
    st = check_bf16("rounded", g, e)
    assert st["max_ulp"] <= 0.5 + 1e-6  # (f64 -> f32 -> bf16 double rounding)
    bad = g + 3 * ulp_bf16(e) * (np.arange(e.size) % 997 == 0)
    with pytest.raises(AssertionError):
        check_bf16("off", bad, e)
