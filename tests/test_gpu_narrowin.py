"""Narrow-input conv kernel (conv3x3_narrowin: bf16, 8 or 16 tap-major input channels, <= 32 outputs) — UNetSmall's
convs (small.py:39-48: 6 -> 8, 8 -> 16, 16 -> 32, 16 -> 8 at 320^2 x 8 in the small_train step).

Against an f64 conv of the same bf16-rounded operands: max-abs error <= 1e-4 of the reference's max-abs for f32
outputs (f32 accumulation order only), one bf16 ulp for bf16 outputs.  The kernel chains the MFMAs over k in the
generic kernel's order with its epilogue, so it must equal conv3x3_mfma (narrowin_kernel=0) bit for bit.
"""

import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"


def _bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy()


def _ref(x, w, b, act):
    xt = torch.from_numpy(x.astype(np.float64)).permute(0, 3, 1, 2)
    wt = torch.from_numpy(w.astype(np.float64)).permute(3, 2, 0, 1)
    y = torch.nn.functional.conv2d(xt, wt, padding=1).permute(0, 2, 3, 1).numpy() + b
    if act == "relu":
        y = np.maximum(y, 0)
    elif act == "sigmoid":
        y = 1 / (1 + np.exp(-y))
    return y


def _run(x, pc, act, out, narrow):
    from vmatting import _lib, ops
    _lib.set_option("narrowin_kernel", 1 if narrow else 0)
    try:
        ops.conv3x3(x, pc, act, out=out, affine=False)
        k = _lib.last_conv_kernel()
    finally:
        _lib.set_option("narrowin_kernel", 1)
    return k


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 13, 37, 6, 8), (1, 5, 3, 8, 16), (3, 20, 41, 16, 32),
                                            (2, 33, 65, 16, 8), (1, 17, 30, 12, 20), (2, 9, 70, 8, 5),
                                            (8, 80, 80, 16, 32)])
@pytest.mark.parametrize("odt,act", [(torch.float32, "none"), (torch.bfloat16, "relu"), (torch.float32, "sigmoid")])
def test_narrowin_conv_vs_f64_and_generic(n, h, w, cin, cout, odt, act):
    from vmatting import ops
    rs = np.random.RandomState(cin * 7 + cout + h)
    cs = (cin + 7) // 8 * 8
    xb = np.zeros((n, h, w, cs), np.float32)
    xb[..., :cin] = _bf(rs.normal(size=(n, h, w, cin)))
    wt = _bf(rs.normal(size=(3, 3, cin, cout)) / np.sqrt(9 * cin))
    b = rs.normal(size=cout).astype(np.float32)
    pc = ops.PackedConv(wt, b, "bf16", DEV)
    x = torch.from_numpy(xb).to(DEV, torch.bfloat16)[..., :cin]
    ys = []
    for narrow in (True, False):
        out = torch.full((n, h, w, cout), 3.0, device=DEV, dtype=odt)
        k = _run(x, pc, act, out, narrow)
        assert k.startswith("vm::conv3x3_narrowin<") == narrow, k
        ys.append(out)
    assert torch.equal(ys[0], ys[1])
    want = _ref(xb[..., :cin], wt, b, act)
    got = ys[0].float().cpu().numpy()
    if odt == torch.float32:
        assert np.abs(got - want).max() <= 1e-4 * np.abs(want).max()
    else:
        assert np.abs(got - want).max() <= 2 ** -8 * np.abs(want).max() + 1e-6


def test_narrowin_conv_into_concat_view():
    """The small_train decoder's form: relu(conv) written into channels 8..15 of a 16-channel bf16 concat
    (small.py:19-20), the other channels untouched."""
    from vmatting import ops
    rs = np.random.RandomState(5)
    n, h, w = 2, 40, 48
    x = torch.from_numpy(_bf(rs.normal(size=(n, h, w, 16)))).to(DEV, torch.bfloat16)
    wt = _bf(rs.normal(size=(3, 3, 16, 8)) / 12)
    pc = ops.PackedConv(wt, None, "bf16", DEV)
    cats = []
    for narrow in (True, False):
        cat = torch.full((n, h, w, 16), 5.0, device=DEV, dtype=torch.bfloat16)
        k = _run(x, pc, "relu", cat[..., 8:], narrow)
        assert k.startswith("vm::conv3x3_narrowin<") == narrow, k
        cats.append(cat)
    assert torch.equal(cats[0], cats[1])
    assert torch.all(cats[0][..., :8] == 5.0)
    want = _ref(x.float().cpu().numpy(), wt, 0.0, "relu")
    assert np.abs(cats[0][..., 8:].float().cpu().numpy() - want).max() <= 2 ** -8 * np.abs(want).max() + 1e-6


@pytest.mark.parametrize("ngroup", [2, 4])
def test_patch_grouped_tile_order_bit_identical(ngroup):
    """ConvArgs::ngroup (the patch kernel's grouped output-tile order) only reorders the blocks: the bf16 UNetVideo
    forward equals the default order's bit for bit, with the grouping forced onto every patch launch."""
    from oracle.models import synthetic_vgg16
    from vmatting import _lib, unet
    rs = np.random.RandomState(1)
    x = rs.uniform(-100, 100, (1, 72, 100, 7)).astype(np.float32)
    outs = []
    for ng, cb in ((0, 4 << 20), (ngroup, 0)):
        _lib.set_option("ngroup", ng)
        _lib.set_option("cband_bytes", cb)
        try:
            np.random.seed(0)
            m = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16")
            m.build(x)
            torch.cuda.synchronize()
            outs.append(m.conv1_3.float().clone())
        finally:
            _lib.set_option("ngroup", 0)
            _lib.set_option("cband_bytes", 4 << 20)
    assert torch.equal(outs[0], outs[1])
