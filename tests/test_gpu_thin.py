"""Narrow-cout conv kernel (conv3x3_thin: bf16, 2..16 output channels) against an f64 conv of the same
bf16-rounded operands — the select convs of unet_simple.py:153-168 (192..1536 channels -> 2..16).

Tolerance: max-abs error <= 1e-4 of the reference's max-abs for f32 outputs (f32 accumulation order only),
one bf16 ulp (2^-8 relative) for bf16 outputs.  Split-K (a workspace, splitk=True) must agree with the unsplit
launch to f32 rounding, and the kernel must agree with the generic MFMA kernels (thin_kernel=0).
"""

import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"


def _ref(x, w, b=None, scale=None, shift=None, act="none"):
    """f64 NHWC conv of the (already bf16-rounded) operands."""
    xt = torch.from_numpy(x.astype(np.float64)).permute(0, 3, 1, 2)
    wt = torch.from_numpy(w.astype(np.float64)).permute(3, 2, 0, 1)
    y = torch.nn.functional.conv2d(xt, wt, padding=1).permute(0, 2, 3, 1).numpy()
    if b is not None:
        y = y + b
    if scale is not None:
        y = y * scale + shift
    if act == "relu":
        y = np.maximum(y, 0)
    return y


def _bf(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(torch.bfloat16).float().numpy()


def _err(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 13, 37, 64, 2), (1, 5, 3, 32, 3), (3, 20, 20, 768, 8),
                                            (2, 9, 70, 192, 4), (1, 40, 40, 1536, 16), (2, 33, 65, 96, 5)])
@pytest.mark.parametrize("splitk", [False, True])
def test_thin_conv_f32_out(n, h, w, cin, cout, splitk):
    from vmatting import _lib, ops
    rs = np.random.RandomState(cin + cout + h)
    x = _bf(rs.normal(size=(n, h, w, cin)))
    wt = _bf(rs.normal(size=(3, 3, cin, cout)) / np.sqrt(9 * cin))
    b = rs.normal(size=cout).astype(np.float32)
    pc = ops.PackedConv(wt, b, "bf16", DEV)
    xd = torch.from_numpy(x).to(DEV, torch.bfloat16)
    y = ops.conv3x3(xd, pc, "none", out_dtype=torch.float32, affine=False, splitk=splitk)
    assert _lib.last_conv_kernel().startswith("vm::conv3x3_thin")
    assert _err(y.cpu().numpy(), _ref(x, wt, b)) <= 1e-4


def test_thin_conv_sources_views_affine_bf16():
    """Tower-major split sources, an unaligned f32 output view, and bf16 output with a folded affine + relu."""
    from vmatting import ops
    rs = np.random.RandomState(7)
    n, h, w, c, cout = 2, 17, 40, 64, 6
    base = _bf(rs.normal(size=(3 * n, h, w, c)))
    src = ops.SourceConcat(torch.from_numpy(base).to(DEV, torch.bfloat16), 3)
    xcat = np.concatenate([base[i * n:(i + 1) * n] for i in range(3)], -1)
    wt = _bf(rs.normal(size=(3, 3, 3 * c, cout)) / 20)
    b = rs.normal(size=cout).astype(np.float32)
    pc = ops.PackedConv(wt, b, "bf16", DEV)
    outb = torch.full((n, h, w, 11), 7.0, device=DEV)
    view = outb[..., 3:3 + cout]
    ops.conv3x3(src, pc, "none", out=view, affine=False, splitk=True)
    want = _ref(xcat, wt, b)
    got = outb.cpu().numpy()
    assert _err(got[..., 3:3 + cout], want) <= 1e-4
    assert np.all(got[..., :3] == 7.0) and np.all(got[..., 3 + cout:] == 7.0)
    sc = rs.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rs.normal(size=cout).astype(np.float32)
    y16 = ops.conv3x3(src, pc, "relu", affine=(torch.from_numpy(sc).to(DEV), torch.from_numpy(sh).to(DEV)))
    want16 = _ref(xcat, wt, b, sc, sh, "relu")
    assert np.abs(y16.float().cpu().numpy() - want16).max() <= 2 ** -8 * np.abs(want16).max() + 1e-6


def test_thin_conv_matches_generic_kernels():
    from vmatting import _lib, ops
    rs = np.random.RandomState(3)
    x = torch.from_numpy(rs.normal(size=(2, 24, 50, 384)).astype(np.float32)).to(DEV, torch.bfloat16)
    pc = ops.PackedConv(rs.normal(size=(3, 3, 384, 8)).astype(np.float32) / 50, None, "bf16", DEV)
    y = ops.conv3x3(x, pc, "none", out_dtype=torch.float32, affine=False)
    _lib.set_option("thin_kernel", 0)
    try:
        y0 = ops.conv3x3(x, pc, "none", out_dtype=torch.float32, affine=False)
        assert not _lib.last_conv_kernel().startswith("vm::conv3x3_thin")
    finally:
        _lib.set_option("thin_kernel", 1)
    assert _err(y.cpu().numpy(), y0.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("th", [8, 4, 16])
@pytest.mark.parametrize("n,h,w,cin,cout,splitk", [(8, 160, 160, 384, 4, False), (6, 80, 80, 768, 8, True),
                                                   (24, 40, 40, 192, 2, False)])
def test_thin_persistent_walk_bit_identical(th, n, h, w, cin, cout, splitk):
    """The persistent grid (blocks walk tiles blockIdx.x, +gridDim.x, ... with the next tile's first chunk in flight)
    equals one block per tile (thin_rounds 0) bit for bit, at sizes with many tiles per block, split-K included."""
    from vmatting import _lib, ops
    rs = np.random.RandomState(n + w + th)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(DEV, torch.bfloat16)
    pc = ops.PackedConv(rs.normal(size=(3, 3, cin, cout)).astype(np.float32) / 40, rs.normal(size=cout).astype(
        np.float32), "bf16", DEV)
    outs = []
    try:
        _lib.set_option("thin_th", th)
        for rounds in (1, 0, 2):
            _lib.set_option("thin_rounds", rounds)
            outs.append(ops.conv3x3(x, pc, "relu", out_dtype=torch.float32, affine=False, splitk=splitk))
            assert _lib.last_conv_kernel() == "vm::conv3x3_thin<%d, true>" % th
    finally:
        _lib.set_option("thin_rounds", 1)
        _lib.set_option("thin_th", 8)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("th", [8, 4, 16])
@pytest.mark.parametrize("n,h,w,cin,cout,splitk", [(8, 80, 80, 768, 8, False), (3, 37, 45, 96, 2, True),
                                                   (2, 40, 40, 1536, 16, True)])
def test_thin_row_reuse_bit_identical(th, n, h, w, cin, cout, splitk):
    """r04: thin_chunk reads each patch row's pixel fragments once for all the output rows they reach; per
    accumulator the MFMAs still run taps 0..8 in order, so the outputs equal the tap-major loop's bit for bit."""
    from vmatting import _lib, ops
    rs = np.random.RandomState(n + cin + th)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(DEV, torch.bfloat16)
    pc = ops.PackedConv(rs.normal(size=(3, 3, cin, cout)).astype(np.float32) / 40, rs.normal(size=cout).astype(
        np.float32), "bf16", DEV)
    outs = []
    try:
        _lib.set_option("thin_th", th)
        for rr in (0, 1):
            _lib.set_option("thin_rowreuse", rr)
            outs.append(ops.conv3x3(x, pc, "none", out_dtype=torch.float32, affine=False, splitk=splitk))
            assert _lib.last_conv_kernel() == "vm::conv3x3_thin<%d, %s>" % (th, "true" if rr else "false")
    finally:
        _lib.set_option("thin_rowreuse", 1)
        _lib.set_option("thin_th", 8)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("n,h,w,cin,cout,splitk", [(8, 320, 320, 192, 2, False), (8, 80, 80, 768, 8, True),
                                                   (3, 37, 45, 96, 4, False)])
def test_thin_xcd_walk_bit_identical(n, h, w, cin, cout, splitk):
    """r04: the XCD-banded tile walk (each XCD's blocks take a contiguous eighth of the tiles) computes every tile
    exactly as the round-robin walk: bit-identical outputs."""
    from vmatting import _lib, ops
    rs = np.random.RandomState(n + cin + w)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(DEV, torch.bfloat16)
    pc = ops.PackedConv(rs.normal(size=(3, 3, cin, cout)).astype(np.float32) / 40, rs.normal(size=cout).astype(
        np.float32), "bf16", DEV)
    outs = []
    try:
        for tw in (0, 1):
            _lib.set_option("thin_twalk", tw)
            outs.append(ops.conv3x3(x, pc, "none", out_dtype=torch.float32, affine=False, splitk=splitk))
            assert _lib.last_conv_kernel().startswith("vm::conv3x3_thin<")
    finally:
        _lib.set_option("thin_twalk", 1)
    assert torch.equal(outs[0], outs[1])
