"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference goldens.

Tolerances (north_star: alpha within 1e-4 max-abs of the CPU reference, fp32):
  * fp32 compute path: alpha max-abs <= 1e-4; logits within 1e-4 relative (+1e-4 abs).
  * bf16 compute path: per-kernel relative error <= 2e-2 (bf16 inputs, f32 accumulate);
    whole-network alpha error is reported and bounded loosely (documented in DESIGN.md).
  * integer / index work (warp_bgr, correct_alpha): bit-exact.
"""

import numpy as np
import pytest
import torch

from bf16check import abs_conv_at, check_bf16
from conftest import golden, gpu_available
from oracle import bf16 as ob
from oracle import flow as oflow
from oracle import models as om
from oracle import ops as oops

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

VGG_MEAN = np.array(oops.VGG_MEAN)
DEV = "cuda"


def T(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def H(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


def test_native_library_is_the_compute_path():
    import vmatting._lib as L
    lib = L.lib()
    assert lib.vm_abi_version() == 1
    import os
    maps = open("/proc/self/maps").read()
    assert os.path.basename(L.LIB_PATH) in maps


# ----------------------------------------------------------------------------- single ops

CONV_CASES = [  # n, h, w, cin, cout, coff_in, act
    (1, 9, 13, 3, 64, 0, "relu"), (2, 11, 7, 7, 64, 0, "relu"), (1, 17, 19, 64, 64, 0, "relu"),
    (1, 8, 40, 64, 128, 0, "none"), (1, 6, 10, 128, 256, 0, "relu"), (1, 5, 6, 512, 512, 0, "relu"),
    (1, 5, 7, 1024, 512, 0, "none"), (1, 12, 12, 9, 2, 0, "relu"), (2, 10, 9, 30, 32, 0, "relu"),
    (1, 13, 21, 128, 1, 0, "sigmoid"), (1, 9, 9, 96, 48, 0, "relu"), (1, 7, 5, 256, 128, 128, "relu"),
    (1, 15, 16, 5, 64, 0, "softmax"), (1, 4, 4, 1536, 16, 0, "relu"), (3, 33, 47, 32, 24, 0, "relu"),
    (2, 10, 17, 128, 1, 8, "sigmoid"), (1, 6, 9, 64, 1, 0, "none"), (1, 3, 8, 256, 1, 0, "relu"),
]


@pytest.fixture(params=["regstage", "lds_dma", "patch"])
def conv_kernel(request):
    """Run a test once per conv kernel: 1 = register-staged, 2 = LDS-DMA pipelined (forced even on small grids),
    3 = patch-reuse kernel (bf16 output only; other cases fall back to the auto choice)."""
    from vmatting import _lib
    _lib.set_option("conv_kernel", {"regstage": 1, "lds_dma": 2, "patch": 3}[request.param])
    yield request.param
    _lib.set_option("conv_kernel", 0)


@pytest.mark.parametrize("cfg", [19, 22, 25, 30])  # every tiling the shipped dispatcher can pick
@pytest.mark.parametrize("case", [(1, 9, 33, 64, 64, "relu"), (2, 17, 70, 128, 128, "none"), (1, 20, 45, 96, 192, "relu"),
                                  (1, 8, 32, 32, 64, "sigmoid"), (1, 3, 5, 256, 128, "relu")])
def test_patch_kernel_configs(case, cfg):
    """Every patch-kernel tiling vs the oracle on bf16-rounded operands (bf16 output), partial tiles included."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, act = case
    rs = np.random.RandomState(cin + cout + h)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16)
    wt = torch.from_numpy((rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32))
    wt = wt.to(torch.bfloat16).float().numpy()
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    _lib.set_option("conv_kernel", 3)
    _lib.set_option("patch_cfg", cfg)
    try:
        y = ops.conv3x3(x.to(DEV), pc, act)
        name = _lib.last_conv_kernel()
    finally:
        _lib.set_option("conv_kernel", 0)
        _lib.set_option("patch_cfg", 0)
    assert name.startswith("vm::conv3x3_patch<"), name
    x64 = x.float().numpy().astype(np.float64)
    ref = oops.conv3x3_same(x64, wt.astype(np.float64)) + b
    ref = {"relu": oops.relu, "sigmoid": oops.sigmoid}.get(act, lambda v: v)(ref)
    # the bf16 rounding bound: >= 99.99 % within 1 ulp, all within 2 ulp or the f32 summation bound
    check_bf16("patch cfg %d" % cfg, H(y), ref, 9 * cin, lambda idx: abs_conv_at(x64, wt, b, idx, ref.shape))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3x3_vs_oracle(case, dtype, conv_kernel):
    from vmatting import ops
    n, h, w, cin, cout, coff, act = case
    rs = np.random.RandomState(cin * 7 + cout)
    x = rs.normal(size=(n, h, w, cin)).astype(np.float32)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    b = rs.normal(size=cout).astype(np.float32) * 0.1
    sc = rs.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rs.normal(size=cout).astype(np.float32) * 0.1
    tdt = ops.TORCH_DTYPE[dtype]
    if dtype == "bf16":  # compare against the oracle on the bf16-rounded operands
        x = torch.from_numpy(x).to(torch.bfloat16).float().numpy()
        wt = torch.from_numpy(wt).to(torch.bfloat16).float().numpy()
    cpad = (cin + 7) // 8 * 8
    buf = torch.zeros((n, h, w, coff + cpad + 8), dtype=tdt, device=DEV)
    buf[..., coff:coff + cin] = T(x, tdt)
    pc = ops.PackedConv(wt, b, tdt, DEV, scale=sc, shift=sh)
    y = ops.conv3x3(buf[..., coff:coff + cin], pc, act, out_dtype=torch.float32)
    ref = (oops.conv3x3_same(x.astype(np.float64), wt.astype(np.float64)) + b) * sc + sh
    ref = {"relu": oops.relu, "sigmoid": oops.sigmoid, "softmax": oops.softmax_lastdim}.get(act, lambda v: v)(ref)
    tol = 1e-5 if dtype == "fp32" else 3e-3
    assert relerr(H(y), ref) < tol, relerr(H(y), ref)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("shape", [(2, 19, 37, 128), (1, 9, 70, 64), (1, 17, 130, 8), (1, 5, 11, 256)])
def test_head_kernels_agree(dtype, shape):
    """cout == 1: the MFMA tap-GEMM, register-strip and generic per-pixel kernels agree with each other and the
    oracle (f32: up to summation order)."""
    from vmatting import _lib, ops
    tdt = ops.TORCH_DTYPE[dtype]
    rs = np.random.RandomState(5)
    xf = rs.normal(size=shape).astype(np.float32)
    wt = (rs.normal(size=(3, 3, shape[-1], 1)) * 0.03).astype(np.float32)
    if dtype == "bf16":
        xf = torch.from_numpy(xf).to(torch.bfloat16).float().numpy()
        wt = torch.from_numpy(wt).to(torch.bfloat16).float().numpy()
    x = T(xf, tdt)
    pc = ops.PackedConv(wt, np.array([0.1], np.float32), tdt, DEV)
    ref = oops.sigmoid(oops.conv3x3_same(xf.astype(np.float64), wt.astype(np.float64)) + 0.1)
    outs, names = [], []
    try:
        for k in (0, 1, 2):
            _lib.set_option("head_kernel", k)
            outs.append(H(ops.conv3x3(x, pc, "sigmoid", out_dtype=torch.float32)))
            names.append(_lib.last_conv_kernel())
    finally:
        _lib.set_option("head_kernel", 0)
    mfma_ok = shape[-1] <= (128 if dtype == "fp32" else 256)  # MFMA head holds <= 8 k-steps of weights
    assert ("head_mfma" in names[0]) == mfma_ok and names[1].startswith("vm::conv3x3_head<"), names
    for y in outs:
        assert np.abs(y - ref).max() < (2e-6 if dtype == "fp32" else 2e-5), np.abs(y - ref).max()


@pytest.mark.parametrize("case", [(1, 9, 13, 3, 64, "relu"), (2, 11, 70, 7, 64, "relu"), (1, 33, 65, 8, 128, "none"),
                                  (1, 1, 1, 7, 64, "relu"), (1, 16, 32, 6, 64, "sigmoid"),
                                  (4, 160, 330, 3, 64, "relu"), (2, 203, 250, 8, 128, "none")])
def test_first_layer_kernel(case):
    """cin <= 8 with bf16 output dispatches conv3x3_first (4 taps x 8 channels per MFMA K-step).  The last two cases
    have more tiles than resident blocks: the persistent walk (next patch in flight, weight-slice reload when the
    output-channel block changes, ragged tiles at both edges)."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, act = case
    rs = np.random.RandomState(cin * 31 + w)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32) * 40).to(torch.bfloat16)
    wt = torch.from_numpy((rs.normal(size=(3, 3, cin, cout)) * 0.02).astype(np.float32)).to(torch.bfloat16)
    wt = wt.float().numpy()
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    buf = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=DEV)
    buf[..., :cin] = x.to(DEV)
    y = ops.conv3x3(buf[..., :cin], pc, act)
    assert _lib.last_conv_kernel() == "vm::conv3x3_first"
    x64 = x.float().numpy().astype(np.float64)
    ref = oops.conv3x3_same(x64, wt.astype(np.float64)) + b
    ref = {"relu": oops.relu, "sigmoid": oops.sigmoid}.get(act, lambda v: v)(ref)
    check_bf16("first", H(y), ref, 9 * cin, lambda idx: abs_conv_at(x64, wt, b, idx, ref.shape))


@pytest.mark.parametrize("shape", [(1, 16, 64, 64, 64), (2, 17, 45, 64, 128), (1, 9, 33, 256, 256),
                                   (1, 135, 240, 32, 64), (1, 1, 1, 64, 64)])
@pytest.mark.parametrize("kernel", [0, 1])
def test_conv_fused_maxpool_matches_separate(shape, kernel):
    """vm_conv3x3_pool_nhwc: the pooled output equals vm_maxpool2x2 of the conv output bit for bit (odd sizes,
    batches, channel-slice outputs), and the conv output itself is unchanged; unsupported kernels fall back."""
    from vmatting import _lib, ops
    n, h, w, cin, cout = shape
    rs = np.random.RandomState(h * w + cin)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, (rs.normal(size=cout) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    _lib.set_option("conv_kernel", kernel)
    _lib.set_option("splitk_tiles", 0)  # the reference conv without split-K (same summation order as the fused one)
    try:
        cat = torch.zeros((n, h, w, 2 * cout), dtype=torch.bfloat16, device=DEV)
        pooled = torch.full((n, (h + 1) // 2, (w + 1) // 2, cout), 7.0, dtype=torch.bfloat16, device=DEV)
        ops.conv3x3(x, pc, "relu", out=cat[..., cout:], pool_out=pooled)
        y_ref = ops.conv3x3(x, pc, "relu")
        p_ref = ops.maxpool2x2(y_ref)
    finally:
        _lib.set_option("conv_kernel", 0)
        _lib.set_option("splitk_tiles", 512)
    assert torch.equal(cat[..., cout:], y_ref)
    assert torch.equal(pooled, p_ref)
    assert float(cat[..., :cout].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(1, 16, 64, 64), (2, 17, 45, 64), (1, 1, 1, 64), (1, 135, 240, 64), (1, 9, 33, 128),
                                   (1, 40, 70, 64)])
@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("xdtype", ["bf16", "fp32"])
@pytest.mark.parametrize("pair_kernel", [0, 1, 2])
def test_conv_pair_first_bit_exact(shape, pool, xdtype, pair_kernel):
    """vm_conv3x3_pair_first_nhwc (conv1_1 evaluated into LDS, then conv1_2 [+ pool1]) equals the two separate
    kernels bit for bit: same bf16 rounding of the 64-channel intermediate, same accumulation order; an f32 frame is
    rounded on load exactly like vm_convert_nhwc."""
    from vmatting import _lib, ops
    n, h, w, cout2 = shape
    rs = np.random.RandomState(h * w + cout2)
    xf = torch.from_numpy((rs.normal(size=(n, h, w, 7)) * 50).astype(np.float32)).to(DEV)
    x8 = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=DEV)
    ops.convert(xf, x8)
    w1 = (rs.normal(size=(3, 3, 7, 64)) * np.sqrt(2.0 / 63)).astype(np.float32)
    w2 = (rs.normal(size=(3, 3, 64, cout2)) * np.sqrt(2.0 / 576)).astype(np.float32)
    pc1 = ops.PackedConv(w1, (rs.normal(size=64) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    pc2 = ops.PackedConv(w2, (rs.normal(size=cout2) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    cat = torch.full((n, h, w, 2 * cout2), 7.0, dtype=torch.bfloat16, device=DEV)
    pooled = torch.zeros((n, (h + 1) // 2, (w + 1) // 2, cout2), dtype=torch.bfloat16, device=DEV) if pool else None
    # pair_kernel 0: the strip-walking kernel (default), 2: the tile-persistent kernel (pair_strip 0), 1: the FIRST
    # patch kernel
    _lib.set_option("pair_kernel", 1 if pair_kernel == 1 else 0)
    _lib.set_option("pair_strip", 1 if pair_kernel == 0 else 0)
    try:
        ops.conv_pair_first(x8[..., :7] if xdtype == "bf16" else xf, pc1, pc2, "relu", out=cat[..., cout2:],
                            pool_out=pooled)
        name = _lib.last_conv_kernel()
    finally:
        _lib.set_option("pair_kernel", 0)
        _lib.set_option("pair_strip", 1)
    # conv3x3_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G>: the fused pair has FIRST = true
    first = name.split("<", 1)[-1].rstrip(">").split(",")[9].strip() if "<" in name else ""
    # (the strip kernel fetches >= 2 KB row windows: smaller frames run the tile kernel)
    strip = pair_kernel == 0 and h * w * (28 if xdtype == "fp32" else 16) >= 2048
    if cout2 != 64 or pair_kernel == 1:
        assert first == "true", name
    else:
        assert name == ("vm::conv3x3_pair_strip" if strip else "vm::conv3x3_pair_persist"), name
    m = ops.conv3x3(x8[..., :7], pc1, "relu")
    y = ops.conv3x3(m, pc2, "relu")
    assert torch.equal(cat[..., cout2:], y)
    assert bool(torch.all(cat[..., :cout2] == 7.0))
    if pool:
        assert torch.equal(pooled, ops.maxpool2x2(y))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("head_kernel", [0, 1, 2])
def test_conv_head_alpha_output(dtype, head_kernel):
    """vm_conv3x3_head_nhwc: the alpha output equals sigmoid of the stored logits exactly as the separate
    vm_convert_nhwc(sigmoid) pass computes it; the logits are unchanged."""
    from vmatting import _lib, ops
    tdt = ops.TORCH_DTYPE[dtype]
    rs = np.random.RandomState(9)
    x = torch.from_numpy(rs.normal(size=(2, 19, 70, 128)).astype(np.float32)).to(tdt).to(DEV)
    pc = ops.PackedConv((rs.normal(size=(3, 3, 128, 1)) * 0.05).astype(np.float32), np.array([0.3], np.float32), tdt)
    _lib.set_option("head_kernel", head_kernel)
    try:
        logits = torch.empty((2, 19, 70, 1), dtype=torch.float32, device=DEV)
        alpha = torch.empty((2, 19, 70, 1), dtype=torch.float32, device=DEV)
        ops.conv_head(x, pc, "none", out=logits, alpha=alpha)
        ref_logits = ops.conv3x3(x, pc, "none", out_dtype=torch.float32)
    finally:
        _lib.set_option("head_kernel", 0)
    assert torch.equal(logits, ref_logits)
    ref_alpha = torch.empty_like(alpha)
    ops.convert(logits, ref_alpha, act="sigmoid")
    assert torch.equal(alpha, ref_alpha)


ROWS_CASES = [(1, 9, 33, 64, 64, "relu"), (2, 17, 70, 128, 128, "none"), (1, 20, 45, 96, 192, "relu"),
              (1, 8, 32, 32, 64, "sigmoid"), (1, 3, 5, 256, 128, "relu"), (1, 37, 70, 512, 256, "relu"),
              (1, 33, 66, 64, 24, "relu"), (3, 16, 32, 160, 64, "none")]


@pytest.mark.parametrize("th", [16, 8])
@pytest.mark.parametrize("case", ROWS_CASES)
def test_rows_kernel(case, th):
    """conv3x3_rows (row-stationary register reuse, conv_rows.hip) vs the oracle on bf16-rounded operands, and
    BIT-identical to the patch kernel (same per-accumulator MFMA sequence: granules in order, taps 0..8), with the
    fused 2x2 SAME max-pool of the same launch, partial tiles and a channel-slice output."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, act = case
    rs = np.random.RandomState(cin + cout + h + th)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16)
    wt = torch.from_numpy((rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32))
    wt = wt.to(torch.bfloat16).float().numpy()
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    outs, pools, names = [], [], []
    for opt in (th, 0):
        cat = torch.full((n, h, w, cout + 16), 7.0, dtype=torch.bfloat16, device=DEV)
        pool = torch.empty((n, (h + 1) // 2, (w + 1) // 2, cout), dtype=torch.bfloat16, device=DEV)
        _lib.set_option("rows_kernel", opt)
        try:
            ops.conv3x3(x.to(DEV), pc, act, out=cat[..., 8:8 + cout], pool_out=pool)
            names.append(_lib.last_conv_kernel())
        finally:
            _lib.set_option("rows_kernel", 1)
        assert bool(torch.all(cat[..., :8] == 7.0)) and bool(torch.all(cat[..., 8 + cout:] == 7.0))
        outs.append(cat[..., 8:8 + cout].clone())
        pools.append(pool)
    assert names[0] == "vm::conv3x3_rows<%d>" % th and names[1].startswith("vm::conv3x3_patch<"), names
    x64 = x.float().numpy().astype(np.float64)
    ref = oops.conv3x3_same(x64, wt.astype(np.float64)) + b
    ref = {"relu": oops.relu, "sigmoid": oops.sigmoid}.get(act, lambda v: v)(ref)
    check_bf16("rows<%d>" % th, H(outs[0]), ref, 9 * cin, lambda idx: abs_conv_at(x64, wt, b, idx, ref.shape))
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(pools[0], pools[1])
    assert np.array_equal(H(pools[0]), oops.max_pool_2x2_same(H(outs[0])))


@pytest.mark.parametrize("case", [(1, 9, 13, 128, 64), (2, 7, 33, 256, 128), (1, 34, 60, 512, 256), (1, 1, 1, 64, 64)])
def test_rows_kernel_folded_upconv(case):
    """The folded 2x upconv (4 phase filters, phase-indexed epilogue scatter) on conv3x3_rows: bit-identical to the
    patch kernel's result."""
    from vmatting import _lib, ops
    n, h, w, cin, cout = case
    rs = np.random.RandomState(h * 7 + cin)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, (rs.normal(size=cout) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    res = []
    for opt in (16, 0):
        _lib.set_option("rows_kernel", opt)
        try:
            res.append(ops.upconv3x3(x, pc, "relu"))
            name = _lib.last_conv_kernel()
        finally:
            _lib.set_option("rows_kernel", 1)
        if opt:
            assert name in ("vm::conv3x3_rows<16>", "vm::conv3x3_up2x_border"), name
    assert torch.equal(res[0], res[1])


UP_CASES = [(1, 9, 13, 128, 64), (2, 7, 33, 256, 128), (1, 1, 1, 64, 64), (1, 3, 2, 32, 64), (1, 34, 60, 512, 256),
            (1, 17, 30, 64, 192), (1, 68, 120, 128, 64)]


@pytest.mark.parametrize("cfg", [0, 19, 22, 25, 30])
@pytest.mark.parametrize("case", UP_CASES)
def test_upconv_folded_resize(case, cfg):
    """vm_conv3x3_up2x_nhwc (resize folded into four phase filters + exact border recompute) vs the oracle's
    resize_images -> conv2d on the same bf16 operands (bf16 tolerance), vs the unfused GPU path (resize kernel +
    conv kernel), with bias + relu through the phase-indexed epilogue and a channel-slice (concat) output."""
    from vmatting import _lib, ops
    n, h, w, cin, cout = case
    rs = np.random.RandomState(h * 31 + cin + cout)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = torch.from_numpy((rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32))
    wt = wt.to(torch.bfloat16).float().numpy()
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    cat = torch.full((n, 2 * h, 2 * w, 2 * cout), 7.0, dtype=torch.bfloat16, device=DEV)
    _lib.set_option("patch_cfg", cfg)
    try:
        ops.upconv3x3(x, pc, "relu", out=cat[..., :cout])
        name = _lib.last_conv_kernel()
    finally:
        _lib.set_option("patch_cfg", 0)
    assert name.startswith("vm::conv3x3_patch<"), name
    assert bool(torch.all(cat[..., cout:] == 7.0))
    y = cat[..., :cout].float().cpu().numpy()
    r = oops.resize_bilinear_tf1(x.float().cpu().numpy(), 2 * h, 2 * w)
    r = torch.from_numpy(r.astype(np.float32)).to(torch.bfloat16).float().numpy().astype(np.float64)
    ref = oops.relu(oops.conv3x3_same(r, wt.astype(np.float64)) + b)
    err = np.abs(y - ref).max() / max(1.0, np.abs(ref).max())
    assert err < 1e-2, err
    # the kernel's own arithmetic (bf16 folded phase filters, unfused bf16 border) to the bf16 rounding bound
    x64 = x.float().cpu().numpy().astype(np.float64)
    refk = oops.relu(ob.upconv2x_folded(x64, wt, round_w=True) + b)
    absk = ob.upconv2x_folded(np.abs(x64), np.abs(wt), round_w=False) + np.abs(b)
    check_bf16("up2x cfg %d" % cfg, y, refk, 9 * cin, lambda idx: 1.01 * absk.reshape(-1)[idx])
    unfused = ops.upconv3x3(x, pc, "relu", fold=False).float().cpu().numpy()
    assert np.abs(y - unfused).max() / max(1.0, np.abs(unfused).max()) < 1e-2
    # border pixels take the unfused arithmetic (bf16 resized taps, plain filter)
    for sl in (np.s_[:, 0], np.s_[:, -1], np.s_[:, :, 0], np.s_[:, :, -1]):
        assert np.abs(y[sl] - unfused[sl]).max() <= 1e-2 * max(1.0, np.abs(unfused[sl]).max())


@pytest.mark.parametrize("cfg", [0, 19, 22, 25])
@pytest.mark.parametrize("case", [(1, 9, 13, 128, 64), (2, 7, 33, 256, 128), (1, 68, 120, 128, 64), (1, 3, 2, 32, 64)])
def test_upconv_folded_zero_tap_skip_bit_identical(case, cfg):
    """The folded upconv's odd phases have exactly-zero filter rows / columns (TF1 legacy 2x bilinear): skipping
    those taps (up_skip 1, the default: 25 of 36 taps) gives bit-identical outputs to running all of them."""
    from vmatting import _lib, ops
    n, h, w, cin, cout = case
    rs = np.random.RandomState(h * 7 + cin)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, (rs.normal(size=cout) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    outs = []
    try:
        _lib.set_option("patch_cfg", cfg)
        for skip in (1, 0):
            _lib.set_option("up_skip", skip)
            outs.append(ops.upconv3x3(x, pc, "relu").clone())
            assert _lib.last_conv_kernel().endswith("true>" if skip else "false>"), _lib.last_conv_kernel()
    finally:
        _lib.set_option("up_skip", 1)
        _lib.set_option("patch_cfg", 0)
    assert torch.equal(outs[0], outs[1])


def test_upconv_fold_f32_uses_unfused_path():
    """f32 has no folded kernel: upconv3x3 runs resize + conv and stays within the f32 parity bound."""
    from vmatting import ops
    rs = np.random.RandomState(3)
    x = torch.from_numpy(rs.normal(size=(1, 5, 7, 64)).astype(np.float32)).to(DEV)
    wt = (rs.normal(size=(3, 3, 64, 64)) * 0.05).astype(np.float32)
    pc = ops.PackedConv(wt, None, torch.float32, DEV)
    assert pc.up2x() is None
    y = ops.upconv3x3(x, pc, "none")
    ref = oops.conv3x3_same(oops.resize_bilinear_tf1(H(x), 10, 14), wt.astype(np.float64))
    assert relerr(H(y), ref) < 1e-5


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_conv3x3_writes_channel_slice_only(dtype):
    """Concat-by-slice: a conv writing channels [64,128) of a 128-ch buffer leaves [0,64) untouched."""
    from vmatting import ops
    tdt = ops.TORCH_DTYPE[dtype]
    x = torch.randn(1, 9, 11, 64, device=DEV).to(tdt)
    pc = ops.PackedConv(np.random.RandomState(0).normal(size=(3, 3, 64, 64)).astype(np.float32) * 0.05, None, tdt)
    buf = torch.full((1, 9, 11, 128), 7.0, device=DEV, dtype=tdt)
    ops.conv3x3(x, pc, "relu", out=buf[..., 64:])
    assert bool(torch.all(buf[..., :64] == 7.0))
    y = ops.conv3x3(x, pc, "relu")
    assert torch.equal(buf[..., 64:], y)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("hw", [(9, 13), (8, 8), (1, 5), (135, 240)])
def test_maxpool_same_vs_oracle(dtype, hw):
    from vmatting import ops
    tdt = ops.TORCH_DTYPE[dtype]
    x = torch.randn(2, hw[0], hw[1], 64, device=DEV).to(tdt)
    y = ops.maxpool2x2(x)
    ref = oops.max_pool_2x2_same(H(x))
    assert np.array_equal(H(y), ref)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("io", [((68, 120), (135, 240)), ((5, 6), (9, 12)), ((3, 4), (3, 4)), ((7, 9), (14, 18))])
def test_resize_tf1_vs_oracle(dtype, io):
    from vmatting import ops
    tdt = ops.TORCH_DTYPE[dtype]
    (ih, iw), (oh, ow) = io
    x = torch.randn(1, ih, iw, 24, device=DEV).to(tdt)
    y = ops.resize_bilinear(x, (oh, ow))
    ref = oops.resize_bilinear_tf1(H(x), oh, ow)
    tol = 1e-6 if dtype == "fp32" else 8e-3
    assert np.abs(H(y) - ref).max() <= tol * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("hw", [(7, 9), (68, 120), (1, 1), (135, 240), (3, 50)])
def test_resize_2x_bit_exact(dtype, hw):
    """Exact-2x fast path: identical to the TF-1 legacy formula evaluated in float32 (then rounded to bf16)."""
    from vmatting import ops
    tdt = ops.TORCH_DTYPE[dtype]
    ih, iw = hw
    x = (torch.randn(2, ih, iw, 32, device=DEV) * 3).to(tdt)
    y = ops.resize_bilinear(x, (2 * ih, 2 * iw))
    xf = x.float().cpu().numpy()  # float32 operands: the oracle then evaluates the formula in float32 like TF
    ref = torch.from_numpy(oops.resize_bilinear_tf1(xf, 2 * ih, 2 * iw)).to(tdt)
    assert torch.equal(y.cpu(), ref)


def test_bn_stats_apply_vs_oracle():
    from vmatting import ops
    x = (torch.randn(2, 17, 23, 40, device=DEV) * 3 + 5).contiguous()
    mean, var = ops.bn_stats(x)
    xn = H(x).reshape(-1, 40)
    assert np.allclose(H(mean), xn.mean(0), rtol=1e-5, atol=1e-5)
    assert np.allclose(H(var), xn.var(0), rtol=1e-4, atol=1e-4)
    g = torch.rand(40, device=DEV) + 0.5
    b = torch.randn(40, device=DEV)
    y = ops.bn_apply(x, mean, var, g, b, 1e-3, "relu", out=torch.empty_like(x))
    ref = oops.relu(oops.batch_norm(H(x), H(g), H(b), True))
    assert np.abs(H(y) - ref).max() < 1e-4


def test_softmax_lastdim():
    from vmatting import ops
    x = torch.randn(1, 5, 7, 64, device=DEV)
    assert np.abs(H(ops.softmax_lastdim(x)) - oops.softmax_lastdim(H(x))).max() < 1e-6


# ----------------------------------------------------------------------------- whole networks vs goldens

@pytest.mark.parametrize("case", ["unet_video_70x90", "unet_video_64x96", "unet_video_70x90_unit", "unet_image_70x90"])
def test_unet_fp32_matches_reference_golden(case, vgg0):
    from vmatting import unet
    g = golden(case)
    cls = unet.UNetVideo if int(g["video"]) else unet.UNetImage
    np.random.seed(int(g["weight_seed"]))
    m = cls(vgg0, dtype="fp32")
    m.build(g["x"])
    torch.cuda.synchronize()
    alpha, logits = H(m.output), H(m.conv1_3)
    assert np.abs(alpha - g["output"]).max() <= 1e-4
    assert np.all(np.abs(logits - g["logits"]) <= 1e-4 * np.abs(g["logits"]).max() + 1e-4)
    for k in ("pool4", "upconv1", "conv2_3"):
        assert relerr(H(getattr(m, k)), g[k]) < 1e-5, k


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_unet_both_conv_kernels_agree_with_golden(dtype, conv_kernel, vgg0):
    from vmatting import unet
    g = golden("unet_video_70x90_unit")
    np.random.seed(int(g["weight_seed"]))
    m = unet.UNetVideo(vgg0, dtype=dtype)
    m.build(g["x"])
    err = np.abs(H(m.output) - g["output"]).max()
    assert err <= (1e-4 if dtype == "fp32" else 2e-2), err


def test_unet_forward_reuse_and_batch_consistency(vgg0):
    """forward() re-evaluates the built net; a frame gives the same matte alone or inside a batch."""
    from vmatting import unet
    g = golden("unet_video_70x90_unit")
    np.random.seed(int(g["weight_seed"]))
    m = unet.UNetVideo(vgg0, dtype="bf16")
    x1 = T(g["x"])
    a1 = m.build(x1).clone()
    x3 = torch.cat([x1 * 0.5, x1, x1 * 2.0])
    a3 = m.forward(x3).clone()
    assert torch.equal(a3[1], a1[0])
    assert torch.equal(m.forward(x1), a1)


def test_unet_bf16_close_to_reference(vgg0):
    from vmatting import unet
    g = golden("unet_video_70x90_unit")
    np.random.seed(int(g["weight_seed"]))
    m = unet.UNetVideo(vgg0, dtype="bf16")
    m.build(g["x"])
    err = np.abs(H(m.output) - g["output"]).max()
    lerr = relerr(H(m.conv1_3), g["logits"])
    print("bf16 UNetVideo 70x90 unit: alpha max-abs err %.3e, logits rel err %.3e" % (err, lerr))
    assert err < 2e-2 and lerr < 5e-2


@pytest.mark.parametrize("shape", [(1, 1080, 1920), (3, 67, 101), (1, 541, 97), (2, 3, 45), (2, 8, 17), (5, 64, 64)])
@pytest.mark.parametrize("xdtype", ["fp32", "bf16"])
def test_pair_strip_matches_tile_kernel(shape, xdtype):
    """The strip-walking pair kernel (conv_pair.hip: row ring of conv1_1 in LDS, filters in registers, segments of
    rows, register epilogue with the DPP pool) against the tile-persistent kernel: conv1_2 output, pool1 and the head
    split's per-tap partials bit for bit, at 1080p (17 segments of 64 rows), odd sizes (partial last strip, odd
    height: the last pooled row from one row), small frames (one segment shorter than the halo; row windows clamped
    at both image ends) and batches."""
    from vmatting import _lib, ops
    n, h, w = shape
    rs = np.random.RandomState(h + 7 * w + n)
    xf = torch.from_numpy((rs.normal(size=(n, h, w, 7)) * 50).astype(np.float32)).to(DEV)
    x8 = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=DEV)
    ops.convert(xf, x8)
    x = xf if xdtype == "fp32" else x8[..., :7]
    w1 = (rs.normal(size=(3, 3, 7, 64)) * np.sqrt(2.0 / 63)).astype(np.float32)
    w2 = (rs.normal(size=(3, 3, 64, 64)) * np.sqrt(2.0 / 576)).astype(np.float32)
    whd = T((rs.normal(size=(3, 3, 128, 1)) * np.sqrt(2.0 / 1152)).astype(np.float32))
    pc1 = ops.PackedConv(w1, (rs.normal(size=64) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    pc2 = ops.PackedConv(w2, (rs.normal(size=64) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    outs = []
    for strip in (1, 0):
        _lib.set_option("pair_strip", strip)
        try:
            y = torch.full((n, h, w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
            p = torch.full((n, (h + 1) // 2, (w + 1) // 2, 64), 7.0, dtype=torch.bfloat16, device=DEV)
            part = torch.full((n, h, w, 12), 3.0, dtype=torch.float32, device=DEV)
            ops.conv_pair_first_head(x, pc1, pc2, whd, 64, part, "relu", out=y, pool_out=p, store_y=True)
            name = _lib.last_conv_kernel()
            y2 = torch.full((n, h, w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
            p2 = torch.full_like(p, 7.0)
            ops.conv_pair_first(x, pc1, pc2, "relu", out=y2, pool_out=p2)
        finally:
            _lib.set_option("pair_strip", 1)
        assert name == ("vm::conv3x3_pair_strip" if strip else "vm::conv3x3_pair_persist"), name
        assert torch.equal(y, y2) and torch.equal(p, p2)
        outs.append((y, p, part))
    (ys, ps, qs), (yt, pt, qt) = outs
    assert torch.equal(ys, yt)
    assert torch.equal(ps, pt)
    assert torch.equal(qs[..., :9], qt[..., :9])
    assert float(qs[..., 9:].abs().max()) == 0.0


@pytest.mark.parametrize("shape", [(24, 320, 320), (3, 67, 101), (1, 1, 1)])
def test_pair_first_keep_mid(shape):
    """ops.conv_pair_first(keep_mid=True) (vm_conv3x3_pair_first_mid_nhwc on the strip kernel; the two convs where
    it cannot run): conv1_1's output, conv1_2 and pool1 equal the separate convs bit for bit — the training towers'
    first pair (unet_simple.py:60-62), whose select convs read conv1_1."""
    from vmatting import ops
    n, h, w = shape
    rs = np.random.RandomState(h + w + n)
    x8 = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=DEV)
    x8[..., :3] = torch.from_numpy((rs.normal(size=(n, h, w, 3)) * 50).astype(np.float32)).to(DEV).to(torch.bfloat16)
    pc1 = ops.PackedConv((rs.normal(size=(3, 3, 3, 64)) * 0.2).astype(np.float32), (rs.normal(size=64) * 0.1).astype(
        np.float32), torch.bfloat16, DEV)
    pc2 = ops.PackedConv((rs.normal(size=(3, 3, 64, 64)) * 0.06).astype(np.float32), (rs.normal(size=64) * 0.1).astype(
        np.float32), torch.bfloat16, DEV)
    mid = torch.full((n, h, w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    y = torch.full((n, h, w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    p = torch.full((n, (h + 1) // 2, (w + 1) // 2, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.conv_pair_first(x8[..., :3], pc1, pc2, "relu", out=y, pool_out=p, mid=mid, keep_mid=True)
    m_ref = ops.conv3x3(x8[..., :3], pc1, "relu")
    y_ref = ops.conv3x3(m_ref, pc2, "relu")
    assert torch.equal(mid, m_ref)
    assert torch.equal(y, y_ref)
    assert torch.equal(p, ops.maxpool2x2(y_ref))


@pytest.mark.parametrize("shape", [(1, 16, 64), (2, 17, 45), (1, 1, 1), (1, 135, 240), (1, 40, 70)])
@pytest.mark.parametrize("store_y", [False, True])
def test_conv_pair_first_head_partials(shape, store_y):
    """vm_conv3x3_pair_first_head_nhwc: pool1 (and y when store_y) bit-identical to the plain pair kernel; the head
    partials partial[p][t] = sum_c y[p][c] * bf16(w)[t][64 + c] of the kernel's own bf16 outputs (f32 MFMA sums vs an
    f64 restatement); taps 9..11 zero; y untouched when not stored.  Then conv_head over the other 64 channels +
    the partials equals the full 128-channel head within f32 summation order."""
    from vmatting import ops
    n, h, w = shape
    rs = np.random.RandomState(h * w + 3)
    xf = torch.from_numpy((rs.normal(size=(n, h, w, 7)) * 50).astype(np.float32)).to(DEV)
    w1 = (rs.normal(size=(3, 3, 7, 64)) * np.sqrt(2.0 / 63)).astype(np.float32)
    w2 = (rs.normal(size=(3, 3, 64, 64)) * np.sqrt(2.0 / 576)).astype(np.float32)
    wh = (rs.normal(size=(3, 3, 128, 1)) * np.sqrt(2.0 / 1152)).astype(np.float32)
    bh = np.array([0.25], np.float32)
    pc1 = ops.PackedConv(w1, (rs.normal(size=64) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    pc2 = ops.PackedConv(w2, (rs.normal(size=64) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    cat = torch.zeros((n, h, w, 128), dtype=torch.bfloat16, device=DEV)
    cat[..., :64] = torch.from_numpy(rs.uniform(0, 2, (n, h, w, 64)).astype(np.float32)).to(DEV).to(torch.bfloat16)
    pooled = torch.zeros((n, (h + 1) // 2, (w + 1) // 2, 64), dtype=torch.bfloat16, device=DEV)
    ops.conv_pair_first(xf, pc1, pc2, "relu", out=cat[..., 64:], pool_out=pooled)
    cat2 = cat.clone()
    cat2[..., 64:] = 7.0
    pooled2 = torch.zeros_like(pooled)
    part = torch.full((n, h, w, 12), 3.0, dtype=torch.float32, device=DEV)
    whd = T(wh)
    ops.conv_pair_first_head(xf, pc1, pc2, whd, 64, part, "relu", out=cat2[..., 64:], pool_out=pooled2,
                             store_y=store_y)
    assert torch.equal(pooled2, pooled)
    if store_y:
        assert torch.equal(cat2, cat)
    else:
        assert float((cat2[..., 64:].float() - 7.0).abs().max()) == 0.0
    y = H(cat[..., 64:].float()).astype(np.float64)
    wb = H(whd.to(torch.bfloat16).float()).astype(np.float64).reshape(9, 128)[:, 64:]
    want = np.einsum("nhwc,tc->nhwt", y, wb)
    got = H(part)
    assert np.abs(got[..., 9:]).max() == 0.0
    assert relerr(got[..., :9], want) < 1e-5, relerr(got[..., :9], want)
    # the split head vs the full head
    full = ops.PackedConv(wh, bh, torch.bfloat16, DEV)
    upper = ops.PackedConv(np.ascontiguousarray(wh[:, :, :64, :]), bh, torch.bfloat16, DEV)
    a_full = torch.empty((n, h, w), dtype=torch.float32, device=DEV)
    a_split = torch.empty_like(a_full)
    l_full = ops.conv_head(cat, full, "none", alpha=a_full)
    l_split = ops.conv_head(cat[..., :64], upper, "none", alpha=a_split, partial=part)
    assert relerr(H(l_split), H(l_full)) < 1e-5, relerr(H(l_split), H(l_full))
    assert float((a_split - a_full).abs().max()) < 1e-5


PERSIST_CASES = [(1, 68, 120, 128, 64, "relu", True), (2, 37, 45, 64, 128, "relu", True),
                 (1, 135, 240, 256, 128, "none", False), (1, 17, 30, 512, 512, "relu", False),
                 (3, 9, 70, 32, 64, "sigmoid", True), (1, 540, 960, 64, 128, "relu", True),
                 (1, 4, 16, 64, 64, "relu", True), (1, 33, 97, 96, 192, "relu", False),
                 (1, 135, 240, 512, 512, "relu", True), (2, 24, 80, 64, 64, "relu", True)]


@pytest.mark.parametrize("case", PERSIST_CASES)
def test_patch_persist_bit_identical(case):
    """The persistent row-slot patch kernel (vm_set_option patch_persist 1: resident grid, tile loop inside the
    kernel, the DMA stream running across tiles) writes exactly the streaming kernel's outputs: conv + bias + act
    (+ fused pool) into a channel slice of a wider buffer, and the folded 2x upconv, with and without the head split."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, act, pool = case
    rs = np.random.RandomState(h * w + cin)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, (rs.normal(size=cout) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    res, names = [], []
    try:
        _lib.set_option("persist_rounds", 0)  # (any grid: the small cases take the persistent kernel too)
        _lib.set_option("persist_up_rounds", 0)
        _lib.set_option("rows_kernel", 0)  # (the row-stationary kernel would take the cin >= 64 1080p-level grids)
        for persist in (0, 1):
            _lib.set_option("patch_persist", persist)
            cat = torch.full((n, h, w, cout + 32), 7.0, dtype=torch.bfloat16, device=DEV)
            po = torch.full((n, (h + 1) // 2, (w + 1) // 2, cout), 5.0, dtype=torch.bfloat16, device=DEV) if pool else None
            ops.conv3x3(x, pc, act, out=cat[..., 16:16 + cout], pool_out=po)
            names.append(_lib.last_conv_kernel())
            outs = [cat, po]
            if cout == 64 or cout == 128:
                up = ops.upconv3x3(x, pc, "relu")
                names.append(_lib.last_conv_kernel())
                outs.append(up)
            if cout == 64:
                whd = T((rs.normal(size=(3, 3, 128, 1)) * 0.05).astype(np.float32)) if persist == 0 else whd
                y = torch.full((n, 2 * h, 2 * w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
                part = torch.full((n, 2 * h, 2 * w, 12), 3.0, dtype=torch.float32, device=DEV)
                assert ops.upconv3x3_head(x, pc, whd, 64, part, "relu", out=y, store_y=True) is not None
                outs += [y, part]
            res.append(outs)
    finally:
        _lib.set_option("patch_persist", 1)
        _lib.set_option("persist_rounds", 2)
        _lib.set_option("persist_up_rounds", 6)
        _lib.set_option("rows_kernel", 1)
    for a, b in zip(res[0], res[1]):
        if a is not None:
            assert torch.equal(a, b)
    assert all("persist" not in nm for nm in names[:len(names) // 2]), names
    if n * h * w >= 8 * 8 * 32 * 2:  # enough pixel tiles for the resident grid (frames not packed): persistent
        assert "conv3x3_patch_persist" in names[len(names) // 2], names


@pytest.mark.parametrize("shape", [(1, 17, 23), (2, 8, 16), (1, 68, 120), (1, 540, 960)])
@pytest.mark.parametrize("store_y", [False, True])
def test_up2x_head_partials(shape, store_y):
    """vm_conv3x3_up2x_head_nhwc (upconv_4 with conv1_5's shares of its own half of cat1 taken in the epilogue,
    unet.py:200-205): y bit-identical to vm_conv3x3_up2x_nhwc (untouched when not stored); the partials
    partial[p][t] = sum_c y[p][c] * bf16(w)[t][c] of the conv's own bf16 outputs, frame border included (the border
    pass), within f32 summation order of an f64 restatement; taps 9..11 zero.  Then vm_conv3x3_head_from_partials
    with the skip half's partials equals the full 128-channel head within f32 summation order."""
    from vmatting import ops
    n, h, w = shape
    rs = np.random.RandomState(h * w + n)
    x = torch.from_numpy(rs.uniform(0, 2, (n, h, w, 128)).astype(np.float32)).to(DEV).to(torch.bfloat16)
    pc = ops.PackedConv((rs.normal(size=(3, 3, 128, 64)) * np.sqrt(2.0 / 1152)).astype(np.float32), None,
                        torch.bfloat16, DEV)
    wh = (rs.normal(size=(3, 3, 128, 1)) * np.sqrt(2.0 / 1152)).astype(np.float32)
    whd = T(wh)
    cat = torch.zeros((n, 2 * h, 2 * w, 128), dtype=torch.bfloat16, device=DEV)
    ops.upconv3x3(x, pc, "none", out=cat[..., :64])
    cat[..., 64:] = torch.from_numpy(rs.uniform(0, 2, (n, 2 * h, 2 * w, 64)).astype(np.float32)).to(DEV).to(
        torch.bfloat16)
    y = torch.full((n, 2 * h, 2 * w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    part = torch.full((n, 2 * h, 2 * w, 12), 3.0, dtype=torch.float32, device=DEV)
    assert ops.upconv3x3_head(x, pc, whd, 0, part, "none", out=y, store_y=store_y) is not None
    if store_y:
        assert torch.equal(y, cat[..., :64])
    else:
        assert float((y.float() - 7.0).abs().max()) == 0.0
    yv = H(cat[..., :64].float()).astype(np.float64)
    wb = H(whd.to(torch.bfloat16).float()).astype(np.float64).reshape(9, 128)[:, :64]
    want = np.einsum("nhwc,tc->nhwt", yv, wb)
    got = H(part)
    assert np.abs(got[..., 9:]).max() == 0.0
    assert relerr(got[..., :9], want) < 1e-5, relerr(got[..., :9], want)
    # the head from the two halves' partials vs the full head over cat1
    bh = np.array([0.25], np.float32)
    full = ops.PackedConv(wh, bh, torch.bfloat16, DEV)
    a_full = torch.empty((n * 4 * h * w,), dtype=torch.float32, device=DEV)
    l_full = ops.conv_head(cat, full, "none", alpha=a_full)
    # the skip half's partials in the pair kernel's layout (f64 restatement, rounded to f32)
    yk = H(cat[..., 64:].float()).astype(np.float64)
    wk = H(whd.to(torch.bfloat16).float()).astype(np.float64).reshape(9, 128)[:, 64:]
    pb = np.zeros((n, 2 * h, 2 * w, 12), np.float32)
    pb[..., :9] = np.einsum("nhwc,tc->nhwt", yk, wk).astype(np.float32)
    a_sp = torch.empty_like(a_full)
    l_sp = ops.head_from_partials(part, T(pb), T(bh), alpha=a_sp)
    assert relerr(H(l_sp), H(l_full)) < 1e-5, relerr(H(l_sp), H(l_full))
    assert float((a_sp - a_full).abs().max()) < 1e-5


def test_unet_bf16_fused_and_unfused_forward_agree(vgg0):
    """bf16 forward: fusing conv1_1->conv1_2 changes nothing (bit for bit, the lazily evaluated .conv1_1 included);
    folding the upconv resizes stays in the bf16 error class of the resize + conv path (logits; alpha of saturated
    He-init logits is not a useful measure here — test_unet_bf16_close_to_reference checks alpha on unit weights)."""
    from vmatting import unet
    rs = np.random.RandomState(11)
    x = np.concatenate([rs.uniform(-120, 130, (1, 66, 130, 6)), rs.choice([-0.5, 0.0, 0.5], (1, 66, 130, 1))], -1)
    xt = torch.from_numpy(x.astype(np.float32)).to(DEV)
    np.random.seed(1)
    m = unet.UNetVideo(vgg0, dtype="bf16")
    m.build(x.astype(np.float32))

    def variant(fuse, fold, split=True):
        v = unet.UNetVideo(vgg0, dtype="bf16").load_params(m.params)
        v.fuse_first, v.fold_upconv, v.split_head = fuse, fold, split
        v.prepare()
        v.forward(xt)
        return v

    m2 = variant(False, m.fold_upconv)
    m4 = variant(True, m.fold_upconv, split=False)
    assert torch.equal(m.conv1_1, m2.conv1_1)
    assert torch.equal(m.pool1, m2.pool1) and torch.equal(m.conv1_2, m2.conv1_2)  # .conv1_2 lazily evaluated (split)
    assert torch.equal(m4.output, m2.output)
    assert torch.equal(m.upconv4, m4.upconv4)
    # the split head (pair-kernel shares of conv1_2's half) only reorders f32 sums
    assert relerr(H(m.conv1_3), H(m4.conv1_3)) < 1e-5, relerr(H(m.conv1_3), H(m4.conv1_3))
    assert float((m.output - m4.output).abs().max()) < 1e-5
    m3 = variant(True, ())
    assert relerr(H(m.conv1_3), H(m3.conv1_3)) < 2e-2, relerr(H(m.conv1_3), H(m3.conv1_3))


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_unet_graph_replay_matches_eager(dtype, vgg0):
    """UNet.capture: the HIP-graph replay reproduces the eager forward bit for bit, also on new frames copied in."""
    from vmatting import unet
    rs = np.random.RandomState(5)
    xs = [np.concatenate([rs.uniform(-120, 130, (2, 40, 72, 6)), rs.choice([-0.5, 0.0, 0.5], (2, 40, 72, 1))],
                         -1).astype(np.float32) for _ in range(2)]
    np.random.seed(1)
    m = unet.UNetVideo(vgg0, dtype=dtype)
    m.build(xs[0])
    g = m.capture(xs[0])
    for x in xs:
        ya = g(x).clone()
        yb = m.forward(torch.from_numpy(x).to(DEV)).clone()
        assert torch.equal(ya, yb)


def test_unet_graph_replay_restores_lazy_attributes(vgg0):
    """After another shape's eager forward and a lazy .conv1_2 evaluation, a replay leaves the model's attributes on
    the replayed frames: .output / .conv1_2 equal a fresh eager forward of the same frames (head split: conv1_2 is
    re-evaluated, not the stale skip half)."""
    from vmatting import unet
    rs = np.random.RandomState(6)
    mk = lambda n, h, w: np.concatenate([rs.uniform(-120, 130, (n, h, w, 6)),  # noqa: E731
                                         rs.choice([-0.5, 0.0, 0.5], (n, h, w, 1))], -1).astype(np.float32)
    x0, x1, other = mk(1, 40, 72), mk(1, 40, 72), mk(2, 24, 40)
    np.random.seed(1)
    m = unet.UNetVideo(vgg0, dtype="bf16")
    m.build(x0)
    g = m.capture(x0)
    g(x1)
    c12_a = m.conv1_2.clone()  # lazily evaluated on x1
    m.forward(torch.from_numpy(other).to(DEV))
    _ = m.conv1_2  # evaluated on the other shape's set
    g(x0)
    out_g, c12_g = m.output.clone(), m.conv1_2.clone()
    m.forward(torch.from_numpy(x0).to(DEV))
    assert torch.equal(out_g, m.output) and torch.equal(c12_g, m.conv1_2)
    assert not torch.equal(c12_a, c12_g)


def test_split_sources_past_the_offset_limit_fall_back():
    """split sources (tower-major SourceConcat) whose byte span passes the 32-bit offsets of the patch
    kernel are refused by the library (VM_EUNSUPPORTED) and ops.conv3x3 runs the materialised concat instead —
    same kernel, same arithmetic: bit-identical to the split-source result, and the oracle within bf16 tolerance."""
    from vmatting import _lib, ops
    rs = np.random.RandomState(17)
    n, h, w, c, cout = 2, 21, 70, 64, 64
    base = T(rs.normal(size=(3 * n, h, w, c)).astype(np.float32), torch.bfloat16)
    sc = ops.SourceConcat(base, 3)
    wt = torch.from_numpy((rs.normal(size=(3, 3, 3 * c, cout)) * 0.05).astype(np.float32))
    wt = wt.to(torch.bfloat16).float().numpy()
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    split = ops.conv3x3(sc, pc, "relu").clone()
    span = (2 * sc.stride + h * w * c) * 2
    try:
        _lib.set_option("src_span_limit", span)  # exactly at the limit: refused
        xv = ops.nhwc(sc.src0)
        y = torch.empty_like(split)
        yv = ops.nhwc(y)
        import ctypes
        rc = _lib.lib().vm_conv3x3_ex_nhwc(ctypes.byref(xv), 3, sc.stride, ops._ptr(pc.packed), pc.cin, pc.cout,
                                           ops._ptr(pc.bias), None, None, _lib.ACT["relu"], ctypes.byref(yv), None, 0,
                                           _lib.stream_handle())
        assert rc == _lib.VM_EUNSUPPORTED
        fell = ops.conv3x3(sc, pc, "relu").clone()
    finally:
        _lib.set_option("src_span_limit", 0x7ffffff0)
    assert torch.equal(fell, split)
    cat = np.concatenate([H(sc.source(i)) for i in range(3)], -1).astype(np.float64)
    ref = oops.relu(oops.conv3x3_same(cat, wt.astype(np.float64)) + b)
    assert np.abs(H(split) - ref).max() <= 1e-2 * max(1.0, np.abs(ref).max())


def test_unet_simple_inference_is_batch_invariant(vgg0):
    """UNetSimple inference (phase False, folded BN affine) runs without split-K, so a frame's alpha
    does not depend on the batch it is evaluated in (bf16 path)."""
    from vmatting import unet_simple
    rs = np.random.RandomState(3)
    c = rs.uniform(-120, 130, (3, 64, 96, 3)).astype(np.float32)
    b = rs.uniform(-120, 130, (3, 64, 96, 3)).astype(np.float32)
    np.random.seed(2)
    m = unet_simple.create_model(c, b, c - b, False, vgg16_npy_path=vgg0, dtype="bf16")
    full = m.output.clone()
    for i in range(3):
        one = m.forward(c[i:i + 1], b[i:i + 1], c[i:i + 1] - b[i:i + 1]).clone()
        assert torch.equal(one[0], full[i]), i


@pytest.mark.parametrize("case", ["unet_simple_256_infer", "unet_simple_64_train"])
def test_unet_simple_fp32_matches_reference_golden(case, vgg0):
    from vmatting import unet_simple
    g = golden(case)
    c = g["cmp_u8"].astype(np.float64) - VGG_MEAN
    b = g["bg_u8"].astype(np.float64) - VGG_MEAN
    np.random.seed(int(g["weight_seed"]))
    m = unet_simple.create_model(c, b, c - b, bool(g["phase"]), vgg16_npy_path=vgg0, dtype="fp32")
    torch.cuda.synchronize()
    assert np.abs(H(m.output) - g["output"]).max() <= 1e-4
    lg = g["logits"]
    assert np.all(np.abs(H(m.logits) - lg) <= 1e-4 * np.abs(lg).max() + 1e-4)
    assert relerr(H(m.upconv4), g["upconv4"]) < 1e-4


@pytest.mark.parametrize("case", ["small_70x90_infer", "small_70x90_train"])
def test_unet_small_fp32_matches_reference_golden(case):
    from vmatting import small
    g = golden(case)
    np.random.seed(int(g["weight_seed"]))
    m = small.UNetSmall(g["x"], bool(g["phase"]), dtype="fp32")
    torch.cuda.synchronize()
    assert np.abs(H(m.output) - g["output"]).max() <= 1e-4
    assert relerr(H(m.upconv2), g["upconv2"]) < 1e-4


def test_refine_fp32_matches_reference_golden():
    from vmatting import refine
    g = golden("refine_40x56")
    np.random.seed(int(g["weight_seed"]))
    m = refine.RefineNet(dtype="fp32")
    m.build(g["x"])
    assert np.abs(H(m.output) - g["output"]).max() <= 1e-5
    assert np.isclose(H(m.conv1).sum(), float(g["conv1_sum"]), rtol=1e-4)  # the lazily-built dead branch


# ----------------------------------------------------------------------------- flow path

def test_warp_img_matches_reference_golden():
    from vmatting import flow
    g = golden("flow_500x1200")
    fb = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_b"]))
    alpha = g["alpha_u8"] / 255.0
    out = flow.warp_img(alpha, fb)  # numpy in -> numpy out, like the reference
    assert out.dtype == np.float64 and out.shape == (500, 1200)
    assert np.abs(out - g["warped"]).max() <= 1e-6
    ex = flow.warp_img(T(alpha), T(fb), mode="exact")
    assert np.abs(H(ex) - oflow.warp_img(alpha, fb, mode="exact")).max() <= 1e-5


def test_warp_bgr_bit_exact_with_reference():
    from vmatting import flow
    g = golden("flow_500x1200")
    assert np.array_equal(flow.warp_bgr(g["bgr_crop"], g["bgr_flow"]), g["bgr_warped"])


def test_correct_alpha_bit_exact_with_reference():
    from vmatting import flow
    g = golden("flow_500x1200")
    fb = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_b"]))
    ff = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_f"]))
    warped = oflow.warp_img(g["alpha_u8"] / 255.0, fb).astype(np.float32)
    a = T(warped)
    flow.correct_alpha(T(fb), T(ff), a, promote="numpy2")
    mask = (H(a) == 0) & (warped != 0)
    assert np.array_equal(np.packbits(mask), g["corrected_zero_mask"])
    small = g["small_alpha"].copy()
    out = flow.correct_alpha(g["small_backward"], g["small_forward"], small, promote="numpy2")
    assert out is small and np.array_equal(out == 0, g["small_corrected"] == 0)
    assert np.allclose(out, g["small_corrected"], rtol=0, atol=1e-7)  # f32 device alpha vs f64 reference
    # numpy-1 semantics (float64 index arithmetic) against the oracle restatement
    a1 = T(warped)
    flow.correct_alpha(T(fb), T(ff), a1, promote="numpy1")
    ref1 = oflow.correct_alpha(fb, ff, warped.copy(), promote="numpy1")
    assert np.array_equal(H(a1), ref1.astype(np.float64))


def test_correct_alpha_index_error_leaves_alpha_untouched():
    from vmatting import flow
    h, w = 16, 20
    bw = np.zeros((h, w, 2), np.float32)
    bw[3, 4, 1] = -40.0  # i0 = 3 - 40 = -37 < -h -> the reference's IndexError
    fw = np.zeros((h, w, 2), np.float32)
    alpha = np.ones((h, w))
    with pytest.raises(IndexError):
        flow.correct_alpha(bw, fw, alpha)
    assert np.all(alpha == 1.0)


def test_matting_loss_matches_reference_golden():
    from vmatting import ops
    g = golden("loss_2x32x32")
    out = H(ops.matting_loss(T(g["pred"]), T(g["gt"]), T(g["raw_fg"]), T(g["in_bg"]), T(g["in_cmp"])))
    assert np.allclose(out, [g["loss"], g["alpha_loss"], g["cmp_loss"]], rtol=2e-5)


# ----------------------------------------------------------------------------- full size (BASELINE configs)

@pytest.mark.slow
def test_unet_video_1080p_fp32_vs_oracle(vgg0):
    """Config 2 at full size: one 1920x1080 7-channel frame, fp32 HIP path vs the float32 numpy oracle."""
    from vmatting import unet
    rs = np.random.RandomState(1234)
    x = np.concatenate([rs.randint(0, 256, (1, 1080, 1920, 3)) - VGG_MEAN,
                        rs.randint(0, 256, (1, 1080, 1920, 3)) - VGG_MEAN,
                        rs.choice([-0.5, 0.0, 0.5], (1, 1080, 1920, 1))], -1).astype(np.float32) / 128.0
    np.random.seed(5)
    m = unet.UNetVideo(vgg0, dtype="fp32")
    m.build(x)
    gpu_alpha, gpu_logits = H(m.output), H(m.conv1_3)
    p = {k: v for k, v in m.params.items()}
    r = om.unet_forward(x, p, dtype=np.float32)
    err = np.abs(gpu_alpha - r["output"]).max()
    print("1080p fp32 alpha max-abs err vs oracle: %.3e" % err)
    assert err <= 1e-4
    assert np.all(np.abs(gpu_logits - r["conv1_3"]) <= 1e-4 * np.abs(r["conv1_3"]).max() + 1e-4)


@pytest.mark.slow
def test_unet_video_1080p_bf16_properties(vgg0):
    """Size-independent properties at 1080p for the bf16 throughput path: determinism, batch
    invariance, alpha in [0,1], and bounded distance from the fp32 path."""
    from vmatting import unet
    torch.manual_seed(0)
    x = torch.randn(2, 1080, 1920, 7, device=DEV) * 0.5
    np.random.seed(5)
    mb = unet.UNetVideo(vgg0, dtype="bf16")
    a2 = mb.build(x).clone()
    a1 = mb.forward(x[1:2].contiguous()).clone()
    assert torch.equal(a1[0], a2[1])
    assert torch.equal(mb.forward(x).clone(), a2)
    assert float(a2.min()) >= 0.0 and float(a2.max()) <= 1.0
    mf = unet.UNetVideo(vgg0, dtype="fp32").load_params(mb.params)
    mf._pack()
    af = mf.forward(x)
    err = float((af - a2).abs().max())
    print("1080p bf16 vs fp32 alpha max-abs diff: %.3e" % err)
    assert err < 5e-2


@pytest.mark.parametrize("xc,yc,ys,odt", [(3, 8, 8, torch.bfloat16), (8, 8, 16, torch.bfloat16), (3, 3, 32, torch.bfloat16),
                                          (7, 16, 16, torch.float32),
                                          (20, 24, 24, torch.bfloat16), (5, 5, 8, torch.float32),
                                          # whole 8-channel runs f32 -> bf16 (the vectorised form when not affine)
                                          (16, 16, 24, torch.bfloat16), (64, 64, 128, torch.bfloat16)])
@pytest.mark.parametrize("affine", [False, True])
def test_convert_views(xc, yc, ys, odt, affine):
    """vm_convert_nhwc (one 16-byte store per pixel for an aligned 8-channel bf16 output, pixel-per-thread form for
    other outputs of <= 16 channels, element form above): x's channels
    through the optional affine + relu into a channel slice of a wider buffer, extra channels zero, the rest of the
    buffer untouched."""
    from vmatting import ops
    rs = np.random.RandomState(xc * 7 + yc)
    n, h, w = 2, 19, 37
    x = rs.normal(size=(n, h, w, xc)).astype(np.float32) * 3
    sc = (rs.normal(size=xc) + 1).astype(np.float32) if affine else None
    sh = rs.normal(size=xc).astype(np.float32) if affine else None
    buf = torch.full((n, h, w, ys), 7.0, dtype=odt, device=DEV)
    off = ys - yc
    ops.convert(T(x), buf[..., off:], scale=None if sc is None else T(sc), shift=None if sh is None else T(sh),
                act="relu" if affine else "none")
    got = H(buf)
    if affine:  # x * scale + shift may be one fused multiply-add on the device: within one rounding of the output
        ref = np.maximum(x.astype(np.float64) * sc + sh, 0)
        tol = 2.0 ** -7 if odt == torch.bfloat16 else 1e-6
        assert np.all(np.abs(got[..., off:off + xc] - ref) <= tol * np.abs(ref) + 1e-6)
    else:
        ref = torch.from_numpy(x).to(odt).float().numpy()
        assert np.array_equal(got[..., off:off + xc], ref)
    assert not got[..., off + xc:].any()
    assert (got[..., :off] == 7.0).all()


PACK_CASES = [  # n, h, w, cin, cout, mode
    (3, 20, 20, 64, 64, "plain"), (5, 40, 40, 128, 128, "pool"), (4, 37, 22, 64, 64, "pool"),
    (3, 19, 21, 64, 128, "plain"), (6, 20, 20, 512, 64, "splitk"), (4, 40, 40, 96, 32, "f32"),
    (8, 20, 20, 64, 64, "sources"), (2, 9, 50, 64, 64, "plain")]


@pytest.mark.parametrize("case", PACK_CASES)
def test_packed_frames_bit_identical(case):
    """Packed frames (narrow frames tiled as one virtual image, ConvArgs::vstride): outputs, fused pool, split-K
    partials, f32 pre-BN output and tower-major split sources equal the per-frame tiling bit for bit, and the
    oracle within the bf16 bound."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, mode = case
    rs = np.random.RandomState(n * 1000 + w + cout)
    nsrc = 2 if mode == "sources" else 1
    x = rs.normal(size=(nsrc * n, h, w, cin)).astype(np.float32)
    wt = (rs.normal(size=(3, 3, nsrc * cin, cout)) * 0.05).astype(np.float32)
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    xd = T(x, torch.bfloat16)
    odt = torch.float32 if mode == "f32" else torch.bfloat16

    def run():
        out = torch.zeros((n, h, w, cout), dtype=odt, device=DEV)
        pool = torch.zeros((n, (h + 1) // 2, (w + 1) // 2, cout), dtype=torch.bfloat16, device=DEV)
        src = ops.SourceConcat(xd, nsrc) if mode == "sources" else xd
        ops.conv3x3(src, pc, "relu", out=out, pool_out=pool if mode == "pool" else None, splitk=mode == "splitk")
        return out, pool, _lib.last_conv_kernel()

    try:
        _lib.set_option("pack_frames", 0)
        y0, p0, k0 = run()
        _lib.set_option("pack_frames", 1)
        y1, p1, k1 = run()
    finally:
        _lib.set_option("pack_frames", 1)
    assert k0 == k1 and k0.startswith("vm::conv3x3_patch"), (k0, k1)
    assert torch.equal(y0, y1) and torch.equal(p0, p1)
    xcat = np.concatenate([H(xd[s * n:(s + 1) * n]) for s in range(nsrc)], -1)
    wb = torch.from_numpy(wt).to(torch.bfloat16).float().numpy().astype(np.float64)
    ref = np.maximum(oops.conv3x3_same(xcat, wb) + b, 0)
    assert relerr(H(y1), ref) < 2e-2


@pytest.mark.parametrize("case", [(1, 17, 30, 256, 512, True), (1, 9, 33, 512, 512, False), (2, 5, 40, 128, 1024, False)])
def test_channel_banded_tiles_bit_identical(case):
    """The channel-banded block -> tile order of the streaming patch kernel (ConvArgs::cband: XCD b % 8 keeps its
    64-channel weight slices L2-resident over every pixel tile; an option, off by default: measured slower) changes
    only which block computes a tile: outputs bit-identical to the pixel-banded order, for folded
    upconvs and plain convs (threshold lowered so these small shapes take it)."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, up = case
    rs = np.random.RandomState(h + cin)
    x = torch.from_numpy(rs.normal(size=(n, h, w, cin)).astype(np.float32)).to(torch.bfloat16).to(DEV)
    wt = (rs.normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, (rs.normal(size=cout) * 0.1).astype(np.float32), torch.bfloat16, DEV)
    outs = []
    try:
        _lib.set_option("patch_persist", 0)
        _lib.set_option("rows_kernel", 0)
        _lib.set_option("cband_bytes", 0)
        for band in (0, 2):
            _lib.set_option("cband", band)
            if up:
                outs.append(ops.upconv3x3(x, pc, "relu"))
            else:
                outs.append(ops.conv3x3(x, pc, "relu"))
            assert _lib.last_conv_kernel().startswith("vm::conv3x3_patch<"), _lib.last_conv_kernel()
    finally:
        _lib.set_option("cband", 0)
        _lib.set_option("cband_bytes", 4 << 20)
        _lib.set_option("patch_persist", 1)
        _lib.set_option("rows_kernel", 1)
    assert torch.equal(outs[0], outs[1])


THIN_CASES = [  # n, h, w, cin (per source x nsrc), cout, nsrc, out dtype, splitk
    (8, 40, 40, 512, 16, 3, "f32", True), (8, 80, 80, 256, 8, 3, "f32", True), (8, 160, 160, 128, 4, 3, "f32", False),
    (8, 320, 320, 64, 2, 3, "f32", False), (3, 37, 45, 96, 8, 1, "bf16", False), (2, 17, 70, 64, 2, 1, "bf16", True),
    (1, 9, 5, 32, 16, 2, "f32", False)]


@pytest.mark.parametrize("case", THIN_CASES)
def test_thin_dma_bit_identical(case):
    """The LDS-DMA narrow-cout kernel (conv3x3_thin_dma, 4 ring / tile configs) against conv3x3_thin: the same MFMA
    order and epilogue, so bit-identical outputs (tower-major split sources, split-K partials, f32 and bf16 outputs,
    ragged tiles, the training step's select shapes); and the oracle within the bf16 bound."""
    from vmatting import _lib, ops
    n, h, w, cin, cout, nsrc, od, splitk = case
    rs = np.random.RandomState(n * 7 + h + cin + cout)
    xd = T(rs.normal(size=(nsrc * n, h, w, cin)).astype(np.float32), torch.bfloat16)
    wt = (rs.normal(size=(3, 3, nsrc * cin, cout)) * 0.05).astype(np.float32)
    b = (rs.normal(size=cout) * 0.1).astype(np.float32)
    pc = ops.PackedConv(wt, b, torch.bfloat16, DEV)
    odt = torch.float32 if od == "f32" else torch.bfloat16

    def run(cfg):
        _lib.set_option("thin_dma", cfg)
        out = torch.zeros((n, h, w, cout), dtype=odt, device=DEV)
        src = ops.SourceConcat(xd, nsrc) if nsrc > 1 else xd
        ops.conv3x3(src, pc, "none", out=out, splitk=splitk)
        return out, _lib.last_conv_kernel()

    try:
        y0, k0 = run(0)
        assert k0.startswith("vm::conv3x3_thin<"), k0
        for cfg in (1, 2, 3, 4):
            y1, k1 = run(cfg)
            assert k1.startswith("vm::conv3x3_thin_dma<"), k1
            assert torch.equal(y0, y1), (cfg, k1, (y0 - y1).abs().max().item())
    finally:
        _lib.set_option("thin_dma", 0)
    if n * h * w > 200000:
        return  # the oracle at the select shapes would take minutes; bit identity carries it from the small cases
    xcat = np.concatenate([H(xd[s * n:(s + 1) * n]) for s in range(nsrc)], -1).astype(np.float64)
    wb = torch.from_numpy(wt).to(torch.bfloat16).float().numpy().astype(np.float64)
    ref = oops.conv3x3_same(xcat, wb) + b
    assert relerr(H(y0), ref) < (1e-4 if od == "f32" else 1e-2)
