"""The timed bf16 UNetVideo forward pinned layer by layer against the float64 oracle at the timed 1080p frame.

bench.py times `unet.UNetVideo(...).forward` on the synthetic 1920x1080 frame of seed 1234 (vmatting/video.py) with the
weights of seeds 0 / 0 (synthetic VGG16, init_conv).  This module runs that exact forward once (eager, so every conv
launch is recorded with the kernel that ran it), copies every activation the forward leaves in HBM, and checks each
of the 20 convs (/root/reference/unet.py:170-205) on the operands the kernel consumed: the GPU's own bf16 input
activation and the bf16-rounded filter, evaluated in float64 by the oracle (oracle/ops.py, oracle/bf16.py) — plus
bias, ReLU, the fused 2x2 SAME pool, the TF1 resize of upconv_1, the folded-resize arithmetic of upconv_2..4 and the
split head's per-tap shares.  Bound (tests/bf16check.py): >= 99.99 % of elements within 1 bf16 ulp, every element
within 2 ulp or the f32 summation bound; f32 outputs (head shares, logits) within the f32 summation bound.

The kernels these layers ran are asserted too (test_timed_kernels): conv3x3_pair_strip, conv3x3_patch_persist
<..., false|true>, conv3x3_rows<16>, the L5 4x32 conv3x3_patch, the 3-slot folded conv3x3_patch for upconv_2 and
head_from_partials — the list bench.py's roofline line reports.
"""

import re

import numpy as np
import pytest
import torch

from bf16check import abs_conv_at, check_bf16, check_f32_sum
from conftest import gpu_available
from oracle import bf16 as ob
from oracle import ops as oops

pytestmark = [pytest.mark.gpu, pytest.mark.slow,
              pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"
H, W = 1080, 1920

# conv launch order of the lean bf16 forward (unet.py:170-205) and the kernel each one must run on
TIMED = [
    ("conv1_1+conv1_2+pool1", r"vm::conv3x3_pair_strip"),
    ("conv2_1", r"vm::conv3x3_rows<16>"),
    ("conv2_2", r"vm::conv3x3_rows<16>"),
    ("conv3_1", r"vm::conv3x3_rows<16>"),
    ("conv3_2", r"vm::conv3x3_rows<16>"),
    ("conv3_3", r"vm::conv3x3_rows<16>"),
    ("conv4_1", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, false>"),
    ("conv4_2", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, false>"),
    ("conv4_3", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, false>"),
    ("conv5_1", r"vm::conv3x3_patch<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3, false>"),
    ("conv5_2", r"vm::conv3x3_patch<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3, false>"),
    ("upconv_1", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, false>"),
    ("conv4_4", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, false>"),
    ("upconv_2", r"vm::conv3x3_patch<64, 8, 1, 3, 8, 1, 9, false, 0, false, 3, true>"),
    ("conv3_4", r"vm::conv3x3_rows<16>"),
    ("upconv_3", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, true>"),
    ("conv2_3", r"vm::conv3x3_rows<16>"),
    ("upconv_4+head shares", r"vm::conv3x3_patch_persist<64, 8, 1, 2, 8, 1, true>"),
    ("conv1_5 (head_from_partials)", r"vm::head_from_partials"),
]


@pytest.fixture(scope="module")
def timed():
    """One eager bf16 forward of the timed frame; host copies (float32, exact for bf16) of every layer's tensors."""
    from vmatting import ops, unet, video
    from vmatting.weights import synthetic_vgg16
    vgg = synthetic_vgg16(0)
    np.random.seed(0)
    m = unet.UNetVideo(vgg, dtype="bf16", device=DEV)
    m.prepare()
    x = video.synthetic_frames(1, H, W, first=0, device=DEV)
    prof = ops.conv_profile(True)
    try:
        m.forward(x)
        torch.cuda.synchronize()
    finally:
        ops.conv_profile(False)
    b = m._ws
    hc = lambda t: t.float().cpu().numpy()  # noqa: E731
    d = {"names": [p[1] for p in prof], "x": hc(x), "params": m.params}
    for k in ("p1", "c21", "cat2", "p2", "c31", "c32", "cat3", "p3", "c41", "c42", "cat4", "p4", "c51", "c52", "r1",
              "c44", "c34", "c23", "hpart", "upart", "logits", "out"):
        d[k] = hc(b[k])
    # the halves of cat1 the lean forward kept on chip, evaluated on first access (bit-identical to its values:
    # test_pair_strip_matches_tile_kernel, test_up2x_head_partials)
    d["c11"] = hc(m.conv1_1)
    d["c12"] = hc(m.conv1_2)
    d["up4"] = hc(m.upconv4[..., :64])
    del m, b
    torch.cuda.empty_cache()
    return d


def _w(d, name):
    w, b = d["params"][name]
    return ob.bf16_round(w), None if b is None else np.asarray(b, np.float64)


def _conv_check(d, name, xin, got, act="relu", pool=None):
    """conv3x3 SAME + bias (+ relu) of the GPU's input ``xin`` with the bf16 filter vs the kernel output ``got``
    (and its fused pool)."""
    wb, bias = _w(d, name)
    x64 = np.asarray(xin, np.float64)
    pre = oops.conv3x3_same(x64, wb, bias)
    e = oops.relu(pre) if act == "relu" else pre
    k = 9 * x64.shape[-1]
    st = [check_bf16(name, got, e, k, lambda idx: abs_conv_at(x64, wb, bias, idx, e.shape))]
    if pool is not None:
        # the fused pool is the max of the stored bf16 outputs (bit for bit), which the check above pins
        assert np.array_equal(pool, oops.max_pool_2x2_same(np.asarray(got, np.float32))), name + " fused pool"
    return st


PLAIN = {  # layer: (input, output (buffer, channel slice), fused pool buffer)
    "conv2_1": ("p1", ("c21", None), None),
    "conv2_2": ("c21", ("cat2", slice(128, 256)), "p2"),
    "conv3_1": ("p2", ("c31", None), None),
    "conv3_2": ("c31", ("c32", None), None),
    "conv3_3": ("c32", ("cat3", slice(256, 512)), "p3"),
    "conv4_1": ("p3", ("c41", None), None),
    "conv4_2": ("c41", ("c42", None), None),
    "conv4_3": ("c42", ("cat4", slice(512, 1024)), "p4"),
    "conv5_1": ("p4", ("c51", None), None),
    "conv5_2": ("c51", ("c52", None), None),
    "conv4_4": ("cat4", ("c44", None), None),
    "conv3_4": ("cat3", ("c34", None), None),
    "conv2_3": ("cat2", ("c23", None), None),
}


def test_timed_kernels(timed):
    names = timed["names"]
    assert len(names) == len(TIMED), names
    for (layer, pat), got in zip(TIMED, names):
        assert re.fullmatch(pat, got), "%s ran %s, expected %s" % (layer, got, pat)


def test_conv1_1_lazy(timed):
    """.conv1_1 (unet.py:170; the lean forward keeps it in LDS, so the attribute is evaluated by conv3x3_first on the
    frame rounded to bf16 like the pair kernel's load)."""
    d = timed
    x = ob.bf16_round(d["x"])
    _conv_check(d, "conv1_1", x, d["c11"])


def test_pair_strip_conv1_2_pool1_head_shares(timed):
    """conv3x3_pair_strip (unet.py:170-172 + conv1_5's conv1_2 half): pool1 and the per-tap head shares it writes,
    against conv1_2 = relu(conv(conv1_1) + b) on the GPU's bf16 conv1_1."""
    d = timed
    _conv_check(d, "conv1_2", d["c11"], d["c12"])
    # the pair kernel's pool1 is the 2x2 SAME max of exactly those (checked) bf16 values
    assert np.array_equal(d["p1"], oops.max_pool_2x2_same(d["c12"])), "pool1 != pool of conv1_2"
    hw = ob.bf16_round(d["params"]["conv1_5"][0])
    y = np.asarray(d["c12"], np.float64)
    e = ob.head_shares(y, hw[:, :, 64:128])
    sa = ob.head_shares(np.abs(y), np.abs(hw[:, :, 64:128]))
    check_f32_sum("pair head shares", d["hpart"], e, 64, sa)


@pytest.mark.parametrize("layer", sorted(PLAIN))
def test_plain_conv_layer(timed, layer):
    d = timed
    src, (dst, sl), pool = PLAIN[layer]
    got = d[dst] if sl is None else d[dst][..., sl]
    _conv_check(d, layer, d[src], got, pool=None if pool is None else d[pool])


def test_upconv_1_resize_and_conv(timed):
    """upconv_1 (unet.py:191): resize_tf1_rows 68x120 -> 135x240 (bf16), then the conv (no bias, no relu) into
    upconv1[..., :512]."""
    d = timed
    c52 = d["c52"]
    er = oops.resize_bilinear_tf1(np.asarray(c52, np.float32), 135, 240)
    check_bf16("upconv_1 resize", d["r1"], er, frac_1ulp=0.0, max_ulp=1.0)
    _conv_check(d, "upconv_1", d["r1"], d["cat4"][..., :512], act="none")


@pytest.mark.parametrize("layer,src,dst", [("upconv_2", "c44", ("cat3", slice(0, 256))),
                                           ("upconv_3", "c34", ("cat2", slice(0, 128))),
                                           ("upconv_4", "c23", ("up4", slice(0, 64)))])
def test_folded_upconv_layer(timed, layer, src, dst):
    """upconv_2 .. upconv_4 (unet.py:193-199) as the folded 2x conv: interior pixels from the bf16 folded phase
    filters on the low-res bf16 input, border pixels from the f32 resize rounded to bf16."""
    d = timed
    x = np.asarray(d[src], np.float64)
    w = d["params"][layer][0]
    e = ob.upconv2x_folded(x, w, round_w=True)
    got = d[dst[0]][..., dst[1]]
    absx = {}

    def abs_terms(idx):
        # fold(|w|) >= |fold(w)| and resize(|x|) >= |resize(x)| elementwise (non-negative blend weights): an upper
        # bound on sum |products| of both the folded interior and the unfused border (x1.01 for the bf16 rounding)
        if "v" not in absx:
            absx["v"] = ob.upconv2x_folded(np.abs(x), np.abs(w), round_w=False)
        return 1.01 * absx["v"].reshape(-1)[idx]

    check_bf16(layer, got, e, 9 * x.shape[-1], abs_terms)
    if layer == "upconv_4":
        hw = ob.bf16_round(d["params"]["conv1_5"][0])
        y = np.asarray(d["up4"], np.float64)
        check_f32_sum("upconv_4 head shares", d["upart"], ob.head_shares(y, hw[:, :, :64]), 64,
                      ob.head_shares(np.abs(y), np.abs(hw[:, :, :64])))


def test_head_logits_alpha(timed):
    """conv1_5 + sigmoid (unet.py:203-205) from the two share sets: logits against the float64 conv1_5 over
    cat1 = [upconv_4, conv1_2] (the GPU's bf16 halves, bf16 head filter), alpha = sigmoid(logits)."""
    d = timed
    hw = ob.bf16_round(d["params"]["conv1_5"][0])
    bias = d["params"]["conv1_5"][1]
    cat1 = np.concatenate([d["up4"], d["c12"]], axis=-1).astype(np.float64)
    e = oops.conv3x3_same(cat1, hw, np.asarray(bias, np.float64))
    sa = oops.conv3x3_same(np.abs(cat1), np.abs(hw), np.abs(np.asarray(bias, np.float64)))
    check_f32_sum("logits", d["logits"], e, 9 * 128, sa)
    # sigmoid in f32 of the kernel's own logits, and the derivative bound against the exact logits
    a_exact = oops.sigmoid(np.asarray(d["logits"], np.float64))
    assert np.abs(d["out"] - a_exact).max() <= 2e-7, np.abs(d["out"] - a_exact).max()
    ae = oops.sigmoid(e)
    tol = 0.25 * np.abs(d["logits"] - e) + 2e-7
    assert (np.abs(d["out"] - ae) <= tol).all()


def test_timed_graph_replay_equals_pinned_eager_pass(timed):
    """bench.py times HIP-graph replays of this forward (`model.capture(x)`, bench.py's timed
    loop), while the layer checks above pin the eager pass.  The replays on the timed frame must equal that eager
    pass bit for bit — alpha and logits — so the pinned numbers are the timed ones (first replay and the 3rd)."""
    from vmatting import unet, video
    from vmatting.weights import synthetic_vgg16
    np.random.seed(0)
    m = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device=DEV)
    m.split_head = True
    m.fuse_up_head = True
    m.prepare()
    x = video.synthetic_frames(1, H, W, first=0, device=DEV)
    g = m.capture(x)
    for i in range(3):
        g.replay()
        torch.cuda.synchronize()
        if i in (0, 2):
            alpha = g.output.float().cpu().numpy()
            logits = m.conv1_3.float().cpu().numpy()
            assert np.array_equal(alpha, timed["out"]), (i, np.abs(alpha - timed["out"]).max())
            assert np.array_equal(logits, timed["logits"]), (i, np.abs(logits - timed["logits"]).max())
    del g, m
    torch.cuda.empty_cache()
