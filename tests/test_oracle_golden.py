"""Pin the CPU oracle against fixtures produced by the reference's own code (CPU only).

The fixtures (tests/golden/*.npz) come from tests/golden/make_golden.py, which
runs /root/reference's graph builders, flow.correct_alpha, reader.read_flow and
the train.py loss helpers verbatim (TF/cv2 ops via tests/golden/tfshim.py).
"""

import os
import tempfile

import numpy as np
import pytest

from conftest import golden
from oracle import flow as oflow
from oracle import models as om
from oracle import ops

VGG_MEAN = np.array(ops.VGG_MEAN)


def _fresh_weight_vars(g, suffix):
    names = [str(n) for n in g["var_names"]]
    idx = [i for i, n in enumerate(names) if n.endswith(suffix)]
    return [names[i] for i in idx], g["var_sums"][idx], g["var_firsts"][idx]


def _close(a, b, rtol, atol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b)
    bound = atol + rtol * np.abs(b)
    assert (err <= bound).all(), "max err %g (worst ratio %g)" % (err.max(), (err / bound).max())


@pytest.mark.parametrize("case", ["unet_video_70x90", "unet_video_64x96", "unet_video_70x90_unit", "unet_image_70x90"])
def test_unet_matches_reference_builder(case, vgg0):
    g = golden(case)
    rs = np.random.RandomState(int(g["weight_seed"]))
    p = om.unet_params(vgg0, rs, video=bool(g["video"]))
    # draw order: the reference's fresh 'weights' variables, in creation order (unet.py:11-17)
    names, sums, firsts = _fresh_weight_vars(g, "/weights")
    assert [n.split("/")[0] for n in names] == [c[0] for c in om.UNET_NEW_CONVS]
    for n, s, f in zip(names, sums, firsts):
        w = p[n.split("/")[0]][0].astype(np.float64)
        assert w.ravel()[0] == f and np.isclose(w.sum(), s, rtol=1e-12, atol=1e-9)
    r = om.unet_forward(g["x"], p)
    _close(r["conv1_3"], g["logits"], 1e-9, 1e-9)
    _close(r["output"], g["output"], 1e-9, 1e-12)
    for k in ("pool4", "upconv1", "conv2_3"):
        _close(r[k], g[k], 1e-6, 1e-4)


@pytest.mark.parametrize("case", ["unet_simple_256_infer", "unet_simple_64_train"])
def test_unet_simple_matches_reference_builder(case, vgg0):
    g = golden(case)
    rs = np.random.RandomState(int(g["weight_seed"]))
    p = om.unet_simple_params(rs)
    names, sums, firsts = _fresh_weight_vars(g, "/weights")
    assert [n.split("/")[-2] for n in names] == [c[0] for c in om.SIMPLE_NEW_CONVS]
    for n, s in zip(names, sums):
        assert np.isclose(p[n.split("/")[-2]][0].astype(np.float64).sum(), s, rtol=1e-12, atol=1e-9)
    c = g["cmp_u8"].astype(np.float64) - VGG_MEAN
    b = g["bg_u8"].astype(np.float64) - VGG_MEAN
    r = om.unet_simple_forward(c, b, c - b, bool(g["phase"]), vgg0, p)
    _close(r["logits"], g["logits"], 1e-8, 1e-8)
    _close(r["output"], g["output"], 1e-8, 1e-12)
    _close(r["upconv4"], g["upconv4"], 1e-5, 1e-4)


@pytest.mark.parametrize("case", ["small_70x90_infer", "small_70x90_train"])
def test_unet_small_matches_reference_builder(case):
    g = golden(case)
    p = om.unet_small_params(np.random.RandomState(int(g["weight_seed"])), cin=6)
    r = om.unet_small_forward(g["x"], bool(g["phase"]), p)
    _close(r["conv1_3"], g["logits"], 1e-9, 1e-9)
    _close(r["output"], g["output"], 1e-9, 1e-12)
    _close(r["upconv2"], g["upconv2"], 1e-5, 1e-5)


def test_refine_matches_reference_builder():
    g = golden("refine_40x56")
    p = om.refine_params(np.random.RandomState(int(g["weight_seed"])), cin=5)
    r = om.refine_forward(g["x"], p)
    _close(r["output"], g["output"], 1e-9, 1e-12)
    assert np.isclose(r["conv1"].sum(), float(g["conv1_sum"]), rtol=1e-9)


def test_read_flow_format_and_roundtrip():
    g = golden("flow_500x1200")
    fb = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_b"]))
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "b.flo")
        oflow.write_flow(p, fb)
        head = open(p, "rb").read(len(g["flo_header"]))
        assert np.array_equal(np.frombuffer(head, np.uint8), g["flo_header"])
        assert np.array_equal(oflow.read_flow(p), fb)


def test_warp_img_matches_reference():
    g = golden("flow_500x1200")
    fb = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_b"]))
    alpha = g["alpha_u8"] / 255.0
    w = oflow.warp_img(alpha, fb, mode="opencv")
    _close(w, g["warped"], 0, 1e-7)
    assert np.isclose(w.sum(), float(g["warped_f64_sum"]), rtol=1e-12)
    # the exact-bilinear mode differs from OpenCV's 1/32-pixel quantisation by at most |grad|/64 per axis
    we = oflow.warp_img(alpha, fb, mode="exact")
    assert np.abs(we - w).max() < 1.0 / 32 + 1e-9


def test_correct_alpha_matches_reference():
    g = golden("flow_500x1200")
    fb = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_b"]))
    ff = oflow.smooth_flow(500, 1200, seed=int(g["flow_seed_f"]))
    warped = oflow.warp_img(g["alpha_u8"] / 255.0, fb)
    out = oflow.correct_alpha(fb, ff, warped.copy(), promote="numpy2")
    mask = (out == 0) & (warped != 0)
    assert np.array_equal(np.packbits(mask), g["corrected_zero_mask"])
    # crafted case: large / negative displacements (numpy-style wrap of negative indices)
    c2 = oflow.correct_alpha(g["small_backward"], g["small_forward"], g["small_alpha"].copy(), promote="numpy2")
    assert np.array_equal(c2, g["small_corrected"])


def test_warp_bgr_matches_reference():
    g = golden("flow_500x1200")
    assert np.array_equal(oflow.warp_bgr(g["bgr_crop"], g["bgr_flow"]), g["bgr_warped"])


def test_loss_matches_reference():
    g = golden("loss_2x32x32")
    loss, al, cl = ops.matting_loss(g["pred"], g["gt"], g["raw_fg"], g["in_bg"], g["in_cmp"])
    assert np.isclose(loss, float(g["loss"]), rtol=1e-12)
    assert np.isclose(al, float(g["alpha_loss"]), rtol=1e-12)
    assert np.isclose(cl, float(g["cmp_loss"]), rtol=1e-12)


def test_oracle_float32_mode_close_to_float64():
    """The float32 oracle (the timed CPU baseline) tracks the float64 goldens."""
    g = golden("unet_video_70x90_unit")
    from oracle.models import synthetic_vgg16
    p = om.unet_params(synthetic_vgg16(0), np.random.RandomState(int(g["weight_seed"])), video=True)
    r = om.unet_forward(g["x"], p, dtype=np.float32)
    _close(r["output"], g["output"], 0, 1e-5)


# ---------------------------------------------------------------- training-sample loader (loader.py)

def _loader_entry(g, i):
    from oracle import loader as ol
    s, fh, fw, bh, bw, v = (int(x) for x in g["entries"][i])
    return ol.synthetic_entry(s, (fh, fw), (bh, bw), bool(v))


def loader_call_outputs(g, ci, entry_fn):
    """Replay golden call ci through entry_fn(entries, seed, input_size, mirror, fn) -> dict of [n,h,w,c]
    arrays; returns (outputs, next global draw)."""
    p = "c%d_" % ci
    seed, sw, sh, mirror, _ = (int(x) for x in g[p + "meta"])
    ents = [int(e) for e in g[p + "entries"]]
    np.random.seed(seed)
    out = entry_fn(ents, (sw, sh), bool(mirror), str(g[p + "fn"]))
    return out, np.random.randint(0, 2 ** 31 - 1)


def check_loader_call(g, ci, out, nxt):
    p = "c%d_" % ci
    assert nxt == int(g[p + "meta"][4]), "np.random draw count differs from the reference's"
    pn, py, px = g[p + "pos"]
    names = [k[len(p):-5] for k in g if k.startswith(p) and k.endswith("_vals")]
    assert names
    for k in names:
        v = np.asarray(out[k], np.float64)[pn, py, px]
        assert np.array_equal(v, g[p + k + "_vals"]), "%s: max diff %g" % (k, np.abs(v - g[p + k + "_vals"]).max())
        s = float(np.asarray(out[k], np.float64).sum())
        assert abs(s - float(g[p + k + "_sum"])) <= 1e-10 * max(1.0, abs(s)), k


@pytest.mark.parametrize("ci", range(11))
def test_loader_oracle_matches_reference_loader(ci):
    """oracle/loader.py reproduces loader.py's outputs bit for bit (float64) and consumes the same draws."""
    from oracle import loader as ol
    g = golden("loader_calls")
    assert int(g["n_calls"]) == 11

    def run(ents, size, mirror, fn):
        out = ol.batch([_loader_entry(g, e) for e in ents], size, mirror=mirror)
        if fn == "get_batch":
            out["input"] = np.concatenate([out["cmp"], out["bg"]], axis=3)
        return out

    out, nxt = loader_call_outputs(g, ci, run)
    check_loader_call(g, ci, out, nxt)


def test_loader_golden_covers_crop_paths():
    """The golden calls exercise every resize path and both get_padded_img branches."""
    from oracle import loader as ol
    g = golden("loader_calls")
    seen = set()
    for ci in range(int(g["n_calls"])):
        p = "c%d_" % ci
        seed, sw, sh = (int(x) for x in g[p + "meta"][:3])
        np.random.seed(seed)
        e = _loader_entry(g, int(g[p + "entries"][0]))
        (ch, _), fr, fc, br, bc = ol.plan_crop(e[0].shape[:2], e[1].shape[:2])
        for ax, img_n in ((fr, e[0].shape[0]), (fc, e[0].shape[1])):
            if ax.shift < 0:
                seen.add("pad-offset")
            elif ax.hi < img_n:
                seen.add("pad-zero-tail")
        seen.add("copy" if ch == sw else ("area" if ch == 2 * sw else "linear"))
        if (br.n, bc.n) == (2 * sh, 2 * sw):
            seen.add("bg-area")
    assert {"pad-offset", "pad-zero-tail", "copy", "area", "linear", "bg-area"} <= seen, seen


@pytest.mark.parametrize("shape", [(37, 23), (640, 640), (480, 320), (5, 3), (64, 64, 3), (300, 700, 3), (41, 1)])
@pytest.mark.parametrize("dsize", [(320, 320), (64, 48), (20, 2), (1, 1)])
def test_cv_resize_restatements_agree(shape, dsize):
    """oracle.loader.resize_linear (vectorised) == tfshim.resize (loop form, OpenCV structure) bit for bit."""
    import sys

    from conftest import GOLDEN
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import tfshim
    from oracle import loader as ol
    if shape[:2] == (640, 640) and dsize != (320, 320):
        pytest.skip("large source only for the area path")
    img = np.random.RandomState(sum(shape)).uniform(0, 255, shape)
    a = ol.resize_linear(img, dsize)
    b = tfshim.resize(img, dsize)
    assert a.shape == b.shape and np.array_equal(a, b)


# ---------------------------------------------------------------- augmentation row

def _tps_case(g, n):
    from oracle import augment as oa
    reg = tuple(int(v) for v in g[n + "_region"])
    ag = float(g[n + "_ag"])
    ag = int(ag) if ag == int(ag) else ag
    planes = [g["img"][:, :, 0], g["img"][:, :, 1], g["img"][:, :, 2], g["alpha"], g[n + "_f32_in"]]
    return oa.warp_images(g[n + "_from"], g[n + "_to"], planes, reg, int(g[n + "_order"]), ag)


@pytest.mark.parametrize("case", ["a", "b", "c", "d"])
def test_tps_oracle_matches_reference_tps(case):
    """oracle.augment.warp_images == the reference's tps.warp_images (run for real on scipy) bit for bit:
    approximate_grid 2 / 1 / 3 / 2.5, order 1 and 0, an offset output region, u8 / f64 / f32 planes."""
    g = golden("tps")
    r = _tps_case(g, case)
    assert np.array_equal(np.stack(r[:3], axis=-1), g[case + "_u8"])
    assert np.array_equal(r[3], g[case + "_f64"])
    assert np.array_equal(r[4], g[case + "_f32"])


def test_tps_deform_matches_reference():
    from oracle import augment as oa
    g = golden("tps")
    np.random.seed(21)
    assert np.array_equal(oa.deform(g["img"]), g["deform_out"])


@pytest.mark.parametrize("dt", [np.uint8, np.float32, np.float64])
@pytest.mark.parametrize("order", [0, 1])
def test_map_coordinates_restatement_matches_scipy(dt, order):
    """scipy (the reference's dependency, present here) vs the restatement on coordinates around every edge."""
    from scipy import ndimage
    from oracle import augment as oa
    rs = np.random.RandomState(order * 7 + len(np.dtype(dt).name))
    img = (rs.rand(7, 9) * 255).astype(dt)
    cr = rs.uniform(-2, 8, size=(40, 50))
    cc = rs.uniform(-2, 10, size=(40, 50))
    cr[::3] = np.round(cr[::3])
    cc[::4] = np.round(cc[::4])
    cr[0, :10] = [0, 6, -0.0, 6.0, -1e-12, 6 + 1e-12, 3, -0.5, 6.5, 1e-7]
    cc[1, :6] = [1e-9, 8 - 1e-9, 8, 8 + 1e-9, -1e-9, 0.5]
    assert np.array_equal(ndimage.map_coordinates(img, [cr, cc], order=order), oa.map_coordinates(img, cr, cc, order))


@pytest.mark.parametrize("i", [0, 1])
def test_augment_oracle_matches_reference(i):
    """augmentation.augment run verbatim (its draws, deform_grid, real tps.py; cv2 from tfshim)."""
    from oracle import augment as oa
    a = golden("augment")
    np.random.seed(int(a["seed%d" % i]))
    fg, bg, al = oa.augment(a["fg%d" % i], a["bg%d" % i], a["alpha%d" % i])
    assert np.array_equal(fg, a["new_fg%d" % i])
    assert np.array_equal(bg, a["new_bg%d" % i])
    assert np.array_equal(al, a["new_alpha%d" % i])
    assert np.random.randint(0, 1 << 30) == int(a["next_draw%d" % i])  # same number of draws consumed
    a2 = golden("augment")
    assert np.array_equal(oa.change_illumination(a2["illum_in"], *a2["illum_abc"]), a2["illum_out"])


def test_cv_warp_affine_and_hsv_restatements_agree():
    """tfshim's per-pixel cv2 restatement (imgwarp.cpp / color.cpp order) == the oracle's vectorised one."""
    import sys

    from conftest import GOLDEN
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import tfshim
    from oracle import augment as oa
    cv2 = tfshim.make_cv2()
    rs = np.random.RandomState(1)
    for src in [(rs.rand(23, 31, 3) * 255).astype(np.uint8), rs.rand(23, 31)]:
        for M in [np.float32([[1, 0, 3], [0, 1, -2]]), cv2.getRotationMatrix2D((15, 11), 7.3, 1.1),
                  cv2.getRotationMatrix2D((16, 8), -9.9, 1.02)]:
            assert np.array_equal(cv2.warpAffine(src, M, (31, 23)), oa.warp_affine(src, M, (31, 23)))
    hsv = np.stack(np.meshgrid(np.arange(180), np.arange(0, 256, 3), np.arange(0, 256, 7), indexing="ij"),
                   -1).reshape(-1, 1, 3).astype(np.uint8)[::7]
    assert np.array_equal(cv2.cvtColor(hsv, cv2.COLOR_HSV2BGR), oa.hsv2bgr(hsv))
    bgr = (rs.rand(30, 40, 3) * 255).astype(np.uint8)
    assert np.array_equal(cv2.cvtColor(bgr, cv2.COLOR_BGR2HSV), oa.bgr2hsv(bgr))


@pytest.mark.parametrize("i", [0, 1, 2])
def test_trimap_oracle_matches_reference(i):
    """data.trimap_from_matte's raster loop (run verbatim for the fixture) == the half-window restatement."""
    from oracle import data as od
    g = golden("trimap")
    assert np.array_equal(od.trimap_from_matte(g["matte%d" % i]), g["trimap%d" % i])
