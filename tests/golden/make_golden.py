"""Generate the committed golden fixtures by running the REFERENCE's own code.

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

Runs in the development container only (it reads /root/reference, which does
not exist on the GPU box; the fixtures it writes are what travels).

What runs for real: the reference modules unet.py, unet_simple.py, small.py,
refine.py, flow.py, reader.py and train.py are imported from /root/reference
unchanged; their graph builders, ``flow.correct_alpha``, ``reader.read_flow``,
``reader.create_composite_image`` and ``train.composite``/``regular_l1`` execute
verbatim.  TensorFlow and OpenCV are absent from the image, so ``tensorflow``
and ``cv2`` resolve to tfshim.py (literal restatements of the TF-1.x / OpenCV
kernels); numpy-2 removed the ``np.float``/``np.int`` aliases the reference
uses, so they are restored; ``np.load`` of the absent weights/vgg16.npy is
answered with a seeded synthetic VGG16 dict.  Weights are never stored: tests
rebuild them from the recorded seeds.
"""

import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import tfshim  # noqa: E402
from oracle.models import synthetic_vgg16  # noqa: E402  (seeded data generator only)
from oracle.flow import smooth_flow, write_flow  # noqa: E402  (fixture data only)

VGG_MEAN = np.array([103.939, 116.779, 123.68])


def load_reference():
    sys.modules["tensorflow"] = tfshim.make_tf()
    sys.modules["cv2"] = tfshim.make_cv2()
    for m in ("progressbar", "skimage", "skimage.io", "skimage.transform"):
        sys.modules[m] = types.ModuleType(m)
    np.float = float  # numpy<1.24 aliases used by reader.py:74, flow.py:38, loader.py:43
    np.int = int
    sys.path.insert(0, REF)
    import unet, unet_simple, small, refine, flow, reader, train, tps, augmentation, data  # noqa: E401
    return types.SimpleNamespace(unet=unet, unet_simple=unet_simple, small=small, refine=refine,
                                 flow=flow, reader=reader, train=train, tps=tps, augmentation=augmentation,
                                 data=data)


_VGG = {}
_orig_load = np.load


def _fake_load(path, *a, **k):
    if isinstance(path, str) and path.endswith(os.path.join("weights", "vgg16.npy")):
        path = vgg_path(0)  # the default path (unet_simple.py:47-51) -> synthetic VGG seed 0
    if isinstance(path, str) and path.startswith("vgg-seed:"):
        arr = np.empty((), dtype=object)
        arr[()] = _VGG[path]
        return arr
    return _orig_load(path, *a, **k)


def vgg_path(seed, scale=1.0):
    key = "vgg-seed:%d:%g" % (seed, scale)
    _VGG[key] = synthetic_vgg16(seed, scale)
    return key


def synth_frames(n, h, w, seed, scale=1.0):
    """7-channel frames like SURVEY.md §8d: cmp/bg BGR U{0..255} - VGG_MEAN, trimap in {0,.5,1} - .5."""
    rs = np.random.RandomState(seed)
    cmp = rs.randint(0, 256, (n, h, w, 3)).astype(np.float64) - VGG_MEAN
    bg = rs.randint(0, 256, (n, h, w, 3)).astype(np.float64) - VGG_MEAN
    yy, xx = np.mgrid[0:h, 0:w]
    tri = np.zeros((n, h, w, 1))
    for i in range(n):
        cy, cx = rs.uniform(0.3, 0.7) * h, rs.uniform(0.3, 0.7) * w
        ry, rx = rs.uniform(0.15, 0.3) * h, rs.uniform(0.15, 0.3) * w
        d = np.sqrt(((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2)
        t = np.where(d < 0.85, 1.0, np.where(d < 1.15, 0.5, 0.0))
        tri[i, :, :, 0] = t
    x = np.concatenate([cmp, bg, tri - 0.5], axis=-1) * scale
    return x.astype(np.float32)


class SigmoidTap:
    """Records the input of every tf.nn.sigmoid call (the pre-sigmoid logits)."""

    def __init__(self, tf):
        self.tf = tf
        self.inputs = []
        self._orig = tf.nn.sigmoid

    def __enter__(self):
        def tap(x, name=None):
            self.inputs.append(np.asarray(x, np.float64))
            return self._orig(x, name)
        self.tf.nn.sigmoid = tap
        return self

    def __exit__(self, *a):
        self.tf.nn.sigmoid = self._orig


def var_summary():
    names = [n for n, _ in tfshim.REG.variables]
    shapes = [str(v.shape) for _, v in tfshim.REG.variables]
    sums = np.array([float(np.asarray(v, np.float64).sum()) for _, v in tfshim.REG.variables])
    firsts = np.array([float(np.asarray(v, np.float64).ravel()[0]) for _, v in tfshim.REG.variables])
    tfshim.REG.variables.clear()
    return {"var_names": np.array(names), "var_shapes": np.array(shapes), "var_sums": sums, "var_firsts": firsts}


def load_png_bgra(path):
    from PIL import Image
    im = np.asarray(Image.open(path))
    if im.ndim == 3 and im.shape[2] == 4:
        return im[:, :, [2, 1, 0, 3]]
    return im[:, :, [2, 1, 0]]


def resize_u8(img, w, h):
    from PIL import Image
    return np.asarray(Image.fromarray(img).resize((w, h), Image.BILINEAR))


def gen_unet(R, out):
    tf = sys.modules["tensorflow"]
    cases = [("unet_video_70x90", R.unet.UNetVideo, 7, 70, 90, 1.0),
             ("unet_video_64x96", R.unet.UNetVideo, 7, 64, 96, 1.0),
             ("unet_video_70x90_unit", R.unet.UNetVideo, 7, 70, 90, 1.0 / 128),
             ("unet_image_70x90", R.unet.UNetImage, 6, 70, 90, 1.0)]
    for i, (name, cls, ch, h, w, in_scale) in enumerate(cases):
        vseed, wseed, xseed = 0, 1 + i, 1234 + i
        x = synth_frames(1, h, w, xseed, in_scale)[..., :ch]
        np.random.seed(wseed)
        m = cls(vgg_path(vseed))
        m.build(x)
        d = dict(x=x, output=np.asarray(m.output), logits=np.asarray(m.conv1_3),
                 pool4=np.asarray(m.pool4, np.float32), upconv1=np.asarray(m.upconv1, np.float32),
                 conv2_3=np.asarray(m.conv2_3, np.float32),
                 vgg_seed=vseed, weight_seed=wseed, video=int(ch == 7))
        d.update(var_summary())
        out[name] = d
        print(name, "logits range", d["logits"].min(), d["logits"].max())
    del tf


def gen_unet_simple(R, out):
    tf = sys.modules["tensorflow"]
    fgimg = load_png_bgra(os.path.join(REF, "test_data", "in0062.png"))
    alpha = fgimg[:, :, 3] / 255.0  # reader.read_fg_img semantics (reader.py:16-17)
    fg = fgimg[:, :, :3]
    sea = load_png_bgra(os.path.join(REF, "test_data", "sea.jpg"))
    bg = resize_u8(sea, fg.shape[1], fg.shape[0])
    cmp = R.reader.create_composite_image(fg, bg, alpha)  # the reference's compositing, for real
    cmp_u8 = np.clip(np.rint(cmp), 0, 255).astype(np.uint8)
    cmp256 = resize_u8(cmp_u8, 256, 256)
    bg256 = resize_u8(bg, 256, 256)
    for name, phase, n, sz in (("unet_simple_256_infer", False, 1, 256), ("unet_simple_64_train", True, 2, 64)):
        if n == 1:
            c8, b8 = cmp256[None], bg256[None]
        else:
            c8 = np.stack([cmp256[:sz, :sz], cmp256[100:100 + sz, 60:60 + sz]])
            b8 = np.stack([bg256[:sz, :sz], bg256[100:100 + sz, 60:60 + sz]])
        c = c8.astype(np.float64) - VGG_MEAN  # loader.py:76-77
        b = b8.astype(np.float64) - VGG_MEAN
        diff = c - b  # train.py:245
        np.random.seed(11)
        with SigmoidTap(tf) as tap:
            m = R.unet_simple.create_model(c, b, diff, phase)
        d = dict(cmp_u8=c8, bg_u8=b8, phase=int(phase), output=np.asarray(m.output),
                 logits=tap.inputs[-1],
                 upconv4=np.asarray(m.upconv4, np.float32), vgg_seed=0, weight_seed=11)
        d.update(var_summary())
        out[name] = d
        print(name, "logits range", d["logits"].min(), d["logits"].max())


def gen_small(R, out):
    tf = sys.modules["tensorflow"]
    for name, phase, n in (("small_70x90_infer", False, 1), ("small_70x90_train", True, 2)):
        x = synth_frames(n, 70, 90, 99, 1.0)[..., :6]
        np.random.seed(21)
        with SigmoidTap(tf) as tap:
            m = R.small.UNetSmall(x, phase)
        d = dict(x=x, phase=int(phase), output=np.asarray(m.output), logits=tap.inputs[-1],
                 upconv2=np.asarray(m.upconv2, np.float32), weight_seed=21)
        d.update(var_summary())
        out[name] = d


def gen_refine(R, out):
    x = synth_frames(1, 40, 56, 77, 1.0 / 128)[..., :5]
    np.random.seed(31)
    m = R.refine.RefineNet()
    m.build(x)
    d = dict(x=x, output=np.asarray(m.output), conv1_sum=float(np.sum(m.conv1)), weight_seed=31)
    d.update(var_summary())
    out["refine_40x56"] = d


def gen_flow(R, out):
    fgimg = load_png_bgra(os.path.join(REF, "test_data", "in0062.png"))
    h, w = fgimg.shape[:2]
    fb = smooth_flow(h, w, seed=7)
    ff = smooth_flow(h, w, seed=8)
    with tempfile.TemporaryDirectory() as td:
        pb, pf = os.path.join(td, "backward.flo"), os.path.join(td, "forward.flo")
        write_flow(pb, fb)
        write_flow(pf, ff)
        rb = R.reader.read_flow(pb)  # the reference reader, for real
        rf = R.reader.read_flow(pf)
        raw_head = open(pb, "rb").read(12 + 4 * 2 * 8)
    assert np.array_equal(rb, fb) and np.array_equal(rf, ff)
    alpha = fgimg[:, :, 3] / 255.0
    warped = R.flow.warp_img(alpha, rb)  # flow.py:9-18 (cv2.remap via tfshim)
    corrected = R.flow.correct_alpha(rb, rf, warped.copy())  # flow.py:36-65, runs for real
    zero_mask = (corrected == 0) & (warped != 0)
    # crafted small case with negative (wrapping) indices and large displacements
    rs = np.random.RandomState(5)
    hb, wb = 48, 64
    b2 = rs.uniform(-40, 25, (hb, wb, 2)).astype(np.float32)
    f2 = rs.uniform(-30, 30, (hb, wb, 2)).astype(np.float32)
    a2 = rs.uniform(0.1, 1.0, (hb, wb))
    c2 = R.flow.correct_alpha(b2, f2, a2.copy())
    # warp_bgr (uint8 path) on a crop
    crop = np.ascontiguousarray(fgimg[100:228, 400:592, :3])
    fc = np.ascontiguousarray(fb[100:228, 400:592])
    bgr = R.flow.warp_bgr(crop, fc)
    out["flow_500x1200"] = dict(
        alpha=alpha.astype(np.float32), alpha_u8=fgimg[:, :, 3], flow_seed_b=7, flow_seed_f=8,
        warped=warped.astype(np.float32), warped_f64_sum=float(warped.sum()),
        corrected_zero_mask=np.packbits(zero_mask), n_zeroed=int(zero_mask.sum()),
        flo_header=np.frombuffer(raw_head, np.uint8),
        small_backward=b2, small_forward=f2, small_alpha=a2, small_corrected=c2,
        bgr_crop=crop, bgr_flow=fc, bgr_warped=bgr)
    print("flow: zeroed", int(zero_mask.sum()), "small zeroed", int((c2 == 0).sum()))


def gen_loss(R, out):
    rs = np.random.RandomState(3)
    n, h, w = 2, 32, 32
    pred = rs.uniform(0, 1, (n, h, w, 1))
    gt = rs.uniform(0, 1, (n, h, w, 1))
    raw_fg = rs.uniform(0, 255, (n, h, w, 3))
    in_bg = rs.uniform(0, 255, (n, h, w, 3)) - VGG_MEAN
    in_cmp = rs.uniform(0, 255, (n, h, w, 3)) - VGG_MEAN
    tf = sys.modules["tensorflow"]
    # train.py:42-47 verbatim expressions over the reference helpers
    alpha_loss = R.train.regular_l1(pred, gt, name="alpha_loss")
    pred_cmp = R.train.composite(raw_fg, in_bg, pred)
    cmp_loss = R.train.regular_l1(pred_cmp, in_cmp, name="compositional_loss")
    s_loss = tf.add(0.5 * alpha_loss, 0.5 * cmp_loss)
    loss = tf.reduce_mean(s_loss, name="loss")
    out["loss_2x32x32"] = dict(pred=pred, gt=gt, raw_fg=raw_fg, in_bg=in_bg, in_cmp=in_cmp,
                               loss=float(loss), alpha_loss=float(np.mean(alpha_loss)),
                               cmp_loss=float(np.mean(cmp_loss)))


# loader entries: (seed, fg_hw, bg_hw, video).  E2's 300 x 700 foreground takes both branches of
# get_padded_img for the 320 crop (rows padded, columns cropped into a zero-tailed canvas).
LOADER_ENTRIES = [(41, (330, 340), (250, 300), True), (42, (330, 340), (640, 640), True),
                  (43, (300, 700), (500, 375), False), (44, (520, 360), (330, 420), False)]
# calls: (fn, entry indices, global np.random seed, input_size, rd_mirror)
LOADER_CALLS = [("video_load_crop", [0], 0, (320, 320), 0), ("video_load_crop", [0], 1, (320, 320), 0),
                ("video_load_crop", [1], 2, (320, 320), 0), ("video_load_crop", [1], 5, (320, 320), 0),
                ("video_load_crop", [0], 3, (200, 200), 0), ("video_load_crop", [1], 4, (160, 160), 0),
                ("simple_load_crop", [2], 6, (320, 320), 0), ("simple_load_crop", [2], 7, (96, 96), 0),
                ("simple_load_crop", [3], 8, (320, 320), 0),
                ("get_batch", [2, 3, 2], 9, (64, 64), 1), ("video_batch", [0, 1], 10, (96, 96), 0)]
LOADER_OUTS = {"video_load_crop": ("cmp", "bg", "label", "warped", "fg"),
               "simple_load_crop": ("cmp", "bg", "label", "fg"),
               "get_batch": ("input", "label", "fg"),
               "video_batch": ("cmp", "bg", "label", "warped", "fg")}


def _write_loader_entry(td, idx):
    from PIL import Image
    from oracle.loader import synthetic_entry
    seed, fg_hw, bg_hw, video = LOADER_ENTRIES[idx]
    ent = synthetic_entry(seed, fg_hw, bg_hw, video)
    p = lambda s: os.path.join(td, "e%d_%s" % (idx, s))  # noqa: E731
    Image.fromarray(np.ascontiguousarray(ent[0][:, :, [2, 1, 0, 3]])).save(p("fg.png"))  # BGRA -> RGBA file
    Image.fromarray(np.ascontiguousarray(ent[1][:, :, ::-1])).save(p("bg.png"))
    if video:
        Image.fromarray(np.ascontiguousarray(ent[2][:, :, [2, 1, 0, 3]])).save(p("prev.png"))
        write_flow(p("flow.flo"), ent[3])
        return (p("fg.png"), p("bg.png"), p("prev.png"), p("flow.flo"))
    a = ent[0][:, :, 3]
    tri = np.where(a == 255, 255, np.where(a == 0, 0, 128)).astype(np.uint8)
    Image.fromarray(tri).save(p("trimap.png"))
    return (p("fg.png"), p("trimap.png"), p("bg.png"))


def gen_loader(R, out):
    """Run the reference's loader.py (load_and_crop via get_batch, simple_load_crop, video_load_crop,
    video_batch) on synthetic PNG / .flo files; keep 1024 sampled pixels of every output plane
    (float64, exact), float64 plane sums, and the next global np.random draw (draw-count check)."""
    sys.path.insert(0, REF)
    import loader  # the reference module, for real
    d = {"entries": np.array([[s, f[0], f[1], b[0], b[1], int(v)] for s, f, b, v in LOADER_ENTRIES]),
         "n_calls": len(LOADER_CALLS)}
    with tempfile.TemporaryDirectory() as td:
        paths = [_write_loader_entry(td, i) for i in range(len(LOADER_ENTRIES))]
        for ci, (fn, ents, seed, size, mirror) in enumerate(LOADER_CALLS):
            np.random.seed(seed)
            if fn == "get_batch":
                res = loader.get_batch([list(paths[e]) for e in ents], size, rd_scale=False, rd_mirror=bool(mirror))
            elif fn.endswith("_batch"):
                res = getattr(loader, fn)([paths[e] for e in ents], size)
            else:
                res = getattr(loader, fn)(paths[ents[0]], size)
            nxt = np.random.randint(0, 2 ** 31 - 1)
            res = [np.asarray(r, np.float64) for r in res]
            if not fn.endswith("batch"):
                res = [r[None] for r in res]
            n, oh, ow = res[0].shape[:3]
            rs = np.random.RandomState(1000 + ci)
            pn, py, px = rs.randint(0, n, 1024), rs.randint(0, oh, 1024), rs.randint(0, ow, 1024)
            pre = "c%d_" % ci
            d[pre + "meta"] = np.array([seed, size[0], size[1], mirror, nxt])
            d[pre + "fn"] = np.array(fn)
            d[pre + "entries"] = np.array(ents)
            d[pre + "pos"] = np.stack([pn, py, px])
            for name, r in zip(LOADER_OUTS[fn], res):
                d[pre + name + "_vals"] = r[pn, py, px]
                d[pre + name + "_sum"] = np.array(float(r.sum()))
            print("loader call", ci, fn, "crop type", [np.random.RandomState(seed).randint(0, 3)], "shape", res[0].shape)
    out["loader_calls"] = d


def gen_tps(R, out):
    """tps.warp_images / tps.deform run for REAL (numpy + scipy 1.15.3 ndimage.map_coordinates; only the unused
    `import cv2` of tps.py resolves to the shim)."""
    d = {}
    fgimg = load_png_bgra(os.path.join(REF, "test_data", "in0062.png"))
    img = resize_u8(np.ascontiguousarray(fgimg[:, :, :3]), 70, 45)          # [45, 70, 3] u8
    alpha = resize_u8(np.ascontiguousarray(fgimg[:, :, 3]), 70, 45) / 255.  # [45, 70] f64
    rs = np.random.RandomState(11)
    cases = [  # (name, region, approximate_grid, order, grid seed, grid h/w)
        ("a", (0, 0, 45, 70), 2, 1, 3),
        ("b", (0, 0, 33, 47), 1, 1, 4),
        ("c", (5, 3, 40, 60), 3, 0, 5),
        ("d", (0, 0, 45, 70), 2.5, 1, 6),
    ]
    for name, region, ag, order, seed in cases:
        np.random.seed(seed)
        h, w = region[2], region[3]
        grid, new_grid = R.augmentation.deform_grid(h, w)
        planes = [img[:, :, 0], img[:, :, 1], img[:, :, 2], alpha, (rs.rand(45, 70) * 4 - 1).astype(np.float32)]
        res = R.tps.warp_images(grid, new_grid, planes, region, interpolation_order=order, approximate_grid=ag)
        d[name + "_from"], d[name + "_to"] = grid, new_grid
        d[name + "_region"], d[name + "_ag"], d[name + "_order"] = np.array(region), np.array(ag), np.array(order)
        d[name + "_f32_in"] = planes[4]
        d[name + "_u8"] = np.stack(res[:3], axis=-1)
        d[name + "_f64"] = res[3]
        d[name + "_f32"] = res[4]
    np.random.seed(21)
    d["deform_out"] = R.tps.deform(img)
    d["img"], d["alpha"] = img, alpha
    out["tps"] = d


def gen_augment(R, out):
    """augmentation.augment (augmentation.py:101-135) run verbatim: its np.random draws, deform_grid, tps.py
    (real scipy) and the cv2 calls (warpAffine / getRotationMatrix2D / cvtColor HSV from tfshim)."""
    d = {}
    fgimg = load_png_bgra(os.path.join(REF, "test_data", "in0062.png"))
    bgimg = load_png_bgra(os.path.join(REF, "test_data", "cmp1.png"))
    for i, (h, w, seed) in enumerate([(48, 64, 31), (57, 83, 32)]):
        fg = resize_u8(np.ascontiguousarray(fgimg[:, :, :3]), w, h)
        alpha = resize_u8(np.ascontiguousarray(fgimg[:, :, 3]), w, h) / 255.
        bg = resize_u8(np.ascontiguousarray(bgimg[:, :, :3]), w, h)
        np.random.seed(seed)
        nfg, nbg, nal = R.augmentation.augment(fg, bg, alpha)
        d["fg%d" % i], d["bg%d" % i], d["alpha%d" % i], d["seed%d" % i] = fg, bg, alpha, np.array(seed)
        d["new_fg%d" % i], d["new_bg%d" % i], d["new_alpha%d" % i] = nfg, nbg, nal
        d["next_draw%d" % i] = np.array(np.random.randint(0, 1 << 30))
    # change_illumination alone over every HSV corner case
    rs = np.random.RandomState(5)
    px = rs.randint(0, 256, (16, 40, 3)).astype(np.uint8)
    px[0, :6] = [[0, 0, 0], [255, 255, 255], [7, 7, 7], [0, 0, 255], [255, 0, 0], [3, 250, 3]]
    d["illum_in"] = px
    d["illum_abc"] = np.array([1.03, 0.81, -0.05])
    d["illum_out"] = R.augmentation.change_illumination(px, 1.03, 0.81, -0.05)
    out["augment"] = d


def gen_trimap(R, out):
    """data.trimap_from_matte (data.py:37-67) run verbatim (pure-Python raster loop) on the in0062.png alpha
    (resized), on a matte with isolated unknown pixels next to 0 and 1, and on image-border cases."""
    d = {}
    fgimg = load_png_bgra(os.path.join(REF, "test_data", "in0062.png"))
    m0 = resize_u8(np.ascontiguousarray(fgimg[:, :, 3]), 60, 144) / 255.
    rs = np.random.RandomState(13)
    m1 = np.where(rs.rand(37, 41) < 0.5, 0., 1.)
    m1[rs.rand(37, 41) < 0.05] = 0.5
    m1[0, 0] = m1[-1, -1] = m1[0, -1] = m1[-1, 0] = 0.25
    m2 = np.zeros((9, 11))
    m2[4, 5] = 0.7
    m2[:, 7:] = 1.
    for i, m in enumerate([m0, m1, m2]):
        d["matte%d" % i] = m
        d["trimap%d" % i] = R.data.trimap_from_matte(m)
    out["trimap"] = d


def main():
    np.load = _fake_load
    R = load_reference()
    out = {}
    if len(sys.argv) > 1:  # regenerate only the named fixtures: make_golden.py loader
        for name in sys.argv[1:]:
            globals()["gen_" + name](R, out)
        for name, d in out.items():
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
            print("wrote", name, os.path.getsize(os.path.join(HERE, name + ".npz")))
        return
    gen_unet(R, out)
    gen_refine(R, out)
    gen_small(R, out)
    gen_flow(R, out)
    gen_loss(R, out)
    gen_unet_simple(R, out)
    gen_loader(R, out)
    gen_tps(R, out)
    gen_augment(R, out)
    gen_trimap(R, out)
    for name, d in out.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, os.path.getsize(os.path.join(HERE, name + ".npz")))


if __name__ == "__main__":
    main()
