"""Numpy restatement of the training-sample loader (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product (video-matting_amd/vmatting/loader.py + csrc/loader.hip) never does.

Restated from the reference, on already-decoded arrays:
  pad_axis / plan_crop  <- get_padded_img (loader.py:10-36) and the np.random draw order of
                           load_and_crop (loader.py:39-85), simple_load_crop (:119-157) and
                           video_load_crop (:285-330): crop type, [canvas placement], crop corner,
                           background canvas placement, background crop corner
  resize_linear         <- cv2.resize(src float64, dsize, INTER_LINEAR) (loader.py:70-73 ...),
                           OpenCV 3.x imgproc/resize.cpp semantics:
                             * dsize == ssize: plain copy;
                             * both scale factors exactly 2: the INTER_AREA fast path,
                               ((a + b) + c) + d over the 2x2 block (row-major), times 0.25f;
                             * otherwise separable bilinear, float32 coefficients, float64 sums:
                               f = (float)((d + 0.5) * scale - 0.5), s = floor(f), f -= s;
                               columns: s < 0 -> (s, f) = (0, 0); s >= n-1 -> (n-1, 0) and the
                               column is copied (S[s] * 1); rows: indices clamped to [0, n-1],
                               coefficients NOT zeroed; row pass H = S[s]*a0 + S[s+1]*a1,
                               column pass D = H[r0]*b0 + H[r1]*b1
  compose               <- reader.create_composite_image (reader.py:72-79) and the VGG_MEAN
                           subtraction (loader.py:76-77, 151-152, 322-323)
  the previous-alpha warp of video_load_crop (loader.py:291-293) is oracle.flow.warp_img
  (cv2.remap, 1/32-px fixed point) on the float64 alpha.

Pinned by tests/golden/loader_*.npz: make_golden.py runs the reference's loader.py itself on
synthetic PNG/.flo files, with cv2.resize / cv2.imread answered by tests/golden/tfshim.py (an
independent loop-form restatement).  Against real OpenCV the resize is "parity unpinned"
(cv2 is not installed in this image).
"""

import numpy as np

from oracle.flow import warp_img

VGG_MEAN = [103.939, 116.779, 123.68]  # params.py:10
CROP_TYPES = [(320, 320), (480, 480), (640, 640)]  # loader.py:47, 124, 294
DBL_EPSILON = np.finfo(np.float64).eps


class Axis:
    """One axis of a padded+cropped source: resize-source index u in [0, n) reads canvas index
    t = u + off; the canvas holds image data on [lo, hi) at image index t + shift, zero elsewhere."""

    __slots__ = ("n", "off", "lo", "hi", "shift")

    def __init__(self, n, off, lo, hi, shift):
        self.n, self.off, self.lo, self.hi, self.shift = int(n), int(off), int(lo), int(hi), int(shift)

    def astuple(self):
        return (self.n, self.off, self.lo, self.hi, self.shift)

    def gather(self, img, axis):
        """The cropped canvas along ``axis`` (zeros outside the image data)."""
        t = np.arange(self.n) + self.off
        ok = (t >= self.lo) & (t < self.hi)
        idx = np.where(ok, t + self.shift, 0)
        out = np.take(img, idx, axis=axis)
        shape = [1] * img.ndim
        shape[axis] = self.n
        return np.where(ok.reshape(shape), out, 0).astype(img.dtype)


def pad_axis(n, crop):
    """get_padded_img along one axis (loader.py:15-34): returns (canvas length, lo, hi, shift).

    crop > n: the image lands at a random offset of a crop-long zero canvas;
    crop <= n: a random crop-long window of the image lands at the START of an n-long canvas
    whose remaining n - crop entries stay zero (the reference's canvas is max(crop, n) long).
    """
    if crop > n:
        beg_out = np.random.randint(0, crop - n + 1)
        return crop, beg_out, beg_out + n, -beg_out
    beg_in = np.random.randint(0, n - crop + 1)
    return n, 0, crop, beg_in


def _slice(canvas, lo, hi, shift, start, length):
    """canvas[start:start+length] with numpy's truncation at the canvas end."""
    n = max(0, min(start + length, canvas) - start)
    return Axis(n, start, lo, hi, shift)


def plan_crop(fg_hw, bg_hw):
    """The draws of load_and_crop / simple_load_crop / video_load_crop, in the reference's order.

    Returns (crop_hw, fg_rows, fg_cols, bg_rows, bg_cols) Axis objects.  Every np.random call has
    the reference's arguments, so a reference-seeded global RandomState is consumed identically.
    """
    fg_h, fg_w = fg_hw
    crop_h, crop_w = CROP_TYPES[np.random.randint(0, len(CROP_TYPES))]  # loader.py:48
    if fg_h < crop_h or fg_w < crop_w:  # loader.py:50-55: pad the (fg, alpha, ...) stack
        rows = pad_axis(fg_h, crop_h)
        cols = pad_axis(fg_w, crop_w)
    else:
        rows = (fg_h, 0, fg_h, 0)
        cols = (fg_w, 0, fg_w, 0)
    ch, cw = rows[0], cols[0]
    i, j = np.random.randint(0, ch - crop_h + 1), np.random.randint(0, cw - crop_w + 1)  # loader.py:59
    # loader.py:60-62 slices [i:i+crop_h, j:j+crop_h] -- crop_h on both axes (the crops are square)
    fr = _slice(ch, rows[1], rows[2], rows[3], i, crop_h)
    fc = _slice(cw, cols[1], cols[2], cols[3], j, crop_h)
    bg_h, bg_w = bg_hw
    # loader.py:65-66: fg.shape is the cropped foreground here
    bg_crop_h = int(np.ceil(crop_h * bg_h / fr.n))
    bg_crop_w = int(np.ceil(crop_w * bg_w / fc.n))
    brows = pad_axis(bg_h, bg_crop_h)  # loader.py:67
    bcols = pad_axis(bg_w, bg_crop_w)
    # loader.py:68: the corner is drawn from the UNPADDED background's shape
    bi, bj = np.random.randint(0, bg_h - bg_crop_h + 1), np.random.randint(0, bg_w - bg_crop_w + 1)
    br = _slice(brows[0], brows[1], brows[2], brows[3], bi, bg_crop_h)
    bc = _slice(bcols[0], bcols[1], bcols[2], bcols[3], bj, bg_crop_w)
    return (crop_h, crop_w), fr, fc, br, bc


# ---------------------------------------------------------------- cv2.resize, INTER_LINEAR, float64

def _col_table(n, dn):
    scale = 1.0 / (float(dn) / float(n))
    f = ((np.arange(dn) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    neg = s < 0
    f[neg] = 0
    s[neg] = 0
    single = s + 1 >= n
    right = s >= n - 1
    f[right] = 0
    s[right] = n - 1
    a0 = (np.float32(1) - f).astype(np.float32)
    return s, a0.astype(np.float64), f.astype(np.float64), single


def _row_table(n, dn):
    scale = 1.0 / (float(dn) / float(n))
    f = ((np.arange(dn) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    b0 = (np.float32(1) - f).astype(np.float32)
    return np.clip(s, 0, n - 1), np.clip(s + 1, 0, n - 1), b0.astype(np.float64), f.astype(np.float64)


def _area2(n, dn):
    scale = 1.0 / (float(dn) / float(n))
    iscale = int(np.rint(scale))
    return abs(scale - iscale) < DBL_EPSILON and iscale == 2


def resize_linear(img, dsize):
    """cv2.resize(img, dsize=(w, h), interpolation=INTER_LINEAR) for a float64 [H,W] or [H,W,C] array.

    A [H,W,1] input returns [h,w] like OpenCV (single-channel Mats come back 2-D)."""
    img = np.asarray(img, np.float64)
    if img.ndim == 3 and img.shape[2] == 1:
        img = img[:, :, 0]
    ow, oh = int(dsize[0]), int(dsize[1])
    h, w = img.shape[:2]
    if (h, w) == (oh, ow):
        return img.copy()
    if _area2(w, ow) and _area2(h, oh):
        s = img[0:2 * oh:2, 0:2 * ow:2] + img[0:2 * oh:2, 1:2 * ow:2]
        s = s + img[1:2 * oh:2, 0:2 * ow:2]
        s = s + img[1:2 * oh:2, 1:2 * ow:2]
        return s * np.float64(np.float32(0.25))
    s, a0, a1, single = _col_table(w, ow)
    s1 = np.minimum(s + 1, w - 1)
    ex = (slice(None),) + (None,) * (img.ndim - 2)
    hrow = img[:, s] * a0[ex] + img[:, s1] * a1[ex]
    hrow[:, single] = img[:, s[single]]
    r0, r1, b0, b1 = _row_table(h, oh)
    ey = (slice(None),) + (None,) * (img.ndim - 1)
    return hrow[r0] * b0[ey] + hrow[r1] * b1[ey]


# ---------------------------------------------------------------- one sample

def crop_sources(fg_bgra, bg_bgr, fr, fc, br, bc, prev_bgra=None, flow=None):
    """The float64 arrays the reference hands to cv2.resize: fg crop [h,w,3], alpha crop [h,w],
    warped-alpha crop [h,w] (or None) and the background crop [hb,wb,3]."""
    fg = np.asarray(fg_bgra[:, :, :3], np.float64)  # loader.py:43 (astype float)
    alpha = fg_bgra[:, :, 3] / 255.  # reader.py:16
    warped = None
    if prev_bgra is not None:
        prev_alpha = prev_bgra[:, :, 3] / 255.
        warped = warp_img(prev_alpha, flow)  # loader.py:292 (flow.py:9-18)
    crop = lambda a: fc.gather(fr.gather(a, 0), 1)  # noqa: E731
    bg = np.asarray(bg_bgr, np.float64)
    return crop(fg), crop(alpha), (crop(warped) if warped is not None else None), bc.gather(br.gather(bg, 0), 1)


def compose(fg_c, alpha_c, bg_c, input_size, warped_c=None):
    """loader.py:70-77 (resize everything to input_size, composite, subtract VGG_MEAN)."""
    bg = resize_linear(bg_c, input_size)
    fg = resize_linear(fg_c, input_size)
    alpha = resize_linear(alpha_c, input_size)
    out = {}
    if warped_c is not None:
        w = resize_linear(warped_c, input_size)
        out["warped"] = np.repeat(w[:, :, None], 3, axis=2)  # loader.py:293 repeats before resizing
    tri = np.repeat(alpha[:, :, None], 3, axis=2)
    cmp = tri * fg + (1. - tri) * bg  # reader.py:78
    out["cmp"] = cmp - VGG_MEAN
    out["bg"] = bg - VGG_MEAN
    out["label"] = alpha.reshape(alpha.shape[0], alpha.shape[1], 1)
    out["fg"] = fg
    return out


def load_sample(fg_bgra, bg_bgr, input_size, prev_bgra=None, flow=None):
    """One *_load_crop call on decoded arrays: draws from the global np.random like the reference
    and returns (plan, outputs).  outputs: cmp, bg (mean-subtracted), label [h,w,1], fg and, when
    prev_bgra/flow are given (video_load_crop), warped [h,w,3]; all float64."""
    crop_hw, fr, fc, br, bc = plan_crop(fg_bgra.shape[:2], bg_bgr.shape[:2])
    fg_c, a_c, w_c, bg_c = crop_sources(fg_bgra, bg_bgr, fr, fc, br, bc, prev_bgra, flow)
    return (crop_hw, fr, fc, br, bc), compose(fg_c, a_c, bg_c, input_size, w_c)


def batch(samples, input_size, mirror=False):
    """get_batch / simple_batch / video_batch (loader.py:93-116, 160-171, 333-345) over decoded
    samples [(fg_bgra, bg_bgr[, prev_bgra, flow])]: per sample one load_sample, then (get_batch with
    rd_mirror) one np.random.uniform draw that flips the sample left-right when > 0.5."""
    outs = []
    for s in samples:
        _, o = load_sample(s[0], s[1], input_size, *(s[2:] if len(s) > 2 else ()))
        if mirror and np.random.uniform(0., 1.) > 0.5:  # loader.py:105-109
            o = {k: np.flip(v, axis=1) for k, v in o.items()}
        outs.append(o)
    return {k: np.stack([o[k] for o in outs]) for k in outs[0]}


# ---------------------------------------------------------------- synthetic decoded inputs (fixtures)

def synthetic_entry(seed, fg_hw, bg_hw, video=True):
    """Deterministic decoded inputs of one loader entry: fg BGRA u8 (smooth colours, soft-edged
    alpha ellipse), bg BGR u8, and for video entries the previous frame's BGRA u8 and a smooth
    backward flow quantised to 1/64 px (float32)."""
    from oracle.flow import smooth_flow
    rs = np.random.RandomState(seed)
    h, w = fg_hw

    def image(hh, ww, ch):
        yy, xx = np.mgrid[0:hh, 0:ww].astype(np.float64)
        out = np.empty((hh, ww, ch))
        for k in range(ch):
            fy, fx, ph = rs.uniform(0.5, 4.0) / hh, rs.uniform(0.5, 4.0) / ww, rs.uniform(0, 6.3)
            out[..., k] = 127.5 + 100 * np.sin(2 * np.pi * (fy * yy + fx * xx) + ph)
        out += rs.uniform(-20, 20, out.shape)
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)

    def matte():
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
        cy, cx = rs.uniform(0.3, 0.7) * h, rs.uniform(0.3, 0.7) * w
        ry, rx = rs.uniform(0.2, 0.4) * h, rs.uniform(0.2, 0.4) * w
        d = np.sqrt(((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2)
        a = np.clip((1.15 - d) / 0.3, 0, 1) * 255
        return np.rint(a).astype(np.uint8)

    fg = np.concatenate([image(h, w, 3), matte()[..., None]], axis=2)
    bg = image(bg_hw[0], bg_hw[1], 3)
    if not video:
        return fg, bg
    prev = np.concatenate([image(h, w, 3), matte()[..., None]], axis=2)
    flow = smooth_flow(h, w, seed=seed + 100, amp=12.0)
    flow = (np.rint(flow.astype(np.float64) * 64) / 64).astype(np.float32)
    return fg, bg, prev, flow
