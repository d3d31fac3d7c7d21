"""Numpy restatement of the two-frame temporal path (TEST INFRASTRUCTURE).

  warp_img        <- flow.warp_img   (flow.py:9-18)   = cv2.remap(INTER_LINEAR, BORDER_CONSTANT 0)
  warp_bgr        <- flow.warp_bgr   (flow.py:21-33)  = the same remap on three uint8 planes
  correct_alpha   <- flow.correct_alpha (flow.py:36-65) forward/backward consistency mask
  read_flow       <- reader.read_flow (reader.py:21-30) Middlebury .flo
  write_flow      -- inverse of read_flow (fixture generation)

OpenCV remap semantics restated (OpenCV 3.x imgproc/imgwarp):
a CV_32FC2 map is converted per pixel to fixed point X = cvRound(x*32)
(round-half-even), integer part X>>5 (floor), fraction X&31; bilinear weights
are products of (1-f/32, f/32) taken from a 32x32 table; a tap outside the
image reads the border value 0; taps are summed TL, TR, BL, BR in that order.
uint8 images use 15-bit integer weights and (sum + 2^14) >> 15.
"""

import numpy as np

FLO_MAGIC = 202021.25  # reader.py:25

INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS
COEF_BITS = 15


def _coords(h, w, flow):
    """identity + flow as float32, like flow.py:12-17 (map = (identity + flow).astype(np.float32))."""
    jj, ii = np.meshgrid(np.arange(w), np.arange(h))
    mx = (jj + flow[..., 0]).astype(np.float32)  # flow.py:16: identity[...,0] is the column index
    my = (ii + flow[..., 1]).astype(np.float32)
    return mx, my


def _taps(img, mx, my, quantize):
    ih, iw = img.shape[:2]
    if quantize:
        X = np.rint(mx.astype(np.float64) * INTER_TAB_SIZE).astype(np.int64)
        Y = np.rint(my.astype(np.float64) * INTER_TAB_SIZE).astype(np.int64)
        x0, y0 = X >> INTER_BITS, Y >> INTER_BITS
        fx = (X & (INTER_TAB_SIZE - 1)).astype(np.float64) / INTER_TAB_SIZE
        fy = (Y & (INTER_TAB_SIZE - 1)).astype(np.float64) / INTER_TAB_SIZE
        fxi = X & (INTER_TAB_SIZE - 1)
        fyi = Y & (INTER_TAB_SIZE - 1)
    else:
        x0 = np.floor(mx).astype(np.int64)
        y0 = np.floor(my).astype(np.int64)
        fx = mx.astype(np.float64) - x0
        fy = my.astype(np.float64) - y0
        fxi = fyi = None

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < iw) & (yy >= 0) & (yy < ih)
        v = np.zeros(xx.shape, dtype=img.dtype)
        v[ok] = img[yy[ok], xx[ok]]
        return v

    return (tap(y0, x0), tap(y0, x0 + 1), tap(y0 + 1, x0), tap(y0 + 1, x0 + 1)), fx, fy, fxi, fyi


def warp_img(img, flow, mode="opencv"):
    """flow.warp_img (flow.py:9-18): out[y,x] = bilinear(img, x+u, y+v).

    mode 'opencv' reproduces cv2.remap's 1/32-pixel coordinate quantisation;
    mode 'exact' is plain bilinear on the float coordinates.
    """
    assert img.ndim == 2  # flow.py:11
    h, w = flow.shape[:2]
    mx, my = _coords(h, w, flow)
    (v00, v01, v10, v11), fx, fy, _, _ = _taps(img, mx, my, mode == "opencv")
    w00 = (1 - fy) * (1 - fx)
    w01 = (1 - fy) * fx
    w10 = fy * (1 - fx)
    w11 = fy * fx
    out = v00 * w00 + v01 * w01 + v10 * w10 + v11 * w11
    return out.astype(np.result_type(img.dtype, np.float32)) if img.dtype.kind == "f" else out


def warp_plane_u8(img, flow):
    """cv2.remap on one uint8 plane: 15-bit fixed-point weights, (sum + 2^14) >> 15, saturate."""
    h, w = flow.shape[:2]
    mx, my = _coords(h, w, flow)
    (v00, v01, v10, v11), _, _, fxi, fyi = _taps(img, mx, my, True)
    fxi = fxi.astype(np.int64)
    fyi = fyi.astype(np.int64)
    # table weights (32-fy)(32-fx)/1024 * 32768 are exact integers: (32-fy)(32-fx)*32
    w00 = (32 - fyi) * (32 - fxi) * 32
    w01 = (32 - fyi) * fxi * 32
    w10 = fyi * (32 - fxi) * 32
    w11 = fyi * fxi * 32
    s = v00.astype(np.int64) * w00 + v01.astype(np.int64) * w01 + v10.astype(np.int64) * w10 + v11.astype(np.int64) * w11
    return np.clip((s + (1 << (COEF_BITS - 1))) >> COEF_BITS, 0, 255).astype(np.uint8)


def warp_bgr(img, flow):
    """flow.warp_bgr (flow.py:21-33): warp each of the 3 uint8 planes, re-stack."""
    return np.stack([warp_plane_u8(img[:, :, k], flow) for k in range(3)], axis=2)


def correct_alpha(backward, forward, alpha, promote="numpy1", thresh=15.0):
    """flow.correct_alpha (flow.py:36-65), vectorised; mutates ``alpha`` in place and returns it.

    For each (i, j): j0 = min(int(bw[i,j,0] + j), w-1); i0 = min(int(bw[i,j,1] + i), h-1)
    (int() truncates toward zero, no lower clamp: a negative index wraps numpy-style,
    an index < -dim raises IndexError); (j1, i1) the same through fw[i0, j0] from (j0, i0);
    err = ||(i1-i, j1-j)||; alpha[err > 15] = 0.

    ``promote`` picks how ``np.float32 + int`` rounds: 'numpy1' (value-based casting of
    the reference's era — float64, exact) or 'numpy2' (NEP 50 — float32 add).
    """
    h, w = backward.shape[:2]
    jj, ii = np.meshgrid(np.arange(w), np.arange(h))

    def step(fl, base_j, base_i, indexes):
        u = fl[..., 0]
        v = fl[..., 1]
        if promote == "numpy1":
            sj = u.astype(np.float64) + base_j
            si = v.astype(np.float64) + base_i
        else:
            sj = u.astype(np.float32) + base_j.astype(np.float32)
            si = v.astype(np.float32) + base_i.astype(np.float32)
        if not (np.all(np.isfinite(sj)) and np.all(np.isfinite(si))):
            raise ValueError("cannot convert float NaN/inf to integer")
        nj = np.minimum(np.trunc(sj).astype(np.int64), w - 1)
        ni = np.minimum(np.trunc(si).astype(np.int64), h - 1)
        if indexes and ((nj < -w).any() or (ni < -h).any()):  # only (j0, i0) index forward[]
            raise IndexError("flow points outside the frame by more than its size")
        return nj, ni

    j0, i0 = step(backward, jj, ii, True)
    fw = forward[i0 % h, j0 % w]
    j1, i1 = step(fw, j0, i0, False)
    d2 = (i1 - ii) ** 2 + (j1 - jj) ** 2
    err = np.sqrt(d2.astype(np.float64))
    alpha[err > thresh] = 0.0
    return alpha


def read_flow(path):
    """reader.read_flow (reader.py:21-30): float32 magic 202021.25, int32 w, int32 h, h*w*2 float32.

    Bad magic prints and continues, like the reference (reader.py:25-26).
    """
    with open(path, "rb") as f:
        key = np.fromfile(f, dtype=np.float32, count=1)
        if FLO_MAGIC != key:
            print("ERROR: invalid key ({})".format(key))
        w = np.fromfile(f, dtype=np.int32, count=1)[0]
        h = np.fromfile(f, dtype=np.int32, count=1)[0]
        data = np.fromfile(f, dtype=np.float32, count=2 * h * w).reshape((h, w, 2))
        return data


def write_flow(path, flow):
    """Inverse of read_flow (the Middlebury writer the reference never ships)."""
    flow = np.asarray(flow, np.float32)
    h, w = flow.shape[:2]
    with open(path, "wb") as f:
        np.array([FLO_MAGIC], np.float32).tofile(f)
        np.array([w, h], np.int32).tofile(f)
        flow.tofile(f)


def smooth_flow(h, w, seed=7, modes=8, amp=20.0):
    """Synthetic smooth flow field (sum of Gaussian modes, |u|,|v| <= amp)."""
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    out = np.zeros((h, w, 2))
    for _ in range(modes):
        cy, cx = rs.uniform(0, h), rs.uniform(0, w)
        s = rs.uniform(0.1, 0.4) * max(h, w)
        g = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        out[..., 0] += rs.uniform(-1, 1) * g
        out[..., 1] += rs.uniform(-1, 1) * g
    out *= amp / max(1e-9, np.abs(out).max())
    return out.astype(np.float32)
