"""Numpy restatement of the augmentation path, SURVEY.md §8(f) rank 3 (TEST INFRASTRUCTURE ONLY:
imported by tests/ and smoke(), never by the product).

  make_warp_coeffs   <- tps._make_warp's L-matrix solve   (tps.py:84-115)
  tps_eval           <- tps._calculate_f / _U             (tps.py:80-81,100-108)
  inverse_warp       <- tps._make_inverse_warp            (tps.py:41-75)
  map_coordinates    <- scipy.ndimage.map_coordinates(order 0/1, mode='constant', cval=0)  (tps.py:34)
  warp_images        <- tps.warp_images                   (tps.py:14-34)
  deform_grid        <- augmentation.deform_grid / the draw loop of tps.deform (augmentation.py:23-39,
                        tps.py:126-143)
  warp_affine        <- cv2.warpAffine(src, M, (w, h))  INTER_LINEAR, BORDER_CONSTANT 0
  rotation_matrix    <- cv2.getRotationMatrix2D
  warp_image         <- augmentation.warp_image           (augmentation.py:42-61)
  bgr2hsv / hsv2bgr  <- cv2.cvtColor(COLOR_BGR2HSV / COLOR_HSV2BGR) on uint8
  change_illumination<- augmentation.change_illumination  (augmentation.py:86-98)
  object_size, fg_center, augment <- augmentation.py:10-20, 101-135

Pinning.  tps.py runs for real in this image on scipy 1.15.3 (a dependency of the reference, not
vendored): tests/golden/make_golden.py calls the reference's own tps.warp_images / tps.deform, and
tests check map_coordinates below against scipy itself.  OpenCV is absent: warp_affine,
rotation_matrix and the HSV conversions are restated from OpenCV 3.x imgwarp.cpp / color.cpp and are
"parity unpinned" (the golden fixtures for augment() run the reference's augmentation.py on
tests/golden/tfshim.py's independent cv2 restatement, which pins the draw order and the wiring).
"""

import math

import numpy as np

AB_BITS = 10          # imgwarp.cpp WarpAffineInvoker: AB_BITS = MAX(10, INTER_BITS)
AB_SCALE = 1 << AB_BITS
INTER_BITS = 5
INTER_TAB_SIZE = 1 << INTER_BITS
ROUND_DELTA = AB_SCALE // INTER_TAB_SIZE // 2  # INTER_LINEAR
HSV_SHIFT = 12


# ------------------------------------------------------------------------------------------------ tps.py

def _U(x):
    """tps.py:80-81: x**2 * log(x), 0 below 1e-100 (x**2 is x*x in numpy)."""
    with np.errstate(divide="ignore"):
        return (x * x) * np.where(x < 1e-100, 0, np.log(x))


def make_warp_coeffs(from_points, to_points):
    """tps._make_warp's solve (tps.py:84-115): coeffs = pinv(L) @ [to; 0], shape [n+3, 2]."""
    from_points = np.asarray(from_points, np.float64)
    to_points = np.asarray(to_points)
    n = len(from_points)
    xd = np.subtract.outer(from_points[:, 0], from_points[:, 0])
    yd = np.subtract.outer(from_points[:, 1], from_points[:, 1])
    k = _U(np.sqrt(xd ** 2 + yd ** 2))
    p = np.ones((n, 3))
    p[:, 1:] = from_points
    ll = np.block([[k, p], [p.T, np.zeros((3, 3))]])
    v = np.resize(to_points, (n + 3, 2))
    v[-3:, :] = 0
    return np.dot(np.linalg.pinv(ll), v)


def tps_eval(coeffs, points, x, y):
    """tps._calculate_f (tps.py:100-108) for one output coordinate: a1 + ax*x + ay*y + sum_i w_i U(r_i)."""
    w = coeffs[:-3]
    a1, ax, ay = coeffs[-3:]
    s = np.zeros(x.shape)
    for wi, pi in zip(w, points):
        dx = x - pi[0]
        dy = y - pi[1]
        s += wi * _U(np.sqrt(dx * dx + dy * dy))
    return a1 + ax * x + ay * y + s


def _mgrid_axis(lo, hi, num):
    """np.mgrid[lo:hi:num*1j] along one axis: int(num) points, i*((hi-lo)/float(int(num)-1)) + lo."""
    cnt = int(abs(num))
    step = (hi - lo) / float(cnt - 1) if cnt != 1 else 1
    return np.arange(cnt, dtype=np.float64) * step + lo, cnt


def inverse_warp(from_points, to_points, output_region, approximate_grid):
    """tps._make_inverse_warp (tps.py:41-75): [row coords, col coords] of the output region."""
    x_min, y_min, x_max, y_max = output_region
    if approximate_grid is None:
        approximate_grid = 1
    x_steps = (x_max - x_min) / approximate_grid
    y_steps = (y_max - y_min) / approximate_grid
    xs, nx = _mgrid_axis(x_min, x_max, x_steps)
    ys, ny = _mgrid_axis(y_min, y_max, y_steps)
    x, y = np.meshgrid(xs, ys, indexing="ij")
    # the reverse transform to -> from (tps.py:50-51)
    points = np.asarray(to_points, np.float64)
    coeffs = make_warp_coeffs(to_points, from_points)
    tx = tps_eval(coeffs[:, 0], points, x, y)
    ty = tps_eval(coeffs[:, 1], points, x, y)
    if approximate_grid == 1:
        return tx, ty

    def axis(lo, hi, steps):
        new = np.arange(lo, hi + 1)
        frac, idx = np.modf((steps - 1) * (new - lo) / float(hi - lo))
        idx = idx.astype(int)
        i1 = np.clip(idx + 1, 0, steps - 1).astype(int)
        return idx, i1, frac, 1 - frac

    xi, xi1, xf, x1 = axis(x_min, x_max, x_steps)
    yi, yi1, yf, y1 = axis(y_min, y_max, y_steps)
    XI, YI = np.meshgrid(xi, yi, indexing="ij")
    XI1, YI1 = np.meshgrid(xi1, yi1, indexing="ij")
    XF, YF = np.meshgrid(xf, yf, indexing="ij")
    X1, Y1 = np.meshgrid(x1, y1, indexing="ij")

    def up(t):  # tps.py:67-69 (left-to-right products and sums)
        return (t[XI, YI] * X1 * Y1 + t[XI, YI1] * X1 * YF + t[XI1, YI] * XF * Y1 + t[XI1, YI1] * XF * YF)

    return up(tx), up(ty)


def map_coordinates(img, cr, cc, order=1):
    """scipy.ndimage.map_coordinates(img, [cr, cc], order=order) for a 2-D image, mode='constant', cval=0
    (scipy 1.15.3 ni_interpolation.c): a coordinate outside [0, n-1] on either axis gives cval; order 1 sums
    the taps (r0,c0), (r0,c1), (r1,c0), (r1,c1) as t += (v * w_row) * w_col in double with weights
    (1 - f, 1 - (1 - f)) (a tap outside the image reads cval); order 0 takes floor(c + 0.5).  Integer
    outputs are (type)(t + 0.5)."""
    img = np.asarray(img)
    h, w = img.shape
    src = img.astype(np.float64)
    inside = (cr >= 0) & (cr <= h - 1) & (cc >= 0) & (cc <= w - 1)
    crs = np.where(inside, cr, 0.0)
    ccs = np.where(inside, cc, 0.0)
    if order == 0:
        r = np.floor(crs + 0.5).astype(np.int64)
        c = np.floor(ccs + 0.5).astype(np.int64)
        t = np.where(inside, src[np.clip(r, 0, h - 1), np.clip(c, 0, w - 1)], 0.0)
    elif order == 1:
        r0 = np.floor(crs)
        c0 = np.floor(ccs)
        fr, fc = crs - r0, ccs - c0
        r0, c0 = r0.astype(np.int64), c0.astype(np.int64)
        # get_spline_interpolation_weights: w0 = 1 - x, and the last weight is 1 - w0 (not x)
        wr = (1.0 - fr, 1.0 - (1.0 - fr))
        wc = (1.0 - fc, 1.0 - (1.0 - fc))
        t = np.zeros(cr.shape)
        for dr in (0, 1):
            for dc in (0, 1):
                rr, ccx = r0 + dr, c0 + dc
                ok = (rr < h) & (ccx < w)
                v = np.where(ok, src[np.minimum(rr, h - 1), np.minimum(ccx, w - 1)], 0.0)
                t = t + (v * wr[dr]) * wc[dc]
        t = np.where(inside, t, 0.0)
    else:
        raise NotImplementedError("map_coordinates: order %d" % order)
    if img.dtype.kind in "ui":
        return np.floor(t + 0.5).astype(img.dtype)
    return t.astype(img.dtype)


def warp_images(from_points, to_points, images, output_region, interpolation_order=1, approximate_grid=2):
    """tps.warp_images (tps.py:14-34)."""
    tx, ty = inverse_warp(from_points, to_points, output_region, approximate_grid)
    return [map_coordinates(np.asarray(im), tx, ty, interpolation_order) for im in images]


def deform_grid(h, w, n=5, fact=0.05):
    """augmentation.deform_grid (augmentation.py:23-39) == tps.deform's draw loop (tps.py:127-143):
    one np.random.uniform per interior coordinate, column (x) before row (y)."""
    bound = min(w, h) * fact
    vec1 = (h / (n - 1)) * np.arange(n)
    vec2 = (w / (n - 1)) * np.arange(n)
    grid = np.transpose([np.repeat(vec1, n), np.tile(vec2, n)])
    new_grid = np.zeros_like(grid)
    for i in range(n * n):
        y, x = grid[i, 0], grid[i, 1]
        new_grid[i] = grid[i]
        if 0. < x < w:
            new_grid[i, 1] += np.random.uniform(-bound, bound)
        if 0. < y < h:
            new_grid[i, 0] += np.random.uniform(-bound, bound)
    return grid, new_grid


def deform(img):
    """tps.deform (tps.py:126-149): TPS-warp the three planes of a BGR image, output (h+1, w+1, 3)."""
    h, w = img.shape[:2]
    grid, new_grid = deform_grid(h, w)
    res = warp_images(grid, new_grid, [img[:, :, 0], img[:, :, 1], img[:, :, 2]], (0, 0, h, w), 1, 2)
    return np.transpose(res, axes=(1, 2, 0)).copy()


# ------------------------------------------------------------------------------------------------ OpenCV

def invert_affine(M):
    """imgwarp.cpp warpAffine: the forward matrix is inverted in double unless WARP_INVERSE_MAP."""
    m = np.asarray(M, np.float64).reshape(6).copy()
    d = m[0] * m[4] - m[1] * m[3]
    d = 1. / d if d != 0 else 0.
    a11, a22 = m[4] * d, m[0] * d
    m[0] = a11
    m[1] *= -d
    m[3] *= -d
    m[4] = a22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return m


def affine_coords(m, h, w):
    """WarpAffineInvoker: X = (cvRound((M1*y + M2)*1024) + 16 + cvRound(M0*x*1024)) >> 5 (same for Y); the
    source tap is (X >> 5, Y >> 5) saturated to short, the table fraction (X & 31, Y & 31)."""
    x = np.arange(w, dtype=np.float64)
    y = np.arange(h, dtype=np.float64)
    adelta = np.rint(m[0] * x * AB_SCALE).astype(np.int64)
    bdelta = np.rint(m[3] * x * AB_SCALE).astype(np.int64)
    x0 = np.rint((m[1] * y + m[2]) * AB_SCALE).astype(np.int64) + ROUND_DELTA
    y0 = np.rint((m[4] * y + m[5]) * AB_SCALE).astype(np.int64) + ROUND_DELTA
    X = (x0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    return sx, sy, X & (INTER_TAB_SIZE - 1), Y & (INTER_TAB_SIZE - 1)


def warp_affine(src, M, dsize):
    """cv2.warpAffine(src, M, dsize=(w, h)), INTER_LINEAR, BORDER_CONSTANT 0 (OpenCV 3.x): affine_coords, then
    remapBilinear with the 32x32 table — uint8: 15-bit integer weights (32-ay)(32-ax)*32 ..., (s + 2^14) >> 15;
    float: exact float weights, v0*w0 + v1*w1 + v2*w2 + v3*w3 in double.  A tap outside the source reads 0."""
    src = np.asarray(src)
    w, h = dsize
    sx, sy, ax, ay = affine_coords(invert_affine(M), h, w)
    sh, sw = src.shape[:2]
    planes = src[..., None] if src.ndim == 2 else src
    out = np.zeros((h, w, planes.shape[2]), src.dtype)
    taps = ((0, 0), (0, 1), (1, 0), (1, 1))
    if src.dtype == np.uint8:
        wts = ((32 - ay) * (32 - ax) * 32, (32 - ay) * ax * 32, ay * (32 - ax) * 32, ay * ax * 32)
    else:
        wts = tuple(((32 - a) / 32.0 if lo_y else a / 32.0) * ((32 - b) / 32.0 if lo_x else b / 32.0)
                    for (lo_y, lo_x), a, b in (((True, True), ay, ax), ((True, False), ay, ax),
                                               ((False, True), ay, ax), ((False, False), ay, ax)))
    for k in range(planes.shape[2]):
        p = planes[..., k]
        acc = None
        for (dy, dx), wt in zip(taps, wts):
            yy, xx = sy + dy, sx + dx
            ok = (yy >= 0) & (yy < sh) & (xx >= 0) & (xx < sw)
            v = np.where(ok, p[np.clip(yy, 0, sh - 1), np.clip(xx, 0, sw - 1)], 0)
            if src.dtype == np.uint8:
                term = v.astype(np.int64) * wt
            else:
                term = v.astype(np.float64) * wt
            acc = term if acc is None else acc + term
        if src.dtype == np.uint8:
            out[..., k] = np.clip((acc + (1 << 14)) >> 15, 0, 255)
        else:
            out[..., k] = acc
    return out[..., 0] if src.ndim == 2 else out


def rotation_matrix(center, angle, scale):
    """cv2.getRotationMatrix2D(center (Point2f), angle in degrees, scale)."""
    cx, cy = float(np.float32(center[0])), float(np.float32(center[1]))
    a = angle * (math.pi / 180)
    alpha = math.cos(a) * scale
    beta = math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]])


def hsv_tables():
    """color.cpp RGB2HSV_b: sdiv[i] = cvRound((255 << 12) / (1.*i)), hdiv180[i] = cvRound((180 << 12) / (6.*i))."""
    i = np.arange(1, 256, dtype=np.float64)
    sdiv = np.zeros(256, np.int64)
    hdiv = np.zeros(256, np.int64)
    sdiv[1:] = np.rint((255 << HSV_SHIFT) / i)
    hdiv[1:] = np.rint((180 << HSV_SHIFT) / (6. * i))
    return sdiv, hdiv


def bgr2hsv(bgr):
    """cv2.cvtColor(bgr, COLOR_BGR2HSV) for uint8 (RGB2HSV_b, hrange 180)."""
    sdiv, hdiv = hsv_tables()
    b, g, r = (bgr[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    s = (diff * sdiv[v] + (1 << (HSV_SHIFT - 1))) >> HSV_SHIFT
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + (~vg & (r - g + 4 * diff))))
    h = (h * hdiv[diff] + (1 << (HSV_SHIFT - 1))) >> HSV_SHIFT
    h = h + np.where(h < 0, 180, 0)
    return np.stack([np.clip(h, 0, 255), s, v], axis=-1).astype(np.uint8)


def hsv2bgr(hsv):
    """cv2.cvtColor(hsv, COLOR_HSV2BGR) for uint8 (HSV2RGB_b -> HSV2RGB_f in float32, hrange 180)."""
    f32 = np.float32
    h = hsv[..., 0].astype(f32)
    s = hsv[..., 1].astype(f32) * f32(1.0 / 255.0)
    v = hsv[..., 2].astype(f32) * f32(1.0 / 255.0)
    h = h * (f32(6.0) / f32(180.0))
    h = np.where(h >= f32(6), h - f32(6), h)  # h < 6 for h <= 179; kept for the literal form
    sector = np.floor(h).astype(np.int64)
    h = (h - sector.astype(f32)).astype(f32)
    one = f32(1)
    tab = np.stack([v, v * (one - s), v * (one - s * h), v * (one - s * (one - h))], axis=0)
    sector_data = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    sec = np.clip(sector, 0, 5)
    out = []
    for c in range(3):
        val = np.take_along_axis(tab, sector_data[sec, c][None], axis=0)[0]
        val = np.where(s == 0, v, val)
        out.append(np.clip(np.rint(val * f32(255)), 0, 255).astype(np.uint8))
    return np.stack(out, axis=-1)


def illumination_lut(a, b, c):
    """augmentation.change_illumination's S/V map (augmentation.py:89-95) on every uint8 value."""
    x = np.arange(256, dtype=np.uint8)
    y = a * np.power(x / 255., b) + c
    return (255. * np.clip(y, 0., 1.)).astype(np.uint8)


def change_illumination(bgr, a, b, c):
    """augmentation.change_illumination (augmentation.py:86-98)."""
    hsv = bgr2hsv(bgr)
    lut = illumination_lut(a, b, c)
    new = np.zeros_like(hsv)
    new[..., 0] = hsv[..., 0]
    new[..., 1] = lut[hsv[..., 1]]
    new[..., 2] = lut[hsv[..., 2]]
    return hsv2bgr(new)


# ------------------------------------------------------------------------------------------------ augmentation.py

def object_size(alpha):
    """augmentation.object_size (augmentation.py:10-14): sqrt(#nonzero alpha)."""
    return np.sqrt(np.count_nonzero(alpha != 0.))


def fg_center(alpha):
    """augmentation.fg_center (augmentation.py:17-20): (int(mean col), int(mean row)) of nonzero alpha."""
    nz = np.where(alpha != 0.)
    return int(np.mean(nz[1])), int(np.mean(nz[0]))


def warp_image(img, params, thin=None):
    """augmentation.warp_image (augmentation.py:42-61): optional TPS (output (h+1, w+1)), then a warpAffine
    translation by (tu, tv) and a warpAffine rotation/scale about `center`, both to (w, h)."""
    (tu, tv), rot, scale, center = params
    h, w = img.shape[:2]
    if thin is not None:
        grid, def_grid = thin
        if img.ndim == 3 and img.shape[2] == 3:
            res = warp_images(grid, def_grid, [img[:, :, 0], img[:, :, 1], img[:, :, 2]], (0, 0, h, w), 1, 2)
            img = np.transpose(res, axes=(1, 2, 0)).copy()
        else:
            img = warp_images(grid, def_grid, [img], (0, 0, h, w), 1, 2)[0]
    mt = np.float32([[1, 0, tu], [0, 1, tv]])
    translated = warp_affine(img, mt, (w, h))
    return warp_affine(translated, rotation_matrix(center, rot, scale), (w, h))


def augment(fg, bg, alpha):
    """augmentation.augment (augmentation.py:101-135): the reference's np.random draws in order."""
    h, w = fg.shape[:2]
    fg_size = object_size(alpha)
    tu_bg = int(np.random.uniform(-w * 0.05, w * 0.05))
    tv_bg = int(np.random.uniform(-h * 0.05, h * 0.05))
    scale_bg = np.random.uniform(1., 1. + 0.15)
    new_bg = warp_image(bg, ((tu_bg, tv_bg), 0., scale_bg, (w // 2, h // 2)))
    grid, def_grid = deform_grid(h, w)
    tu_fg = int(np.random.uniform(-fg_size * 0.05, fg_size * 0.05))
    tv_fg = int(np.random.uniform(-fg_size * 0.05, fg_size * 0.05))
    rot_fg = np.random.uniform(-10, 10)
    scale_fg = np.random.uniform(1., 1. + 0.15)
    params_fg = (tu_fg, tv_fg), rot_fg, scale_fg, fg_center(alpha)
    new_fg = warp_image(fg, params_fg, thin=(grid, def_grid))
    new_alpha = warp_image(alpha, params_fg, thin=(grid, def_grid))
    a = np.random.uniform(1. - 0.05, 1. + 0.05)
    b = np.random.uniform(1. - 0.3, 1. + 0.3)
    c = np.random.uniform(-0.07, 0.07)
    return change_illumination(new_fg, a, b, c), change_illumination(new_bg, a, b, c), new_alpha
