"""Eager numpy stand-ins for the TF-1.x / OpenCV calls the reference's hot path makes.

Used ONLY by make_golden.py to execute the reference's own graph-builder code
(/root/reference/unet.py, unet_simple.py, small.py, refine.py, flow.py,
train.py loss helpers) verbatim, since TensorFlow and OpenCV are not in this
image.  Written literally from the library kernels' documented behaviour and
deliberately independent of oracle/ops.py (different code paths: einsum
convolution, per-axis interpolation tables, explicit window loops), so the
golden-vs-oracle test cross-checks two restatements.

Every variable the reference creates is recorded (scope path, shape, values)
so that tests can check the product's weight construction against the
reference's draw order.
"""

import contextlib
import types

import numpy as np

DTYPE = np.float64


class _Registry:
    def __init__(self):
        self.scope = []
        self.variables = []  # (full_name, array)

    def add(self, name, value):
        full = "/".join(self.scope + [name])
        self.variables.append((full, np.array(value)))
        return np.asarray(value)


REG = _Registry()


@contextlib.contextmanager
def variable_scope(name, *a, **k):
    REG.scope.append(name)
    try:
        yield
    finally:
        REG.scope.pop()


def get_variable(name=None, initializer=None, **k):
    return REG.add(name, initializer)


def Variable(value, name=None, **k):
    return REG.add(name or "Variable", value)


def constant(value, name=None, **k):
    return np.asarray(value)


# ------------------------------------------------------------------ nn ops

def conv2d(x, filt, strides, padding, **k):
    assert list(strides) == [1, 1, 1, 1] and padding == "SAME"
    x = np.asarray(x, DTYPE)
    filt = np.asarray(filt, DTYPE)
    kh, kw, ci, co = filt.shape
    n, h, w, c = x.shape
    assert c == ci, (x.shape, filt.shape)
    ph, pw = (kh - 1) // 2, (kw - 1) // 2  # SAME, stride 1, odd kernel: pad_before = (k-1)//2
    xp = np.pad(x, ((0, 0), (ph, kh - 1 - ph), (pw, kw - 1 - pw), (0, 0)))
    out = np.zeros((n, h, w, co), DTYPE)
    for a in range(kh):
        for b in range(kw):
            out += np.einsum("nhwc,co->nhwo", xp[:, a:a + h, b:b + w, :], filt[a, b], optimize=True)
    return out


def bias_add(x, b, **k):
    return np.asarray(x, DTYPE) + np.asarray(b, DTYPE)


def relu(x, name=None):
    x = np.asarray(x, DTYPE)
    return np.where(x > 0, x, 0.0)


def sigmoid(x, name=None):
    from scipy.special import expit
    return expit(np.asarray(x, DTYPE))


def softmax(x, axis=-1, name=None):
    x = np.asarray(x, DTYPE)
    z = np.exp(x - x.max(axis=axis, keepdims=True))
    return z / z.sum(axis=axis, keepdims=True)


def max_pool(x, ksize, strides, padding, name=None):
    assert padding == "SAME"
    x = np.asarray(x, DTYPE)
    n, h, w, c = x.shape
    k, s = ksize[1], strides[1]
    oh, ow = -(-h // s), -(-w // s)
    pad_h = max((oh - 1) * s + k - h, 0)
    pad_w = max((ow - 1) * s + k - w, 0)
    top, left = pad_h // 2, pad_w // 2
    out = np.full((n, oh, ow, c), -np.inf, DTYPE)
    for a in range(k):
        for b in range(k):
            rows = np.arange(oh) * s - top + a
            cols = np.arange(ow) * s - left + b
            rv = (rows >= 0) & (rows < h)
            cv = (cols >= 0) & (cols < w)
            tap = np.full((n, oh, ow, c), -np.inf, DTYPE)
            sub = x[:, np.clip(rows, 0, h - 1)][:, :, np.clip(cols, 0, w - 1)]
            mask = rv[None, :, None, None] & cv[None, None, :, None]
            tap = np.where(mask, sub, tap)
            out = np.maximum(out, tap)
    return out


def _interp_table(out_size, in_size):
    # tensorflow/core/kernels/resize_bilinear_op.cc, legacy scaler: scale = (float)in/out,
    # in = (float)i * scale, lower = floor(in), upper = min(ceil(in), in-1), lerp = in - floor(in)
    scale = np.float32(in_size) / np.float32(out_size)
    lo = np.empty(out_size, np.int64)
    hi = np.empty(out_size, np.int64)
    lerp = np.empty(out_size, np.float32)
    for i in range(out_size):
        v = np.float32(i) * scale
        f = np.floor(v)
        lo[i] = max(int(f), 0)
        hi[i] = min(int(np.ceil(v)), in_size - 1)
        lerp[i] = v - f
    return lo, hi, lerp


def resize_images(images, size, **k):
    images = np.asarray(images, DTYPE)
    n, ih, iw, c = images.shape
    oh, ow = int(size[0]), int(size[1])
    if (oh, ow) == (ih, iw):
        return images
    ylo, yhi, ylerp = _interp_table(oh, ih)
    xlo, xhi, xlerp = _interp_table(ow, iw)
    out = np.empty((n, oh, ow, c), DTYPE)
    for y in range(oh):
        top_row = images[:, ylo[y]]
        bot_row = images[:, yhi[y]]
        tl, tr = top_row[:, xlo], top_row[:, xhi]
        bl, br = bot_row[:, xlo], bot_row[:, xhi]
        xl = xlerp.astype(DTYPE)[None, :, None]
        top = tl + (tr - tl) * xl
        bot = bl + (br - bl) * xl
        out[:, y] = top + (bot - top) * DTYPE(ylerp[y])
    return out


def batch_norm(x, center=True, scale=True, is_training=False, scope=None, epsilon=0.001, **k):
    x = np.asarray(x, DTYPE)
    c = x.shape[-1]
    with variable_scope(scope or "BatchNorm"):
        beta = get_variable("beta", np.zeros(c, np.float32)) if center else np.zeros(c)
        gamma = get_variable("gamma", np.ones(c, np.float32)) if scale else np.ones(c)
        mm = get_variable("moving_mean", np.zeros(c, np.float32))
        mv = get_variable("moving_variance", np.ones(c, np.float32))
    if bool(is_training):
        mean = x.reshape(-1, c).mean(axis=0)
        var = np.square(x.reshape(-1, c) - mean).mean(axis=0)  # fused_batch_norm normalises with the biased variance
    else:
        mean, var = mm.astype(DTYPE), mv.astype(DTYPE)
    return (x - mean) / np.sqrt(var + epsilon) * gamma.astype(DTYPE) + beta.astype(DTYPE)


def concat(values=None, axis=0, name=None, **k):
    return np.concatenate([np.asarray(v, DTYPE) for v in values], axis=axis)


def split(value, num_or_size_splits, axis=0, **k):
    v = np.asarray(value, DTYPE)
    if isinstance(num_or_size_splits, int):
        return np.split(v, num_or_size_splits, axis=axis)
    idx = np.cumsum(num_or_size_splits)[:-1]
    return np.split(v, idx, axis=axis)


def _binary(f):
    return lambda a, b, name=None: f(np.asarray(a, DTYPE), np.asarray(b, DTYPE))


def make_tf():
    tf = types.ModuleType("tensorflow")
    tf.variable_scope = variable_scope
    tf.get_variable = get_variable
    tf.Variable = Variable
    tf.constant = constant
    tf.concat = concat
    tf.split = split
    tf.add = _binary(np.add)
    tf.subtract = _binary(np.subtract)
    tf.multiply = _binary(np.multiply)
    tf.square = lambda x, name=None: np.square(np.asarray(x, DTYPE))
    tf.sqrt = lambda x, name=None: np.sqrt(np.asarray(x, DTYPE))
    tf.reduce_mean = lambda x, axis=None, name=None: np.mean(np.asarray(x, DTYPE), axis=axis)
    tf.nn = types.SimpleNamespace(conv2d=conv2d, bias_add=bias_add, relu=relu, sigmoid=sigmoid,
                                  softmax=softmax, max_pool=max_pool)
    tf.image = types.SimpleNamespace(resize_images=resize_images)
    tf.contrib = types.SimpleNamespace(layers=types.SimpleNamespace(batch_norm=batch_norm))
    return tf


# ------------------------------------------------------------------ OpenCV stand-in (remap, resize, imread, warpAffine, cvtColor HSV)

INTER_LINEAR = 1


def remap(src, map1, map2, interpolation):
    """cv2.remap(src, map1 CV_32FC2, None, INTER_LINEAR), BORDER_CONSTANT 0 — per OpenCV 3.x
    imgwarp.cpp: X = cvRound(x*32), sx = X>>5, table index (Y&31)*32+(X&31); fully-inside
    pixels sum S0*w0+S1*w1+S2*w2+S3*w3; border pixels take 0 for every tap outside."""
    assert map2 is None and interpolation == INTER_LINEAR
    src = np.asarray(src)
    h, w = map1.shape[:2]
    X = np.rint(map1[..., 0].astype(np.float64) * 32).astype(np.int64)
    Y = np.rint(map1[..., 1].astype(np.float64) * 32).astype(np.int64)
    sx, sy = X >> 5, Y >> 5
    ax, ay = X & 31, Y & 31
    if src.dtype == np.uint8:
        def wt(fy_lo, fx_lo):  # itab = saturate_cast<short>(tab * INTER_REMAP_COEF_SCALE)
            t = (np.where(fy_lo, 1 - ay / 32.0, ay / 32.0).astype(np.float32)
                 * np.where(fx_lo, 1 - ax / 32.0, ax / 32.0).astype(np.float32))
            return np.rint(t.astype(np.float64) * 32768).astype(np.int64)
        ws = [wt(True, True), wt(True, False), wt(False, True), wt(False, False)]
    else:
        wy0, wy1 = (1 - ay / 32.0).astype(np.float32), (ay / 32.0).astype(np.float32)
        wx0, wx1 = (1 - ax / 32.0).astype(np.float32), (ax / 32.0).astype(np.float32)
        ws = [(wy0 * wx0).astype(np.float64), (wy0 * wx1).astype(np.float64),
              (wy1 * wx0).astype(np.float64), (wy1 * wx1).astype(np.float64)]
    out = np.zeros((h, w), np.int64 if src.dtype == np.uint8 else np.float64)
    taps = [(0, 0), (0, 1), (1, 0), (1, 1)]
    vals = []
    for dy, dx in taps:
        yy, xx = sy + dy, sx + dx
        ok = (yy >= 0) & (yy < src.shape[0]) & (xx >= 0) & (xx < src.shape[1])
        v = np.zeros((h, w), src.dtype)
        v[ok] = src[yy[ok], xx[ok]]
        vals.append(v)
    if src.dtype == np.uint8:
        s = sum(vals[i].astype(np.int64) * ws[i] for i in range(4))
        return np.clip((s + (1 << 14)) >> 15, 0, 255).astype(np.uint8)
    for i in range(4):
        out = out + vals[i].astype(np.float64) * ws[i]
    return out.astype(src.dtype)


def resize(src, dsize, interpolation=INTER_LINEAR, **k):
    """cv2.resize(src, dsize, interpolation=INTER_LINEAR) for float64 sources, written after the
    structure of OpenCV 3.x imgproc/resize.cpp: dsize == ssize copies; an exact 2x reduction in both
    axes switches to the INTER_AREA fast path (sum += S[ofs0]+S[ofs1]+S[ofs2]+S[ofs3]; D = sum*scale);
    otherwise resizeGeneric_ with HResizeLinear<double,double,float> / VResizeLinear: per-column
    (xofs, alpha) and per-row (yofs, beta) tables built one entry at a time in float32, rows fetched
    through clip(sy, 0, ssize.height)."""
    src = np.asarray(src)
    assert interpolation == INTER_LINEAR and src.dtype == np.float64
    if src.ndim == 3 and src.shape[2] == 1:
        src = src[:, :, 0]
    sh, sw = src.shape[:2]
    dw, dh = int(dsize[0]), int(dsize[1])
    if (sh, sw) == (dh, dw):
        return src.copy()
    inv_x, inv_y = float(dw) / sw, float(dh) / sh
    scale_x, scale_y = 1.0 / inv_x, 1.0 / inv_y
    ix, iy = int(round(scale_x)), int(round(scale_y))
    eps = np.finfo(np.float64).eps
    if abs(scale_x - ix) < eps and abs(scale_y - iy) < eps and ix == 2 and iy == 2:
        dst = np.zeros((dh, dw) + src.shape[2:], np.float64)
        scale = float(np.float32(1.0) / np.float32(4))
        for dy in range(dh):
            for dx in range(dw):
                S = [src[2 * dy + a, 2 * dx + b] for a in range(2) for b in range(2)]
                total = 0.0 + (((S[0] + S[1]) + S[2]) + S[3])
                dst[dy, dx] = total * scale
        return dst
    xofs, alpha, xmax = [], [], dw
    for dx in range(dw):
        fx = np.float32((dx + 0.5) * scale_x - 0.5)
        sx = int(np.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0), 0
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                fx, sx = np.float32(0), sw - 1
        xofs.append(sx)
        alpha.append((float(np.float32(1) - fx), float(fx)))
    yofs, beta = [], []
    for dy in range(dh):
        fy = np.float32((dy + 0.5) * scale_y - 0.5)
        sy = int(np.floor(fy))
        fy = np.float32(fy - np.float32(sy))
        yofs.append(sy)
        beta.append((float(np.float32(1) - fy), float(fy)))

    def hresize(row):
        out = np.empty((dw,) + row.shape[1:], np.float64)
        for dx in range(dw):
            sx = xofs[dx]
            if dx < xmax:
                out[dx] = row[sx] * alpha[dx][0] + row[sx + 1] * alpha[dx][1]
            else:
                out[dx] = row[sx] * 1.0
        return out

    dst = np.empty((dh, dw) + src.shape[2:], np.float64)
    cache = {}
    for dy in range(dh):
        rows = []
        for k in range(2):
            sy = min(max(yofs[dy] + k, 0), sh - 1)
            if sy not in cache:
                cache[sy] = hresize(src[sy])
            rows.append(cache[sy])
        dst[dy] = rows[0] * beta[dy][0] + rows[1] * beta[dy][1]
    return dst


def imread(path, flags=1):
    """cv2.imread via PIL: flags -1 (IMREAD_UNCHANGED) keeps BGRA / 16-bit, 0 = grayscale, else BGR u8."""
    from PIL import Image
    im = Image.open(path)
    if flags == 0:
        return np.asarray(im.convert("L"))
    if flags == -1:
        a = np.asarray(im)
        if a.ndim == 3 and a.shape[2] == 4:
            return a[:, :, [2, 1, 0, 3]]
        if a.ndim == 3:
            return a[:, :, ::-1]
        return a
    return np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])


# warpAffine / getRotationMatrix2D / cvtColor(HSV) — written after OpenCV 3.x imgwarp.cpp (WarpAffineInvoker +
# remapBilinear) and color.cpp (RGB2HSV_b, HSV2RGB_b/_f), per pixel in C order; independent of oracle/augment.py.

def _cv_round(v):
    return int(np.rint(v))  # cvRound: round half to even


def warpAffine(src, M, dsize, flags=INTER_LINEAR):
    assert flags == INTER_LINEAR
    src = np.asarray(src)
    assert src.dtype in (np.uint8, np.float64, np.float32), src.dtype
    m = [float(v) for v in np.asarray(M, np.float64).reshape(6)]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1. / D if D != 0 else 0.
    A11, A22 = m[4] * D, m[0] * D
    m[0] = A11
    m[1] *= -D
    m[3] *= -D
    m[4] = A22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    W, H = dsize
    sh, sw = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    S = src.reshape(sh, sw, cn)
    dst = np.zeros((H, W, cn), src.dtype)
    adelta = [_cv_round(m[0] * x * 1024) for x in range(W)]
    bdelta = [_cv_round(m[3] * x * 1024) for x in range(W)]
    for y in range(H):
        X0 = _cv_round((m[1] * y + m[2]) * 1024) + 16
        Y0 = _cv_round((m[4] * y + m[5]) * 1024) + 16
        for x in range(W):
            X = (X0 + adelta[x]) >> 5
            Y = (Y0 + bdelta[x]) >> 5
            sx = max(-32768, min(32767, X >> 5))
            sy = max(-32768, min(32767, Y >> 5))
            fx, fy = X & 31, Y & 31
            if sx >= sw or sx + 1 < 0 or sy >= sh or sy + 1 < 0:
                continue  # BORDER_CONSTANT: the whole pixel is the border value 0
            for k in range(cn):
                v = [S[yy, xx, k] if (0 <= yy < sh and 0 <= xx < sw) else 0
                     for yy, xx in ((sy, sx), (sy, sx + 1), (sy + 1, sx), (sy + 1, sx + 1))]
                if src.dtype == np.uint8:
                    wt = [(32 - fy) * (32 - fx) * 32, (32 - fy) * fx * 32, fy * (32 - fx) * 32, fy * fx * 32]
                    t = int(v[0]) * wt[0] + int(v[1]) * wt[1] + int(v[2]) * wt[2] + int(v[3]) * wt[3]
                    dst[y, x, k] = max(0, min(255, (t + (1 << 14)) >> 15))
                else:
                    ty = (np.float32(1 - fy / 32.), np.float32(fy / 32.))
                    tx = (np.float32(1 - fx / 32.), np.float32(fx / 32.))
                    wt = [float(ty[0] * tx[0]), float(ty[0] * tx[1]), float(ty[1] * tx[0]), float(ty[1] * tx[1])]
                    dst[y, x, k] = float(v[0]) * wt[0] + float(v[1]) * wt[1] + float(v[2]) * wt[2] + float(v[3]) * wt[3]
    return dst[..., 0] if src.ndim == 2 else dst


def getRotationMatrix2D(center, angle, scale):
    import math
    cx, cy = float(np.float32(center[0])), float(np.float32(center[1]))
    angle = angle * (math.pi / 180)
    alpha = math.cos(angle) * scale
    beta = math.sin(angle) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy], [-beta, alpha, beta * cx + (1 - alpha) * cy]])


COLOR_BGR2HSV = 40
COLOR_HSV2BGR = 54


def _hsv_tables():
    sdiv = [0] * 256
    hdiv = [0] * 256
    for i in range(1, 256):
        sdiv[i] = _cv_round((255 << 12) / (1. * i))
        hdiv[i] = _cv_round((180 << 12) / (6. * i))
    return sdiv, hdiv


def cvtColor(src, code):
    src = np.asarray(src)
    assert src.dtype == np.uint8 and src.ndim == 3 and src.shape[2] == 3
    out = np.zeros_like(src)
    if code == COLOR_BGR2HSV:
        sdiv, hdiv = _hsv_tables()
        for (y, x), _ in np.ndenumerate(src[..., 0]):
            b, g, r = (int(v) for v in src[y, x])
            v = max(b, g, r)
            vmin = min(b, g, r)
            diff = v - vmin
            vr = -1 if v == r else 0
            vg = -1 if v == g else 0
            s = (diff * sdiv[v] + (1 << 11)) >> 12
            h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))))
            h = (h * hdiv[diff] + (1 << 11)) >> 12
            h += 180 if h < 0 else 0
            out[y, x] = (h, s, v)
        return out
    assert code == COLOR_HSV2BGR
    f = np.float32
    hscale = f(6.) / f(180.)
    sector_data = ((1, 3, 0), (1, 0, 2), (3, 0, 1), (0, 2, 1), (0, 1, 3), (2, 1, 0))
    for (y, x), _ in np.ndenumerate(src[..., 0]):
        h = f(src[y, x, 0])
        s = f(src[y, x, 1]) * f(1. / 255.)
        v = f(src[y, x, 2]) * f(1. / 255.)
        if s == 0:
            b = g = r = v
        else:
            h = f(h * hscale)
            while h < 0:
                h = f(h + f(6))
            while h >= 6:
                h = f(h - f(6))
            sector = int(np.floor(h))
            h = f(h - f(sector))
            if not 0 <= sector < 6:
                sector, h = 0, f(0)
            tab = (v, f(v * f(f(1) - s)), f(v * f(f(1) - f(s * h))), f(v * f(f(1) - f(s * f(f(1) - h)))))
            b, g, r = (tab[sector_data[sector][k]] for k in range(3))
        out[y, x] = [max(0, min(255, int(np.rint(f(c * f(255)))))) for c in (b, g, r)]
    return out


def make_cv2():
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = INTER_LINEAR
    cv2.NORM_MINMAX = 32
    cv2.IMREAD_UNCHANGED = -1
    cv2.remap = remap
    cv2.resize = resize
    cv2.imread = imread
    cv2.warpAffine = warpAffine
    cv2.getRotationMatrix2D = getRotationMatrix2D
    cv2.cvtColor = cvtColor
    cv2.COLOR_BGR2HSV = COLOR_BGR2HSV
    cv2.COLOR_HSV2BGR = COLOR_HSV2BGR
    cv2.normalize = lambda *a, **k: None
    cv2.imshow = lambda *a, **k: None
    cv2.waitKey = lambda *a, **k: 0
    return cv2
