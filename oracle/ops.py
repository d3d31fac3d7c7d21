"""Numpy restatement of the TF-1.x / OpenCV ops on the hot path (TEST INFRASTRUCTURE).

Every function names the reference call site(s) it stands in for and the
library semantics it restates.  Arrays are NHWC like
the reference (unet.py:15 builds HWIO filters, TF's default data_format).
All functions keep the input dtype (float64 for goldens, float32 for the
timed CPU baseline).
"""

import numpy as np

# params.py:10, unet.py:8, unet_simple.py:7
VGG_MEAN = (103.939, 116.779, 123.68)

BN_EPS = 1e-3  # tf.contrib.layers.batch_norm default epsilon (unet_simple.py:25, small.py:32)


def conv3x3_same(x, w, b=None, row_chunk=None):
    """tf.nn.conv2d(x, w, [1,1,1,1], 'SAME') (+ tf.nn.bias_add) for a 3x3 filter.

    Reference call sites: unet.py:39,60,70; unet_simple.py:23,35,102;
    small.py:19,30; refine.py:22.  SAME + stride 1 + 3x3 = zero pad 1 on every
    side; cross-correlation y[n,h,w,o] = sum_{kh,kw,c} x[n,h+kh-1,w+kw-1,c] w[kh,kw,c,o].
    Computed as 9 shifted GEMMs, chunked over output rows to bound memory.
    """
    n, h, wd, c = x.shape
    assert w.shape[:3] == (3, 3, c), (w.shape, x.shape)
    o = w.shape[3]
    w = w.astype(x.dtype, copy=False)
    xp = np.zeros((n, h + 2, wd + 2, c), dtype=x.dtype)
    xp[:, 1:-1, 1:-1, :] = x
    y = np.empty((n, h, wd, o), dtype=x.dtype)
    if row_chunk is None:
        # keep each shifted slab around 64 MB
        row_chunk = max(1, int(64e6 // max(1, n * wd * max(c, o) * x.dtype.itemsize)))
    for r0 in range(0, h, row_chunk):
        r1 = min(h, r0 + row_chunk)
        acc = np.zeros((n * (r1 - r0) * wd, o), dtype=x.dtype)
        for kh in range(3):
            for kw in range(3):
                sl = xp[:, r0 + kh:r1 + kh, kw:kw + wd, :].reshape(-1, c)
                acc += sl @ w[kh, kw]
        y[:, r0:r1] = acc.reshape(n, r1 - r0, wd, o)
    if b is not None:
        y += b.astype(x.dtype, copy=False)
    return y


def relu(x):
    """tf.nn.relu (unet.py:96-192 and throughout)."""
    return np.maximum(x, 0)


def sigmoid(x):
    """tf.nn.sigmoid (unet.py:145,205; unet_simple.py:142; small.py:50), overflow-safe."""
    out = np.empty_like(x)
    pos = x >= 0
    out[pos] = 1.0 / (1.0 + np.exp(-x[pos]))
    e = np.exp(x[~pos])
    out[~pos] = e / (1.0 + e)
    return out


def softmax_lastdim(x):
    """tf.nn.softmax over the last axis (refine.py:31)."""
    m = x.max(axis=-1, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=-1, keepdims=True)


def max_pool_2x2_same(x):
    """tf.nn.max_pool(ksize 2, stride 2, 'SAME') (unet.py:33; unet_simple.py:96; small.py:40,42).

    out = ceil(n/2); pad_total = max((out-1)*2 + 2 - n, 0); pad_before = 0, so on an
    odd size the last window holds a single row/column (padded taps never win).
    """
    n, h, w, c = x.shape
    oh, ow = (h + 1) // 2, (w + 1) // 2
    xp = np.full((n, oh * 2, ow * 2, c), -np.inf, dtype=x.dtype)
    xp[:, :h, :w, :] = x
    xp = xp.reshape(n, oh, 2, ow, 2, c)
    return xp.max(axis=(2, 4))


def resize_bilinear_tf1(x, oh, ow):
    """tf.image.resize_images(x, [oh, ow]) with TF-1.x defaults (unet.py:58; unet_simple.py:33; small.py:17).

    Bilinear, align_corners=False, legacy (no half-pixel) coordinates, float32 scalers:
    scale = in/out, src = dst*scale, i0 = floor(src), i1 = min(i0+1, in-1), f = src-i0;
    top = tl + (tr-tl)*fx; bot = bl + (br-bl)*fx; out = top + (bot-top)*fy.
    TF-1.x resize_images returns the input unchanged when the size already matches.
    """
    n, ih, iw, c = x.shape
    if (ih, iw) == (oh, ow):
        return x.copy()
    # TF computes scale = (float)in/out and src = (float)dst * scale in float32
    sy = np.float32(ih) / np.float32(oh)
    sx = np.float32(iw) / np.float32(ow)
    ys = np.arange(oh, dtype=np.float32) * sy
    xs = np.arange(ow, dtype=np.float32) * sx
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    y1 = np.minimum(y0 + 1, ih - 1)
    x1 = np.minimum(x0 + 1, iw - 1)
    fy = (ys - np.floor(ys)).astype(x.dtype)[None, :, None, None]
    fx = (xs - np.floor(xs)).astype(x.dtype)[None, None, :, None]
    tl = x[:, y0][:, :, x0]
    tr = x[:, y0][:, :, x1]
    bl = x[:, y1][:, :, x0]
    br = x[:, y1][:, :, x1]
    top = tl + (tr - tl) * fx
    bot = bl + (br - bl) * fx
    return top + (bot - top) * fy


def batch_norm(x, gamma, beta, training, moving_mean=None, moving_var=None, eps=BN_EPS):
    """tf.contrib.layers.batch_norm(center=True, scale=True, is_training=phase) (unet_simple.py:25,41; small.py:22,32).

    training: batch statistics over N,H,W with the biased variance.
    inference: the moving statistics, which the reference never updates
    (UPDATE_OPS is not wired into the train op: train.py:180,304; small_train.py:48),
    so they stay at their initial values mean=0, var=1.
    """
    c = x.shape[-1]
    if training:
        axes = tuple(range(x.ndim - 1))
        mean = x.mean(axis=axes)
        var = ((x - mean) ** 2).mean(axis=axes)
    else:
        mean = np.zeros(c, x.dtype) if moving_mean is None else moving_mean
        var = np.ones(c, x.dtype) if moving_var is None else moving_var
    inv = 1.0 / np.sqrt(var + eps)
    return (x - mean) * (inv * gamma) + beta


def composite(fg, bg, alpha):
    """train.composite / small_train.composite / reader.create_composite_image.

    alpha*fg + (1-alpha)*bg per channel (train.py:14-18; small_train.py:17-21; reader.py:72-79).
    """
    return alpha * fg + (1.0 - alpha) * bg


def charbonnier(out, gt):
    """train.regular_l1: sqrt((out-gt)^2 + (1e-6)^2) (train.py:21-28; small_train.py:24-31)."""
    return np.sqrt(np.square(out - gt) + np.square(1e-6))


def matting_loss(pred, gt, raw_fg, in_bg, in_cmp):
    """The training loss (train.py:42-47, 294-299; small_train.py:39-44).

    loss = mean(0.5*L_alpha[N,H,W,1] + 0.5*L_cmp[N,H,W,3]) — the broadcast sum is
    [N,H,W,3], so the mean equals 0.5*mean(L_alpha) + 0.5*mean(L_cmp).
    Returns (loss, mean alpha loss, mean compositional loss).
    """
    a = charbonnier(pred, gt)
    pred_cmp = composite(raw_fg, in_bg, pred)
    cl = charbonnier(pred_cmp, in_cmp)
    s = 0.5 * a + 0.5 * cl
    return s.mean(), a.mean(), cl.mean()
