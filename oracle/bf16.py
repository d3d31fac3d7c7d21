"""bf16 operand arithmetic of the timed path, restated on the CPU (TEST INFRASTRUCTURE).

The throughput path computes every conv of unet.UNetVideo (unet.py:161-205) on bf16 operands with f32
accumulation.  To pin those kernels layer by layer at their timed shapes, the oracle evaluates each layer in float64
on EXACTLY the operands the kernel consumes — the GPU's own bf16 input activation and the bf16-rounded filter — so
that the only difference left is the kernel's f32 summation and its final bf16 rounding (<= 1 bf16 ulp).

Restated here (beyond oracle/ops.py, which restates the reference's TF ops):
  * bf16_round: round-to-nearest-even to bfloat16 (v_cvt_pk_bf16_f32, the kernels' only rounding mode);
  * fold_up2x_weights / upconv2x_folded: tf.image.resize_images 2x (TF1 legacy, scale 0.5) followed by the 3x3 SAME
    conv of unet.py:44-63 is linear in the low-res frame, so output pixel (2i+a, 2j+b) is a 3x3 conv of the low-res
    frame at (i, j) with a phase filter W'_ab = R_a W R_b^T.  ``upconv2x_folded(..., round_w=False)`` equals
    resize -> conv exactly in float64 (tests/test_oracle_bf16.py pins that identity); with ``round_w`` the folded
    filter is rounded to bf16 like the kernel's packed copy, and the frame-border pixels (which see the resized
    image's zero padding) are evaluated the unfused way from the bf16-rounded f32 resize, as the border pass does;
  * head_shares: conv1_5's per-tap shares sum_c bf16(w[tap][c]) * y[c] of one half of cat1 (unet.py:200-205).
"""

import numpy as np

from . import ops

# TF1 legacy 2x resize as a 3x3 mixing matrix per output phase: rows = low-res offset u-1, columns = kernel row kh
_R = (np.array([[.5, 0., 0.], [.5, 1., .5], [0., 0., .5]]),
      np.array([[0., 0., 0.], [1., .5, 0.], [0., .5, 1.]]))


def bf16_round(a):
    """Round to the nearest bfloat16 (ties to even), returned as float64 (via float32, exact for bf16 values)."""
    f = np.ascontiguousarray(a, np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32).astype(np.float64)


def fold_up2x_weights(w, dtype=np.float32):
    """[3,3,cin,cout] HWIO -> [3,3,cin,4*cout]: output channel p*cout + co is phase p = 2a+b of channel co, summed in
    float64 and returned as float32 like the packed source filter (``dtype`` float64: unrounded)."""
    w = np.asarray(w, np.float64)
    cin, cout = w.shape[2], w.shape[3]
    out = np.empty((3, 3, cin, 4 * cout), np.float64)
    for p in range(4):
        ra, rb = _R[p >> 1], _R[p & 1]
        # W'[u][v] = sum_{kh,kw} R_a[u][kh] R_b[v][kw] W[kh][kw]
        out[..., p * cout:(p + 1) * cout] = np.einsum("uh,vk,hkco->uvco", ra, rb, w)
    return out.astype(dtype)


def _pad_replicate_br(x):
    """Zero row/column before the frame, a replicated row/column after it (the folded conv's low-res padding)."""
    n, h, w, c = x.shape
    xp = np.zeros((n, h + 2, w + 2, c), x.dtype)
    xp[:, 1:-1, 1:-1] = x
    xp[:, -1, 1:-1] = x[:, -1]
    xp[:, :, -1] = xp[:, :, -2]
    return xp


def _conv_padded(xp, w):
    """3x3 VALID conv of an already padded [n,h+2,w+2,c] frame (float64)."""
    n, hp, wp, c = xp.shape
    h, wd, o = hp - 2, wp - 2, w.shape[3]
    y = np.zeros((n, h, wd, o), np.float64)
    rows = max(1, int(64e6 // max(1, n * wd * max(c, o) * 8)))
    for r0 in range(0, h, rows):
        r1 = min(h, r0 + rows)
        acc = np.zeros((n * (r1 - r0) * wd, o), np.float64)
        for kh in range(3):
            for kw in range(3):
                acc += xp[:, r0 + kh:r1 + kh, kw:kw + wd, :].reshape(-1, c) @ w[kh, kw]
        y[:, r0:r1] = acc.reshape(n, r1 - r0, wd, o)
    return y


def resize2x_at(x, rows, cols):
    """tf.image.resize_images(x, [2H, 2W]) (TF1 legacy bilinear, float32 arithmetic like the kernels) evaluated only
    at output rows ``rows`` x columns ``cols`` -> float32 [n, len(rows), len(cols), c]."""
    x = np.asarray(x, np.float32)
    n, h, w, c = x.shape
    ys = np.asarray(rows, np.float32) * np.float32(0.5)
    xs = np.asarray(cols, np.float32) * np.float32(0.5)
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    y1, x1 = np.minimum(y0 + 1, h - 1), np.minimum(x0 + 1, w - 1)
    fy = (ys - np.floor(ys)).astype(np.float32)[None, :, None, None]
    fx = (xs - np.floor(xs)).astype(np.float32)[None, None, :, None]
    tl, tr = x[:, y0][:, :, x0], x[:, y0][:, :, x1]
    bl, br = x[:, y1][:, :, x0], x[:, y1][:, :, x1]
    top = tl + (tr - tl) * fx
    bot = bl + (br - bl) * fx
    return (top + (bot - top) * fy).astype(np.float32)


def upconv2x_folded(x, w, round_w=True):
    """conv3x3_SAME(resize2x(x), w) for an [n,h,w,cin] frame -> float64 [n,2h,2w,cout] (no bias, no activation: the
    upconv half of unet.py:44-63).

    round_w=False: the exact linear identity in float64 (equals oracle.ops resize_bilinear_tf1 -> conv3x3_same).
    round_w=True: the bf16 kernel's arithmetic — interior pixels from the folded filter rounded to bf16, the frame's
    border rows/columns (0 and 2h-1 / 2w-1) from the f32 resize rounded to bf16 and the bf16 filter."""
    x = np.asarray(x, np.float64)
    n, h, wd, cin = x.shape
    cout = w.shape[3]
    wf = bf16_round(fold_up2x_weights(w)) if round_w else fold_up2x_weights(w, np.float64)
    yl = _conv_padded(_pad_replicate_br(x), wf)  # [n,h,w,4*cout]
    oh, ow = 2 * h, 2 * wd
    y = np.empty((n, oh, ow, cout), np.float64)
    for p in range(4):
        y[:, (p >> 1)::2, (p & 1)::2] = yl[..., p * cout:(p + 1) * cout]
    # border rows / columns see the resized image's zero padding: evaluate them unfused
    wb = bf16_round(w) if round_w else np.asarray(w, np.float64)
    q = (lambda t: bf16_round(t)) if round_w else (lambda t: np.asarray(t, np.float64))
    if round_w:
        rz = lambda rr, cc: q(resize2x_at(x, rr, cc))  # noqa: E731
    else:
        xr = ops.resize_bilinear_tf1(x, oh, ow)
        rz = lambda rr, cc: xr[:, rr][:, :, cc]  # noqa: E731
    allc, allr = np.arange(ow), np.arange(oh)
    top = ops.conv3x3_same(rz([0, 1], allc), wb)          # output row 0 (row -1 is zero padding)
    bot = ops.conv3x3_same(rz([oh - 2, oh - 1], allc), wb)  # output row oh-1
    left = ops.conv3x3_same(rz(allr, [0, 1]), wb)         # output column 0
    right = ops.conv3x3_same(rz(allr, [ow - 2, ow - 1]), wb)
    y[:, 0] = top[:, 0]
    y[:, oh - 1] = bot[:, 1]
    y[:, :, 0] = left[:, :, 0]
    y[:, :, ow - 1] = right[:, :, 1]
    return y


def head_shares(y, w_half):
    """Per-tap shares of a cout == 1 head over one half of its input: s[..., tap] = sum_c w_half[tap][c] * y[..., c]
    for taps 0..8 (taps 9..11 zero) -> float64 [n,h,w,12].  ``w_half`` [3,3,c,1] (already bf16-rounded when pinning
    the kernels' shares)."""
    y = np.asarray(y, np.float64)
    wt = np.asarray(w_half, np.float64).reshape(9, -1)  # [tap][c]
    s = np.zeros(y.shape[:3] + (12,), np.float64)
    s[..., :9] = y @ wt.T
    return s


def head_from_shares(pa, pb, bias):
    """logits[p] = bias + sum_tap (pa + pb)[p + off(tap)][tap], off(tap) = (tap/3 - 1, tap%3 - 1), zero outside."""
    s = np.asarray(pa, np.float64) + np.asarray(pb, np.float64)
    n, h, w, _ = s.shape
    sp = np.zeros((n, h + 2, w + 2, 12), np.float64)
    sp[:, 1:-1, 1:-1] = s
    out = np.full((n, h, w, 1), 0.0 if bias is None else float(np.asarray(bias).reshape(-1)[0]), np.float64)
    for tap in range(9):
        kh, kw = divmod(tap, 3)
        out[..., 0] += sp[:, kh:kh + h, kw:kw + w, tap]
    return out
