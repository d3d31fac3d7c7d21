"""CPU restatement of the config-5 training step (TEST INFRASTRUCTURE — only tests/, smoke() and bench.py's
cpu_baseline may use it; the product never does).

  train_step_grads  one iteration of train.py's video_procedure / simple_procedure (train.py:288-343 / 176-227):
                    create_model(cmp, bg, warped, phase=True) (unet_simple.py:145-171) with the frozen VGG towers
                    taken from the numpy oracle (models.vgg16_tower), then UNetSimple restated in torch float64 so
                    that autograd gives d loss / d every variable of 'model/simple_unet' (train.py:289)
  small_step_grads  one iteration of small_train.py's small_training (small_train.py:34-88, entry train() at
                    :91-112): UNetSmall(concat(cmp, bg), phase=True) (small.py:37-50) restated in torch float64, the
                    same loss (small_train.py:39-44), autograd over ALL its variables (small_train.py:47-48: Adam on
                    every trainable variable — conv weights / biases and BN gamma / beta; the upconvs' drawn biases
                    feed nothing and get no gradient).  max_pool's gradient goes to each window's first maximum in
                    row-major order (TF MaxPoolGrad's strict '>' scan; parity unpinned, TF is absent)
  image_step_grads  one iteration of train.py's training_procedure (train.py:37-109, entry train() at :112-135):
                    unet.UNetImage.build(x = concat(cmp, bg)) (unet.py:86-148: 12 VGG convs, 4 SAME max-pools, 4
                    upconv_concat = resize -> conv (no bias, no relu) -> [up, skip], conv1_5 + sigmoid) restated in
                    torch float64, the same loss (train.py:41-47), autograd over EVERY variable (train.py:51-52:
                    minimize() with the default var_list — the VGG filters and biases, UNetImage's halved conv1_1
                    and the fresh convs; the upconvs' drawn biases feed nothing and get no gradient)
  adam_tf           tf.train.AdamOptimizer's ApplyAdam (train.py:302-304) in numpy float32, including TF's f32
                    beta-power variables and lr_t = lr*sqrt(1-beta2^t)/(1-beta1^t)

The forward is the same op sequence as models.unet_simple_forward (pinned by the reference builders' goldens,
tests/golden/unet_simple_64_train.npz); tests check the two agree before trusting the gradients.  No TF gradient
goldens exist (TF is absent), so the backward is pinned by autograd on that forward: "parity unpinned" against
real TF 1.x gradients.
"""

import numpy as np
import torch
import torch.nn.functional as F

from . import models as om

BN_EPS = 1e-3

LEVELS = (
    ("conv4", ("select4_1", "select4_2", "select4_3"), "upconv4", "conv4"),
    ("conv3", ("select3_1", "select3_2", "select3_3"), "upconv3", "conv3"),
    ("conv2", ("select2_1", "select2_2"), "upconv2", "conv2"),
    ("conv1", ("select1_1", "select1_2", "select1_3"), "upconv1", "conv1"),
)


def _conv(x, w, b=None):
    """tf.nn.conv2d 3x3 SAME (+ bias_add) on NHWC with an HWIO filter."""
    y = F.conv2d(x.permute(0, 3, 1, 2).contiguous(), w.permute(3, 2, 0, 1).contiguous(), b, padding=1)
    return y.permute(0, 2, 3, 1)


def _bn(x, gamma, beta):
    mean = x.mean(dim=(0, 1, 2))
    var = ((x - mean) ** 2).mean(dim=(0, 1, 2))
    return (x - mean) * (gamma / torch.sqrt(var + BN_EPS)) + beta


def _resize(x, oh, ow):
    """TF-1 legacy bilinear (models/ops.resize_bilinear_tf1) as differentiable gathers."""
    n, ih, iw, c = x.shape
    if (ih, iw) == (oh, ow):
        return x
    sy = np.float32(ih) / np.float32(oh)
    sx = np.float32(iw) / np.float32(ow)
    ys = np.arange(oh, dtype=np.float32) * sy
    xs = np.arange(ow, dtype=np.float32) * sx
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    y1 = np.minimum(y0 + 1, ih - 1)
    x1 = np.minimum(x0 + 1, iw - 1)
    dev = x.device
    fy = torch.from_numpy((ys - np.floor(ys)).astype(np.float64))[None, :, None, None].to(dev)
    fx = torch.from_numpy((xs - np.floor(xs)).astype(np.float64))[None, None, :, None].to(dev)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    tl = x[:, T(y0)][:, :, T(x0)]
    tr = x[:, T(y0)][:, :, T(x1)]
    bl = x[:, T(y1)][:, :, T(x0)]
    br = x[:, T(y1)][:, :, T(x1)]
    top = tl + (tr - tl) * fx
    bot = bl + (br - bl) * fx
    return top + (bot - top) * fy


def _loss(la, lc, sample_weights):
    """mean(0.5*L_alpha + 0.5*L_cmp) (train.py:294-298); with per-sample weights w: sum_i w_i * (sample i's mean) —
    e.g. the objective data-parallel replicas jointly minimise, the sum of each replica's batch-mean loss."""
    s = 0.5 * la + 0.5 * lc
    if sample_weights is None:
        return s.mean()
    w = torch.as_tensor(np.asarray(sample_weights, np.float64), device=s.device)
    return (s.mean(dim=(1, 2, 3)) * w).sum()


def train_step_grads(cmp, bg, warped, gt, raw_fg, vgg, params, bn=None, towers=None, device="cpu",
                     sample_weights=None):
    """-> (loss terms (loss, alpha_loss, cmp_loss), alpha, grads {(scope, kind): ndarray})

    device: where the float64 autograd runs ("cpu"; a GPU only for large test shapes — float64 there too, the
    checker, not the product).

    params: {scope: (w_hwio, bias|None)} (models.unet_simple_params); bn: {scope: (gamma, beta)} or fresh (1, 0).
    kinds: 'w', 'b' (new_conv scopes), 'gamma', 'beta' — the trainable variables of unet_simple.py:19-42.
    towers: optional precomputed frozen-tower features (3 dicts layer -> [N,H,W,C], plus 'in9' in the first) to
    isolate the trainable head (a test of a reduced-precision path's head against its own tower features)."""
    f64 = lambda a: np.asarray(a, np.float64)  # noqa: E731
    cmp, bg, warped = f64(cmp), f64(bg), f64(warped)
    in9 = np.concatenate([cmp, bg, warped], -1)
    if towers is None:
        towers = [om.vgg16_tower(t, vgg) for t in (cmp, bg, warped)]
    elif "in9" in towers[0]:
        in9 = towers[0]["in9"]
    # tower features may be numpy arrays or tensors (a device test hands over the trainer's own, already on device)
    dd = lambda a: a.to(device, torch.float64) if isinstance(a, torch.Tensor) else torch.from_numpy(f64(a)).to(device)  # noqa: E731,E501
    cat = lambda k: torch.cat([dd(t[k]) for t in towers], -1)  # noqa: E731
    layers = {
        "conv1": [dd(in9), cat("conv1_1"), cat("conv1_2")],
        "conv2": [cat("conv2_1"), cat("conv2_2")],
        "conv3": [cat("conv3_1"), cat("conv3_2"), cat("conv3_3")],
        "conv4": [cat("conv4_1"), cat("conv4_2"), cat("conv4_3")],
        "conv5": [cat("conv5_1"), cat("conv5_2"), cat("conv5_3")],
    }
    V = {}
    for scope, (w, b) in params.items():
        V[scope, "w"] = torch.tensor(f64(w), requires_grad=True, device=device)
        if not scope.startswith("upconv"):
            V[scope, "b"] = torch.tensor(f64(b), requires_grad=True, device=device)
    widths = {"upconv4": 96, "upconv3": 48, "upconv2": 32, "upconv1": 30}
    for scope, (w, b) in params.items():
        c = widths.get(scope, w.shape[3])
        g, be = (np.ones(c), np.zeros(c)) if bn is None or scope not in bn else bn[scope]
        V[scope, "gamma"] = torch.tensor(f64(g), requires_grad=True, device=device)
        V[scope, "beta"] = torch.tensor(f64(be), requires_grad=True, device=device)

    def new_conv(x, s):
        return _bn(_conv(x, V[s, "w"], V[s, "b"]), V[s, "gamma"], V[s, "beta"])

    prev = layers["conv5"][-1]
    for key, sels, up, conv in LEVELS:
        srcs = layers[key]
        outs = [torch.relu(new_conv(srcs[i], s)) for i, s in enumerate(sels)]
        h, w = outs[0].shape[1:3]
        u = torch.relu(_conv(_resize(prev, h, w), V[up, "w"]))
        catn = _bn(torch.cat(outs + [u], -1), V[up, "gamma"], V[up, "beta"])
        prev = torch.relu(new_conv(catn, conv))
    alpha = torch.sigmoid(new_conv(prev, "output"))
    gt_t, fg_t, bg_t, cmp_t = (torch.from_numpy(f64(a)).to(device) for a in (gt, raw_fg, bg, cmp))
    eps2 = np.float64(np.float32(1e-6) ** 2)
    la = torch.sqrt((alpha - gt_t) ** 2 + eps2)
    lc = torch.sqrt((alpha * fg_t + (1 - alpha) * bg_t - cmp_t) ** 2 + eps2)
    loss = _loss(la, lc, sample_weights)
    loss.backward()
    grads = {k: v.grad.cpu().numpy().copy() for k, v in V.items()}
    terms = (float(loss.detach()), float(la.mean().detach()), float(lc.mean().detach()))
    return terms, alpha.detach().cpu().numpy(), grads


def _pool(x):
    """tf.nn.max_pool 2x2/2 SAME (small.py:40,42): pad past odd edges with -inf; torch.max over the row-major window
    returns (and back-propagates to) the first maximum, TF's tie rule."""
    n, h, w, c = x.shape
    oh, ow = (h + 1) // 2, (w + 1) // 2
    xp = F.pad(x, (0, 0, 0, 2 * ow - w, 0, 2 * oh - h), value=float("-inf"))
    win = xp.reshape(n, oh, 2, ow, 2, c).permute(0, 1, 3, 5, 2, 4).reshape(n, oh, ow, c, 4)
    return win.max(dim=-1).values


SMALL_BN_WIDTH = {"upconv1": 32, "upconv2": 16}


def small_step_grads(cmp, bg, gt, raw_fg, params, bn=None, device="cpu", sample_weights=None):
    """-> (loss terms, alpha, grads {(scope, kind): ndarray}, forward dict) for small_train.py's step on
    input = concat(cmp, bg) (small_train.py:95).  params: models.unet_small_params (cin 6); bn: {scope: (gamma,
    beta)} or fresh (1, 0)."""
    f64 = lambda a: np.asarray(a, np.float64)  # noqa: E731
    T = lambda a: torch.from_numpy(f64(a)).to(device)  # noqa: E731
    x = torch.cat([T(cmp), T(bg)], -1)
    V = {}
    for scope, (w, b) in params.items():
        V[scope, "w"] = torch.tensor(f64(w), requires_grad=True, device=device)
        if not scope.startswith("upconv"):
            V[scope, "b"] = torch.tensor(f64(b), requires_grad=True, device=device)
        c = SMALL_BN_WIDTH.get(scope, w.shape[3])
        g, be = (np.ones(c), np.zeros(c)) if bn is None or scope not in bn else bn[scope]
        V[scope, "gamma"] = torch.tensor(f64(g), requires_grad=True, device=device)
        V[scope, "beta"] = torch.tensor(f64(be), requires_grad=True, device=device)

    def new_conv(t, s):  # small.py:26-34
        return _bn(_conv(t, V[s, "w"], V[s, "b"]), V[s, "gamma"], V[s, "beta"])

    def upconv_concat(prev_layer, down, s):  # small.py:13-23: resize -> conv (no bias) -> relu -> [skip, up] -> BN
        h, w = prev_layer.shape[1:3]
        up = torch.relu(_conv(_resize(down, h, w), V[s, "w"]))
        return _bn(torch.cat([prev_layer, up], -1), V[s, "gamma"], V[s, "beta"])

    r = {}
    r["conv1_1"] = torch.relu(new_conv(x, "conv1_1"))
    r["pool1"] = _pool(r["conv1_1"])
    r["conv2_1"] = torch.relu(new_conv(r["pool1"], "conv2_1"))
    r["pool2"] = _pool(r["conv2_1"])
    r["conv3_1"] = torch.relu(new_conv(r["pool2"], "conv3_1"))
    r["conv3_2"] = torch.relu(new_conv(r["conv3_1"], "conv3_2"))
    r["upconv1"] = upconv_concat(r["conv2_1"], r["conv3_2"], "upconv1")
    r["conv2_2"] = torch.relu(new_conv(r["upconv1"], "conv2_2"))
    r["upconv2"] = upconv_concat(r["conv1_1"], r["conv2_2"], "upconv2")
    r["conv1_2"] = torch.relu(new_conv(r["upconv2"], "conv1_2"))
    r["conv1_3"] = new_conv(r["conv1_2"], "conv1_3")
    alpha = torch.sigmoid(r["conv1_3"])
    gt_t, fg_t, bg_t, cmp_t = (T(a) for a in (gt, raw_fg, bg, cmp))
    eps2 = np.float64(np.float32(1e-6) ** 2)
    la = torch.sqrt((alpha - gt_t) ** 2 + eps2)
    lc = torch.sqrt((alpha * fg_t + (1 - alpha) * bg_t - cmp_t) ** 2 + eps2)
    loss = _loss(la, lc, sample_weights)
    loss.backward()
    grads = {k: v.grad.cpu().numpy().copy() for k, v in V.items() if v.grad is not None}
    terms = (float(loss.detach()), float(la.mean().detach()), float(lc.mean().detach()))
    fwd = {k: v.detach().cpu().numpy() for k, v in r.items()}
    fwd["output"] = alpha.detach().cpu().numpy()
    return terms, fwd["output"], grads, fwd


IMAGE_LAYERS = ("conv1_1", "conv1_2", "conv2_1", "conv2_2", "conv3_1", "conv3_2", "conv3_3", "conv4_1", "conv4_2",
                "conv4_3", "conv5_1", "conv5_2", "upconv_1", "conv4_4", "upconv_2", "conv3_4", "upconv_3", "conv2_3",
                "upconv_4", "conv1_5")


def image_step_grads(cmp, bg, gt, raw_fg, params, device="cpu", sample_weights=None):
    """-> (loss terms (loss, alpha_loss, cmp_loss), alpha, grads {(scope, kind): ndarray}, forward dict) for
    train.py's training_procedure on x = concat(cmp, bg) (train.py:41: in_cmp, in_bg = split(x, [3, 3])).
    params: {scope: (w_hwio, bias|None)} of UNetImage (models.unet_params(video=False)); kinds 'w' and 'b'.
    The forward is models.unet_forward's op sequence (a test checks the two agree)."""
    f64 = lambda a: np.asarray(a, np.float64)  # noqa: E731
    T = lambda a: torch.from_numpy(f64(a)).to(device)  # noqa: E731
    x = torch.cat([T(cmp), T(bg)], -1)
    V = {}
    for scope in IMAGE_LAYERS:
        w, b = params[scope]
        V[scope, "w"] = torch.tensor(f64(w), requires_grad=True, device=device)
        if b is not None:
            V[scope, "b"] = torch.tensor(f64(b), requires_grad=True, device=device)
    cv = lambda t, s: _conv(t, V[s, "w"], V.get((s, "b")))  # noqa: E731

    def upconv_concat(a, skip, s):  # unet.py:44-63
        h, w = skip.shape[1:3]
        return torch.cat([cv(_resize(a, h, w), s), skip], -1)

    r = {}
    r["conv1_1"] = torch.relu(cv(x, "conv1_1"))
    r["conv1_2"] = torch.relu(cv(r["conv1_1"], "conv1_2"))
    r["pool1"] = _pool(r["conv1_2"])
    r["conv2_1"] = torch.relu(cv(r["pool1"], "conv2_1"))
    r["conv2_2"] = torch.relu(cv(r["conv2_1"], "conv2_2"))
    r["pool2"] = _pool(r["conv2_2"])
    r["conv3_1"] = torch.relu(cv(r["pool2"], "conv3_1"))
    r["conv3_2"] = torch.relu(cv(r["conv3_1"], "conv3_2"))
    r["conv3_3"] = torch.relu(cv(r["conv3_2"], "conv3_3"))
    r["pool3"] = _pool(r["conv3_3"])
    r["conv4_1"] = torch.relu(cv(r["pool3"], "conv4_1"))
    r["conv4_2"] = torch.relu(cv(r["conv4_1"], "conv4_2"))
    r["conv4_3"] = torch.relu(cv(r["conv4_2"], "conv4_3"))
    r["pool4"] = _pool(r["conv4_3"])
    r["conv5_1"] = torch.relu(cv(r["pool4"], "conv5_1"))
    r["conv5_2"] = torch.relu(cv(r["conv5_1"], "conv5_2"))
    r["upconv1"] = upconv_concat(r["conv5_2"], r["conv4_3"], "upconv_1")
    r["conv4_4"] = torch.relu(cv(r["upconv1"], "conv4_4"))
    r["upconv2"] = upconv_concat(r["conv4_4"], r["conv3_3"], "upconv_2")
    r["conv3_4"] = torch.relu(cv(r["upconv2"], "conv3_4"))
    r["upconv3"] = upconv_concat(r["conv3_4"], r["conv2_2"], "upconv_3")
    r["conv2_3"] = torch.relu(cv(r["upconv3"], "conv2_3"))
    r["upconv4"] = upconv_concat(r["conv2_3"], r["conv1_2"], "upconv_4")
    r["conv1_3"] = cv(r["upconv4"], "conv1_5")
    alpha = torch.sigmoid(r["conv1_3"])
    gt_t, fg_t, bg_t, cmp_t = (T(a) for a in (gt, raw_fg, bg, cmp))
    eps2 = np.float64(np.float32(1e-6) ** 2)
    la = torch.sqrt((alpha - gt_t) ** 2 + eps2)
    lc = torch.sqrt((alpha * fg_t + (1 - alpha) * bg_t - cmp_t) ** 2 + eps2)
    loss = _loss(la, lc, sample_weights)
    loss.backward()
    grads = {k: v.grad.cpu().numpy().copy() for k, v in V.items()}
    terms = (float(loss.detach()), float(la.mean().detach()), float(lc.mean().detach()))
    fwd = {k: v.detach().cpu().numpy() for k, v in r.items()}
    fwd["output"] = alpha.detach().cpu().numpy()
    return terms, fwd["output"], grads, fwd


def adam_tf(var, m, v, grad, t, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
    """ApplyAdam after ``t`` steps' beta-power updates (t >= 1), numpy float32 -> (var, m, v)."""
    f = np.float32
    b1p, b2p = f(1.0), f(1.0)
    for _ in range(t):
        b1p, b2p = f(b1p * f(beta1)), f(b2p * f(beta2))
    lr_t = f(f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p))
    g = np.asarray(grad, f)
    m = (m + (g - m) * (f(1) - f(beta1))).astype(f)
    v = (v + (g * g - v) * (f(1) - f(beta2))).astype(f)
    var = (var - (m * lr_t) / (np.sqrt(v) + f(eps))).astype(f)
    return var, m, v
