"""Numpy restatement of the reference's model graphs (TEST INFRASTRUCTURE).

Each forward mirrors one graph builder op-for-op (unfused, NHWC):
  unet_forward        <- unet.UNetImage.build / unet.UNetVideo.build   (unet.py:86-217)
  unet_simple_forward <- unet_simple.create_model / UNetSimple         (unet_simple.py:45-171)
  unet_small_forward  <- small.UNetSmall                               (small.py:37-50)
  refine_forward      <- refine.RefineNet.build                        (refine.py:14-32)

Weights follow the reference's own construction so that the same seeds give
the same numbers: VGG filters come from a ``data_dict`` {name: [W_hwio, b]}
(unet.py:29 loads it from vgg16.npy), fresh filters come from ``init_conv``
draws on a legacy ``RandomState`` in graph-build order (unet.py:11-17 — the
bias is drawn even where it is discarded, unet.py:59).
"""

import numpy as np

from . import ops

VGG_LAYERS = (
    ("conv1_1", 3, 64), ("conv1_2", 64, 64),
    ("conv2_1", 64, 128), ("conv2_2", 128, 128),
    ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256),
    ("conv4_1", 256, 512), ("conv4_2", 512, 512), ("conv4_3", 512, 512),
    ("conv5_1", 512, 512), ("conv5_2", 512, 512), ("conv5_3", 512, 512),
)


def synthetic_vgg16(seed=0, scale=1.0):
    """Stand-in for the absent weights/vgg16.npy (unet.py:25; .gitignore:3).

    Same dict layout as the real file ({name: [W(3,3,cin,cout) f32, b(cout) f32]});
    He-normal draws from RandomState(seed) in VGG layer order.  ``scale``
    multiplies every filter (used to build non-saturating fixtures).
    """
    rs = np.random.RandomState(seed)
    d = {}
    for name, cin, cout in VGG_LAYERS:
        std = np.sqrt(2.0 / (9 * cin))
        w = (rs.normal(0.0, std, (3, 3, cin, cout)) * scale).astype(np.float32)
        b = rs.normal(0.0, std, cout).astype(np.float32)
        d[name] = [w, b]
    return d


def init_conv(rs, cin, cout):
    """unet.init_conv (unet.py:11-17; same in unet_simple.py:10-16, small.py:5-10, refine.py:5-11)."""
    std = np.sqrt(2.0 / (3 * 3 * int(cin)))
    w = rs.normal(loc=0.0, scale=std, size=(3, 3, cin, cout)).astype(np.float32)
    b = rs.normal(loc=0.0, scale=std, size=cout).astype(np.float32)
    return w, b


# ----------------------------------------------------------------------------- U-Net (unet.py)

UNET_NEW_CONVS = (  # graph-build order of the fresh convs (unet.py:191-203)
    ("upconv_1", 512, 512, False), ("conv4_4", 1024, 512, True),
    ("upconv_2", 512, 256, False), ("conv3_4", 512, 256, True),
    ("upconv_3", 256, 128, False), ("conv2_3", 256, 128, True),
    ("upconv_4", 128, 64, False), ("conv1_5", 128, 1, True),
)


def unet_params(vgg, rs, video=True):
    """All 20 filters of UNetVideo (video=True) / UNetImage, keyed by reference scope name.

    conv1_1: UNetVideo -> [VGG, VGG, 0] over 7 input channels (unet.py:210-217);
             UNetImage -> [VGG/2, VGG/2] over 6 (unet.py:150-157).
    Fresh convs: init_conv draws in build order; upconvs keep no bias (unet.py:59).
    """
    p = {}
    for name, cin, cout in VGG_LAYERS[:12]:  # conv5_3 is commented out (unet.py:117)
        w, b = vgg[name]
        if name == "conv1_1":
            if video:
                t = np.zeros((3, 3, 7, 64), np.float32)
                t[:, :, :3] = w
                t[:, :, 3:6] = w
            else:
                t = np.zeros((3, 3, 6, 64), np.float32)
                t[:, :, :3] = w / 2.0
                t[:, :, 3:6] = w / 2.0
            w = t
        p[name] = (np.asarray(w, np.float32), np.asarray(b, np.float32))
    for name, cin, cout, keep_bias in UNET_NEW_CONVS:
        w, b = init_conv(rs, cin, cout)
        p[name] = (w, b if keep_bias else None)
    return p


def unet_forward(x, p, dtype=np.float64):
    """unet.UNetVideo.build / UNetImage.build (unet.py:161-205 / 87-145) as an eager forward.

    Returns a dict of every public attribute the reference sets (conv1_1 ... conv1_3,
    upconv1..4, pool1..4) plus 'output' = sigmoid(conv1_3).
    """
    f = lambda t: np.asarray(t, dtype)  # noqa: E731
    x = f(x)
    cv = lambda t, name: ops.conv3x3_same(t, f(p[name][0]), None if p[name][1] is None else f(p[name][1]))  # noqa: E731
    r = {}
    r["conv1_1"] = ops.relu(cv(x, "conv1_1"))
    r["conv1_2"] = ops.relu(cv(r["conv1_1"], "conv1_2"))
    r["pool1"] = ops.max_pool_2x2_same(r["conv1_2"])
    r["conv2_1"] = ops.relu(cv(r["pool1"], "conv2_1"))
    r["conv2_2"] = ops.relu(cv(r["conv2_1"], "conv2_2"))
    r["pool2"] = ops.max_pool_2x2_same(r["conv2_2"])
    r["conv3_1"] = ops.relu(cv(r["pool2"], "conv3_1"))
    r["conv3_2"] = ops.relu(cv(r["conv3_1"], "conv3_2"))
    r["conv3_3"] = ops.relu(cv(r["conv3_2"], "conv3_3"))
    r["pool3"] = ops.max_pool_2x2_same(r["conv3_3"])
    r["conv4_1"] = ops.relu(cv(r["pool3"], "conv4_1"))
    r["conv4_2"] = ops.relu(cv(r["conv4_1"], "conv4_2"))
    r["conv4_3"] = ops.relu(cv(r["conv4_2"], "conv4_3"))
    r["pool4"] = ops.max_pool_2x2_same(r["conv4_3"])
    r["conv5_1"] = ops.relu(cv(r["pool4"], "conv5_1"))
    r["conv5_2"] = ops.relu(cv(r["conv5_1"], "conv5_2"))

    def upconv_concat(a, skip, name):  # unet.py:44-63: resize -> conv (no bias/relu) -> concat [up, skip]
        h, w = skip.shape[1:3]
        up = ops.resize_bilinear_tf1(a, h, w)
        return np.concatenate([cv(up, name), skip], axis=-1)

    r["upconv1"] = upconv_concat(r["conv5_2"], r["conv4_3"], "upconv_1")
    r["conv4_4"] = ops.relu(cv(r["upconv1"], "conv4_4"))
    r["upconv2"] = upconv_concat(r["conv4_4"], r["conv3_3"], "upconv_2")
    r["conv3_4"] = ops.relu(cv(r["upconv2"], "conv3_4"))
    r["upconv3"] = upconv_concat(r["conv3_4"], r["conv2_2"], "upconv_3")
    r["conv2_3"] = ops.relu(cv(r["upconv3"], "conv2_3"))
    r["upconv4"] = upconv_concat(r["conv2_3"], r["conv1_2"], "upconv_4")
    r["conv1_3"] = cv(r["upconv4"], "conv1_5")  # attribute conv1_3 holds scope conv1_5 (unet.py:203)
    r["output"] = ops.sigmoid(r["conv1_3"])
    return r


# ----------------------------------------------------------------------------- UNetSimple (unet_simple.py)

SIMPLE_NEW_CONVS = (  # graph-build order inside UNetSimple.__init__ (unet_simple.py:119-142)
    ("select4_1", 1536, 16), ("select4_2", 1536, 16), ("select4_3", 1536, 16),
    ("upconv4", 1536, 48), ("conv4", 96, 48),
    ("select3_1", 768, 8), ("select3_2", 768, 8), ("select3_3", 768, 8),
    ("upconv3", 48, 24), ("conv3", 48, 24),
    ("select2_1", 384, 4), ("select2_2", 384, 4),
    ("upconv2", 24, 24), ("conv2", 32, 32),
    ("select1_1", 9, 2), ("select1_2", 192, 2), ("select1_3", 192, 2),
    ("upconv1", 32, 24), ("conv1", 30, 32),
    ("output", 32, 1),
)


def unet_simple_params(rs):
    """init_conv draws of UNetSimple in build order (bias drawn but unused for upconv*, unet_simple.py:34)."""
    p = {}
    for name, cin, cout in SIMPLE_NEW_CONVS:
        w, b = init_conv(rs, cin, cout)
        p[name] = (w, None if name.startswith("upconv") else b)
    return p


def vgg16_tower(x, vgg, dtype=np.float64):
    """unet_simple.Vgg16.build (unet_simple.py:57-89): frozen VGG16 conv1_1..conv5_3, 4 max-pools."""
    f = lambda t: np.asarray(t, dtype)  # noqa: E731
    cv = lambda t, n: ops.relu(ops.conv3x3_same(t, f(vgg[n][0]), f(vgg[n][1])))  # noqa: E731
    t = {}
    t["conv1_1"] = cv(f(x), "conv1_1")
    t["conv1_2"] = cv(t["conv1_1"], "conv1_2")
    p = ops.max_pool_2x2_same(t["conv1_2"])
    t["conv2_1"] = cv(p, "conv2_1")
    t["conv2_2"] = cv(t["conv2_1"], "conv2_2")
    p = ops.max_pool_2x2_same(t["conv2_2"])
    t["conv3_1"] = cv(p, "conv3_1")
    t["conv3_2"] = cv(t["conv3_1"], "conv3_2")
    t["conv3_3"] = cv(t["conv3_2"], "conv3_3")
    p = ops.max_pool_2x2_same(t["conv3_3"])
    t["conv4_1"] = cv(p, "conv4_1")
    t["conv4_2"] = cv(t["conv4_1"], "conv4_2")
    t["conv4_3"] = cv(t["conv4_2"], "conv4_3")
    p = ops.max_pool_2x2_same(t["conv4_3"])
    t["conv5_1"] = cv(p, "conv5_1")
    t["conv5_2"] = cv(t["conv5_1"], "conv5_2")
    t["conv5_3"] = cv(t["conv5_2"], "conv5_3")
    return t


def unet_simple_forward(cmp, bg, diff, phase, vgg, p, dtype=np.float64, bn=None):
    """unet_simple.create_model(cmp, bg, diff, phase) (unet_simple.py:145-171) -> dict of attributes.

    ``bn`` optionally maps scope -> (gamma, beta); default gamma=1, beta=0 (fresh variables).
    """
    f = lambda t: np.asarray(t, dtype)  # noqa: E731
    cmp, bg, diff = f(cmp), f(bg), f(diff)
    towers = [vgg16_tower(t, vgg, dtype) for t in (cmp, bg, diff)]
    cat = lambda k: np.concatenate([t[k] for t in towers], axis=-1)  # noqa: E731
    layers = {
        "conv1": [np.concatenate([cmp, bg, diff], -1), cat("conv1_1"), cat("conv1_2")],
        "conv2": [cat("conv2_1"), cat("conv2_2")],
        "conv3": [cat("conv3_1"), cat("conv3_2"), cat("conv3_3")],
        "conv4": [cat("conv4_1"), cat("conv4_2"), cat("conv4_3")],
        "conv5": [cat("conv5_1"), cat("conv5_2"), cat("conv5_3")],
    }

    def bnorm(t, scope):
        g, b = (1.0, 0.0) if bn is None or scope not in bn else bn[scope]
        return ops.batch_norm(t, g, b, training=bool(phase))

    def new_conv(t, scope):  # unet_simple.py:19-27: conv + bias -> BN
        w, b = p[scope]
        return bnorm(ops.conv3x3_same(t, f(w), f(b)), scope)

    def upconv_concat(prev_layers, prev, scope):  # unet_simple.py:30-42
        h, w = prev_layers[0].shape[1:3]
        up = ops.resize_bilinear_tf1(prev, h, w)
        up = ops.relu(ops.conv3x3_same(up, f(p[scope][0])))
        return bnorm(np.concatenate(list(prev_layers) + [up], axis=-1), scope)

    r = {}
    R = lambda t, s: ops.relu(new_conv(t, s))  # noqa: E731
    r["select4_1"] = R(layers["conv4"][0], "select4_1")
    r["select4_2"] = R(layers["conv4"][1], "select4_2")
    r["select4_3"] = R(layers["conv4"][2], "select4_3")
    r["upconv4"] = upconv_concat([r["select4_1"], r["select4_2"], r["select4_3"]], layers["conv5"][-1], "upconv4")
    r["conv4"] = R(r["upconv4"], "conv4")
    r["select3_1"] = R(layers["conv3"][0], "select3_1")
    r["select3_2"] = R(layers["conv3"][1], "select3_2")
    r["select3_3"] = R(layers["conv3"][2], "select3_3")
    r["upconv3"] = upconv_concat([r["select3_1"], r["select3_2"], r["select3_3"]], r["conv4"], "upconv3")
    r["conv3"] = R(r["upconv3"], "conv3")
    r["select2_1"] = R(layers["conv2"][0], "select2_1")
    r["select2_2"] = R(layers["conv2"][1], "select2_2")
    r["upconv2"] = upconv_concat([r["select2_1"], r["select2_2"]], r["conv3"], "upconv2")
    r["conv2"] = R(r["upconv2"], "conv2")
    r["select1_1"] = R(layers["conv1"][0], "select1_1")
    r["select1_2"] = R(layers["conv1"][1], "select1_2")
    r["select1_3"] = R(layers["conv1"][2], "select1_3")
    r["upconv1"] = upconv_concat([r["select1_1"], r["select1_2"], r["select1_3"]], r["conv2"], "upconv1")
    r["conv1"] = R(r["upconv1"], "conv1")
    r["logits"] = new_conv(r["conv1"], "output")  # BN output before the sigmoid (unet_simple.py:142)
    r["output"] = ops.sigmoid(r["logits"])
    return r


# ----------------------------------------------------------------------------- UNetSmall (small.py)

SMALL_NEW_CONVS = (  # small.py:39-49 build order; cin of conv1_1 is the caller's (6 in small_train.py:95)
    ("conv1_1", None, 8), ("conv2_1", 8, 16), ("conv3_1", 16, 32), ("conv3_2", 32, 32),
    ("upconv1", 32, 16), ("conv2_2", 32, 16), ("upconv2", 16, 8), ("conv1_2", 16, 8),
    ("conv1_3", 8, 1),
)


def unet_small_params(rs, cin=6):
    p = {}
    for name, ci, co in SMALL_NEW_CONVS:
        w, b = init_conv(rs, cin if ci is None else ci, co)
        p[name] = (w, None if name.startswith("upconv") else b)
    return p


def unet_small_forward(x, phase, p, dtype=np.float64, bn=None):
    """small.UNetSmall(input, phase) (small.py:37-50); upconv concat order is [skip, up] (small.py:20)."""
    f = lambda t: np.asarray(t, dtype)  # noqa: E731

    def bnorm(t, scope):
        g, b = (1.0, 0.0) if bn is None or scope not in bn else bn[scope]
        return ops.batch_norm(t, g, b, training=bool(phase))

    def new_conv(t, scope):  # small.py:26-34
        w, b = p[scope]
        return bnorm(ops.conv3x3_same(t, f(w), f(b)), scope)

    def upconv_concat(prev_layer, down, scope):  # small.py:13-23
        h, w = prev_layer.shape[1:3]
        up = ops.resize_bilinear_tf1(down, h, w)
        up = ops.relu(ops.conv3x3_same(up, f(p[scope][0])))
        return bnorm(np.concatenate([prev_layer, up], axis=-1), scope)

    r = {}
    r["conv1_1"] = ops.relu(new_conv(f(x), "conv1_1"))
    r["pool1"] = ops.max_pool_2x2_same(r["conv1_1"])
    r["conv2_1"] = ops.relu(new_conv(r["pool1"], "conv2_1"))
    r["pool2"] = ops.max_pool_2x2_same(r["conv2_1"])
    r["conv3_1"] = ops.relu(new_conv(r["pool2"], "conv3_1"))
    r["conv3_2"] = ops.relu(new_conv(r["conv3_1"], "conv3_2"))
    r["upconv1"] = upconv_concat(r["conv2_1"], r["conv3_2"], "upconv1")
    r["conv2_2"] = ops.relu(new_conv(r["upconv1"], "conv2_2"))
    r["upconv2"] = upconv_concat(r["conv1_1"], r["conv2_2"], "upconv2")
    r["conv1_2"] = ops.relu(new_conv(r["upconv2"], "conv1_2"))
    r["conv1_3"] = new_conv(r["conv1_2"], "conv1_3")
    r["output"] = ops.sigmoid(r["conv1_3"])
    return r


# ----------------------------------------------------------------------------- RefineNet (refine.py)

def refine_params(rs, cin):
    """conv1..conv4 init_conv draws (refine.py:18-31), each keeps its bias."""
    return {n: init_conv(rs, cin, 64) for n in ("conv1", "conv2", "conv3", "conv4")}


def refine_forward(x, p, dtype=np.float64):
    """refine.RefineNet.build (refine.py:27-32): four independent convs of the SAME input;
    conv1..3 = relu (never used), conv4 = softmax over 64 channels = output."""
    f = lambda t: np.asarray(t, dtype)  # noqa: E731
    x = f(x)
    r = {}
    for n in ("conv1", "conv2", "conv3"):
        r[n] = ops.relu(ops.conv3x3_same(x, f(p[n][0]), f(p[n][1])))
    r["conv4"] = ops.softmax_lastdim(ops.conv3x3_same(x, f(p["conv4"][0]), f(p["conv4"][1])))
    r["output"] = r["conv4"]
    return r
