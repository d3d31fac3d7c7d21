"""Weight construction with the reference's exact semantics.

* VGG16 filters come from a ``data_dict`` {layer: [W_hwio f32, b f32]} — the
  format of weights/vgg16.npy that unet.py:29 / unet_simple.py:54 load.  That
  file is not shipped with the reference (.gitignore:3); ``synthetic_vgg16``
  stands in with seeded He-normal draws (generator spec: RandomState(seed),
  layers conv1_1..conv5_3 in order, filter then bias, std sqrt(2/(9*cin))).
* Fresh filters follow ``init_conv`` (unet.py:11-17): drawn from numpy's
  GLOBAL legacy RNG (np.random.normal), filter then bias — the bias is drawn
  even where the graph discards it (unet.py:59, unet_simple.py:34, small.py:18).
  So ``np.random.seed(s)`` before ``build()`` reproduces the reference's weights.
"""

import os

import numpy as np

VGG16_LAYERS = (
    ("conv1_1", 3, 64), ("conv1_2", 64, 64),
    ("conv2_1", 64, 128), ("conv2_2", 128, 128),
    ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256),
    ("conv4_1", 256, 512), ("conv4_2", 512, 512), ("conv4_3", 512, 512),
    ("conv5_1", 512, 512), ("conv5_2", 512, 512), ("conv5_3", 512, 512),
)

DEFAULT_VGG_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "weights", "vgg16.npy")


def synthetic_vgg16(seed=0, scale=1.0):
    rs = np.random.RandomState(seed)
    out = {}
    for name, cin, cout in VGG16_LAYERS:
        std = np.sqrt(2.0 / (9 * cin))
        w = rs.normal(0.0, std, (3, 3, cin, cout))
        if scale != 1.0:
            w = w * scale
        out[name] = [w.astype(np.float32), rs.normal(0.0, std, cout).astype(np.float32)]
    return out


def save_vgg16_npz(data_dict, path):
    """Write a data_dict as a plain-array .npz ("<layer>/W", "<layer>/b"): no pickle, loadable with
    allow_pickle=False by load_vgg16."""
    arrays = {}
    for name, (w, b) in data_dict.items():
        arrays[name + "/W"] = np.asarray(w, np.float32)
        arrays[name + "/b"] = np.asarray(b, np.float32)
    np.savez(path, **arrays)


def _load_npz(path):
    out = {}
    with np.load(path, allow_pickle=False) as z:
        for key in z.files:
            name, kind = key.rsplit("/", 1)
            ent = out.setdefault(name, [None, None])
            ent[0 if kind == "W" else 1] = z[key]
    bad = [k for k, (w, b) in out.items() if w is None or b is None]
    if bad:
        raise ValueError("%s: layers without both W and b: %s" % (path, bad))
    return out


def load_vgg16(path_or_dict, allow_pickle=None):
    """Accept a data_dict, a weights-only ``.npz`` (save_vgg16_npz / tools/vgg_npy_to_npz.py), or a pickled
    ``vgg16.npy`` as unet.py:29 / unet_simple.py:54 load it.

    A pickled .npy can execute code when loaded, so it is refused unless the caller opts in with
    ``allow_pickle=True`` or VMATTING_ALLOW_PICKLE=1 (trusted files only).  With the default path, a
    ``weights/vgg16.npz`` next to the reference's ``weights/vgg16.npy`` is preferred."""
    if isinstance(path_or_dict, dict):
        return path_or_dict
    path = DEFAULT_VGG_PATH if path_or_dict is None else os.fspath(path_or_dict)
    # only the default location is redirected to its converted sibling: a path the caller named is loaded as named
    if path_or_dict is None and os.path.exists(path[:-4] + ".npz"):
        path = path[:-4] + ".npz"
    if not os.path.exists(path):
        raise FileNotFoundError("[Errno 2] No such file or directory: %r (pass a data_dict, e.g. "
                                "vmatting.weights.synthetic_vgg16(0), or a vgg16 .npz / .npy)" % path)
    if path.endswith(".npz"):
        return _load_npz(path)
    if allow_pickle is None:
        allow_pickle = os.environ.get("VMATTING_ALLOW_PICKLE", "") == "1"
    if not allow_pickle:
        raise ValueError("%s is a pickled data_dict, which can run code when loaded.  Convert it once with "
                         "tools/vgg_npy_to_npz.py (weights-only .npz), or pass allow_pickle=True / set "
                         "VMATTING_ALLOW_PICKLE=1 for a file you trust" % path)
    return np.load(path, encoding="latin1", allow_pickle=True).item()


def init_conv(cin, cout, rng=None):
    """unet.init_conv: He-normal filter [3,3,cin,cout] then bias [cout], both f32."""
    r = np.random if rng is None else rng
    std = np.sqrt(2.0 / (3 * 3 * int(cin)))
    w = r.normal(loc=0.0, scale=std, size=(3, 3, cin, cout)).astype(np.float32)
    b = r.normal(loc=0.0, scale=std, size=cout).astype(np.float32)
    return w, b


def bn_inference_affine(gamma, beta, moving_mean=None, moving_var=None, eps=1e-3):
    """tf.contrib batch_norm with is_training=False as y = x*scale + shift (moving stats never
    updated by the reference: mean 0, var 1)."""
    gamma = np.asarray(gamma, np.float64)
    beta = np.asarray(beta, np.float64)
    mm = np.zeros_like(gamma) if moving_mean is None else np.asarray(moving_mean, np.float64)
    mv = np.ones_like(gamma) if moving_var is None else np.asarray(moving_var, np.float64)
    s = gamma / np.sqrt(mv + eps)
    return s.astype(np.float32), (beta - mm * s).astype(np.float32)
