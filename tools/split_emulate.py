"""Float64 emulation of unet.py's forward (unet.py:161-205) under split-operand conv schemes (study tool, CPU).

Each conv's operands are cut into parts the way a split MFMA forward would carry them, the kept cross products are
summed exactly (float64 conv), and the conv output is rounded to f32 (the kernels' f32 epilogue).  Bias, relu, pool
and resize run in float64.  The result is compared with the exact float64 forward on the same frame and weights:
the representation error of a scheme, before the f32 accumulation order every f32 path shares.

  bf16x3   x = h + l (bf16), W likewise;   y = l*Wh + h*Wl + h*Wh
  bf16x6   x = h + m + l (bf16);           y = l*Wh + m*Wm + h*Wl + m*Wh + h*Wm + h*Wh
  f16x3    x*2^s = h + l (fp16), W*2^t = Wh + Wl (fp16), y = (l*Wh + h*Wl + h*Wh) * 2^-(s+t): power-of-two scales put
           max|x*2^s| at 2^AMAX and max|W*2^t| at 2^WMAX, so no part leaves fp16's normal range where it matters
  f16x3w   the filter scale only (activations unscaled: max |x| stays far below fp16's 65504 on this net)
  f16x3u   the same without scales
  bf16     y = bf16(x) * bf16(W)
  f16x2a   x3 without l*Wh (the activation rounded to fp16), f16x2w without h*Wl (the filter rounded), f16 h*Wh only

    python tools/split_emulate.py --size 1080x1920 --scheme f16x3 bf16x3
    python tools/split_emulate.py --size 540x960 --scheme f16x3 --only conv1_2     # one layer split, the rest exact
    python tools/split_emulate.py --scheme f16x2a --per-layer --rest f16x3         # per-layer sensitivity on x3
"""

import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "video-matting_amd"))

from oracle import models as om  # noqa: E402
from oracle import ops as oo  # noqa: E402

AMAX, WMAX = 12, 12


def _bf(t):
    return t.float().bfloat16().double()


def _hf(t):
    return t.float().half().double()


def _p2(m, top):
    """power-of-two scale putting max |.| = m just under 2^top"""
    if m == 0:
        return 1.0
    return 2.0 ** (top - int(np.ceil(np.log2(m))))


def parts(x, w, scheme):
    """-> list of (activation part, filter part) pairs and the output scale"""
    if scheme == "exact":
        return [(x, w)], 1.0
    if scheme == "bf16":
        return [(_bf(x), _bf(w))], 1.0
    if scheme == "bf16x3":
        xh, wh = _bf(x), _bf(w)
        xl, wl = _bf(x - xh), _bf(w - wh)
        return [(xl, wh), (xh, wl), (xh, wh)], 1.0
    if scheme == "bf16x6":
        xh, wh = _bf(x), _bf(w)
        xm, wm = _bf(x - xh), _bf(w - wh)
        xl, wl = _bf(x - xh - xm), _bf(w - wh - wm)
        return [(xl, wh), (xm, wm), (xh, wl), (xm, wh), (xh, wm), (xh, wh)], 1.0
    if scheme in ("f16x3", "f16x3u", "f16x3w"):
        s = _p2(x.abs().max().item(), AMAX) if scheme == "f16x3" else 1.0
        t = _p2(w.abs().max().item(), WMAX) if scheme != "f16x3u" else 1.0
        xs, ws = x * s, w * t
        xh, wh = _hf(xs), _hf(ws)
        xl, wl = _hf(xs - xh), _hf(ws - wh)
        assert torch.isfinite(xh).all() and torch.isfinite(wh).all()
        return [(xl, wh), (xh, wl), (xh, wh)], 1.0 / (s * t)
    if scheme in ("f16x2a", "f16x2w", "f16"):  # x3 minus a cross term: the activation (a) or filter (w) fp16-rounded
        t = _p2(w.abs().max().item(), WMAX)
        ws = w * t
        xh, wh = _hf(x), _hf(ws)
        xl, wl = _hf(x - xh), _hf(ws - wh)
        pr = {"f16x2a": [(xh, wl), (xh, wh)], "f16x2w": [(xl, wh), (xh, wh)], "f16": [(xh, wh)]}[scheme]
        return pr, 1.0 / t
    raise ValueError(scheme)


class Emu:
    def __init__(self, params, scheme, only=None, rest="exact"):
        self.p = params
        self.scheme, self.only, self.rest = scheme, only, rest
        self.amax = {}

    def conv(self, x, name, exact=False):
        """x NCHW f64 -> conv3x3 SAME (+ bias), output rounded to f32 unless exact"""
        w, b = self.p[name]
        wt = torch.from_numpy(np.asarray(w, np.float64)).permute(3, 2, 0, 1).contiguous()
        self.amax[name] = max(self.amax.get(name, 0.0), x.abs().max().item())
        sch = "exact" if exact else self.rest if (self.only is not None and name not in self.only) else self.scheme
        pr, sc = parts(x, wt, sch)
        y = None
        for xa, wa in pr:
            c = F.conv2d(xa, wa, padding=1)
            y = c if y is None else y + c
        y = y * sc
        if not exact:
            y = y.float().double()
        if b is not None:
            y = y + torch.from_numpy(np.asarray(b, np.float64))[None, :, None, None]
            if not exact:
                y = y.float().double()
        return y

    def forward(self, x, exact=False):
        relu = torch.relu
        pool = lambda t: F.max_pool2d(t, 2, 2, ceil_mode=True)  # noqa: E731  (SAME, pad after, for ceil sizes)
        cv = lambda t, n: self.conv(t, n, exact)  # noqa: E731
        r = {}
        c12 = relu(cv(relu(cv(x, "conv1_1")), "conv1_2"))
        c22 = relu(cv(relu(cv(pool(c12), "conv2_1")), "conv2_2"))
        c33 = relu(cv(relu(cv(relu(cv(pool(c22), "conv3_1")), "conv3_2")), "conv3_3"))
        c43 = relu(cv(relu(cv(relu(cv(pool(c33), "conv4_1")), "conv4_2")), "conv4_3"))
        c52 = relu(cv(relu(cv(pool(c43), "conv5_1")), "conv5_2"))

        def up(a, skip, name):
            h, w = skip.shape[2:]
            a_n = a.permute(0, 2, 3, 1).numpy()
            rs = torch.from_numpy(oo.resize_bilinear_tf1(a_n, h, w)).permute(0, 3, 1, 2).contiguous()
            return torch.cat([cv(rs, name), skip], 1)

        c44 = relu(cv(up(c52, c43, "upconv_1"), "conv4_4"))
        c34 = relu(cv(up(c44, c33, "upconv_2"), "conv3_4"))
        c23 = relu(cv(up(c34, c22, "upconv_3"), "conv2_3"))
        lg = cv(up(c23, c12, "upconv_4"), "conv1_5")
        r["logits"] = lg
        r["alpha"] = torch.sigmoid(lg)
        return r


def frame(h, w, seed=0):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "video-matting_amd"))
    from vmatting import video
    return video.synthetic_frames(1, h, w, first=seed, device="cpu")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1080x1920")
    ap.add_argument("--scheme", nargs="+", default=["f16x3", "bf16x3"])
    ap.add_argument("--only", nargs="*", default=None, help="split only these convs (the rest exact)")
    ap.add_argument("--per-layer", action="store_true", help="one run per conv, that conv split, the rest exact")
    ap.add_argument("--golden", default=None, help="a tests/golden case: its frame and weights (size ignored)")
    ap.add_argument("--rest", default="exact", help="the scheme of the convs --only / --per-layer leave out")
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    h, w = map(int, args.size.split("x"))
    g = None
    if args.golden:
        g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", args.golden + ".npz"))
        params = om.unet_params(om.synthetic_vgg16(0), np.random.RandomState(int(g["weight_seed"])),
                                video=bool(g["video"]))
        x = torch.from_numpy(np.asarray(g["x"], np.float64)).permute(0, 3, 1, 2).contiguous()
    else:
        np.random.seed(0)
        params = om.unet_params(om.synthetic_vgg16(0), np.random.mtrand._rand, video=True)
        x = frame(h, w).permute(0, 3, 1, 2).double().contiguous()
    t0 = time.time()
    ex = Emu(params, "exact").forward(x, exact=True)
    print("exact forward %.1f s; max |logit| %.4g" % (time.time() - t0, ex["logits"].abs().max().item()), flush=True)
    if g is not None:
        ga = torch.from_numpy(np.asarray(g["output"], np.float64)).permute(0, 3, 1, 2)
        print("golden alpha vs exact: max-abs %.3e" % (ga - ex["alpha"]).abs().max().item(), flush=True)
    names = [n for n, _, _ in om.VGG_LAYERS[:12]] + [n for n, _, _, _ in om.UNET_NEW_CONVS]
    for sch in args.scheme:
        runs = [[n] for n in names] if args.per_layer else [args.only]
        for only in runs:
            t0 = time.time()
            e = Emu(params, sch, only, args.rest)
            r = e.forward(x)
            da = (r["alpha"] - ex["alpha"]).abs().max().item()
            dl = (r["logits"] - ex["logits"]).abs().max().item() / ex["logits"].abs().max().item()
            print("%-8s %-12s alpha max-abs %.3e  logits rel %.3e  (%.0f s)" % (
                sch, "all" if only is None else ",".join(only), da, dl, time.time() - t0), flush=True)
            if only is None:
                print("  max |input| per conv: " + " ".join("%s %.3g" % (k, v) for k, v in e.amax.items()))


if __name__ == "__main__":
    main()
