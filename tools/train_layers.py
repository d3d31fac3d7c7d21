"""Per-conv timing of one config-5 training step (VideoTrainer, 8 x 320^2 bf16, one stream) or small_train step.

    python tools/train_layers.py [--small] [--steps 5]

Prints every conv launch of a step in order: input shape, cin -> cout, the kernel that ran, HIP-event ms, TFLOP/s.
"""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmatting import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--option", action="append", default=[])
    args = ap.parse_args()
    from vmatting import _lib
    for kv in args.option:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    dev = torch.device("cuda")
    n, size = 8, 320
    rs = np.random.RandomState(0)
    mean = np.array([103.939, 116.779, 123.68])
    fg = rs.uniform(0, 255, (n, size, size, 3))
    bg = rs.uniform(0, 255, (n, size, size, 3))
    gt = rs.uniform(0, 1, (n, size, size, 1))
    cmp = gt * fg + (1 - gt) * bg - mean
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    cmp_d, bg_d, gt_d, fg_d, w_d = T(cmp), T(bg - mean), T(gt), T(fg), T(np.repeat(gt, 3, -1))
    np.random.seed(1)
    if args.small:
        from vmatting.small_train import SmallTrainer
        trn = SmallTrainer(6, "bf16", dev)
        step = lambda: trn.step(cmp_d, bg_d, gt_d, fg_d)  # noqa: E731
    else:
        from vmatting.train import VideoTrainer
        from vmatting.weights import synthetic_vgg16
        trn = VideoTrainer(synthetic_vgg16(0), "bf16", dev, streams=0)
        step = lambda: trn.step(cmp_d, bg_d, w_d, gt_d, fg_d)  # noqa: E731
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    prof = ops.conv_profile(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ops.conv_profile(False)
    per = len(prof) // args.steps
    tot = 0.0
    for i in range(per):
        rows = prof[i::per]
        t = sum(r[2].elapsed_time(r[3]) for r in rows) / len(rows)
        tot += t
        sh = rows[0][4] if len(rows[0]) > 4 else ()
        print("%3d %-28s %-62s %.4f ms %7.1f TFLOP/s" % (i, "x".join(str(v) for v in sh), rows[0][1][:62], t,
                                                          rows[0][0] / (t * 1e-3) / 1e12), flush=True)
    print("sum of conv launches %.3f ms per step" % tot)


if __name__ == "__main__":
    main()
