"""Is the config-5 training step host-bound?  Times the host's issue of K eager steps while the GPU is held busy by a
spin kernel queued ahead of them (the host never waits on the device), against the wall time of K steps.

    python tools/train_host.py [--steps 10] [--streams 3]
"""
import argparse
import os
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--streams", type=int, default=3)
    args = ap.parse_args()
    from vmatting.train import VideoTrainer
    from vmatting.weights import synthetic_vgg16
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n, size = 8, 320
    rs = np.random.RandomState(100)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    cmp, bg, fg = (T(rs.uniform(-120, 120, (n, size, size, 3))) for _ in range(3))
    gt = T(rs.uniform(0, 1, (n, size, size, 1)))
    warped = gt.expand(n, size, size, 3).contiguous()
    np.random.seed(1)
    trn = VideoTrainer(synthetic_vgg16(0), "bf16", dev, streams=args.streams)
    for _ in range(3):
        trn.step(cmp, bg, warped, gt, fg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trn.step(cmp, bg, warped, gt, fg)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps * 1e3
    # host issue alone: a spin kernel holds the GPU long enough that no launch below waits for the device
    torch.cuda._sleep(int(2.0e9))  # ~1 s at ~2 GHz
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trn.step(cmp, bg, warped, gt, fg)
    issue = (time.perf_counter() - t0) / args.steps * 1e3
    torch.cuda.synchronize()
    # forward only / backward only issue
    torch.cuda._sleep(int(2.0e9))
    t0 = time.perf_counter()
    trn.forward(cmp, bg, warped)
    f_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    trn.backward(gt, fg, bg, cmp)
    b_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    trn.apply_gradients()
    a_ms = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    print(f"wall {wall:.3f} ms/step, host issue {issue:.3f} ms/step (forward {f_ms:.3f}, backward {b_ms:.3f}, "
          f"update {a_ms:.3f})")


if __name__ == "__main__":
    main()
