"""Host-side profile (cProfile, tottime) of the config-5 chained bench (bench.train_chain_bench): where the host's
per-step issue time goes (numpy draws / TPS solves, ctypes launches, torch allocator calls).

    python tools/chain_host_profile.py [--serial] [--steps 10]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    pr = cProfile.Profile()  # enabled over the timed steps only
    rec = bench.train_chain_bench(dev, args.steps, 3, overlap=not args.serial, profiler=pr)
    print("ms_per_step", rec["ms_per_step"])
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    print(s.getvalue()[:9000])


if __name__ == "__main__":
    main()
