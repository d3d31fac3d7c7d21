"""Run a few config-5 training steps (8 x 320x320 bf16 per GPU) for rocprofv3 kernel traces."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rec = bench.train_bench(torch.device("cuda:0"), steps, 2, 1, 0, cpu=False)
    print(rec["ms_per_step"], rec["device_ms"])
