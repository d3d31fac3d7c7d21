"""Run a few config-5 training steps (8 x 320x320 bf16 per GPU) for rocprofv3 kernel traces.

    python tools/train_step.py [steps] [dtype]
Prints the step time and the per-phase device times; under rocprofv3 --stats divide totals by steps + 3 warm-up.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    rec = bench.train_bench(torch.device("cuda:0"), steps, 3, 1, 0, 1, cpu=False, dtype=dtype)
    print(rec["ms_per_step"], rec["device_ms"], flush=True)
