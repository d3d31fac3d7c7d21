"""Config-5 training step timed with the trainer's main stream at high priority (1) or default (0):
    python tools/train_prio.py 0|1 [steps]
(the side streams keep the default priority; hipDeviceGetStreamPriorityRange is printed)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    hi = bool(int(sys.argv[1]))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    print("priority range", torch.cuda.Stream.priority_range(), flush=True)
    s = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1]) if hi else torch.cuda.current_stream()
    with torch.cuda.stream(s):
        rec = bench.train_bench(torch.device("cuda:0"), steps, 5, 1, 0, 1, cpu=False, dtype="bf16")
    print("main_hi=%d ms_per_step %.3f" % (hi, rec["ms_per_step"]), rec["device_ms"], flush=True)
