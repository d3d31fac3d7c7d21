"""Does the UNetImage step's speed depend on which pooled stream its side stream gets (study tool, GPU)?  The step
is timed, then one more torch stream is taken from the pool, repeatedly: a period of GPU_MAX_HW_QUEUES in the step
time says the side stream shares a hardware queue with the main stream for some pool positions.

    python tools/img_streams.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-matting_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    keep = []
    print("GPU_MAX_HW_QUEUES=%s" % os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
    for k in range(9):
        r = bench.train_image_bench(dev, 20, 5, 1, 0, 16, cpu=False)
        print("extra pool streams taken %d: train_image %.4f ms/step (backward %.4f)" % (
            k, r["ms_per_step"], r["device_ms"]["backward"]), flush=True)
        keep.append(torch.cuda.Stream(device=dev))


if __name__ == "__main__":
    main()
