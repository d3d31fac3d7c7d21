"""Does the UNetImage step's speed depend on which pooled stream its side stream gets (study tool, GPU)?  The step
is timed, then one more torch stream is taken from the pool, repeatedly: a period of GPU_MAX_HW_QUEUES in the step
time says the side stream shares a hardware queue with the main stream for some pool positions.

    python tools/img_streams.py [masked|pool|high]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-matting_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from vmatting.image_train import ImageTrainer
    if len(sys.argv) > 1:  # the trainers' side stream kind: masked (default) / pool / high
        ImageTrainer.side_kind = sys.argv[1]
    dev = torch.device("cuda", 0)
    keep = []
    print("GPU_MAX_HW_QUEUES=%s side_kind=%s" % (os.environ.get("GPU_MAX_HW_QUEUES"), ImageTrainer.side_kind),
          flush=True)
    for k in range(9):
        r = bench.train_image_bench(dev, 20, 5, 1, 0, 16, cpu=False)
        print("extra pool streams taken %d: train_image %.4f ms/step (backward %.4f)" % (
            k, r["ms_per_step"], r["device_ms"]["backward"]), flush=True)
        keep.append(torch.cuda.Stream(device=dev))


if __name__ == "__main__":
    main()
