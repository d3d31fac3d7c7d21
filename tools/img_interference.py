"""Why the UNetImage step (bench.py's train_image record) runs slower inside the full bench than alone (study tool,
GPU): its ms_per_step alone, then after each record that precedes it in bench.main, then alone again.

    python tools/img_interference.py
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "video-matting_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def img(tag, dev, threads, cpu=False):
    r = bench.train_image_bench(dev, 25, 5, 1, 0, threads, cpu=cpu)
    print("%-34s train_image %.4f ms/step (device %.4f)" % (tag, r["ms_per_step"], sum(r["device_ms"].values())),
          flush=True)


def main():
    dev = torch.device("cuda", 0)
    threads = 16
    torch.set_num_threads(threads)
    img("alone", dev, threads)
    img("alone again", dev, threads)
    bench.train_bench(dev, 25, 3, 1, 0, threads, cpu=False)
    img("after train", dev, threads)
    bench.train_chain_bench(dev, 5, 2)
    img("after train_chain", dev, threads)
    time.sleep(5)
    img("after train_chain + 5 s", dev, threads)
    bench.train_small_bench(dev, 25, 3, 1, 0, threads, cpu=False)
    img("after train_small", dev, threads)
    bench.train_bench(dev, 25, 3, 1, 0, threads, cpu=True)
    img("after train with its CPU baseline", dev, threads)
    img("alone, cpu leg on", dev, threads, cpu=True)
    img("after its own CPU leg", dev, threads)


if __name__ == "__main__":
    main()
