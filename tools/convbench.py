"""Single-layer conv microbenchmark (for kernel tuning and rocprofv3 --pmc runs).

    python tools/convbench.py --shape 135x240x512x512 --kernel 2 --iters 50
    python tools/convbench.py --unet-layers            # every UNetVideo 1080p conv shape

Prints one line per shape: ms per launch (HIP events) and TFLOP/s.
"""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmatting import _lib, ops  # noqa: E402

# (name, h, w, cin, cout) of UNetVideo at 1920x1080
UNET_1080 = [("conv1_1", 1080, 1920, 7, 64), ("conv1_2", 1080, 1920, 64, 64), ("conv2_1", 540, 960, 64, 128),
             ("conv2_2", 540, 960, 128, 128), ("conv3_1", 270, 480, 128, 256), ("conv3_2", 270, 480, 256, 256),
             ("conv4_1", 135, 240, 256, 512), ("conv4_2", 135, 240, 512, 512), ("conv5_1", 68, 120, 512, 512),
             ("upconv_1", 135, 240, 512, 512), ("conv4_4", 135, 240, 1024, 512), ("upconv_2", 270, 480, 512, 256),
             ("conv3_4", 270, 480, 512, 256), ("upconv_3", 540, 960, 256, 128), ("conv2_3", 540, 960, 256, 128),
             ("upconv_4", 1080, 1920, 128, 64)]


SPLITK = False


def run(name, h, w, cin, cout, dtype, iters, n=1):
    tdt = ops.TORCH_DTYPE[dtype]
    cpad = (cin + 7) // 8 * 8
    x = (torch.randn(n, h, w, cpad, device="cuda") * 0.5).to(tdt)[..., :cin]
    wt = (np.random.RandomState(0).normal(size=(3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    pc = ops.PackedConv(wt, np.zeros(cout, np.float32), tdt)
    y = torch.empty(n, h, w, cout, dtype=tdt, device="cuda")
    for _ in range(3):
        ops.conv3x3(x, pc, "relu", out=y, splitk=SPLITK)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.conv3x3(x, pc, "relu", out=y, splitk=SPLITK)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 2.0 * n * h * w * 9 * cin * cout
    print("%-10s %4dx%-4d %4d->%-4d  %.4f ms  %7.1f TFLOP/s  %s" % (name, h, w, cin, cout, ms, fl / ms / 1e9,
                                                                  _lib.last_conv_kernel()), flush=True)
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", default=[], help="HxWxCINxCOUT")
    ap.add_argument("--unet-layers", action="store_true")
    ap.add_argument("--kernel", type=int, default=0, help="conv_kernel option: 0 auto, 1 regstage, 2 LDS-DMA, 3 patch")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--glds-rb", type=int, default=128)
    ap.add_argument("--patch-cfg", type=int, default=0)
    ap.add_argument("--ablate", type=int, default=0, help="patch kernel timing ablation (1 no MFMA, 2 no DMA, 4 no sync)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--option", action="append", default=[], help="extra vm_set_option key=value")
    ap.add_argument("--ab", default="", help="key=v1,v2,...: time every value per shape, interleaved in rounds")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--splitk", action="store_true", help="allow split-K (a workspace; the training path's setting)")
    args = ap.parse_args()
    global SPLITK
    SPLITK = args.splitk
    for kv in args.option:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    _lib.set_option("conv_kernel", args.kernel)
    _lib.set_option("glds_rb", args.glds_rb)
    if args.patch_cfg:
        _lib.set_option("patch_cfg", args.patch_cfg)  # sweep tilings other than 19/22/25/30: the study build
    if args.ablate:  # timing-only ablations exist in the study build only:
        _lib.set_option("patch_ablate", args.ablate)  # VM_LIB_PATH=video-matting_amd/study/libvmatting_study.so
    shapes = [("shape",) + tuple(int(v) for v in s.split("x")) for s in args.shape]
    if args.unet_layers:
        shapes += UNET_1080
    if args.ab:  # same-process interleaved A/B (one variant after the other, several rounds; median per variant)
        key, vals = args.ab.split("=")
        vals = [int(v) for v in vals.split(",")]
        tot = {v: 0.0 for v in vals}
        for s in shapes:
            t = {v: [] for v in vals}
            for _ in range(args.rounds):
                for v in vals:
                    _lib.set_option(key, v)
                    t[v].append(run(*s, dtype=args.dtype, iters=args.iters))
            for v in vals:
                tot[v] += float(np.median(t[v]))
            print("AB %-10s " % s[0] + "  ".join("%s=%d: %.4f ms" % (key, v, np.median(t[v])) for v in vals), flush=True)
        print("AB total " + "  ".join("%s=%d: %.3f ms" % (key, v, tot[v]) for v in vals))
        return
    tot = 0.0
    for s in shapes:
        tot += run(*s, dtype=args.dtype, iters=args.iters)
    print("total %.3f ms" % tot)


if __name__ == "__main__":
    main()
