"""Contention stress for the UNetVideo bf16 forward: N processes share cuda:0, each replaying chunked HIP graphs
(video.matte_video, chunks of 2) and the eager forward() of the same 4 frames for SECONDS, counting frames whose
mattes differ.  Used to find the r03 ring-slot LDS race: races that only show when another process
shares the CUs.

    python tools/contention_stress.py [NPROC=2] [SECONDS=60]
    VM_HW=1080x1920 (frame size), VM_OPTS="patch_cfg=25,up_skip=0" (vm_set_option knobs),
    VM_FLAGS="fuse_up_head=0" (UNetVideo attributes)

Prints per rank (rank, iterations, mismatching frames, the first few as (iteration, frame, max |diff|, pixels,
first pixel, last pixel)) and a SUMMARY line."""
import os, sys, time
import numpy as np
import torch
import multiprocessing as mp
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-matting_amd"))


def worker(rank, q, seconds, h, w):
    from vmatting import unet, video, _lib
    from vmatting.weights import synthetic_vgg16
    torch.cuda.set_device(0)
    for kv in filter(None, os.environ.get("VM_OPTS", "").split(",")):
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    np.random.seed(100)
    model = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device="cuda:0")
    for kv in filter(None, os.environ.get("VM_FLAGS", "").split(",")):
        k, v = kv.split("=")
        setattr(model, k, bool(int(v)))
    model.prepare()
    n = 4
    frames = video.synthetic_frames(n, h, w, first=rank * n, device="cuda:0")
    t0 = time.time()
    it, bad = 0, []
    while time.time() - t0 < seconds:
        full, vm = video.matte_video(model, frames, n, chunk=2)
        torch.cuda.synchronize()
        got = full.clone()
        for i in range(n):
            ref = model.forward(frames[i:i + 1].clone())[0]
            if not torch.equal(ref, got[i]):
                d = (ref.float() - got[i].float()).abs()
                nz = (d > 0).nonzero()
                bad.append((it, i, float(d.max()), int((d > 0).sum()), tuple(int(v) for v in nz[0]),
                            tuple(int(v) for v in nz[-1])))
        it += 1
    q.put((rank, it, bad[:20], len(bad)))


if __name__ == "__main__":
    nproc = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 60
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    hh, ww = (int(v) for v in os.environ.get("VM_HW", "270x480").split("x"))
    ps = [ctx.Process(target=worker, args=(r, q, secs, hh, ww)) for r in range(nproc)]
    for p in ps:
        p.start()
    tot = []
    for _ in ps:
        r = q.get(timeout=secs + 200)
        tot.append((r[0], r[1], r[3]))
        print(r[0], r[1], r[3], r[2][:3], flush=True)
    print("SUMMARY", os.environ.get("VM_OPTS", ""), os.environ.get("VM_FLAGS", ""), tot, flush=True)
    for p in ps:
        p.join(30)
