"""Benchmark: alpha-mattes/sec of unet.UNetVideo at 1920x1080 (BASELINE.json configs[1]; configs[3] at N>1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16|fp32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one UNetVideo forward over B synthetic 1080p 7-channel frames per GPU (inputs resident
in HBM before timing).  Frame-parallel: every rank runs its own frames, no collective in the data
path (scaling "weak"); the packed weights are RCCL-broadcast from rank 0 once, before timing.
Rank 0 prints ONE JSON line (value = frames processed by all ranks / max-over-ranks time).
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vmatting import ops, parallel, unet  # noqa: E402
from vmatting.weights import synthetic_vgg16  # noqa: E402

METRIC = "alpha-mattes/sec at 1920×1080, 1/2/4/8 MI355X + achieved HBM GB/s"
PEAK_TFLOPS = {"bf16": 2516.6, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBPS = 8000.0
VGG_MEAN = (103.939, 116.779, 123.68)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_frames(n, h, w, first, device):
    """frame f (seed 1234+f): cmp/bg BGR U{0..255} - VGG_MEAN; trimap {0,.5,1} - .5
    from a random ellipse with an unknown band.  Generated on the device."""
    out = torch.empty((n, h, w, 7), dtype=torch.float32, device=device)
    mean = torch.tensor(VGG_MEAN, device=device)
    yy = torch.arange(h, device=device, dtype=torch.float32)[:, None]
    xx = torch.arange(w, device=device, dtype=torch.float32)[None, :]
    for i in range(n):
        g = torch.Generator(device=device)
        g.manual_seed(1234 + first + i)
        out[i, :, :, 0:3] = torch.randint(0, 256, (h, w, 3), generator=g, device=device).float() - mean
        out[i, :, :, 3:6] = torch.randint(0, 256, (h, w, 3), generator=g, device=device).float() - mean
        c = torch.rand(4, generator=g, device=device)
        cy, cx = (0.3 + 0.4 * c[0]) * h, (0.3 + 0.4 * c[1]) * w
        ry, rx = (0.15 + 0.15 * c[2]) * h, (0.15 + 0.15 * c[3]) * w
        d = torch.sqrt(((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2)
        band = 8.0 / float(min(ry, rx))
        tri = torch.where(d < 1 - band, 1.0, torch.where(d < 1 + band, 0.5, 0.0))
        out[i, :, :, 6] = tri - 0.5
    return out


def video_batch(graphed, n_frames, h, w, rank, world, dev):
    """BASELINE config 4: ``n_frames`` synthetic 1080p frames (seeds 1234..) sharded frame-parallel in contiguous
    blocks, each rank runs its block through the captured forward, then ONE all-gather (RCCL ring over xGMI) hands
    every rank the whole [n_frames, H, W, 1] fp32 matte batch.  Timed between barriers, max over ranks."""
    a, b = parallel.shard_range(n_frames, rank, world)
    frames = synth_frames(b - a, h, w, a, dev)
    out_shape = tuple(graphed.output.shape[1:])
    local = torch.empty((b - a,) + out_shape, dtype=graphed.output.dtype, device=dev)
    mx = max(q - p for p, q in (parallel.shard_range(n_frames, r, world) for r in range(world)))
    recv = torch.empty((world * mx,) + out_shape, dtype=local.dtype, device=dev) if world > 1 else None
    graphed(frames[:1])  # warm
    if world > 1:
        parallel.gather_frames(local, n_frames, out=recv)  # warm the communicator
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(b - a):
        local[i].copy_(graphed(frames[i:i + 1])[0])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    full = parallel.gather_frames(local, n_frames, out=recv)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    ts = torch.tensor([t2 - t0, t1 - t0, t2 - t1], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
    total, comp, gath = (float(v) for v in ts.tolist())
    assert full.shape[0] == n_frames
    return {"workload": "config 4: %d synthetic %dx%d frames sharded frame-parallel, mattes all-gathered to every rank"
                        % (n_frames, w, h),
            "frames": n_frames, "frames_per_s": round(n_frames / total, 3), "ms_total": round(1e3 * total, 3),
            "ms_compute_max_rank": round(1e3 * comp, 3), "ms_all_gather": round(1e3 * gath, 3),
            "all_gather_bytes": int(full.numel() * full.element_size()),
            "includes": "per-frame input copy into the graph's static buffer + graph replay + matte copy-out"}


def cpu_baseline(h, w, sample_h, sample_w):
    """The oracle (numpy f32 restatement of unet.py) timed on host cores on a bounded sample."""
    from oracle import models as om
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    vgg = synthetic_vgg16(0)
    p = om.unet_params(vgg, np.random.RandomState(0), video=True)
    rs = np.random.RandomState(1234)
    x = np.concatenate([rs.randint(0, 256, (1, sample_h, sample_w, 6)).astype(np.float32) - np.tile(VGG_MEAN, 2),
                        rs.choice([-0.5, 0.0, 0.5], (1, sample_h, sample_w, 1))], -1).astype(np.float32)
    t0 = time.perf_counter()
    om.unet_forward(x, p, dtype=np.float32)
    dt = time.perf_counter() - t0
    scale = (h * w) / float(sample_h * sample_w)  # conv work is linear in pixels
    return {"value": round(1.0 / (dt * scale), 5), "unit": "frames/s", "cores": int(threads), "kind": "port",
            "sample": "oracle/ numpy-f32 UNetVideo forward on one %dx%d 7-ch frame (%.1f s), scaled x%.0f to "
                      "1920x1080 by pixel count" % (sample_w, sample_h, dt, scale)}


def loader_inputs(n, h, w, seed=0):
    """Decoded video-loader entries (fg/prev BGRA, bg BGR u8, piecewise-constant f32 flow) at h x w."""
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        lo = rs.uniform(-12, 12, ((h + 63) // 64, (w + 63) // 64, 2)).astype(np.float32)
        flow = np.repeat(np.repeat(lo, 64, 0), 64, 1)[:h, :w]  # |u|, |v| <= 12 px
        out.append({"fg": rs.randint(0, 256, (h, w, 4), dtype=np.uint8),
                    "bg": rs.randint(0, 256, (h, w, 3), dtype=np.uint8),
                    "prev": rs.randint(0, 256, (h, w, 4), dtype=np.uint8), "flow": np.ascontiguousarray(flow)})
    return out


def loader_bench(dev, steps, cpu=True, n=8, size=320, h=1080, w=1920):
    """video_batch's per-pixel work (csrc/loader.hip) on a batch of n 1080p video entries resized
    to size x size; inputs resident in HBM, the host's np.random draws replayed once outside the timed region."""
    from vmatting import loader as vl
    host = loader_inputs(n, h, w)
    np.random.seed(0)
    for s in host:
        s["plan"] = vl.plan_crop((h, w), (h, w))
    samples = [dict(s, **{k: torch.from_numpy(s[k]).to(dev) for k in ("fg", "bg", "prev", "flow")}) for s in host]
    names = ("cmp", "bg", "label", "warped", "fg")
    for _ in range(3):
        vl.compose_batch(samples, (size, size), names, device=dev)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(steps):
        vl.compose_batch(samples, (size, size), names, device=dev)
    ev[1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    dev_ms = ev[0].elapsed_time(ev[1]) / steps
    # algorithmic bytes per batch: the f32 outputs (13 channels) + each source byte the resize can touch, once
    # (min(window area, 4 taps per output pixel) per plane: fg BGRA 4 B, flow 8 B, prev BGRA 4 B, bg 3 B)
    taps = 4 * size * size
    src = 0
    for s in host:
        fr, fc, br, bc = s["plan"]
        src += min(fr[0] * fc[0], taps) * (4 + 8 + 4) + min(br[0] * bc[0], taps) * 3
    algo = n * size * size * 13 * 4 + src
    rec = {"workload": "loader.video_batch per-pixel work: %d entries %dx%d -> %dx%d, f32 out" % (n, w, h, size, size),
           "samples_per_s": round(n / wall, 1), "ms_per_batch": round(1000 * wall, 4),
           "device_ms_per_batch": round(dev_ms, 4), "algorithmic_bytes_per_batch": int(algo),
           "achieved_gbps": round(algo / (dev_ms * 1e-3) / 1e9, 1), "peak_gbps": PEAK_HBM_GBPS,
           "crops": [int(s["plan"][0][0]) for s in host]}
    if cpu:
        from oracle import loader as ol  # the CPU-baseline leg only
        k = 2
        t0 = time.perf_counter()
        for s in host[:k]:
            fr, fc, br, bc = (ol.Axis(*a) for a in s["plan"])
            srcs = ol.crop_sources(s["fg"], s["bg"], fr, fc, br, bc, s["prev"], s["flow"])
            ol.compose(srcs[0], srcs[1], srcs[3], (size, size), srcs[2])
        dt = (time.perf_counter() - t0) / k
        rec["cpu_baseline"] = {"value": round(1.0 / dt, 3), "unit": "samples/s", "cores": 1, "kind": "port",
                               "sample": "oracle/loader.py (numpy float64, with the reference's full-frame warp) on "
                                         "%d of the %d entries (%.2f s each)" % (k, n, dt)}
    return rec


def augment_bench(dev, steps, cpu=True, h=1080, w=1920):
    """augmentation.augment on one 1080p (fg, bg, alpha) sample resident in HBM: host draws +
    TPS solve + one stats sync + the csrc/augment.hip kernels.  Device time from HIP events on the launch stream."""
    from vmatting import augmentation as va
    rs = np.random.RandomState(9)
    yy, xx = np.mgrid[0:h, 0:w]
    alpha_h = np.clip(1.2 - np.sqrt(((yy - 0.46 * h) / (0.28 * h)) ** 2 + ((xx - 0.47 * w) / (0.21 * w)) ** 2), 0, 1)
    fg_h = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    bg_h = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    fg, bg, alpha = (torch.from_numpy(a).to(dev) for a in (fg_h, bg_h, alpha_h))
    np.random.seed(0)
    for _ in range(3):
        va.augment(fg, bg, alpha)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record()
    for _ in range(steps):
        va.augment(fg, bg, alpha)
    ev[1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    dev_ms = ev[0].elapsed_time(ev[1]) / steps
    # algorithmic bytes per sample (per pixel): alpha stats 8; bg 2 warps 2*(3+3); TPS grid (h/2)(w/2)*16 = 4;
    # fg TPS 3+3, alpha TPS 8+8; fg 2 warps 2*(3+3); alpha 2 warps 2*(8+8); illumination fg+bg 2*(3+3)
    algo = h * w * (8 + 12 + 4 + 6 + 16 + 12 + 32 + 12)
    rec = {"workload": "augmentation.augment: one %dx%d sample (u8 fg/bg, f64 alpha), inputs in HBM" % (w, h),
           "samples_per_s": round(1.0 / wall, 1), "ms_per_sample": round(1000 * wall, 4),
           "device_ms_per_sample": round(dev_ms, 4), "algorithmic_bytes_per_sample": int(algo),
           "achieved_gbps": round(algo / (dev_ms * 1e-3) / 1e9, 1), "peak_gbps": PEAK_HBM_GBPS}
    if cpu:
        from oracle import augment as oa  # the CPU-baseline leg only
        sh, sw = h // 2, w // 2
        np.random.seed(0)
        t0 = time.perf_counter()
        oa.augment(fg_h[:sh, :sw].copy(), bg_h[:sh, :sw].copy(), alpha_h[::2, ::2].copy())
        dt = (time.perf_counter() - t0) * (h * w) / float(sh * sw)
        rec["cpu_baseline"] = {"value": round(1.0 / dt, 3), "unit": "samples/s", "cores": 1, "kind": "port",
                               "sample": "oracle/augment.py (numpy, scipy-order TPS + OpenCV restatement) on one "
                                         "%dx%d sample, scaled x%d to %dx%d by pixel count" % (sw, sh, (h * w) // (sh * sw),
                                                                                         w, h)}
    return rec


def train_flops(n, h, w):
    """Algorithmic FLOPs of one config-5 step: 3 frozen VGG16 towers + UNetSimple forward (unet_simple.py:45-171),
    the filter gradient of every trainable conv and the data gradient of the convs whose input is trainable."""
    from vmatting.train import DGRAD, LEVELS
    from vmatting.unet_simple import NEW_CONVS, _levels
    L = _levels(h, w)
    vgg = [(0, 3, 64), (0, 64, 64), (1, 64, 128), (1, 128, 128), (2, 128, 256), (2, 256, 256), (2, 256, 256),
           (3, 256, 512), (3, 512, 512), (3, 512, 512), (4, 512, 512), (4, 512, 512), (4, 512, 512)]
    f = lambda lv, ci, co: 2.0 * n * L[lv][0] * L[lv][1] * 9 * ci * co  # noqa: E731
    fwd = 3 * sum(f(*v) for v in vgg)
    lvl = {"output": 0}
    for lv, _, _, sels, up, _, conv, _ in LEVELS:
        for s, _ in sels:
            lvl[s] = lv
        lvl[up] = lvl[conv] = lv
    head = sum(f(lvl[s], ci, co) for s, ci, co in NEW_CONVS)
    dgrad = sum(f(lvl[s], ci, co) for s, ci, co in NEW_CONVS if s in DGRAD)
    return fwd + head, head + dgrad


def train_bench(dev, steps, warmup, world, rank, cpu=True, n=8, size=320, dtype="bf16"):
    """BASELINE config 5: one train.py video_procedure iteration per step (train.py:288-343) — batch of 8 320x320
    samples per GPU (params.py:8-9) resident in HBM: 3 VGG16 towers + UNetSimple (batch-statistics BN) forward,
    loss, backward through the trainable layers, one RCCL all-reduce of the gradients (DDP), TF-Adam, re-pack.
    Device time per phase from HIP events on the launch stream; step time = max over ranks."""
    from vmatting.train import VideoTrainer
    from vmatting.weights import synthetic_vgg16
    rs = np.random.RandomState(100 + rank)
    mean = np.array([103.939, 116.779, 123.68])
    fg = rs.uniform(0, 255, (n, size, size, 3))
    bg = rs.uniform(0, 255, (n, size, size, 3))
    yy, xx = np.mgrid[:size, :size]
    gt = np.clip(1.2 - np.hypot((yy - size / 2) / (size / 3), (xx - size / 2) / (size / 4)), 0, 1)
    gt = np.repeat(gt[None, :, :, None], n, 0)
    cmp = gt * fg + (1 - gt) * bg - mean
    warped = np.repeat(gt, 3, -1)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    cmp_d, bg_d, warped_d, gt_d, fg_d = T(cmp), T(bg - mean), T(warped), T(gt), T(fg)
    np.random.seed(1)
    trn = VideoTrainer(synthetic_vgg16(0), dtype, dev)
    for _ in range(warmup):
        trn.step(cmp_d, bg_d, warped_d, gt_d, fg_d)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    fwd_ms = bwd_ms = upd_ms = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        ev[0].record()
        trn.forward(cmp_d, bg_d, warped_d)
        from vmatting import ops
        trn._tb["loss"].copy_(ops.matting_loss(trn._tb["alpha"], gt_d, fg_d, bg_d, cmp_d))
        ev[1].record()
        trn.grad.zero_()
        trn.backward(gt_d, fg_d, bg_d, cmp_d)
        ev[2].record()
        trn.apply_gradients()
        ev[3].record()
        torch.cuda.synchronize()
        fwd_ms += ev[0].elapsed_time(ev[1])
        bwd_ms += ev[1].elapsed_time(ev[2])
        upd_ms += ev[2].elapsed_time(ev[3])
    wall = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall)
    fwd_f, bwd_f = train_flops(n, size, size)
    rec = {"workload": "train.py video_procedure step (config 5): %d x %dx%d per GPU, 3 VGG16 towers + UNetSimple "
                       "fwd/bwd, loss, DDP all-reduce, TF-Adam" % (n, size, size),
           "dtype": dtype + " forward, f32 gradients/optimizer", "n_gpus": world,
           "samples_per_s": round(n * world / wall, 1), "ms_per_step": round(1000 * wall, 3),
           "device_ms": {"forward_loss": round(fwd_ms / steps, 3), "backward": round(bwd_ms / steps, 3),
                         "allreduce_adam_repack": round(upd_ms / steps, 3)},
           "flops_per_step_per_gpu": {"forward": fwd_f, "backward": bwd_f},
           "achieved_tflops_per_gpu": round((fwd_f + bwd_f) / wall / 1e12, 1),
           "loss_last": [round(float(v), 5) for v in trn._tb["loss"].cpu()]}
    if cpu and world == 1:
        from oracle import models as om  # the CPU-baseline leg only
        from oracle import train_ref as tr
        sh = 128
        p = om.unet_simple_params(np.random.RandomState(1))
        sl = lambda a: np.asarray(a[:1, :sh, :sh], np.float64)  # noqa: E731
        t0 = time.perf_counter()
        tr.train_step_grads(sl(cmp), sl(bg - mean), sl(warped), sl(gt), sl(fg), synthetic_vgg16(0), p)
        dt = (time.perf_counter() - t0) * (size * size) / float(sh * sh)
        rec["cpu_baseline"] = {"value": round(1.0 / dt, 4), "unit": "samples/s", "cores": torch.get_num_threads(),
                               "kind": "port",
                               "sample": "oracle/train_ref.py (numpy-f64 VGG towers + torch-f64 autograd head) on one "
                                         "%dx%d sample, scaled x%.2f to %dx%d by pixel count" %
                                         (sh, sh, (size * size) / float(sh * sh), size, size)}
    return rec


def load_traffic(args, full=False):
    """Per-launch HBM bytes per kernel from the committed PMC pass (tools/traffic.py -> profiles/*_traffic.json),
    used only when it was collected on this exact workload."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json")), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        c = t.get("config", {})
        if (c.get("dtype"), c.get("height"), c.get("width"), c.get("batch")) == (args.dtype, args.height, args.width,
                                                                               args.batch):
            return (path, t) if full else (path, t.get("kernels", {}))
    return None, ({} if not full else None)


def conv_roofline(prof, args):
    """Roofline of the dominant conv kernel (largest share of conv time): ALGORITHMIC flops per launch
    (2*H*W*9*cin*cout of each launch) / its average launch duration from HIP events on
    the launch stream, recorded over a K-step pass identical to the timed region (run right after it)."""
    per = {}
    for fl, name, e0, e1 in prof:
        d = per.setdefault(name, [0, 0.0, 0])
        d[0] += fl
        d[1] += e0.elapsed_time(e1)
        d[2] += 1
    name, (fl, ms, n) = max(per.items(), key=lambda kv: kv[1][1])
    achieved = fl / (ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    src, traffic = load_traffic(args)
    tr = traffic.get(name)
    all_fl = sum(v[0] for k, v in per.items() if "head" not in k)
    all_ms = sum(v[1] for k, v in per.items() if "head" not in k)
    if args.layers:
        per_step = len(prof) // max(1, args.steps)
        for i in range(per_step):
            rows = prof[i::per_step]
            t_ms = sum(e0.elapsed_time(e1) for _, _, e0, e1 in rows) / len(rows)
            log("  conv #%2d %-55s %.3f ms  %.1f TFLOP/s" % (i, rows[0][1], t_ms, rows[0][0] / (t_ms * 1e-3) / 1e12))
    for k, (f, t, c) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        log("%-58s %3d launches %.3f ms/step %.1f TFLOP/s" % (k, c, t / args.steps, f / (t * 1e-3) / 1e12))
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": tr["bytes_per_launch"] if tr else None,
            "kernel": name, "launches": n, "avg_launch_ms": round(ms / n, 4), "flops_per_launch": int(fl / n),
            "traffic_source": ("%s (FETCH_SIZE x2 + WRITE_SIZE, per launch)" % os.path.relpath(src, REPO)) if tr
            else None,
            "all_mfma_convs": {"tflops": round(all_fl / (all_ms * 1e-3) / 1e12, 2),
                               "ms_per_step": round(all_ms / args.steps, 4),
                               "frac": round(all_fl / (all_ms * 1e-3) / 1e12 / peak, 4)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1, help="frames per step per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="540x960", help="HxW of the CPU-baseline sample frame")
    ap.add_argument("--no-profile", action="store_true", help="skip per-conv HIP events")
    ap.add_argument("--layers", action="store_true", help="per-conv timing breakdown on stderr")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches instead of the captured HIP graph")
    ap.add_argument("--no-loader", action="store_true", help="skip the training-sample loader record (rank 0, N=1)")
    ap.add_argument("--no-augment", action="store_true", help="skip the augmentation record (rank 0, N=1)")
    ap.add_argument("--no-train", action="store_true", help="skip the config-5 training-step record (all ranks)")
    ap.add_argument("--video-frames", type=int, default=256,
                    help="config-4 record: frames sharded over the ranks + matte all-gather (0 = skip)")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="vm_set_option kernel knob before the run (A/B comparisons), repeatable")
    args = ap.parse_args()

    rank, world, local = parallel.init_from_env("nccl")
    if world != args.gpus:
        log("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    for kv in args.option:
        k, v = kv.split("=")
        from vmatting import _lib
        _lib.set_option(k, int(v))

    # identical weights everywhere: every rank draws from the same seeds, then rank 0's packed
    # buffers are broadcast (one RCCL collective) so replicas are bit-identical by construction
    vgg = synthetic_vgg16(0)
    np.random.seed(0)
    model = unet.UNetVideo(vgg, dtype=args.dtype, device=dev).prepare()
    parallel.broadcast_tensors(model.weights_flat(), src=0)

    B, H, W = args.batch, args.height, args.width
    x = synth_frames(B, H, W, rank * B, dev)
    flops_per_frame = model.conv_flops(1, H, W)

    # the timed step is the whole forward replayed from a HIP graph (captured once: one host call per step, no
    # per-launch host cost); --no-graph times the eager launch sequence instead
    graphed = model.capture(x) if not args.no_graph else None
    step = graphed.replay if graphed is not None else (lambda: model.forward(x))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    # per-kernel HIP events cost ~10% of the step (a marker between every launch), so the roofline pass is a
    # second, identical K-step pass with an event pair on the launch stream around every conv
    prof = None
    if not args.no_profile:
        prof = ops.conv_profile(True)
        for _ in range(args.steps):
            model.forward(x)
        torch.cuda.synchronize()
        ops.conv_profile(False)

    video = None
    if args.video_frames > 0 and graphed is not None and args.batch == 1:
        video = video_batch(graphed, args.video_frames, H, W, rank, world, dev)

    train = None
    if not args.no_train:  # every rank: the DDP all-reduce is part of the step
        train = train_bench(dev, max(args.steps // 2, 5), 2, world, rank, cpu=not args.no_cpu_baseline)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames = world * B * args.steps
    value = frames / elapsed
    ms_step = 1000.0 * elapsed / args.steps

    roofline = None
    if prof:
        roofline = conv_roofline(prof, args)
    if rank == 0:
        rec = {"metric": METRIC, "value": round(value, 3), "unit": "frames/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic (seeded 1080p cmp/bg/trimap frames; synthetic VGG16 + init_conv weights)",
               "config": {"workload": "unet.UNetVideo forward (20 3x3 convs, 3.233 TFLOP/frame), %dx%d 7-ch NHWC"
                                      % (W, H),
                          "frames_per_step_per_gpu": B, "height": H, "width": W,
                          "launch": "eager" if args.no_graph else "hip-graph replay",
                          "parallelism": "frame-parallel dp%d" % world},
               "achieved_tflops_whole_forward": round(value / world * flops_per_frame / 1e12, 2),
               "roofline": roofline, "cpu_baseline": None}
        src, tr = load_traffic(args, full=True)
        if tr and tr.get("bytes_per_forward"):
            # whole-forward HBM traffic (PMC FETCH_SIZE x2 + WRITE_SIZE summed over every kernel of one forward,
            # one-time weight packing excluded) at this run's frame rate
            bpf = tr["bytes_per_forward"] / float(args.batch)
            rec["achieved_hbm_gbps"] = round(bpf * value / world / 1e9, 1)
            rec["hbm"] = {"bytes_per_frame": int(bpf), "achieved_gbps_per_gpu": rec["achieved_hbm_gbps"],
                          "peak_gbps": PEAK_HBM_GBPS, "frac": round(bpf * value / world / 1e9 / PEAK_HBM_GBPS, 4),
                          "source": os.path.relpath(src, REPO)}
        if video:
            rec["video_batch"] = video
        if train:
            rec["train"] = train
        if world == 1 and not args.no_cpu_baseline:
            sh, sw = (int(v) for v in args.cpu_sample.split("x"))
            rec["cpu_baseline"] = cpu_baseline(H, W, sh, sw)
        if world == 1 and not args.no_loader:
            rec["loader"] = loader_bench(dev, max(args.steps, 10), cpu=not args.no_cpu_baseline)
        if world == 1 and not args.no_augment:
            rec["augment"] = augment_bench(dev, max(args.steps, 10), cpu=not args.no_cpu_baseline)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
