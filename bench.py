"""Benchmark: alpha-mattes/sec of unet.UNetVideo at 1920x1080 (BASELINE.json configs[1]; configs[3] at N>1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16|fp32]
    python bench.py --gpus N --dist-selftest      # CPU-only (gloo) check of the N-rank launcher and collectives

With --gpus N > 1 bench.py starts its own N ranks (one child process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT in their environment) before anything touches a GPU, waits for them and exits
with rank 0's code (the first failing rank's, if any fails).  Launched by torchrun instead (WORLD_SIZE already set),
it is one of those ranks.  Either way a run whose initialised world differs from --gpus exits non-zero.

A step = one UNetVideo forward over B synthetic 1080p 7-channel frames per GPU (inputs resident
in HBM before timing).  Frame-parallel: every rank runs its own frames, no collective in the data
path (scaling "weak"); the packed weights are RCCL-broadcast from rank 0 once, before timing.
Rank 0 prints ONE JSON line (value = frames processed by all ranks / max-over-ranks time).

Sub-records on the same line: video_batch (config 4: 256 frames sharded + all-gathered), temporal
(config 3: warp + occlusion + refine), fp32 (the path that meets north_star's 1e-4 bound), parity
(bf16 vs fp32 vs the CPU oracle on the timed frame), train (config 5), loader and augment.
"""

import argparse
import json
import os
import platform
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vmatting import ops, parallel, unet, video  # noqa: E402
from vmatting.weights import synthetic_vgg16  # noqa: E402

METRIC = "alpha-mattes/sec at 1920×1080, 1/2/4/8 MI355X + achieved HBM GB/s"
PEAK_TFLOPS = {"bf16": 2516.6, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md chip table)
PEAK_HBM_GBPS = 8000.0
VGG_MEAN = video.VGG_MEAN
N_SIMD = 1024  # 256 CUs x 4 SIMDs


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_info():
    """Host CPU model and the thread count the CPU baselines use (BLAS pool; OMP_NUM_THREADS on the box)."""
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return model, int(threads)


class Events:
    """HIP events on the CURRENT stream (the one every vm_* launch of this process uses)."""

    def __init__(self):
        self.e = []

    def mark(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.e.append(ev)
        return ev


def ms(e0, e1):
    return e0.elapsed_time(e1)


# ------------------------------------------------------------------------------------------------ config 4

def video_batch(model, n_frames, h, w, rank, world, dev, chunk, solo_frames=32):
    """BASELINE config 4 through the product path (vmatting/video.py): n_frames synthetic 1080p frames sharded
    frame-parallel in contiguous blocks, each rank's block replayed in HIP graphs of `chunk` frames (input read
    in place, alpha written in place), then ONE all-gather (RCCL ring over xGMI) hands every rank the whole
    [n_frames, H, W, 1] f32 matte batch.  Timed between barriers, max over ranks.

    parallel_efficiency (N > 1) = frames/s / (N x the same video path's frames/s on ONE GPU, measured in this run:
    rank 0 alone replays `solo_frames` frames' chunk graphs while the other ranks wait at a barrier)."""
    solo = None
    if world > 1:
        if rank == 0:
            sf = video.synthetic_frames(solo_frames, h, w, first=0, device=dev)
            svm = video.VideoMatter(model, sf, chunk=chunk)
            svm.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            svm.run()
            torch.cuda.synchronize()
            solo = solo_frames / (time.perf_counter() - t0)
            del svm, sf
        dist.barrier()
    a, b = video.shard(n_frames, rank, world)
    frames = video.synthetic_frames(b - a, h, w, first=a, device=dev)
    vm = video.VideoMatter(model, frames, chunk=chunk)
    mx = max(q - p for p, q in (parallel.shard_range(n_frames, r, world) for r in range(world)))
    recv = torch.empty((world * mx, h, w, 1), dtype=torch.float32, device=dev) if world > 1 else None
    vm.run()  # warm
    if world > 1:
        parallel.gather_frames(vm.alpha, n_frames, out=recv)  # warm the communicator
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vm.run()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    full = parallel.gather_frames(vm.alpha, n_frames, out=recv)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    ts = torch.tensor([t2 - t0, t1 - t0, t2 - t1], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
    total, comp, gath = (float(v) for v in ts.tolist())
    assert full.shape[0] == n_frames
    fps = n_frames / total
    rec = {"workload": "config 4: %d synthetic %dx%d frames sharded frame-parallel over %d GPU(s), mattes "
                       "all-gathered to every rank (vmatting/video.py)" % (n_frames, w, h, world),
           "frames": n_frames, "frames_per_s": round(fps, 3), "ms_total": round(1e3 * total, 3),
           "ms_compute_max_rank": round(1e3 * comp, 3), "chunk_frames": chunk, "graphs_per_rank": len(vm.spans),
           "includes": "chunked HIP-graph replay reading the frames in place" + (" + the matte all-gather"
                                                                                 if world > 1 else "")}
    if world > 1 and solo is not None:  # rank 0 (the one that prints)
        rec.update({"ms_all_gather": round(1e3 * gath, 3),
                    "all_gather_bytes": int(full.numel() * full.element_size()),
                    "solo_frames_per_s": round(solo, 3), "parallel_efficiency": round(fps / (world * solo), 4),
                    "parallel_efficiency_def": "frames_per_s / (n_gpus x the same chunked video path's frames/s on "
                                               "rank 0 alone, %d frames, measured in this run)" % solo_frames})
    else:
        rec["parallel_efficiency_def"] = ("N = 1: this record IS the single-GPU reference of the video path; "
                                          "efficiency is defined at N > 1 against it")
    return rec


# ------------------------------------------------------------------------------------------------ config 3

def synthetic_flow(h, w, seed, modes=8, amp=20.0):
    """smooth random flow, sum of `modes` Gaussian modes scaled to |u|,|v| <= amp (seed 7)."""
    rs = np.random.RandomState(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    out = np.zeros((h, w, 2), np.float32)
    for _ in range(modes):
        cy, cx = rs.uniform(0, h), rs.uniform(0, w)
        s = rs.uniform(0.1, 0.4) * max(h, w)
        g = np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / np.float32(2 * s * s))
        out[..., 0] += np.float32(rs.uniform(-1, 1)) * g
        out[..., 1] += np.float32(rs.uniform(-1, 1)) * g
    out *= np.float32(amp / max(1e-9, float(np.abs(out).max())))
    return out


def temporal_case(h, w, seed=7):
    rs = np.random.RandomState(seed)
    bw = synthetic_flow(h, w, seed)
    fw = -bw
    yy, xx = np.mgrid[0:h, 0:w]
    fw[((yy - 0.4 * h) ** 2 + (xx - 0.6 * w) ** 2) < (0.15 * min(h, w)) ** 2] += 40.0  # an occluded disk
    prev = np.clip(1.3 - np.hypot((yy - h / 2) / (h / 3), (xx - w / 2) / (w / 4)), 0, 1).astype(np.float32)
    cur = np.clip(prev + rs.normal(0, 0.02, prev.shape), 0, 1).astype(np.float32)
    cmp = (rs.uniform(0, 255, (h, w, 3)) - np.array(VGG_MEAN)).astype(np.float32)
    return prev, cur, cmp, bw, fw


def temporal_bench(dev, steps, dtypes, sizes, cpu, threads):
    """BASELINE config 3: flow warp (flow.py:9-18) + occlusion check (flow.py:36-65) + RefineNet (refine.py:27-32,
    Cin 5) on synthetic smooth flows, inputs resident in HBM, for each compute dtype: fp32 is the reference's
    precision (the config-3 number), bf16 the throughput variant.  Device ms per stage from HIP events on the
    launch stream; the refine stage's roofline is the larger of its HBM time (algorithmic bytes) and its MFMA time
    (algorithmic FLOPs at the dtype's dense peak)."""
    from vmatting import temporal
    recs, cpu_rec = [], None
    for dtype, (h, w) in [(d, hw) for d in dtypes for hw in sizes]:
        prev, cur, cmp, bw, fw = temporal_case(h, w)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        args = [T(a) for a in (prev, cur, cmp, bw, fw)]
        np.random.seed(3)
        tp = temporal.TemporalRefiner(dtype=dtype, device=dev)
        for _ in range(3):
            tp(*args, check_index=False)
        torch.cuda.synchronize()
        ev = Events()
        t0 = time.perf_counter()
        for _ in range(steps):
            ev.mark()
            x = tp.prepare_input(*args, check_index=False)
            ev.mark()
            tp.refine.forward_prepared(x, out=tp._bufs[(h, w)]["out"])
            ev.mark()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps
        assert int(tp._bufs[(h, w)]["err"].item()) == 0
        e = ev.e
        t_in = sum(ms(e[3 * i], e[3 * i + 1]) for i in range(steps)) / steps
        t_rf = sum(ms(e[3 * i + 1], e[3 * i + 2]) for i in range(steps)) / steps
        px = h * w
        ob = 2 if dtype == "bf16" else 4
        # input pass: flow_b 8 + flow_f gather 8 + prev gather 4 + cmp 12 + alpha_t 4 + warped out 4 + row 8*ob
        b_in = px * (8 + 8 + 4 + 12 + 4 + 4 + 8 * ob)
        # refine: input row 8*ob + f32 64-ch softmax out 256; FLOPs of conv4 at the reference's Cin = 5
        b_rf = px * (8 * ob + 256)
        f_rf = 2.0 * px * 9 * 5 * 64
        pk = PEAK_TFLOPS[dtype]
        t_hbm, t_mfma = b_rf / (PEAK_HBM_GBPS * 1e9), f_rf / (pk * 1e12)
        rf = {"bound": "hbm" if t_hbm >= t_mfma else "mfma", "algorithmic_bytes": int(b_rf),
              "algorithmic_flops": int(f_rf), "achieved_gbps": round(b_rf / (t_rf * 1e-3) / 1e9, 1),
              "peak_gbps": PEAK_HBM_GBPS, "tflops": round(f_rf / (t_rf * 1e-3) / 1e12, 2), "peak_tflops": pk,
              "roofline_ms": round(1e3 * max(t_hbm, t_mfma), 4),
              "frac": round(1e3 * max(t_hbm, t_mfma) / t_rf, 4),
              "frac_def": "roofline time (max of HBM bytes / 8 TB/s and FLOPs / dense peak) / measured device time"}
        rec = {"workload": "config 3: warp + correct_alpha + RefineNet(Cin 5) at %dx%d, %s" % (w, h, dtype),
               "dtype": dtype,
               "role": "reference precision (fp32, the config-3 number)" if dtype == "fp32" else
                       "throughput variant (bf16 operands, f32 accumulate and softmax)",
               "pairs_per_s": round(1.0 / wall, 1), "ms_per_pair": round(1e3 * wall, 4),
               "device_ms": {"warp_occlusion_input": round(t_in, 4), "refine_conv_softmax": round(t_rf, 4)},
               "refine_kernel": _lib_last_kernel(),
               "roofline": {
                   "warp_occlusion_input": {"bound": "hbm", "algorithmic_bytes": int(b_in),
                                            "achieved_gbps": round(b_in / (t_in * 1e-3) / 1e9, 1),
                                            "peak_gbps": PEAK_HBM_GBPS,
                                            "frac": round(b_in / (t_in * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4)},
                   "refine_conv_softmax": rf},
               "occluded_px": int((tp.warped == 0).sum().item())}
        if cpu and (h, w) == sizes[0] and cpu_rec is None:
            from oracle import flow as oflow  # the CPU-baseline leg only
            from oracle import ops as oops
            p4 = tp.refine.params["conv4"]
            times = []
            for _ in range(2):
                t0 = time.perf_counter()
                a = oflow.correct_alpha(bw, fw, oflow.warp_img(prev, bw), promote="numpy1")
                xin = np.concatenate([cmp, cur[..., None], a[..., None].astype(np.float32)], -1)[None]
                oops.softmax_lastdim(oops.conv3x3_same(xin, p4[0], p4[1]))
                times.append(time.perf_counter() - t0)
            dt = min(times)
            cpu_rec = {"value": round(1.0 / dt, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
                       "sample": "oracle/flow.py warp_img + vectorised correct_alpha + oracle/ops.py "
                                 "conv3x3 + softmax (RefineNet conv4, f32) on one %dx%d pair, best of 2" % (w, h)}
        if cpu_rec is not None and (h, w) == sizes[0]:
            rec["cpu_baseline"] = cpu_rec
        recs.append(rec)
    return recs


def _lib_last_kernel():
    from vmatting import _lib
    return _lib.last_conv_kernel()


# ------------------------------------------------------------------------------------------------ CPU baseline + parity

def cpu_baseline(x_host, params, frames, threads, model_name, flops_per_frame):
    """The oracle (numpy f32 restatement of unet.py, the reference's op sequence) on the host cores: 1 warm-up
    frame at 270x480, then `frames` full 1920x1080 frames timed, median.  Returns (record, oracle output of the
    first timed frame) — the latter is the fp32 parity check of the timed frame."""
    from oracle import models as om  # the CPU-baseline leg only
    om.unet_forward(np.ascontiguousarray(x_host[:, :270, :480]), params, dtype=np.float32)
    times, ref = [], None
    for _ in range(frames):
        t0 = time.perf_counter()
        r = om.unet_forward(x_host, params, dtype=np.float32)
        times.append(time.perf_counter() - t0)
        if ref is None:
            ref = r
    med = statistics.median(times)
    rec = {"value": round(1.0 / med, 5), "unit": "frames/s", "cores": threads, "kind": "port",
           "host_cpu": model_name, "implied_tflops": round(flops_per_frame / med / 1e12, 3),
           "affinity_cpus": len(os.sched_getaffinity(0)),
           "threads_def": "cores = BLAS pool threads the oracle ran on (numpy's OpenBLAS, OMP_NUM_THREADS on the box); "
                          "affinity_cpus = CPUs in this process's affinity mask; the loader / augment / train / "
                          "temporal CPU legs use the same thread count",
           # BASELINE.md's plan sets the pool to the affinity mask; on this pool a 1-GPU job's CPU share is
           # OMP_NUM_THREADS (16) of a host whose whole mask (256) is shared with the other GPUs' jobs, so the
           # measurement keeps that share, and the linear scaling to the full mask is given as an upper bound
           "threads_subset_reason": "the pool gives each GPU job OMP_NUM_THREADS=%s of the %d host CPUs in the "
                                    "affinity mask (shared with the other GPUs' jobs); the baseline runs on that share"
                                    % (os.environ.get("OMP_NUM_THREADS", "?"), len(os.sched_getaffinity(0))),
           "upper_bound_at_affinity_cpus": round(len(os.sched_getaffinity(0)) / max(1, threads) / med, 4),
           "sample": "oracle/models.py numpy-f32 UNetVideo forward (the reference's op sequence) on the timed "
                     "1920x1080 frame: 1 warm-up (270x480), median of %d full frames (%s s)"
                     % (frames, ", ".join("%.1f" % t for t in times))}
    return rec, ref


def fp32_record(model, x, steps, vgg, params):
    """The fp32 path (exact-f32 MFMA, the one north_star's 1e-4 alpha bound holds for) at 1080p: graph-replayed
    forward timed over `steps` frames, plus per-conv events for its roofline against the f32 MFMA peak."""
    m32 = unet.UNetVideo(vgg, dtype="fp32", device=x.device).load_params(params).prepare()
    g = m32.capture(x)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    prof = ops.conv_profile(True)
    m32.forward(x)
    torch.cuda.synchronize()
    ops.conv_profile(False)
    fl = sum(p[0] for p in prof)
    t = sum(ms(p[2], p[3]) for p in prof)
    flops = m32.conv_flops(x.shape[0], x.shape[1], x.shape[2])
    rec = {"workload": "unet.UNetVideo forward, fp32 (v_mfma_f32_16x16x4_f32), 1920x1080, hip-graph replay",
           "frames_per_s": round(x.shape[0] / dt, 3), "ms_per_frame": round(1e3 * dt / x.shape[0], 3),
           "tflops_whole_forward": round(flops / dt / 1e12, 2),
           "roofline": {"bound": "mfma", "achieved": round(fl / (t * 1e-3) / 1e12, 2), "peak": PEAK_TFLOPS["fp32"],
                        "unit": "TFLOP/s", "frac": round(fl / (t * 1e-3) / 1e12 / PEAK_TFLOPS["fp32"], 4),
                        "scope": "all convs of one forward (HIP events per launch)"}}
    return rec, m32


SPLIT_DESC = {
    "bf16x6": ("split-bf16 x6 (three bf16 parts per operand, 6 cross products on v_mfma_f32_16x16x32_bf16, f32 sums)",
               6),
    "f16x3": ("split-fp16 x3 (two fp16 parts per operand, the filter pre-scaled by a power of two; l*Wh + h*Wl + h*Wh "
              "on v_mfma_f32_16x16x32_f16, f32 sums)", 3),
}


def split_record(x, steps, vgg, params, mode):
    """A split-operand path (vmatting/split6.py "bf16x6", vmatting/split3.py "f16x3": conv operands carried as
    16-bit parts whose cross products are exact, f32 epilogues) at 1080p — the paths that meet north_star's 1e-4
    alpha bound on the 16-bit MFMA pipes.  Graph-replayed forward over `steps` frames.  roofline: the ALGORITHMIC
    conv FLOPs (2*H*W*9*cin*cout, 3.233 TFLOP per frame) over the whole forward's time at the bf16 dense peak
    (what the path delivers); executed_products: the products the MFMA pipes run (k x those FLOPs) over the convs'
    own launch time (how busy the pipes are)."""
    desc, k = SPLIT_DESC[mode]
    m = unet.UNetVideo(vgg, dtype=mode, device=x.device).load_params(params).prepare()
    g = m.capture(x)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    prof = ops.conv_profile(True)
    m.forward(x)
    torch.cuda.synchronize()
    ops.conv_profile(False)
    fl = sum(p[0] for p in prof)
    t = sum(ms(p[2], p[3]) for p in prof)
    flops = m.conv_flops(x.shape[0], x.shape[1], x.shape[2])
    pk = PEAK_TFLOPS["bf16"]
    algo = flops / dt / 1e12
    rec = {"workload": "unet.UNetVideo forward, %s, 1920x1080, hip-graph replay" % desc,
           "frames_per_s": round(x.shape[0] / dt, 3), "ms_per_frame": round(1e3 * dt / x.shape[0], 3),
           "tflops_whole_forward": round(algo, 2),
           "roofline": {"bound": "mfma", "achieved": round(algo, 2), "peak": pk, "unit": "TFLOP/s",
                        "frac": round(algo / pk, 4),
                        "scope": "algorithmic conv FLOPs of the forward (3.233 TFLOP per 1080p frame) over the whole "
                                 "forward's time (graph replay) at the bf16 dense peak"},
           "executed_products": {"tflops": round(fl / (t * 1e-3) / 1e12, 2), "frac": round(fl / (t * 1e-3) / 1e12 / pk, 4),
                                 "conv_ms": round(t, 3), "products_per_algorithmic_flop": k,
                                 "scope": "the %dx products the MFMA pipes execute (the conv over %d stacked operand "
                                          "slabs) over the convs' own launch time (HIP events per launch)" % (k, k)}}
    if mode == "f16x3":
        rec["overflow"] = m.overflowed()  # an activation past fp16's range would void the frame (bf16x6 fallback)
    return rec, m


# ------------------------------------------------------------------------------------------------ loader / augment

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


def _pool_rate(fn, items, threads):
    """Wall-clock rate of fn over items on a pool of `threads` host threads (numpy releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(fn, items))
    return len(items) / (time.perf_counter() - t0)


def loader_bench(dev, steps, threads, cpu=True, n=8, size=320, h=1080, w=1920):
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
    ev = Events()
    t0 = time.perf_counter()
    ev.mark()
    for _ in range(steps):
        vl.compose_batch(samples, (size, size), names, device=dev)
    ev.mark()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    dev_ms = ms(*ev.e) / steps
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

        def one(s):
            fr, fc, br, bc = (ol.Axis(*a) for a in s["plan"])
            srcs = ol.crop_sources(s["fg"], s["bg"], fr, fc, br, bc, s["prev"], s["flow"])
            ol.compose(srcs[0], srcs[1], srcs[3], (size, size), srcs[2])
        items = [host[i % n] for i in range(threads)]
        rate = _pool_rate(one, items, threads)
        rec["cpu_baseline"] = {"value": round(rate, 3), "unit": "samples/s", "cores": threads, "kind": "port",
                               "sample": "oracle/loader.py (numpy float64, with the reference's full-frame warp), "
                                         "%d entries on a pool of %d host threads" % (len(items), threads)}
    return rec


def augment_bench(dev, steps, threads, cpu=True, h=1080, w=1920, batch=8):
    """augmentation.augment on 1080p (fg, bg, alpha) samples resident in HBM, `batch` at a time
    through augment_many (config 5's path: host draws + TPS solves, one statistics readback, one landmark upload,
    vm_augment_batch).  Per-sample figures; device time from HIP events on the launch stream."""
    from vmatting import augmentation as va
    rs = np.random.RandomState(9)
    yy, xx = np.mgrid[0:h, 0:w]
    alpha_h = np.clip(1.2 - np.sqrt(((yy - 0.46 * h) / (0.28 * h)) ** 2 + ((xx - 0.47 * w) / (0.21 * w)) ** 2), 0, 1)
    fg_h = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    bg_h = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    fg, bg, alpha = (torch.from_numpy(a).to(dev) for a in (fg_h, bg_h, alpha_h))
    triples = [(fg, bg, alpha)] * batch
    np.random.seed(0)
    for _ in range(3):
        va.augment_many(triples)
    torch.cuda.synchronize()
    ev = Events()
    va._EVENTS = kev = []  # the device pipeline's own time: events around each vm_augment_batch launch
    t0 = time.perf_counter()
    ev.mark()
    for _ in range(steps):
        va.augment_many(triples)
    ev.mark()
    torch.cuda.synchronize()
    va._EVENTS = None
    wall = (time.perf_counter() - t0) / steps / batch
    span_ms = ms(*ev.e) / steps / batch
    dev_ms = sum(ms(a, b) for a, b in kev) / steps / batch
    # algorithmic bytes per sample (per pixel): alpha stats 8; bg 2 warps 2*(3+3); TPS grid (h/2)(w/2)*16 = 4;
    # fg TPS 3+3, alpha TPS 8+8; fg 2 warps 2*(3+3); alpha 2 warps 2*(8+8); illumination fg+bg 2*(3+3)
    algo = augment_bytes(h, w)
    rec = {"workload": "augmentation.augment: %dx%d samples (u8 fg/bg, f64 alpha), %d per augment_many call, inputs in "
                       "HBM; per-sample figures" % (w, h, batch),
           "algorithmic_bytes_def": "the reference's passes (stats, two warpAffine per image, TPS lattice + resampling, "
                                    "illumination), each image read and written once per pass",
           "samples_per_s": round(1.0 / wall, 1), "ms_per_sample": round(1000 * wall, 4),
           "device_ms_per_sample": round(dev_ms, 4),
           "device_ms_def": "HIP events around each vm_augment_batch launch (the per-pixel pipeline); the stream span "
                            "per sample, host draws / TPS solves / statistics readback included, is stream_ms_per_sample",
           "stream_ms_per_sample": round(span_ms, 4), "algorithmic_bytes_per_sample": int(algo),
           "achieved_gbps": round(algo / (dev_ms * 1e-3) / 1e9, 1), "peak_gbps": PEAK_HBM_GBPS,
           "roofline": {"bound": "hbm", "achieved": round(algo / (dev_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBPS,
                        "unit": "GB/s", "frac": round(algo / (dev_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4)}}
    if cpu:
        from oracle import augment as oa  # the CPU-baseline leg only
        np.random.seed(0)
        rate = _pool_rate(lambda _: oa.augment(fg_h, bg_h, alpha_h), list(range(threads)), threads)
        rec["cpu_baseline"] = {"value": round(rate, 3), "unit": "samples/s", "cores": threads, "kind": "port",
                               "sample": "oracle/augment.py (numpy, scipy-order TPS + OpenCV restatement): %d "
                                         "%dx%d samples (the config's size, not scaled) on a pool of %d host threads"
                                         % (threads, w, h, threads)}
    return rec


# ------------------------------------------------------------------------------------------------ config 5

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


def train_step_traffic(n, h, w, dtype_bytes=2):
    """Algorithmic HBM bytes of the memory-bound part of one config-5 step (unet_simple.py:116-142 at phase=True,
    train.py:288-304), the way small_train_traffic counts small_train.py's: the select convs read every tower
    feature level twice (forward, and again for their filter gradients) — the concat of the three towers, in the
    compute dtype; every decoder tensor (1-96 channels: select / upconv / conv pre-BN outputs in f32, BN'd
    activations and resized inputs in the compute dtype) written once and read once per consumer, and their f32
    gradients likewise; the trainable parameters, gradients and Adam slots once.  The tower convs themselves (their
    activations included) are the MFMA-bound part, priced by train_flops."""
    from vmatting.train import param_layout
    from vmatting.unet_simple import _levels
    L = _levels(h, w)
    px = [n * a * b for a, b in L]
    T, F = dtype_bytes, 4
    # tower features the select convs read (unet_simple.py:153-168: cmp | bg | diff per level; in9 = the 9-channel
    # input concat at L0), and conv5_3's concat that upconv4 resizes
    feats = [(0, 9 + 3 * 64 + 3 * 64), (1, 3 * 128 * 2), (2, 3 * 256 * 3), (3, 3 * 512 * 3), (4, 3 * 512)]
    tower = sum(px[lv] * c * T * 2 for lv, c in feats)
    # per level (selects k x nsel, upconv cout u, concat width W, conv cout c, the upconv's input width ci at lv+1)
    lvls = [(3, 48, 48, 96, 48, None), (2, 24, 24, 48, 24, 48), (1, 8, 24, 32, 32, 24), (0, 6, 24, 30, 32, 32)]
    dec = 0
    for lv, sel, u, W, c, ci in lvls:
        ent = [(lv, sel, F, 2), (lv, u, F, 2),             # select / upconv pre-BN outputs (stats + apply)
               (lv, W, T, 1 + 1),                          # BN'd concat: conv input + its filter gradient
               (lv, c, F, 2), (lv, c, T, 2)]               # conv pre-BN output, its BN'd relu activation
        if ci is not None:
            ent.append((lv, ci, T, 2))                     # the resized upconv input (conv + filter gradient)
        grads = [(lv, W, F, 2), (lv, c, F, 2), (lv, u, F, 1), (lv, sel, F, 1)]  # dconcat, dconv, dupconv, dselect
        reread = [(lv, sel + u + c, F, 1)]                 # the BN backward re-reads its pre-BN inputs
        dec += sum(px[l] * ch * b * (1 + r) for l, ch, b, r in ent + grads) + sum(px[l] * ch * b for l, ch, b, _ in
                                                                                     reread)
    dec += px[0] * (1 * F * 3 + 1 * F * 2 + 3 * 4 * 3 + 1 * 4 * 2)  # output conv, alpha, the loss's inputs, dalpha
    nparam = param_layout()[1]
    return tower + dec + nparam * 4 * (1 + 1 + 2 + 2)


def step_roofline(flops, nbytes, dev_ms, peak_tflops):
    """Two-part roofline of a step: its MFMA-bound convs at the dense peak plus its memory-bound work at the HBM peak
    (dependent phases: the sum is the bound), over the measured device time."""
    t_mfma = flops / (peak_tflops * 1e12) * 1e3
    t_hbm = nbytes / (PEAK_HBM_GBPS * 1e9) * 1e3
    rl = t_mfma + t_hbm
    return {"bound": "mfma+hbm", "roofline_ms": round(rl, 4), "measured_device_ms": round(dev_ms, 4),
            "frac": round(rl / dev_ms, 4), "mfma_ms": round(t_mfma, 4), "hbm_ms": round(t_hbm, 4),
            "flops": int(flops), "algorithmic_bytes": int(nbytes), "peak_tflops": peak_tflops,
            "peak_gbps": PEAK_HBM_GBPS, "achieved_tflops": round(flops / (dev_ms * 1e-3) / 1e12, 2),
            "frac_max": round(max(t_mfma, t_hbm) / dev_ms, 4),
            "def": "roofline_ms = algorithmic conv FLOPs / dense MFMA peak + algorithmic bytes of the memory-bound work "
                   "/ 8 TB/s (phases in sequence); frac = roofline_ms / measured device ms; frac_max uses the larger "
                   "of the two instead (perfect overlap)"}


def set_train_side(kind):
    """--train-side: the config-5 trainer's side-stream kind (VideoTrainer.side_kind), set in the ranks only."""
    if kind:
        from vmatting.train import VideoTrainer
        VideoTrainer.side_kind = kind


def train_bench(dev, steps, warmup, world, rank, threads, cpu=True, n=8, size=320, dtype="bf16", graph=False,
                streams=3, wgrad_stream=True):
    """BASELINE config 5: one train.py video_procedure iteration per step (train.py:288-343) — batch of 8 320x320
    samples per GPU (params.py:8-9) resident in HBM: 3 VGG16 towers + UNetSimple (batch-statistics BN) forward,
    loss, backward through the trainable layers, one RCCL all-reduce of the gradients (DDP), TF-Adam, re-pack.
    Device time per phase from HIP events on the launch stream; step time = max over ranks."""
    from vmatting.train import VideoTrainer
    rs = np.random.RandomState(100 + rank)
    mean = np.array(VGG_MEAN)
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
    trn = VideoTrainer(synthetic_vgg16(0), dtype, dev, streams=streams, wgrad_stream=wgrad_stream)
    # eager launches (the select chains overlap the decoder on side streams); graph: forward + loss and backward
    # replayed from HIP graphs (VideoTrainer.capture), DDP exchange + Adam eager
    g = trn.capture(cmp_d, bg_d, warped_d, gt_d, fg_d) if graph else None
    for _ in range(warmup):
        if g is not None:
            g.step()
        else:
            trn.step(cmp_d, bg_d, warped_d, gt_d, fg_d)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = Events()
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.mark()
        if g is not None:
            g.g_fwd.replay()
        else:
            trn.forward(cmp_d, bg_d, warped_d)
            trn._tb["loss"].copy_(ops.matting_loss(trn._tb["alpha"], gt_d, fg_d, bg_d, cmp_d))
        ev.mark()
        if g is not None:
            g.g_bwd.replay()
        else:
            trn.grad.zero_()
            trn.backward(gt_d, fg_d, bg_d, cmp_d)
        ev.mark()
        trn.apply_gradients()
        ev.mark()
    torch.cuda.synchronize()
    wall = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall)
    e = ev.e
    ph = [sum(ms(e[4 * i + k], e[4 * i + k + 1]) for i in range(steps)) / steps for k in range(3)]
    fwd_f, bwd_f = train_flops(n, size, size)
    rec = {"workload": "train.py video_procedure step (config 5): %d x %dx%d per GPU, 3 VGG16 towers + UNetSimple "
                       "fwd/bwd, loss, DDP all-reduce, TF-Adam" % (n, size, size),
           "dtype": dtype + " forward, f32 gradients/optimizer", "n_gpus": world,
           "launch": ("hip-graph replay of forward+loss and of backward, eager all-reduce + Adam + re-pack" if graph
                      else "eager") + ("; select chains on %d side streams%s" % (
                          streams, ", decoder filter gradients on one more" if wgrad_stream else "") if streams
                                       else ""),
           "samples_per_s": round(n * world / wall, 1), "ms_per_step": round(1000 * wall, 3),
           "device_ms": {"forward_loss": round(ph[0], 3), "backward": round(ph[1], 3),
                         "allreduce_adam_repack": round(ph[2], 3)},
           "flops_per_step_per_gpu": {"forward": fwd_f, "backward": bwd_f},
           "achieved_tflops_per_gpu": round((fwd_f + bwd_f) / wall / 1e12, 1),
           "roofline": step_roofline(fwd_f + bwd_f, train_step_traffic(n, size, size, 2 if dtype == "bf16" else 4),
                                     sum(ph), PEAK_TFLOPS[dtype]),
           "loss_last": [round(float(v), 5) for v in trn._tb["loss"].cpu()]}
    if cpu and world == 1:
        from oracle import models as om  # the CPU-baseline leg only
        from oracle import train_ref as tr
        p = om.unet_simple_params(np.random.RandomState(1))
        sl = lambda a: np.asarray(a[:1], np.float64)  # noqa: E731
        t0 = time.perf_counter()
        tr.train_step_grads(sl(cmp), sl(bg - mean), sl(warped), sl(gt), sl(fg), synthetic_vgg16(0), p)
        dt = time.perf_counter() - t0
        rec["cpu_baseline"] = {"value": round(1.0 / dt, 4), "unit": "samples/s", "cores": threads,
                               "kind": "port",
                               "sample": "oracle/train_ref.py (numpy-f64 VGG towers + torch-f64 autograd head) on one "
                                         "%dx%d sample (the config's sample size, timed, not scaled)" % (size, size)}
    return rec


def small_train_traffic(n, h, w, dtype_bytes=2):
    """Algorithmic HBM bytes of one small_train.py step (8 x 320^2): every tensor the step materialises written once
    and read once per consumer — activations in the compute dtype, pre-BN outputs and gradients in f32 — plus the
    parameters, gradients and Adam slots once (the roofline of a step whose convs are 1-32 channels wide)."""
    from vmatting.small_train import param_layout
    L = [(h, w), ((h + 1) // 2, (w + 1) // 2)]
    L.append(((L[1][0] + 1) // 2, (L[1][1] + 1) // 2))
    px = [n * a * b for a, b in L]
    T, F = dtype_bytes, 4
    # (level, channels, bytes per element, reads) of each tensor of the forward and backward (small.py:37-50)
    fwd = [(0, 6, F, 1), (0, 8, T, 1),                      # input, its bf16 copy
           (0, 8, F, 2), (0, 8, T, 3), (1, 8, T, 2),          # conv1_1 z, act, pool1
           (1, 16, F, 2), (1, 16, T, 3), (2, 16, T, 2),       # conv2_1 z, act, pool2
           (2, 32, F, 2), (2, 32, T, 2), (2, 32, F, 2), (2, 32, T, 2),   # conv3_1, conv3_2
           (1, 32, T, 1), (1, 16, T, 3), (1, 32, T, 2),       # resize, upconv1, BN(cat1)
           (1, 16, F, 2), (1, 16, T, 2), (0, 16, T, 1), (0, 8, T, 3), (0, 16, T, 2),  # conv2_2, resize, upconv2, BN
           (0, 8, F, 2), (0, 8, T, 2), (0, 1, F, 2), (0, 1, F, 2)]                   # conv1_2, conv1_3, alpha
    bwd = [(0, 1, F, 2), (0, 8, F, 3), (0, 16, F, 2), (0, 16, F, 2), (0, 8, F, 1), (0, 8, F, 2), (0, 16, F, 1),
           (1, 16, F, 2), (1, 32, F, 2), (1, 32, F, 2), (1, 16, F, 1), (1, 16, F, 2), (1, 32, F, 1), (2, 32, F, 2),
           (2, 32, F, 2), (2, 16, F, 1), (1, 16, F, 2), (1, 8, F, 1), (0, 8, F, 2)]
    act = sum(px[lv] * c * b * (1 + r) for lv, c, b, r in fwd + bwd)
    nparam = param_layout(6)[1]
    return act + nparam * 4 * (1 + 1 + 2 + 2)  # params read+write, gradients, Adam m / v read+write


def train_small_bench(dev, steps, warmup, world, rank, threads, cpu=True, n=8, size=320, dtype="bf16", graph=True):
    """small_train.py's step (small_train.py:34-88 with train()'s graph, :91-112): UNetSmall(concat(cmp, bg),
    phase=True) forward, the loss, backward through EVERY variable (max-pool, BN and resize adjoints, filter and data
    gradients), DDP all-reduce, TF-Adam at lr 1e-5, re-pack — batch 8 x 320^2 per GPU (params.py:8-9) resident in
    HBM.  Forward + loss and backward are replayed from HIP graphs (the step is ~110 tiny launches)."""
    from vmatting.small_train import SmallTrainer
    rs = np.random.RandomState(200 + rank)
    mean = np.array(VGG_MEAN)
    fg = rs.uniform(0, 255, (n, size, size, 3))
    bg = rs.uniform(0, 255, (n, size, size, 3))
    yy, xx = np.mgrid[:size, :size]
    gt = np.clip(1.2 - np.hypot((yy - size / 2) / (size / 3), (xx - size / 2) / (size / 4)), 0, 1)
    gt = np.repeat(gt[None, :, :, None], n, 0)
    cmp = gt * fg + (1 - gt) * bg - mean
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    cmp_d, bg_d, gt_d, fg_d = T(cmp), T(bg - mean), T(gt), T(fg)
    np.random.seed(2)
    trn = SmallTrainer(6, dtype, dev)
    g = trn.capture(cmp_d, bg_d, gt_d, fg_d) if graph else None
    for _ in range(warmup):
        if g is not None:
            g.step()
        else:
            trn.step(cmp_d, bg_d, gt_d, fg_d)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = Events()
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.mark()
        if g is not None:
            g.g_fwd.replay()
        else:
            trn.forward(cmp_d, bg_d)
            trn._b["loss"].copy_(ops.matting_loss(trn._b["alpha"], gt_d, fg_d, bg_d, cmp_d))
        ev.mark()
        if g is not None:
            g.g_bwd.replay()
        else:
            trn.grad.zero_()
            trn.backward(gt_d, fg_d, bg_d, cmp_d)
        ev.mark()
        trn.apply_gradients()
        ev.mark()
    torch.cuda.synchronize()
    wall = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall)
    e = ev.e
    ph = [sum(ms(e[4 * i + k], e[4 * i + k + 1]) for i in range(steps)) / steps for k in range(3)]
    dev_ms = sum(ph)
    nbytes = small_train_traffic(n, size, size, 2 if dtype == "bf16" else 4)
    rec = {"workload": "small_train.py step: %d x %dx%d per GPU, UNetSmall(concat(cmp, bg)) fwd/bwd over all "
                       "variables, loss, DDP all-reduce, TF-Adam" % (n, size, size),
           "dtype": dtype + " forward, f32 gradients/optimizer", "n_gpus": world,
           "launch": "hip-graph replay of forward+loss and of backward, eager all-reduce + Adam + re-pack" if graph
                     else "eager",
           "samples_per_s": round(n * world / wall, 1), "ms_per_step": round(1000 * wall, 4),
           "device_ms": {"forward_loss": round(ph[0], 4), "backward": round(ph[1], 4),
                         "allreduce_adam_repack": round(ph[2], 4)},
           "roofline": {"bound": "hbm", "algorithmic_bytes": int(nbytes),
                        "achieved_gbps": round(nbytes / (dev_ms * 1e-3) / 1e9, 1), "peak_gbps": PEAK_HBM_GBPS,
                        "frac": round(nbytes / (dev_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4),
                        "def": "bench.small_train_traffic: every tensor of the step written once and read once per "
                               "consumer + parameters / gradients / Adam slots, over the step's device time"},
           "loss_last": [round(float(v), 5) for v in trn._b["loss"].cpu()]}
    if cpu and world == 1:
        from oracle import models as om  # the CPU-baseline leg only
        from oracle import train_ref as tr
        p = om.unet_small_params(np.random.RandomState(1), cin=6)
        sl = lambda a: np.asarray(a[:2], np.float64)  # noqa: E731
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            tr.small_step_grads(sl(cmp), sl(bg - mean), sl(gt), sl(fg), p)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        rec["cpu_baseline"] = {"value": round(2.0 / best, 3), "unit": "samples/s", "cores": threads, "kind": "port",
                               "sample": "oracle/train_ref.py small_step_grads (torch-f64 autograd of UNetSmall) on 2 "
                                         "of the %dx%d samples, best of 2" % (size, size)}
    return rec


def train_image_bench(dev, steps, warmup, world, rank, threads, cpu=True, n=8, size=320, dtype="bf16", graph=False,
                      streams=1):
    """train.py's training_procedure step (train.py:37-109 with train()'s graph, :112-135):
    unet.UNetImage(x = [cmp, bg]) forward (the 20 convs, pools, TF-1 resizes, concats), the loss, backward through
    EVERY variable (VGG filters and biases included: wide MFMA filter gradients, data gradients on the forward conv
    kernels over flipped filters, pool / resize adjoints), DDP all-reduce, TF-Adam at lr 1e-5, re-pack — batch 8 x
    320^2 per GPU (params.py BATCH_SIZE / INPUT_SIZE) resident in HBM.  Eager launches with the filter gradients on
    a side stream beside the data-gradient chain (6.0 ms against 6.5 on one stream; a HIP-graph replay runs the
    captured fork's branches serially, 6.7 — so ``graph`` captures without the side stream); roofline: the step's
    algorithmic conv FLOPs over its device time at the bf16 dense MFMA peak."""
    from vmatting.image_train import ImageTrainer
    from vmatting.weights import synthetic_vgg16 as svgg
    rs = np.random.RandomState(300 + rank)
    mean = np.array(VGG_MEAN)
    fg = rs.uniform(0, 255, (n, size, size, 3))
    bg = rs.uniform(0, 255, (n, size, size, 3))
    yy, xx = np.mgrid[:size, :size]
    gt = np.clip(1.2 - np.hypot((yy - size / 2) / (size / 3), (xx - size / 2) / (size / 4)), 0, 1)
    gt = np.repeat(gt[None, :, :, None], n, 0)
    cmp = gt * fg + (1 - gt) * bg - mean
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    cmp_d, bg_d, gt_d, fg_d = T(cmp), T(bg - mean), T(gt), T(fg)
    np.random.seed(4)
    trn = ImageTrainer(svgg(0), dtype, dev, streams=streams)
    g = trn.capture(cmp_d, bg_d, gt_d, fg_d) if graph else None
    for _ in range(warmup):
        if g is not None:
            g.step()
        else:
            trn.step(cmp_d, bg_d, gt_d, fg_d)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = Events()
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.mark()
        if g is not None:
            g.g_fwd.replay()
        else:
            trn.forward(cmp_d, bg_d)
            trn._g["loss"].copy_(ops.matting_loss(trn.model.output, gt_d, fg_d, bg_d, cmp_d))
        ev.mark()
        if g is not None:
            g.g_bwd.replay()
        else:
            trn.grad.zero_()
            trn.backward(gt_d, fg_d, bg_d, cmp_d)
        ev.mark()
        trn.apply_gradients()
        ev.mark()
    torch.cuda.synchronize()
    wall = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall)
    e = ev.e
    ph = [sum(ms(e[4 * i + k], e[4 * i + k + 1]) for i in range(steps)) / steps for k in range(3)]
    dev_ms = sum(ph)
    per_step = sorted(ms(e[4 * i], e[4 * i + 3]) for i in range(steps))
    fwd_f, bwd_f = trn.conv_flops(n, size, size)
    pk = PEAK_TFLOPS[dtype]
    tf = (fwd_f + bwd_f) / (dev_ms * 1e-3) / 1e12
    rec = {"workload": "train.py training_procedure step: %d x %dx%d per GPU, unet.UNetImage([cmp, bg]) fwd/bwd over "
                       "all variables (VGG included), loss, DDP all-reduce, TF-Adam" % (n, size, size),
           "dtype": dtype + " forward / MFMA gradients, f32 gradients/optimizer", "n_gpus": world,
           "launch": "hip-graph replay of forward+loss and of backward (one stream), eager all-reduce + Adam + "
                     "re-pack" if graph else "eager" + ("; filter gradients on a side stream" if streams else ""),
           "samples_per_s": round(n * world / wall, 1), "ms_per_step": round(1000 * wall, 4),
           "device_ms": {"forward_loss": round(ph[0], 4), "backward": round(ph[1], 4),
                         "allreduce_adam_repack": round(ph[2], 4)},
           "device_ms_per_step": {"min": round(per_step[0], 4), "median": round(per_step[len(per_step) // 2], 4),
                                  "max": round(per_step[-1], 4)},
           "flops_per_step_per_gpu": {"forward": fwd_f, "backward": bwd_f},
           "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": pk, "unit": "TFLOP/s",
                        "frac": round(tf / pk, 4),
                        "def": "algorithmic conv FLOPs of the step (forward 20 convs + 20 filter gradients + 19 data "
                               "gradients, 2*H*W*9*cin*cout each) over the step's device time (HIP events)"},
           "loss_last": [round(float(v), 5) for v in trn._g["loss"].cpu()]}
    if cpu and world == 1:
        from oracle import models as om  # the CPU-baseline leg only
        from oracle import train_ref as tr
        p = om.unet_params(om.synthetic_vgg16(0), np.random.RandomState(4), video=False)
        sl = lambda a: np.asarray(a[:1], np.float64)  # noqa: E731
        best = None
        for _ in range(2):
            t0 = time.perf_counter()
            tr.image_step_grads(sl(cmp), sl(bg - mean), sl(gt), sl(fg), p)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        rec["cpu_baseline"] = {"value": round(1.0 / best, 4), "unit": "samples/s", "cores": threads, "kind": "port",
                               "sample": "oracle/train_ref.py image_step_grads (torch-f64 autograd of UNetImage) on "
                                         "one %dx%d sample (the config's sample size), best of 2" % (size, size)}
    return rec


def train_chain_bench(dev, steps, warmup, n=8, size=320, h=1080, w=1920, dtype="bf16", graph=False, overlap=True,
                      profiler=None, prio=False):
    """BASELINE config 5 as ONE pipeline per step (rank 0, N=1): augmentation.augment makes frame t of each of n
    1080p source samples resident in HBM (augmentation.py:102-135: host np.random draws + TPS solves, the device
    statistics / TPS lattice / resampling / fused warps + illumination — augment_many, one landmark upload, no sync),
    the video loader's crops / warp / resize / composite turn the n (frame t, bg, frame t-1, flow) entries into an
    n x size^2 batch (loader.py:285-330, host crop draws) written straight into the captured training step's input
    buffers, then the step (train.py:318-332) replays from its HIP graphs.  Pipelined: the next batch's foreground
    statistics are launched on a side stream before this step, so the host's only wait (their readback) overlaps the
    training step, and the next batch's draws / TPS solves / launches happen while it runs.  graph=False: the step's
    eager launches with the select chains on side streams (HIP graph replay runs those branches one after another:
    slower when the host keeps ahead, as it does here).  No decoding: the source
    images are synthetic device tensors (PNG/JPEG decode is host I/O outside the path).  Wall ms per phase and device
    ms per phase (HIP events on the launch stream)."""
    from vmatting import augmentation as va
    from vmatting import loader as vl
    from vmatting.train import VideoTrainer
    rs = np.random.RandomState(12)
    yy, xx = np.mgrid[0:h, 0:w]
    src = []
    for i in range(n):
        al = np.clip(1.2 - np.sqrt(((yy - (0.4 + 0.02 * i) * h) / (0.28 * h)) ** 2 +
                                   ((xx - 0.47 * w) / (0.21 * w)) ** 2), 0, 1)
        src.append(tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
                         ((rs.rand(h, w, 3) * 255).astype(np.uint8), (rs.rand(h, w, 3) * 255).astype(np.uint8), al)))
    alphas = [t[2] for t in src]
    flow = torch.from_numpy(synthetic_flow(h, w, 11, amp=12.0)).to(dev)
    np.random.seed(7)
    # (prio: the step's streams at the greatest priority, the producer at 0 — measured on MI355X: the step at high
    # queue priority ran 9.4 ms against 5.6, so the overlap keeps every stream at the default priority)
    hi = torch.cuda.Stream.priority_range()[1] if (overlap and prio) else 0
    trn = VideoTrainer(synthetic_vgg16(0), dtype, dev, stream_priority=hi)
    names = ("cmp", "bg", "label", "warped", "fg")

    def batch(stats, out=None):
        samples = va.video_samples(src, flow, stats=stats)
        for smp in samples:
            smp["plan"] = vl.plan_crop((h, w), (h, w))
        return samples

    if overlap:
        if hi != 0:
            with torch.cuda.stream(torch.cuda.Stream(device=dev, priority=hi)):
                rec = _train_chain_overlap(dev, steps, warmup, trn, batch, alphas, n, size, names, dtype, graph,
                                           profiler)
            rec["launch"] += "; step streams at priority %d, producer at 0" % hi
            return rec
        return _train_chain_overlap(dev, steps, warmup, trn, batch, alphas, n, size, names, dtype, graph, profiler)
    r = vl.compose_batch(batch(va.StatsPrefetch(alphas).result()), (size, size), names, device=dev)
    if graph:
        g = trn.capture(r["cmp"], r["bg"], r["warped"], r["label"], r["fg"])
        ins = g.inputs
    else:
        g, ins = None, [r["cmp"], r["bg"], r["warped"], r["label"], r["fg"]]
    outs = dict(zip(("cmp", "bg", "warped", "label", "fg"), ins))
    state = {"pending": va.StatsPrefetch(alphas)}

    def one(ev=None, wall=None):
        t0 = time.perf_counter()
        ev and ev.mark()
        samples = batch(state["pending"].result())
        t1 = time.perf_counter()
        ev and ev.mark()
        vl.compose_batch(samples, (size, size), names, device=dev, out=outs)
        state["pending"] = va.StatsPrefetch(alphas)  # the next batch's statistics, ahead of this step
        t2 = time.perf_counter()
        ev and ev.mark()
        loss = g.step() if g is not None else trn.step(*ins)
        ev and ev.mark()
        t3 = time.perf_counter()
        if wall is not None:
            wall.append((t1 - t0, t2 - t1, t3 - t2))
        return loss

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    ev, wall = Events(), []
    profiler and profiler.enable()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = one(ev, wall)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    profiler and profiler.disable()
    e = ev.e
    dev_ms = [sum(ms(e[4 * i + k], e[4 * i + k + 1]) for i in range(steps)) / steps for k in range(3)]
    host_ms = [1e3 * sum(wl[k] for wl in wall) / steps for k in range(3)]
    return {"workload": "config 5 chained: augmentation.augment on %d 1080p sources -> loader video_batch per-pixel "
                        "work -> %dx%d -> VideoTrainer step (%s forward, f32 gradients / Adam)" % (n, size, size, dtype),
            "samples_per_s": round(n / dt, 1), "ms_per_step": round(1e3 * dt, 3),
            "device_ms": {"augment": round(dev_ms[0], 3), "loader": round(dev_ms[1], 3),
                          "train_step": round(dev_ms[2], 3)},
            "host_issue_ms": {"augment_stats_wait_draws_tps_solve_launch": round(host_ms[0], 3),
                              "loader_crop_draws_launch_next_stats": round(host_ms[1], 3),
                              "train_step_launches_adam": round(host_ms[2], 3)},
            "launch": "augment + loader eager (one statistics readback per batch, prefetched on a side stream), "
                      "training step %s" % ("replayed from HIP graphs" if graph else
                                            "eager with the select chains on side streams"),
            "decode": "none: synthetic source images resident in HBM (PNG/JPEG decoding is host I/O outside the path)",
            "loss_last": [round(float(v), 5) for v in loss.cpu()]}


def augment_bytes(h, w):
    """augment_bench's algorithmic bytes of one augmentation.augment sample (per pixel: alpha stats 8; bg two warps
    2*(3+3); TPS grid (h/2)(w/2)*16 = 4; fg TPS 3+3, alpha TPS 8+8; fg two warps 2*(3+3); alpha two warps 2*(8+8);
    illumination fg+bg 2*(3+3))."""
    return h * w * (8 + 12 + 4 + 6 + 16 + 12 + 32 + 12)


def chain_roofline_and_baseline(rec, n, size, h, w, dtype, threads, cpu):
    """train.chained's roofline and CPU baseline: the pipeline's algorithmic work per batch —
    augment of n 1080p sources + the loader's per-pixel work + one config-5 step (its MFMA FLOPs and memory-bound
    bytes) — at the MFMA / HBM peaks, over the measured wall time per step (the phases overlap on two streams, so
    wall, not a phase sum, is what the roofline is compared with).  CPU baseline: the oracle's augment of one 1080p
    source, the oracle loader on one 1080p video entry and oracle/train_ref's step on one 320^2 sample, in turn."""
    fwd_f, bwd_f = train_flops(n, size, size)
    nbytes = (n * augment_bytes(h, w) + n * size * size * 13 * 4 + n * 4 * size * size * (4 + 8 + 4 + 3)
              + train_step_traffic(n, size, size, 2 if dtype == "bf16" else 4))
    rl = step_roofline(fwd_f + bwd_f, nbytes, rec["ms_per_step"], PEAK_TFLOPS[dtype])
    rl["def"] = ("roofline_ms = the step's algorithmic conv FLOPs / dense MFMA peak + (augment of %d 1080p sources + "
                 "loader per-pixel bytes + the step's memory-bound bytes) / 8 TB/s; frac = roofline_ms / measured "
                 "wall ms per step (augment + loader of batch k+1 overlap step k)" % n)
    rl.pop("measured_device_ms")
    rl["measured_wall_ms"] = rec["ms_per_step"]
    rec["roofline"] = rl
    if not cpu:
        return rec
    from oracle import augment as oa  # the CPU-baseline leg only
    from oracle import loader as ol
    from oracle import models as om
    from oracle import train_ref as tr
    rs = np.random.RandomState(13)
    yy, xx = np.mgrid[0:h, 0:w]
    al = np.clip(1.2 - np.sqrt(((yy - 0.4 * h) / (0.28 * h)) ** 2 + ((xx - 0.47 * w) / (0.21 * w)) ** 2), 0, 1)
    fg = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    bg = (rs.rand(h, w, 3) * 255).astype(np.uint8)
    np.random.seed(0)
    t0 = time.perf_counter()
    oa.augment(fg, bg, al)
    t_aug = time.perf_counter() - t0
    ent = loader_inputs(1, h, w)[0]
    np.random.seed(0)
    from vmatting import loader as vl
    plan = vl.plan_crop((h, w), (h, w))
    t0 = time.perf_counter()
    fr, fc, br, bc = (ol.Axis(*a) for a in plan)
    srcs = ol.crop_sources(ent["fg"], ent["bg"], fr, fc, br, bc, ent["prev"], ent["flow"])
    ol.compose(srcs[0], srcs[1], srcs[3], (size, size), srcs[2])
    t_ldr = time.perf_counter() - t0
    mean = np.array(VGG_MEAN)
    rs = np.random.RandomState(100)
    f1 = rs.uniform(0, 255, (1, size, size, 3))
    b1 = rs.uniform(0, 255, (1, size, size, 3))
    g1 = rs.uniform(0, 1, (1, size, size, 1))
    c1 = g1 * f1 + (1 - g1) * b1 - mean
    p = om.unet_simple_params(np.random.RandomState(1))
    t0 = time.perf_counter()
    tr.train_step_grads(c1, b1 - mean, np.repeat(g1, 3, -1), g1, f1, synthetic_vgg16(0), p)
    t_step = time.perf_counter() - t0
    tot = t_aug + t_ldr + t_step
    rec["cpu_baseline"] = {"value": round(1.0 / tot, 5), "unit": "samples/s", "cores": threads, "kind": "port",
                           "sample": "one sample through the oracle chain in turn: oracle/augment.py augment of one "
                                     "%dx%d source (%.2f s), oracle/loader.py crop + warp + resize + composite of one "
                                     "%dx%d video entry to %dx%d (%.2f s), oracle/train_ref.py step of one %dx%d "
                                     "sample (%.2f s)" % (w, h, t_aug, w, h, size, size, t_ldr, size, size, t_step)}
    return rec


def _train_chain_overlap(dev, steps, warmup, trn, batch, alphas, n, size, names, dtype, graph, profiler=None):
    """train_chain_bench's pipelined form: batch k+1's augment + loader run on a producer stream while step k runs
    on the caller's stream (the data pipeline of a training job overlapping its step, as a prefetching loader
    does).  Two batch slots: the producer fills slot (k+1) % 2 after the step that read it has finished (event),
    the step waits for its slot's ready event.  Same batches, same order, same step: only the overlap differs
    from the serial form.  Host per step: the step's launches (graph: two replays), then batch k+1's draws / TPS
    solves / launches."""
    from vmatting import augmentation as va
    from vmatting import loader as vl
    main = torch.cuda.current_stream(dev)
    prod = torch.cuda.Stream(device=dev)
    ready = [torch.cuda.Event(), torch.cuda.Event()]
    freed = [torch.cuda.Event(), torch.cuda.Event()]
    slots = [None, None]
    pev = {}  # producer-stream timing events of the timed steps

    def produce(k, stats, timed):
        s = k % 2
        with torch.cuda.stream(prod):
            prod.wait_event(freed[s])  # the step that read this slot is done (never-recorded events: no wait)
            e0 = torch.cuda.Event(enable_timing=True) if timed else None
            e0 and e0.record()
            samples = batch(stats)
            e1 = torch.cuda.Event(enable_timing=True) if timed else None
            e1 and e1.record()
            slots[s] = vl.compose_batch(samples, (size, size), names, device=dev, out=slots[s])
            ready[s].record(prod)
            if timed:
                e2 = torch.cuda.Event(enable_timing=True)
                e2.record()
                pev[k] = (e0, e1, e2)
            # the next batch's foreground statistics, behind this batch on the producer stream
            return va.StatsPrefetch(alphas)

    # batch 0 = the serial form's first batch: it sizes the slots (and is what a graph is captured on), the steps
    # start at batch 1 in both forms
    pending = produce(0, va.StatsPrefetch(alphas).result(), False)
    main.wait_event(ready[0])
    g = None
    if graph:
        r = slots[0]
        g = trn.capture(r["cmp"], r["bg"], r["warped"], r["label"], r["fg"])
    freed[0].record(main)
    pending = produce(1, pending.result(), False)

    def one(k, timed, sev=None):
        s = k % 2
        r = slots[s]
        main.wait_event(ready[s])
        if sev is not None:
            sev.append(torch.cuda.Event(enable_timing=True))
            sev[-1].record(main)
        ins = (r["cmp"], r["bg"], r["warped"], r["label"], r["fg"])
        if g is not None:
            g.load(*ins)  # the graph's static inputs (on the caller's stream), then the slot is free again
            freed[s].record(main)
            loss = g.step()
        else:
            loss = trn.step(*ins)
            freed[s].record(main)
        if sev is not None:
            sev.append(torch.cuda.Event(enable_timing=True))
            sev[-1].record(main)
        return loss, produce(k + 1, pending_box[0].result(), timed)

    pending_box = [pending]
    k = 1
    for _ in range(warmup):
        loss, pending_box[0] = one(k, False)
        k += 1
    torch.cuda.synchronize()
    sev = []
    k0 = k
    profiler and profiler.enable()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss, pending_box[0] = one(k, True, sev)
        k += 1
    # both streams drained: the timed region also holds the batch produced behind the last step (the first timed
    # step's batch was produced before it), so it is one full pipeline period per step
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    profiler and profiler.disable()
    step_ms = sum(ms(sev[2 * i], sev[2 * i + 1]) for i in range(steps)) / steps
    aug_ms = sum(ms(pev[k][0], pev[k][1]) for k in range(k0 + 1, k0 + steps + 1)) / steps
    ldr_ms = sum(ms(pev[k][1], pev[k][2]) for k in range(k0 + 1, k0 + steps + 1)) / steps
    return {"workload": "config 5 chained: augmentation.augment on %d 1080p sources -> loader video_batch per-pixel "
                        "work -> %dx%d -> VideoTrainer step (%s forward, f32 gradients / Adam)" % (n, size, size, dtype),
            "samples_per_s": round(n / dt, 1), "ms_per_step": round(1e3 * dt, 3),
            "device_ms": {"augment": round(aug_ms, 3), "loader": round(ldr_ms, 3), "train_step": round(step_ms, 3)},
            "device_ms_def": "HIP events on each phase's own stream; augment + loader of batch k+1 (producer stream) "
                             "run concurrently with step k (training stream), so the phases overlap",
            "launch": "pipelined: augment + loader of the next batch on a producer stream (two batch slots, events) "
                      "beside the training step %s" % ("replayed from HIP graphs" if graph else
                                                       "(eager, select chains on side streams)"),
            "decode": "none: synthetic source images resident in HBM (PNG/JPEG decoding is host I/O outside the path)",
            "loss_last": [round(float(v), 5) for v in loss.cpu()]}


# ------------------------------------------------------------------------------------------------ roofline

def load_profile(kind, args):
    """Per-launch PMC values per kernel from the committed rocprofv3 passes (tools/pmc_passes.py ->
    profiles/*_<kind>.json), used only when collected on this exact workload."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_%s.json" % kind)), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        c = t.get("config", {})
        if (c.get("dtype"), c.get("height"), c.get("width"), c.get("batch")) == (args.dtype, args.height, args.width,
                                                                               args.batch):
            return os.path.relpath(path, REPO), t
    return None, None


def conv_roofline(prof, args):
    """Roofline of the dominant conv kernel (largest share of conv time): ALGORITHMIC flops per launch
    (2*H*W*9*cin*cout of each launch) / its average launch duration from HIP events on
    the launch stream, recorded over a K-step pass identical to the timed region (run right after it)."""
    per = {}
    for fl, name, e0, e1, *_ in prof:
        d = per.setdefault(name, [0, 0.0, 0])
        d[0] += fl
        d[1] += ms(e0, e1)
        d[2] += 1
    name, (fl, t, n) = max(per.items(), key=lambda kv: kv[1][1])
    achieved = fl / (t * 1e-3) / 1e12
    peak = PEAK_TFLOPS[args.dtype]
    src_t, traffic = load_profile("traffic", args)
    tr = (traffic or {}).get("kernels", {}).get(name)
    src_m, mf = load_profile("mfma", args)
    mk = (mf or {}).get("kernels", {}).get(name)
    all_fl = sum(v[0] for k, v in per.items() if "head" not in k)
    all_ms = sum(v[1] for k, v in per.items() if "head" not in k)
    if args.layers:
        per_step = len(prof) // max(1, args.steps)
        for i in range(per_step):
            rows = prof[i::per_step]
            t_ms = sum(ms(r[2], r[3]) for r in rows) / len(rows)
            log("  conv #%2d %-55s %.3f ms  %.1f TFLOP/s" % (i, rows[0][1], t_ms, rows[0][0] / (t_ms * 1e-3) / 1e12))
    for k, (f, tt, c) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        log("%-58s %3d launches %.3f ms/step %.1f TFLOP/s" % (k, c, tt / args.steps, f / (tt * 1e-3) / 1e12))
    rec = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
           "frac": round(achieved / peak, 4), "traffic": tr["bytes_per_launch"] if tr else None,
           "kernel": name, "launches": n, "avg_launch_ms": round(t / n, 4), "flops_per_launch": int(fl / n),
           "traffic_source": ("%s (FETCH_SIZE x2 + WRITE_SIZE, per launch)" % src_t) if tr else None,
           "all_mfma_convs": {"tflops": round(all_fl / (all_ms * 1e-3) / 1e12, 2),
                              "ms_per_step": round(all_ms / args.steps, 4),
                              "frac": round(all_fl / (all_ms * 1e-3) / 1e12 / peak, 4)}}
    if mk:
        # SQ_VALU_MFMA_BUSY_CYCLES: SIMD-cycles the matrix pipes were busy (all SIMDs, one launch);
        # GRBM_GUI_ACTIVE / 8: the launch's GPU cycles (summed over the 8 XCDs by rocprofv3)
        cyc = mk["GRBM_GUI_ACTIVE"] / 8.0
        rec["mfma_util"] = round(mk["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * cyc), 4)
        rec["mfma_counters"] = {"source": src_m, "measured_in_this_run": False,
                                "note": "copied from the committed rocprofv3 --pmc pass over the same workload "
                                        "(tools/prof_bench.sh), not measured by this process", "SQ_VALU_MFMA_BUSY_CYCLES": mk["SQ_VALU_MFMA_BUSY_CYCLES"],
                                "GRBM_GUI_ACTIVE": mk["GRBM_GUI_ACTIVE"], "SQ_BUSY_CYCLES": mk.get("SQ_BUSY_CYCLES"),
                                "effective_clock_ghz": round(cyc / (t / n * 1e-3) / 1e9, 3),
                                "def": "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8): "
                                       "matrix-pipe busy fraction at the clock the chip actually held"}
    return rec


# ------------------------------------------------------------------------------------------------ launcher

def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """One child process of this script per rank (BASELINE metric at 1/2/4/8 GPUs), with torchrun's
    environment contract.  The parent never touches a GPU (no HIP call, no torch.cuda initialisation) and never
    re-execs itself: it only waits.  When a rank fails the others are stopped (they would block in a collective).
    Returns rank 0's exit code, or the first failing rank's."""
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
        rcs = [None] * n
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            failed = [r for r in range(n) if rcs[r] not in (None, 0)]
            if failed:
                log("bench launcher: rank %d exited with %d; stopping the other ranks" % (failed[0], rcs[failed[0]]))
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                for p in procs:
                    try:
                        p.wait(30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        p.wait()
                return rcs[failed[0]]
            time.sleep(0.2)
        return rcs[0]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()


def dist_selftest(rank, world):
    """CPU-only (gloo) check of what the multi-GPU run relies on, through the same launcher: the weight broadcast
    from rank 0 (parallel.broadcast_tensors) and the matte all-gather of an uneven frame split
    (parallel.gather_frames, config 4).  Rank 0 prints one JSON line."""
    n_frames = 2 * world + 1  # uneven: the first ranks get 2 frames, the last 3
    wts = [torch.arange(64, dtype=torch.float32) * (rank + 1), torch.full((3, 5), float(rank), dtype=torch.float64)]
    parallel.broadcast_tensors(wts, src=0)
    ok_b = torch.equal(wts[0], torch.arange(64, dtype=torch.float32)) and bool((wts[1] == 0).all())
    a, b = parallel.shard_range(n_frames, rank, world)
    local = torch.arange(a, b, dtype=torch.float32).view(-1, 1, 1, 1).expand(b - a, 4, 6, 1).contiguous()
    full = parallel.gather_frames(local, n_frames)
    ok_g = tuple(full.shape) == (n_frames, 4, 6, 1) and all(bool((full[i] == i).all()) for i in range(n_frames))
    ok = torch.tensor([1 if ok_b and ok_g else 0], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"selftest": "dist", "n_gpus": world, "backend": dist.get_backend(), "frames": n_frames,
                          "split": [list(parallel.shard_range(n_frames, r, world)) for r in range(world)],
                          "broadcast_ok": ok_b, "gather_ok": ok_g, "ok": bool(ok.item())}), flush=True)
    return 0 if ok.item() else 1


# ------------------------------------------------------------------------------------------------ main

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1, help="frames per step per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=3, help="full 1080p frames timed for the CPU baseline (median)")
    ap.add_argument("--no-profile", action="store_true", help="skip per-conv HIP events")
    ap.add_argument("--layers", action="store_true", help="per-conv timing breakdown on stderr")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches instead of the captured HIP graph")
    ap.add_argument("--no-up-head", action="store_true",
                    help="upconv_4 stores its output and the head reads it (A/B of the fused up-head)")
    ap.add_argument("--no-split-head", action="store_true",
                    help="conv1_5 over the whole cat1 instead of the pair kernel's head split (A/B)")
    ap.add_argument("--no-loader", action="store_true", help="skip the training-sample loader record (rank 0, N=1)")
    ap.add_argument("--no-augment", action="store_true", help="skip the augmentation record (rank 0, N=1)")
    ap.add_argument("--no-train", action="store_true", help="skip the config-5 training-step record (all ranks)")
    ap.add_argument("--no-temporal", action="store_true", help="skip the config-3 record (rank 0)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 record and the parity block (rank 0)")
    ap.add_argument("--video-frames", type=int, default=256,
                    help="config-4 record: frames sharded over the ranks + matte all-gather (0 = skip)")
    ap.add_argument("--video-chunk", type=int, default=8, help="frames per HIP graph in the config-4 record")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="vm_set_option kernel knob before the run (A/B comparisons), repeatable")
    ap.add_argument("--train-graph", action="store_true",
                    help="config-5 record from HIP-graph replays (VideoTrainer.capture) instead of eager launches: "
                         "the step is not host-bound, and the graph runs the side-stream select chains serially")
    ap.add_argument("--chain-prio", action="store_true",
                    help="config-5 chained record: the step's streams at the greatest priority (A/B; slower)")
    ap.add_argument("--chain-serial", action="store_true",
                    help="config-5 chained record without the producer-stream overlap (augment, loader, step in turn)")
    ap.add_argument("--train-streams", type=int, default=3,
                    help="side streams of the config-5 trainer's select chains (0: one stream, for serial profiles)")
    ap.add_argument("--train-wgrad-stream", type=int, default=1,
                    help="config-5 trainer: 1 = the decoder chain's filter gradients on their own side stream")
    ap.add_argument("--image-graph", action="store_true",
                    help="train_image record from HIP-graph replays (one stream) instead of eager launches")
    ap.add_argument("--image-streams", type=int, default=1,
                    help="train_image: 1 = filter gradients on a side stream beside the data-gradient chain, 0 = one")
    ap.add_argument("--only", choices=["train", "train_chain", "train_small", "train_image", "temporal", "augment",
                                       "loader"],
                    help="profiling passes: run just this record (rank 0 / N=1) and print it")
    ap.add_argument("--temporal-sizes", default="500x1200,1080x1920", help="config-3 sizes HxW, comma separated")
    ap.add_argument("--temporal-dtypes", default="fp32,bf16", help="config-3 compute dtypes, comma separated")
    ap.add_argument("--train-side", default=None, choices=["pool", "probe"],
                    help="config-5 trainer side streams: torch pool streams, or pool streams probed to run beside the "
                         "caller's (VideoTrainer.side_kind; default: the class default)")
    ap.add_argument("--cooldown", type=float, default=5.0,
                    help="seconds of GPU idle before each training record (outside the timed regions)")
    ap.add_argument("--dummy-streams", type=int, default=0,
                    help="(study) create this many idle HIP streams first: how the trainers' side streams map onto "
                         "the hardware queues when a process already holds streams")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU-only: the N-rank launcher + gloo broadcast / uneven all-gather, no GPU")
    args = ap.parse_args()
    t_sizes = [tuple(int(v) for v in hw.split("x")) for hw in args.temporal_sizes.split(",")]
    t_dtypes = args.temporal_dtypes.split(",")

    if args.gpus < 1:
        log("bench: --gpus must be >= 1")
        return 2
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # this process is the launcher: it starts the N ranks and makes no torch.cuda / HIP call at all (on ROCm
        # torch.cuda.device_count() can fall back to a HIP-initialising query; a child started from a GPU-initialised
        # parent is the pattern this pool forbids) — each rank checks the visible GPUs itself
        return launch_ranks(args.gpus, sys.argv[1:])
    if not args.dist_selftest:
        need = int(os.environ.get("WORLD_SIZE", args.gpus))
        if torch.cuda.device_count() < need:  # a rank process (or the N=1 run): checked before any GPU work
            log("bench: %d rank(s) need %d GPU(s), %d visible" % (need, need, torch.cuda.device_count()))
            return 2

    rank, world, local = parallel.init_from_env("gloo" if args.dist_selftest else "nccl")
    if world != args.gpus:
        log("bench: --gpus %d but the initialised world has %d rank(s)" % (args.gpus, world))
        if dist.is_initialized():
            dist.destroy_process_group()
        return 2
    if args.dist_selftest:
        rc = dist_selftest(rank, world) if world > 1 else 0
        if world == 1:
            print(json.dumps({"selftest": "dist", "n_gpus": 1, "ok": True}), flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()
        return rc
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    for kv in args.option:
        k, v = kv.split("=")
        from vmatting import _lib
        _lib.set_option(k, int(v))
    cpu_model, threads = host_info()
    _dummy = [torch.cuda.Stream(device=dev) for _ in range(args.dummy_streams)]  # noqa: F841 (study knob)
    if args.only:  # one record alone (rocprofv3 passes per record: tools/prof_bench.sh)
        if args.only == "train":
            set_train_side(args.train_side)
            rec = train_bench(dev, args.steps, args.warmup, world, rank, threads, cpu=False, graph=args.train_graph,
                              streams=args.train_streams, wgrad_stream=bool(args.train_wgrad_stream))
        elif args.only == "train_chain":
            rec = chain_roofline_and_baseline(
                train_chain_bench(dev, args.steps, args.warmup, graph=args.train_graph, overlap=not args.chain_serial,
                                  prio=args.chain_prio), 8, 320, 1080, 1920, "bf16", threads, False)
        elif args.only == "train_small":
            rec = train_small_bench(dev, args.steps, args.warmup, world, rank, threads, cpu=False)
        elif args.only == "train_image":
            rec = train_image_bench(dev, args.steps, args.warmup, world, rank, threads, cpu=False,
                                    graph=args.image_graph, streams=args.image_streams)
        elif args.only == "augment":
            rec = augment_bench(dev, args.steps, threads, cpu=False)
        elif args.only == "loader":
            rec = loader_bench(dev, args.steps, threads, cpu=False)
        else:
            rec = temporal_bench(dev, args.steps, t_dtypes, t_sizes, False, threads)
        if rank == 0:
            print(json.dumps({"only": args.only, "record": rec}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    # identical weights everywhere: every rank draws from the same seeds, then rank 0's packed
    # buffers are broadcast (one RCCL collective) so replicas are bit-identical by construction
    vgg = synthetic_vgg16(0)
    np.random.seed(0)
    model = unet.UNetVideo(vgg, dtype=args.dtype, device=dev)
    model.split_head = not args.no_split_head
    model.fuse_up_head = not args.no_up_head
    model.prepare()
    parallel.broadcast_tensors(model.weights_flat(), src=0)

    B, H, W = args.batch, args.height, args.width
    x = video.synthetic_frames(B, H, W, first=rank * B, device=dev)
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
    alpha_timed = (graphed.output if graphed is not None else model.output).clone()
    logits_timed = model.conv1_3.clone()

    # per-kernel HIP events cost ~10% of the step (a marker between every launch), so the roofline pass is a
    # second, identical K-step pass with an event pair on the launch stream around every conv
    prof = None
    if not args.no_profile:
        prof = ops.conv_profile(True)
        for _ in range(args.steps):
            model.forward(x)
        torch.cuda.synchronize()
        ops.conv_profile(False)

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = world * B * args.steps
    value = frames / elapsed
    ms_step = 1000.0 * elapsed / args.steps

    vrec = None
    if args.video_frames > 0:
        vrec = video_batch(model, args.video_frames, H, W, rank, world, dev, args.video_chunk)

    # each training / config-3 / loader / augment record starts from an idle GPU (no record inherits its predecessor's
    # queued work); the pause is outside every timed region.  (It does not decide the UNetImage step's slow mode:
    # DESIGN §3.9, profiles/r06m_img_trainer_instances.log)
    def cool():
        if args.cooldown > 0:
            torch.cuda.synchronize()
            time.sleep(args.cooldown)

    train = None
    if not args.no_train:  # every rank: the DDP all-reduce is part of the step
        cool()
        set_train_side(args.train_side)
        train = train_bench(dev, max(args.steps // 4, 10), 3, world, rank, threads, cpu=not args.no_cpu_baseline,
                            graph=args.train_graph, streams=args.train_streams,
                            wgrad_stream=bool(args.train_wgrad_stream))
        if world == 1:
            cool()
            train["chained"] = chain_roofline_and_baseline(
                train_chain_bench(dev, 5, 2, graph=args.train_graph, overlap=not args.chain_serial,
                                  prio=args.chain_prio), 8, 320, 1080, 1920, "bf16", threads, not args.no_cpu_baseline)
        cool()
        train_small = train_small_bench(dev, max(args.steps // 4, 10), 3, world, rank, threads,
                                        cpu=not args.no_cpu_baseline)
        cool()
        train_image = train_image_bench(dev, max(args.steps // 4, 10), 5, world, rank, threads,
                                        cpu=not args.no_cpu_baseline, graph=args.image_graph,
                                        streams=args.image_streams)

    roofline = conv_roofline(prof, args) if prof else None
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
        src, tr = load_profile("traffic", args)
        if tr and tr.get("bytes_per_forward"):
            # whole-forward HBM traffic (PMC FETCH_SIZE x2 + WRITE_SIZE summed over every kernel of one forward,
            # one-time weight packing excluded) at this run's frame rate
            bpf = tr["bytes_per_forward"] / float(args.batch)
            rec["achieved_hbm_gbps"] = round(bpf * value / world / 1e9, 1)
            rec["hbm"] = {"bytes_per_frame": int(bpf), "achieved_gbps_per_gpu": rec["achieved_hbm_gbps"],
                          "peak_gbps": PEAK_HBM_GBPS, "frac": round(bpf * value / world / 1e9 / PEAK_HBM_GBPS, 4),
                          "source": src}
        if world == 1 and not args.no_fp32:
            params = model.params
            fp32, m32 = fp32_record(model, x, 10, vgg, params)
            rec["fp32"] = fp32
            a32 = m32.output.clone()
            l32 = m32.conv1_3.clone()
            del m32
            x3, m3 = split_record(x, 10, vgg, params, "f16x3")
            rec["f16x3"] = x3
            a3 = m3.output.clone()
            del m3
            x6, m6 = split_record(x, 10, vgg, params, "bf16x6")
            rec["bf16x6"] = x6
            a6 = m6.output.clone()
            del m6
            par = {"frame": "the timed %dx%d frame (seed 1234)" % (W, H),
                   "bf16_vs_fp32_alpha_maxabs": float((alpha_timed - a32).abs().max()) if args.dtype == "bf16"
                   else 0.0,
                   "bf16_logits_rel": float((logits_timed - l32).abs().max() / l32.abs().max())
                   if args.dtype == "bf16" else 0.0,
                   # the max sits on the few pixels whose logit crosses 0 with a steep sigmoid (|logits| reach
                   # O(100) with synthetic weights): also the mean and the 99.9th percentile of |alpha error|
                   "bf16_vs_fp32_alpha_meanabs": float((alpha_timed - a32).abs().mean()) if args.dtype == "bf16"
                   else 0.0,
                   "bf16_vs_fp32_alpha_p999": float(torch.quantile((alpha_timed - a32).abs().flatten()[::7].float(),
                                                                   0.999)) if args.dtype == "bf16" else 0.0,
                   "fp32_logits_absmax": float(l32.abs().max()),
                   "bound": 1e-4, "bound_applies_to": "fp32 alpha vs the reference CPU forward (north_star)"}
            if not args.no_cpu_baseline:
                crec, ref = cpu_baseline(x[:1].cpu().numpy(), params, args.cpu_frames, threads, cpu_model,
                                         flops_per_frame)
                rec["cpu_baseline"] = crec
                par["fp32_vs_oracle_alpha_maxabs"] = float(np.abs(a32[:1].cpu().numpy() - ref["output"]).max())
                par["fp32_vs_oracle_logits_rel"] = float(np.abs(l32[:1].cpu().numpy() - ref["conv1_3"]).max()
                                                         / np.abs(ref["conv1_3"]).max())
                par["bf16_vs_oracle_alpha_maxabs"] = float(np.abs(alpha_timed[:1].cpu().numpy()
                                                                  - ref["output"]).max())
                par["bf16x6_vs_oracle_alpha_maxabs"] = float(np.abs(a6[:1].cpu().numpy() - ref["output"]).max())
                par["f16x3_vs_oracle_alpha_maxabs"] = float(np.abs(a3[:1].cpu().numpy() - ref["output"]).max())
                par["f16x3_meets_bound"] = par["f16x3_vs_oracle_alpha_maxabs"] <= 1e-4
                par["fp32_meets_bound"] = par["fp32_vs_oracle_alpha_maxabs"] <= 1e-4
                par["bf16_meets_bound"] = par["bf16_vs_oracle_alpha_maxabs"] <= 1e-4
                par["bf16x6_meets_bound"] = par["bf16x6_vs_oracle_alpha_maxabs"] <= 1e-4
            rec["parity"] = par
        if vrec:
            rec["video_batch"] = vrec
        if world == 1 and not args.no_temporal:
            cool()
            rec["temporal"] = temporal_bench(dev, 20, t_dtypes, t_sizes, not args.no_cpu_baseline, threads)
        if train:
            rec["train"] = train
            rec["train_small"] = train_small
            rec["train_image"] = train_image
            for r in (train, train_small, train_image):
                r["idle_before_s"] = args.cooldown
        if world == 1 and not args.no_loader:
            cool()
            rec["loader"] = loader_bench(dev, max(args.steps // 4, 10), threads, cpu=not args.no_cpu_baseline)
        if world == 1 and not args.no_augment:
            cool()
            rec["augment"] = augment_bench(dev, max(args.steps // 4, 10), threads, cpu=not args.no_cpu_baseline)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
