"""augmentation.py (synthetic video-matting samples) on gfx950 kernels — SURVEY.md §8(f) rank 3.

Same names and call shapes as the reference's augmentation.py:10-135.  The np.random draws stay on the host in
the reference's order (so a seeded run draws the same parameters); everything per pixel runs on the device:
the foreground statistics behind object_size / fg_center (vm_nonzero_stats), the TPS deformation (tps.py via
vm_tps_grid / vm_tps_sample), cv2.warpAffine (vm_warp_affine) and the HSV illumination change
(vm_change_illumination_u8, whose 256-entry S/V map is built on the host with the reference's float64
arithmetic).  numpy in -> numpy out; torch device tensors stay on the device.  The dataset-writing driver
augmentation() (file listing, imread/imwrite, progress bar) is I/O and out of scope.
"""

import ctypes
import math

import numpy as np
import torch

from . import _lib, ops
from . import tps
from .tps import deform_grid  # noqa: F401  (augmentation.deform_grid, augmentation.py:23-39)


def _device(a):
    if isinstance(a, torch.Tensor):
        return a if a.is_cuda else a.cuda()
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _out(t, like):
    return t if isinstance(like, torch.Tensor) else t.cpu().numpy()


def _stats(alpha):
    return [int(v) for v in ops.nonzero_stats(_device(alpha)).cpu().tolist()]


def object_size(alpha):
    """augmentation.object_size (augmentation.py:10-14): sqrt of the number of nonzero alpha pixels."""
    return np.sqrt(_stats(alpha)[0])


def fg_center(alpha):
    """augmentation.fg_center (augmentation.py:17-20): (int(mean column), int(mean row)) of the nonzero pixels.
    An all-zero alpha raises ValueError, as int(np.mean([])) does in the reference."""
    cnt, sr, sc = _stats(alpha)
    if cnt == 0:
        raise ValueError("cannot convert float NaN to integer")
    return int(sc / cnt), int(sr / cnt)  # exact integer sums, one float64 division (numpy's mean)


def rotation_matrix(center, angle, scale):
    """cv2.getRotationMatrix2D(center, angle, scale) (center is a Point2f)."""
    cx, cy = float(np.float32(center[0])), float(np.float32(center[1]))
    a = angle * (math.pi / 180)
    alpha = math.cos(a) * scale
    beta = math.sin(a) * scale
    return np.array([[alpha, beta, (1 - alpha) * cx - beta * cy],
                     [-beta, alpha, beta * cx + (1 - alpha) * cy]])


def _warp_image_dev(img, params, inv=None):
    (tu, tv), rot, scale, center = params
    h, w = img.shape[:2]
    if inv is not None:
        img = inv.sample(img, 1)
        if img.shape[2] == 1:
            img = img[:, :, 0]
    # cv2.warpAffine by [[1, 0, tu], [0, 1, tv]] then by getRotationMatrix2D(center, rot, scale), one fused pass
    return ops.warp_image(img, tu, tv, rotation_matrix(center, rot, scale), (w, h))


def warp_image(img, params, thin=None):
    """augmentation.warp_image (augmentation.py:42-61): optional TPS deformation thin = (grid, def_grid)
    (output (h+1, w+1)), then cv2.warpAffine by the translation (tu, tv) and by getRotationMatrix2D(center, rot,
    scale), both to (w, h)."""
    d = _device(img)
    h, w = d.shape[:2]
    inv = None
    if thin is not None:
        grid, def_grid = thin
        inv = tps.InverseWarp(grid, def_grid, (0, 0, h, w), 2, d.device)
    return _out(_warp_image_dev(d, params, inv), img)


def identity(m, n):
    """augmentation.identity (augmentation.py:64-68): arr[i, j] = [i+1, j+1] (int64, host)."""
    vec1 = np.arange(1, n + 1)
    vec2 = np.arange(1, m + 1)
    return np.transpose([np.repeat(vec2, n), np.tile(vec1, m)]).reshape(m, n, 2)


def synthetize_flow(fg_params, bg_params, grids, warped_alpha):
    """augmentation.synthetize_flow (augmentation.py:71-83) passes int64 identity() maps to cv2.warpAffine,
    which OpenCV rejects (no 64-bit integer depth); the reference therefore always raises here, and so does
    this drop-in.  It has no caller in the reference."""
    raise TypeError("src data type = 9 is not supported (cv2.warpAffine on the int64 identity map, "
                    "augmentation.py:78)")


def illumination_lut(a, b, c):
    """change_illumination's S/V map (augmentation.py:89-95) for every uint8 value, float64 like the reference."""
    x = np.arange(256, dtype=np.uint8)
    return (255. * np.clip(a * np.power(x / 255., b) + c, 0., 1.)).astype(np.uint8)


def change_illumination(bgr, a, b, c):
    """augmentation.change_illumination (augmentation.py:86-98): HSV round trip with S, V -> a * x**b + c."""
    return _out(ops.change_illumination(_device(bgr), illumination_lut(a, b, c)), bgr)


def augment(fg, bg, alpha):
    """augmentation.augment (augmentation.py:101-135): camera motion on bg, TPS + similarity motion on fg and
    alpha, one illumination change for both.  Returns (new_fg u8, new_bg u8, new_alpha f64)."""
    nfg, nbg, nal = augment_many([(fg, bg, alpha)])[0]
    return _out(nfg, fg), _out(nbg, bg), _out(nal, alpha)


def _stats_into(alphas, st):
    """Every alpha's (count, row sum, column sum) into the device [n, 3] buffer st: one vm_nonzero_stats_batch launch
    per 8 f64 alphas (the augment pipeline's), else one vm_nonzero_stats per alpha."""
    al = [a.contiguous() for a in alphas]
    if all(a.dtype == torch.float64 and a.dim() == 2 for a in al):
        n = len(al)
        ptrs = (ctypes.c_void_p * n)(*[a.data_ptr() for a in al])
        hs = (ctypes.c_int * n)(*[a.shape[0] for a in al])
        ws = (ctypes.c_int * n)(*[a.shape[1] for a in al])
        ops.check(ops.lib().vm_nonzero_stats_batch(ptrs, hs, ws, n, ops._ptr(st), ops.stream_handle()),
                  "nonzero_stats_batch")
        return al
    for i, a in enumerate(al):
        ops.nonzero_stats(a, out=st[i])
    return al


def nonzero_stats_many(alphas):
    """(count, row sum, column sum) of every alpha's nonzero pixels (object_size / fg_center) with ONE host sync:
    one batched launch into one [n, 3] device buffer, read back once."""
    st = torch.empty((len(alphas), 3), dtype=torch.int64, device=alphas[0].device)
    _stats_into(alphas, st)
    return [tuple(int(v) for v in row) for row in st.cpu().tolist()]


class StatsPrefetch:
    """nonzero_stats_many launched ahead on a side stream: it waits only for the work queued on the caller's stream
    so far (e.g. the upload of the next batch's sources), not for what is queued after (the current training step),
    and ``result()`` blocks only until those few launches are done."""

    def __init__(self, alphas):
        dev = alphas[0].device
        cur = torch.cuda.current_stream(dev)
        self.stream = torch.cuda.Stream(device=dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            st = torch.empty((len(alphas), 3), dtype=torch.int64, device=dev)
            for a in alphas:
                a.record_stream(self.stream)
            _stats_into(alphas, st)
            self.host = torch.empty((len(alphas), 3), dtype=torch.int64, pin_memory=True)
            self.host.copy_(st, non_blocking=True)
            self.done = torch.cuda.Event()
            self.done.record(self.stream)
        self._st = st

    def result(self):
        self.done.synchronize()
        return [tuple(int(v) for v in row) for row in self.host.tolist()]


def _upload_f64(arrays, device):
    """Small host float64 arrays -> device views, through ONE pinned buffer and one asynchronous copy (the caching
    pinned allocator keeps the buffer until the copy has run)."""
    flat = [np.ascontiguousarray(a, np.float64).ravel() for a in arrays]
    host = torch.empty(sum(f.size for f in flat), dtype=torch.float64, pin_memory=True)
    hn = host.numpy()
    off, spans = 0, []
    for f in flat:
        hn[off:off + f.size] = f
        spans.append((off, f.size))
        off += f.size
    dev = host.to(device, non_blocking=True)
    return [dev[o:o + n].view(np.shape(a)) for (o, n), a in zip(spans, arrays)]


def augment_many(triples, stats=None):
    """augment() over several samples: see _augment_many.  Returns [(new_fg u8, new_bg u8, new_alpha f64)]."""
    return [r[:3] for r in _augment_many(triples, stats)]


def _augment_many(triples, stats=None, bgra=False):
    """augment() over several (fg, bg, alpha) samples as one device pipeline: the foreground statistics of every
    sample with one readback (or ``stats`` already read, e.g. by a StatsPrefetch), then every sample's host draws in
    augment's order (sample by sample, so a seeded global RandomState gives the per-call draws), the TPS solves, one
    upload of all landmarks / coefficients, and per sample: the TPS lattice, fg / alpha TPS resampling, and the fused
    translate + similarity warps with the illumination change (vm_warp_image).  No host sync after the statistics.
    Returns [(new_fg u8, new_bg u8, new_alpha f64, new BGRA frame u8 or None)] as device tensors (the BGRA frame,
    augmentation.augmentation's frame t, only with bgra=True)."""
    bound_translate, bound_rotate, bound_scale = 0.05, 10, 0.15
    devs = [(_device(fg), _device(bg), _device(al)) for fg, bg, al in triples]
    if stats is None:
        stats = nonzero_stats_many([d[2] for d in devs])
    plans, uploads = [], []
    for (dfg, dbg, dal), (cnt, sr, sc) in zip(devs, stats):
        h, w = dfg.shape[:2]
        fg_size = np.sqrt(cnt)
        # camera motion (bg)
        tu_bg = int(np.random.uniform(-w * bound_translate, w * bound_translate))
        tv_bg = int(np.random.uniform(-h * bound_translate, h * bound_translate))
        scale_bg = np.random.uniform(1., 1. + bound_scale)
        # object motion (fg): TPS deformation + similarity
        grid, def_grid = deform_grid(h, w)
        tu_fg = int(np.random.uniform(-fg_size * bound_translate, fg_size * bound_translate))
        tv_fg = int(np.random.uniform(-fg_size * bound_translate, fg_size * bound_translate))
        rot_fg = np.random.uniform(-bound_rotate, bound_rotate)
        scale_fg = np.random.uniform(1., 1. + bound_scale)
        if cnt == 0:
            raise ValueError("cannot convert float NaN to integer")
        center = (int(sc / cnt), int(sr / cnt))
        a = np.random.uniform(1. - 0.05, 1. + 0.05)
        b = np.random.uniform(1. - 0.3, 1. + 0.3)
        c = np.random.uniform(-0.07, 0.07)
        # one TPS map serves fg and alpha (the reference evaluates the same map twice): the reverse transform
        # def_grid -> grid (tps.py:50-51), solved on the host like the reference (numpy's pinv: L is numerically
        # singular, cond ~1e16, so pinv's cut of the small singular values IS the map — no faster LU solve)
        uploads += [def_grid, tps._coefficients(def_grid, grid)]
        plans.append((h, w, grid, def_grid, (tu_bg, tv_bg, scale_bg), (tu_fg, tv_fg, rot_fg, scale_fg, center),
                      illumination_lut(a, b, c)))
    dev_arrays = _upload_f64(uploads, devs[0][0].device) if uploads else []
    batched = _BATCH and all(dfg.dtype == torch.uint8 and dfg.dim() == 3 and dfg.shape[2] == 3 and dbg.dtype == torch.uint8 and
                  dbg.dim() == 3 and dbg.shape[2] == 3 and dal.dtype == torch.float64 and dal.dim() == 2 and
                  tuple(dal.shape) == tuple(dfg.shape[:2]) and min(dfg.shape[:2]) >= 4 for dfg, dbg, dal in devs)
    if batched:
        return _augment_batch(devs, plans, dev_arrays, bgra)
    out = []
    for k, ((dfg, dbg, dal), (h, w, grid, def_grid, pbg, pfg, lut)) in enumerate(zip(devs, plans)):
        tu_bg, tv_bg, scale_bg = pbg
        # the camera motion warps the background to its own size (augmentation.py:56-63 with h, w = bg's)
        new_bg = ops.warp_image(dbg, tu_bg, tv_bg, rotation_matrix((w // 2, h // 2), 0., scale_bg),
                                (dbg.shape[1], dbg.shape[0]), lut)
        inv = tps.InverseWarp(grid, def_grid, (0, 0, h, w), 2, dfg.device,
                              solved=(dev_arrays[2 * k], dev_arrays[2 * k + 1]))
        tu_fg, tv_fg, rot_fg, scale_fg, center = pfg
        m = rotation_matrix(center, rot_fg, scale_fg)
        new_fg = ops.warp_image(inv.sample(dfg, 1), tu_fg, tv_fg, m, (w, h), lut)
        tal = inv.sample(dal, 1)
        new_alpha = ops.warp_image(tal[:, :, 0] if tal.dim() == 3 else tal, tu_fg, tv_fg, m, (w, h))
        out.append((new_fg, new_bg, new_alpha, ops.bgra(new_fg, new_alpha) if bgra else None))
    return out


_BATCH = True  # False: the per-sample launches (the batched kernels' bit-identity test)
_EVENTS = None  # a list: HIP events around every vm_augment_batch launch are appended (bench.py's kernel time)


def _augment_batch(devs, plans, dev_arrays, bgra=False):
    """augment_many's device work for u8 BGR fg / bg and f64 alpha samples: vm_augment_batch (the TPS lattice, one
    fg + alpha resampling pass, the fused warps with the illumination change; four launches per 4 samples)."""
    lib = ops.lib()
    n = len(devs)
    jobs = (_lib.VmAugmentJob * n)()
    out, keep = [], []
    for k, ((dfg, dbg, dal), (h, w, grid, def_grid, pbg, pfg, lut)) in enumerate(zip(devs, plans)):
        dfg, dbg, dal = dfg.contiguous(), dbg.contiguous(), dal.contiguous()
        dev = dfg.device
        scratch = torch.empty(lib.vm_augment_scratch_bytes(h, w), dtype=torch.uint8, device=dev)
        new_fg = torch.empty((h, w, 3), dtype=torch.uint8, device=dev)
        new_bg = torch.empty(dbg.shape, dtype=torch.uint8, device=dev)
        new_alpha = torch.empty((h, w), dtype=torch.float64, device=dev)
        new_bgra = torch.empty((h, w, 4), dtype=torch.uint8, device=dev) if bgra else None
        pts, co = dev_arrays[2 * k], dev_arrays[2 * k + 1]
        tu_bg, tv_bg, scale_bg = pbg
        tu_fg, tv_fg, rot_fg, scale_fg, center = pfg
        j = jobs[k]
        j.fg, j.bg, j.alpha = dfg.data_ptr(), dbg.data_ptr(), dal.data_ptr()
        j.tps_points, j.tps_coeffs, j.scratch = pts.data_ptr(), co.data_ptr(), scratch.data_ptr()
        j.new_fg, j.new_bg, j.new_alpha = new_fg.data_ptr(), new_bg.data_ptr(), new_alpha.data_ptr()
        j.new_bgra = new_bgra.data_ptr() if bgra else None
        j.h, j.w, j.bg_h, j.bg_w, j.npts = h, w, dbg.shape[0], dbg.shape[1], pts.shape[0]
        j.tu_bg, j.tv_bg, j.tu_fg, j.tv_fg = int(tu_bg), int(tv_bg), int(tu_fg), int(tv_fg)
        j.m_bg[:] = [float(v) for v in rotation_matrix((w // 2, h // 2), 0., scale_bg).reshape(6)]
        j.m_fg[:] = [float(v) for v in rotation_matrix(center, rot_fg, scale_fg).reshape(6)]
        ctypes.memmove(j.lut, np.ascontiguousarray(lut, np.uint8).ctypes.data, 256)
        keep += [dfg, dbg, dal, scratch]
        out.append((new_fg, new_bg, new_alpha, new_bgra))
    ev = _EVENTS is not None and (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev and ev[0].record()
    ops.check(lib.vm_augment_batch(jobs, n, ops.stream_handle()), "augment_batch")
    ev and ev[1].record()
    ev and _EVENTS.append(ev)
    return out


def bgra(fg, alpha):
    """The BGRA image augmentation.augmentation writes for a (fg, alpha) pair (augmentation.py:152-153,163-164):
    concat(fg u8, (255. * alpha).astype(uint8)) — on the device for device tensors (float64 product, truncation)."""
    dfg, dal = _device(fg), _device(alpha)
    return _out(ops.bgra(dfg, dal), fg)


def bgra_many(pairs):
    """bgra() of several (fg u8 [h, w, 3], alpha f64 [h, w]) device pairs: one vm_bgra_u8_batch launch per 8."""
    pairs = [(f.contiguous(), a.contiguous()) for f, a in pairs]
    if not all(f.dtype == torch.uint8 and a.dtype == torch.float64 and f.dim() == 3 and f.shape[2] == 3 and
               a.numel() == f.shape[0] * f.shape[1] for f, a in pairs):
        return [ops.bgra(f, a) for f, a in pairs]
    n = len(pairs)
    outs = [torch.empty((f.shape[0], f.shape[1], 4), dtype=torch.uint8, device=f.device) for f, _ in pairs]
    P = ctypes.c_void_p * n
    ops.check(ops.lib().vm_bgra_u8_batch(P(*[f.data_ptr() for f, _ in pairs]), P(*[a.data_ptr() for _, a in pairs]),
                                         (ctypes.c_long * n)(*[a.numel() for _, a in pairs]),
                                         P(*[o.data_ptr() for o in outs]), n, ops.stream_handle()), "bgra_batch")
    return outs


def video_sample(fg, bg, alpha, flow):
    """One training entry of loader.video_batch made in memory the way augmentation.augmentation makes it on disk
    (augmentation.py:141-168): frame t-1 = the reference BGRA (fg + alpha), frame t = augment(fg, bg, alpha) as
    BGRA with its augmented background.  ``flow`` is the entry's .flo (the reference computes it offline with an
    optical-flow estimator between the two frames; any [h, w, 2] f32).  Returns the dict loader.compose_batch takes
    (fg, bg, prev, flow; add "plan" = loader.plan_crop(...)), all on the device."""
    return video_samples([(fg, bg, alpha)], flow)[0]


def video_samples(sources, flow, stats=None):
    """video_sample over several (fg, bg, alpha) sources as one augment_many pipeline (one statistics readback, or
    none with ``stats`` from a StatsPrefetch)."""
    devs = [(_device(fg), _device(bg), _device(al)) for fg, bg, al in sources]
    aug = _augment_many(devs, stats=stats, bgra=True)  # frame t's BGRA written by the object-motion pass
    prev = bgra_many([(d[0], d[2]) for d in devs])      # frame t-1: the source itself
    d_flow = _device(flow)
    return [{"fg": a[3], "bg": a[1], "prev": p, "flow": d_flow} for a, p in zip(aug, prev)]
