"""Training-sample loader (reference loader.py) with the per-pixel work on the GPU.

Same names, arguments and return shapes as loader.py: ``load_and_crop`` / ``get_batch``,
``simple_load_crop`` / ``simple_batch``, ``video_load_crop`` / ``video_batch``, ``get_padded_img``,
``get_file_list``, ``get_batch_list``, ``epoch_is_over``.

Split of the work:
  * host — file decoding (PIL; cv2 is not in this image) and the np.random draws, made with the
    reference's arguments in the reference's order (crop type, canvas placement, crop corner,
    background canvas placement, background corner, [mirror coin]), so a seeded global RandomState
    yields the reference's crops;
  * GPU — everything per pixel, for the whole batch in one vm_loader_compose launch
    (csrc/loader.hip): canvases and crops as index maps, the flow warp of the previous alpha at the
    pixels the crop reads, cv2.resize (INTER_LINEAR, OpenCV's float64 rounding), compositing and
    VGG-mean subtraction.

Outputs are device tensors, float32 by default (the network's input type); ``dtype=torch.float64``
returns the reference's float64 values bit for bit.  ``compose_batch`` takes already-decoded arrays
or device tensors (a decode pipeline, or inputs resident in HBM).
"""

import ctypes
import os

import numpy as np
import torch

from . import _lib, reader

CROP_TYPES = [(320, 320), (480, 480), (640, 640)]  # loader.py:47, 124, 294


# ---------------------------------------------------------------- host: window planning (the random draws)

def _pad_axis(n, crop):
    """get_padded_img along one axis (loader.py:15-34) -> (canvas length, lo, hi, shift).

    crop > n: the image sits at a random offset of a crop-long zero canvas; crop <= n: a random
    crop-long window of the image sits at the start of an n-long canvas, the rest stays zero."""
    if crop > n:
        beg_out = np.random.randint(0, crop - n + 1)
        return crop, beg_out, beg_out + n, -beg_out
    beg_in = np.random.randint(0, n - crop + 1)
    return n, 0, crop, beg_in


def _window(canvas, start, length):
    """canvas[start:start+length] (numpy truncates at the canvas end) -> (n, off, lo, hi, shift)."""
    size, lo, hi, shift = canvas
    return (max(0, min(start + length, size) - start), start, lo, hi, shift)


def plan_crop(fg_hw, bg_hw):
    """The draws of one *_load_crop call (loader.py:48-69, 125-145, 295-315), as window maps.

    Returns (fg_rows, fg_cols, bg_rows, bg_cols), each (n, off, lo, hi, shift): resize-source
    index u reads canvas index u + off, which holds image index u + off + shift when in [lo, hi)."""
    fg_h, fg_w = int(fg_hw[0]), int(fg_hw[1])
    crop_h, crop_w = CROP_TYPES[np.random.randint(0, len(CROP_TYPES))]
    if fg_h < crop_h or fg_w < crop_w:
        rows, cols = _pad_axis(fg_h, crop_h), _pad_axis(fg_w, crop_w)
    else:
        rows, cols = (fg_h, 0, fg_h, 0), (fg_w, 0, fg_w, 0)
    i, j = np.random.randint(0, rows[0] - crop_h + 1), np.random.randint(0, cols[0] - crop_w + 1)
    fr = _window(rows, i, crop_h)
    fc = _window(cols, j, crop_h)  # loader.py:60: [j:j+crop_h] on the column axis too
    bg_h, bg_w = int(bg_hw[0]), int(bg_hw[1])
    bg_crop_h = int(np.ceil(crop_h * bg_h / fr[0]))  # loader.py:65-66 (fg.shape = the crop's)
    bg_crop_w = int(np.ceil(crop_w * bg_w / fc[0]))
    brows, bcols = _pad_axis(bg_h, bg_crop_h), _pad_axis(bg_w, bg_crop_w)
    bi, bj = np.random.randint(0, bg_h - bg_crop_h + 1), np.random.randint(0, bg_w - bg_crop_w + 1)
    return fr, fc, _window(brows, bi, bg_crop_h), _window(bcols, bj, bg_crop_w)


def get_padded_img(img, crop_h, crop_w):
    """loader.py:10-36 on a host array: the image randomly placed in / cropped to a max(crop, size) canvas."""
    h, w = img.shape[:2]
    rows, cols = _pad_axis(h, crop_h), _pad_axis(w, crop_w)
    out = np.zeros((rows[0], cols[0]) + img.shape[2:], dtype=img.dtype)
    out[rows[1]:rows[2], cols[1]:cols[2]] = img[rows[1] + rows[3]:rows[2] + rows[3], cols[1] + cols[3]:cols[2] + cols[3]]
    return out


# ---------------------------------------------------------------- host: decoding

def read_bgra(path):
    """The decode of reader.read_fg_img (reader.py:10-18) kept as u8 BGRA (16-bit PNGs rescaled as there)."""
    from PIL import Image
    im = np.asarray(Image.open(path))
    if im.dtype == np.uint16:
        im = (((im + 1) / 256.) - 1).astype(np.uint8)  # reader.py:13-14
    if im.ndim != 3 or im.shape[2] != 4:
        raise IndexError("%s: foreground images are RGBA (reader.py:16 reads channel 3)" % path)
    return np.ascontiguousarray(im[:, :, [2, 1, 0, 3]])


def read_bgr(path):
    """cv2.imread(path) (IMREAD_COLOR): u8 BGR."""
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(path).convert("RGB"))[:, :, ::-1])


def _check_image(path):
    """loader.py:45 reads the trimap, which no output uses; only its readability is kept."""
    from PIL import Image
    with Image.open(path) as im:
        im.size  # noqa: B018


# ---------------------------------------------------------------- GPU: one launch per batch

_OUT_CH = {"cmp": 3, "bg": 3, "label": 1, "warped": 3, "fg": 3, "input": 6}


def _dev(a, dtype, device):
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dtype)


class _PinnedDescRing:
    """Pinned host memory for the per-batch sample descriptors vm_loader_compose copies to the device: a copy from
    pageable memory would make hipMemcpyAsync wait for the stream (the previous training step); from pinned memory
    it stays asynchronous.  A slot is reused only after the event recorded behind its copy has completed."""

    def __init__(self, slots=4):
        self.slots = [[None, None] for _ in range(slots)]
        self.i = 0

    def take(self, n):
        slot = self.slots[self.i]
        self.i = (self.i + 1) % len(self.slots)
        buf, ev = slot
        if ev is not None:
            ev.synchronize()
        nbytes = n * ctypes.sizeof(_lib.VmLoaderSample)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 4096), dtype=torch.uint8, pin_memory=True)
            slot[0] = buf
        desc = (_lib.VmLoaderSample * n).from_address(buf.data_ptr())
        ctypes.memset(buf.data_ptr(), 0, nbytes)
        return desc, slot

    @staticmethod
    def issued(slot):
        ev = torch.cuda.Event()
        ev.record()
        slot[1] = ev


_DESC = _PinnedDescRing()


def compose_batch(samples, input_size, outputs=("cmp", "bg", "label", "fg"), mirror=None, dtype=torch.float32,
                  device="cuda", out=None):
    """Run vm_loader_compose on decoded samples.

    samples: list of dicts with fg (u8 BGRA [h,w,4]), bg (u8 BGR), plan (from plan_crop) and, for
    video samples, prev (u8 BGRA) + flow (f32 [h,w,2]); numpy arrays or device tensors.
    outputs: names from cmp, bg, label, warped, fg and input (= cmp | bg, get_batch's layout).
    out: optional {name: contiguous tensor} to write into (e.g. a captured training graph's static inputs).
    Returns {name: tensor [n, input_size[1], input_size[0], C]}."""
    if dtype not in (torch.float32, torch.float64):
        raise ValueError("loader outputs are float32 or float64")
    n = len(samples)
    if n == 0:
        raise ValueError("empty batch")
    if "input" in outputs and ("cmp" in outputs or "bg" in outputs):
        raise ValueError("'input' already holds cmp and bg (channels 0-2 / 3-5)")
    ow, oh = int(input_size[0]), int(input_size[1])
    keep = []
    desc, slot = _DESC.take(n)
    for i, s in enumerate(samples):
        fg = _dev(s["fg"], torch.uint8, device)
        bg = _dev(s["bg"], torch.uint8, device)
        if fg.dim() != 3 or fg.shape[2] != 4 or bg.dim() != 3 or bg.shape[2] != 3:
            raise ValueError("sample %d: fg must be [h,w,4] BGRA and bg [h,w,3] BGR" % i)
        d = desc[i]
        d.fg, d.bg = fg.data_ptr(), bg.data_ptr()
        d.fg_h, d.fg_w, d.bg_h, d.bg_w = fg.shape[0], fg.shape[1], bg.shape[0], bg.shape[1]
        keep += [fg, bg]
        if s.get("prev") is not None:
            prev = _dev(s["prev"], torch.uint8, device)
            flow = _dev(s["flow"], torch.float32, device)
            if tuple(flow.shape) != (fg.shape[0], fg.shape[1], 2) or prev.dim() != 3 or prev.shape[2] != 4:
                raise ValueError("sample %d: flow must be [fg_h, fg_w, 2] and prev [h,w,4]" % i)
            d.prev, d.flow, d.prev_h, d.prev_w = prev.data_ptr(), flow.data_ptr(), prev.shape[0], prev.shape[1]
            keep += [prev, flow]
        fr, fc, br, bc = s["plan"]
        d.fg_rows, d.fg_cols = _lib.VmCropAxis(*fr), _lib.VmCropAxis(*fc)
        d.bg_rows, d.bg_cols = _lib.VmCropAxis(*br), _lib.VmCropAxis(*bc)
        d.mirror = int(bool(mirror[i])) if mirror is not None else 0
    res = {}
    for k in outputs:
        shape = (n, oh, ow, _OUT_CH[k])
        t = None if out is None else out.get(k)
        if t is not None and (tuple(t.shape) != shape or t.dtype != dtype or not t.is_contiguous()):
            raise ValueError("compose_batch: out[%r] must be a contiguous %s tensor of shape %s" % (k, dtype, shape))
        res[k] = t if t is not None else torch.empty(shape, dtype=dtype, device=device)
    o = _lib.VmLoaderOutputs()
    esz = 8 if dtype == torch.float64 else 4
    for k, t in res.items():
        if k == "input":
            o.ptr[0], o.pixstride[0] = t.data_ptr(), 6
            o.ptr[1], o.pixstride[1] = t.data_ptr() + 3 * esz, 6
        else:
            o.ptr[_lib.LOADER_PLANES[k]], o.pixstride[_lib.LOADER_PLANES[k]] = t.data_ptr(), _OUT_CH[k]
    lib = _lib.lib()
    work = torch.empty(max(1, lib.vm_loader_workspace_bytes(n)), dtype=torch.uint8, device=device)
    with torch.cuda.device(work.device):
        _lib.check(lib.vm_loader_compose(desc, n, oh, ow, _lib.VM_F64 if dtype == torch.float64 else _lib.VM_F32,
                                         ctypes.byref(o), ctypes.c_void_p(work.data_ptr()), _lib.stream_handle()),
                   "loader_compose")
        _DESC.issued(slot)
    return res


def _decode(fg_path, bg_path, prev_path=None, flo_path=None):
    s = {"fg": read_bgra(fg_path), "bg": read_bgr(bg_path)}
    if flo_path is not None:
        s["flow"] = reader.read_flow(flo_path)
        s["prev"] = read_bgra(prev_path)
    return s


def _planned(s):
    s["plan"] = plan_crop(s["fg"].shape[:2], s["bg"].shape[:2])
    return s


def _square(input_size):
    if int(input_size[0]) != int(input_size[1]):
        # the reference's batch arrays are (input_size[0], input_size[1]) but cv2.resize makes
        # (input_size[1], input_size[0]) images: the assignment fails for non-square sizes
        raise ValueError("batch loaders need a square input_size (loader.py:96 vs :70)")


def load_and_crop(entry, input_size, dtype=torch.float32, device="cuda"):
    """loader.py:39-85 -> (inp [h,w,6] = cmp | bg, label [h,w,1], fg [h,w,3])."""
    fg_path, tr_path, bg_path = entry
    s = _decode(fg_path, bg_path)
    _check_image(tr_path)
    r = compose_batch([_planned(s)], input_size, ("input", "label", "fg"), dtype=dtype, device=device)
    return r["input"][0], r["label"][0], r["fg"][0]


def get_batch(file_list, input_size, rd_scale=False, rd_mirror=False, dtype=torch.float32, device="cuda"):
    """loader.py:93-116 -> (input [N,h,w,6], label [N,h,w,1], raw_fgs [N,h,w,3])."""
    if rd_scale:
        raise ValueError("rd_scale: random_scale is an unimplemented stub in the reference (loader.py:88-90)")
    _square(input_size)
    samples, flips = [], []
    for fg_path, tr_path, bg_path in file_list:
        s = _decode(fg_path, bg_path)
        _check_image(tr_path)
        samples.append(_planned(s))
        flips.append(bool(rd_mirror) and np.random.uniform(0., 1.) > 0.5)  # loader.py:105-106
    r = compose_batch(samples, input_size, ("input", "label", "fg"), flips, dtype, device)
    return r["input"], r["label"], r["fg"]


def simple_load_crop(entry, input_size, dtype=torch.float32, device="cuda"):
    """loader.py:119-157 -> (cmp, bg, label, fg) for one entry (fg_path, tr_path, bg_path)."""
    fg_path, _, bg_path = entry
    r = compose_batch([_planned(_decode(fg_path, bg_path))], input_size, dtype=dtype, device=device)
    return r["cmp"][0], r["bg"][0], r["label"][0], r["fg"][0]


def simple_batch(file_list, input_size, dtype=torch.float32, device="cuda"):
    """loader.py:160-171 -> (cmps, bgs, label, raw_fgs)."""
    _square(input_size)
    samples = [_planned(_decode(e[0], e[2])) for e in file_list]
    r = compose_batch(samples, input_size, dtype=dtype, device=device)
    return r["cmp"], r["bg"], r["label"], r["fg"]


_VIDEO_OUT = ("cmp", "bg", "label", "warped", "fg")


def video_load_crop(entry, input_size, dtype=torch.float32, device="cuda"):
    """loader.py:285-330 -> (cmp, bg, label, warped_alpha [h,w,3], fg) for (fg, bg, previous, flo) paths."""
    fg_path, bg_path, prev_path, flo_path = entry
    r = compose_batch([_planned(_decode(fg_path, bg_path, prev_path, flo_path))], input_size, _VIDEO_OUT,
                      dtype=dtype, device=device)
    return tuple(r[k][0] for k in _VIDEO_OUT)


def video_batch(file_list, input_size, dtype=torch.float32, device="cuda"):
    """loader.py:333-345 -> (cmps, bgs, label, warped, raw_fgs)."""
    _square(input_size)
    samples = [_planned(_decode(*e)) for e in file_list]
    r = compose_batch(samples, input_size, _VIDEO_OUT, dtype=dtype, device=device)
    return tuple(r[k] for k in _VIDEO_OUT)


# ---------------------------------------------------------------- file-list helpers (host, as loader.py:190-211)

def get_file_list(root_dir, list_path):
    """loader.py:190-198: lines 'fg tr bg' (space separated) joined to root_dir."""
    files = []
    with open(list_path, "r") as f:
        for line in f:
            files.append([os.path.join(root_dir, p) for p in line[:-1].split(" ")])
    return files


def get_batch_list(file_list, batch_size):
    """loader.py:201-206: pops batch_size entries off the END of file_list."""
    return [file_list.pop() for _ in range(batch_size)]


def epoch_is_over(file_list, batch_size):
    """loader.py:209-211."""
    return len(file_list) < batch_size
