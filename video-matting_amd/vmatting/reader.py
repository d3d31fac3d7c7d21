"""Formats on the path (reference reader.py): Middlebury .flo I/O and compositing.

``read_flow`` keeps reader.py:21-30's semantics exactly (float32 magic 202021.25, int32 w,
int32 h, h*w*2 float32, little-endian; a bad magic prints and continues).  The rest of
reader.py (PNG decoding via cv2, GUI playback, HSV flow visualisation) is outside the hot
path — ``read_fg_img`` is provided through PIL for convenience only.
"""

import numpy as np
import torch

FLO_MAGIC = 202021.25


def read_flow(flow_path, device=None):
    """reader.read_flow; ``device='cuda'`` returns a device tensor (pinned host staging)."""
    with open(flow_path, "rb") as f:
        key = np.fromfile(f, dtype=np.float32, count=1)
        if FLO_MAGIC != key:
            print("ERROR: invalid key ({})".format(key))
        w = np.fromfile(f, dtype=np.int32, count=1)[0]
        h = np.fromfile(f, dtype=np.int32, count=1)[0]
        data = np.fromfile(f, dtype=np.float32, count=2 * h * w).reshape((h, w, 2))
    if device is None:
        return data
    host = torch.from_numpy(data).pin_memory()
    return host.to(device, non_blocking=True)


def write_flow(flow_path, flow):
    """The .flo writer matching read_flow (the reference ships none)."""
    if isinstance(flow, torch.Tensor):
        flow = flow.detach().cpu().numpy()
    flow = np.asarray(flow, np.float32)
    h, w = flow.shape[:2]
    with open(flow_path, "wb") as f:
        np.array([FLO_MAGIC], np.float32).tofile(f)
        np.array([w, h], np.int32).tofile(f)
        flow.tofile(f)


def create_composite_image(fg, bg, alpha, out_dtype=torch.float64):
    """reader.create_composite_image (reader.py:72-79): alpha*fg + (1-alpha)*bg per channel.

    numpy in -> float64 numpy out (like the reference); device tensors -> float64 device tensor from the
    vm_composite_image kernel (bit-identical to the numpy expression; pass out_dtype=torch.float32 to halve
    the write).
    """
    if isinstance(fg, torch.Tensor):
        from vmatting import ops
        return ops.composite_image(fg, bg, alpha, out_dtype=out_dtype)
    a = np.asarray(alpha, np.float64)[..., None]
    return a * np.asarray(fg) + (1.0 - a) * np.asarray(bg)


def read_fg_img(img_path):
    """reader.read_fg_img (reader.py:10-18) via PIL: returns (alpha in [0,1] float64, BGR uint8)."""
    from PIL import Image
    im = np.asarray(Image.open(img_path))
    if im.dtype == np.uint16:
        im = (((im + 1) / 256.0) - 1).astype(np.uint8)  # reader.py:13-14
    bgr = im[:, :, [2, 1, 0]]
    alpha = im[:, :, 3] / 255.0
    return alpha, bgr
