"""Two-frame temporal helpers (reference flow.py) on gfx950 kernels.

Same names and call shapes as flow.py:9-65.  numpy arguments are accepted like the
reference (uploaded, computed on the GPU, returned as numpy; ``correct_alpha`` still
mutates the caller's array in place); torch device tensors stay on the device.
"""

import numpy as np
import torch

from . import ops


def _dev(a, dtype=torch.float32):
    if isinstance(a, torch.Tensor):
        return a.to("cuda" if not a.is_cuda else a.device, dtype)
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dtype)


def warp_img(img, flow, mode="opencv"):
    """flow.warp_img (flow.py:9-18): backward-warp a single-channel image by a dense flow.

    mode 'opencv' = cv2.remap's 1/32-pixel fixed-point coordinates (reference behaviour),
    'exact' = plain bilinear.  img [H,W] (or [N,H,W] with flow [N,H,W,2]).
    """
    if isinstance(img, torch.Tensor):
        if img.dim() not in (2, 3):
            raise AssertionError("warp_img: image must be 1 channel")
        return ops.remap_f32(_dev(img), _dev(flow), mode)
    assert len(img.shape) == 2  # flow.py:11
    out = ops.remap_f32(_dev(img), _dev(flow), mode)
    return out.cpu().numpy().astype(img.dtype if img.dtype.kind == "f" else np.float32)


def warp_bgr(img, flow):
    """flow.warp_bgr (flow.py:21-33): uint8 [H,W,3], OpenCV fixed-point bilinear per plane."""
    if isinstance(img, torch.Tensor):
        return ops.remap_u8(img.to(torch.uint8), _dev(flow))
    out = ops.remap_u8(torch.from_numpy(np.ascontiguousarray(img, np.uint8)).cuda(), _dev(flow))
    return out.cpu().numpy()


def correct_alpha(backward, forward, alpha, promote="numpy1", thresh=15.0):
    """flow.correct_alpha (flow.py:36-65): zero alpha where the forward/backward round trip misses by > 15 px.

    Mutates ``alpha`` in place and returns it.  ``promote``: 'numpy1' (the reference's numpy-1.x
    float64 index arithmetic) or 'numpy2' (float32, what the same code does under numpy 2).
    Raises IndexError, leaving alpha untouched, where the reference would (flow.py:46).
    The reference's GUI side effects (cv2.imshow of the error map, flow.py:51-52) are not reproduced.
    """
    if isinstance(alpha, torch.Tensor) and alpha.is_cuda and alpha.dtype == torch.float32 and alpha.is_contiguous():
        return ops.fb_consistency(_dev(backward), _dev(forward), alpha, thresh, promote)
    a = _dev(alpha).contiguous()
    ops.fb_consistency(_dev(backward), _dev(forward), a, thresh, promote)
    res = a.cpu()
    if isinstance(alpha, torch.Tensor):
        alpha.copy_(res.to(alpha.dtype))
    else:
        alpha[...] = res.numpy()
    return alpha
