"""data.py's per-pixel dataset preparation on gfx950 kernels — SURVEY.md §8(f) rank 4.

``trimap_from_matte`` (data.py:37-67) is the reference's pure-Python O(h*w*49) raster loop; here it is one
LDS-tiled kernel (vm_trimap_from_matte) with the loop's exact result, raster-order overwrites included.  The
dataset drivers around it (create_bgra / convert_dataset / generate_trimaps: directory walks, imread/imwrite)
are file I/O and stay out of scope.
"""

import numpy as np
import torch

from . import ops


def trimap_from_matte(matte, dilate=1, crop=3):
    """data.trimap_from_matte: 255 where the matte is 1, 0 where it is 0, 128 in the unknown band (see module doc).
    numpy float64 in -> numpy uint8 out (the reference asserts float64, data.py:42); device tensors stay on the
    device.  ``dilate``/``crop`` are the reference's hard-coded 1 and 3."""
    if isinstance(matte, torch.Tensor):
        return ops.trimap_from_matte(matte if matte.is_cuda else matte.cuda(), dilate, crop)
    assert matte.dtype == np.float64
    d = torch.from_numpy(np.ascontiguousarray(matte)).cuda()
    return ops.trimap_from_matte(d, dilate, crop).cpu().numpy()
