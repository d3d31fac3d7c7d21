"""Numpy restatement of data.trimap_from_matte (data.py:37-67) — TEST INFRASTRUCTURE ONLY.

The reference walks the matte in raster order: a pixel whose matte is exactly 1 (0) is set to 255 (0), any
other pixel to 128 and, in the same iteration, it re-marks as 128 its neighbours with matte 1 within `crop`
and with matte 0 within `dilate`.  A known pixel's own assignment overwrites every mark made before it, so its
final value is 128 exactly when an unknown pixel LATER in raster order lies within its radius (crop for 1,
dilate for 0); that is what is restated here, vectorised over offsets.  Pinned bit-exactly by
tests/golden/trimap.npz, produced by running the reference's own loop.
"""

import numpy as np


def trimap_from_matte(matte, dilate=1, crop=3):
    assert matte.dtype == np.float64
    h, w = matte.shape
    one, zero = matte == 1., matte == 0.
    unknown = ~(one | zero)
    trimap = np.where(one, 255, np.where(zero, 0, 128)).astype(np.uint8)
    side = max(dilate, crop)
    marked = np.zeros((h, w), bool)
    pad = np.zeros((h + 2 * side, w + 2 * side), bool)
    pad[side:side + h, side:side + w] = unknown
    for dk in range(0, side + 1):
        for dl in range(-side, side + 1):
            if dk == 0 and dl <= 0:
                continue  # only pixels after p in raster order survive p's own assignment
            q = pad[side + dk:side + dk + h, side + dl:side + dl + w]
            r = max(dk, abs(dl))
            marked |= q & ((one & (r <= crop)) | (zero & (r <= dilate)))
    trimap[marked] = 128
    return trimap
