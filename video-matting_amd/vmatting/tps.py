# The host-side TPS solve below (_U, _interpoint_distances, _make_L_matrix, _coefficients and the
# deform_grid draw sequence) follows the reference's tps.py, which is
#   Copyright 2007 Zachary Pincus, part of CellTool,
#   free software under version 2 of the GNU General Public License (tps.py:1-6).
# Those ~30 lines stay close to the original so that numpy's pinv solve and np.random draw order are
# reproduced bit for bit; they are distributed under the same GPLv2 terms as the original.
"""tps.py (thin-plate-spline warp, Bookstein) on gfx950 kernels — SURVEY.md §8(f) rank 3.

Same names and call shapes as the reference's tps.py:14-149.  The host keeps what the reference does once per
warp on 28 numbers — the L-matrix build and its pinv solve (tps._make_warp, tps.py:110-115), with the
reference's own numpy arithmetic — and the device does the per-pixel work: the TPS evaluated on the approximate
grid (vm_tps_grid), its bilinear upsampling fused with scipy's map_coordinates resampling of every plane
(vm_tps_sample).  numpy inputs are uploaded and numpy results returned (drop-in); torch device tensors stay on
the device.  No CPU fallback: without the gfx950 library every call raises.
"""

import numpy as np
import torch

from . import ops

_small = 1e-100  # tps.py:77


def _U(x):
    """tps.py:80-81 (host side: the 25x25 kernel matrix only)."""
    with np.errstate(divide="ignore"):
        return (x ** 2) * np.where(x < _small, 0, np.log(x))


def _interpoint_distances(points):
    """tps.py:84-87."""
    xd = np.subtract.outer(points[:, 0], points[:, 0])
    yd = np.subtract.outer(points[:, 1], points[:, 1])
    return np.sqrt(xd ** 2 + yd ** 2)


def _make_L_matrix(points):
    """tps.py:90-97: [[K, P], [P^T, 0]]."""
    n = len(points)
    k = _U(_interpoint_distances(points))
    p = np.ones((n, 3))
    p[:, 1:] = points
    return np.block([[k, p], [p.T, np.zeros((3, 3))]])


def _coefficients(from_points, to_points):
    """tps._make_warp's solve (tps.py:110-115): pinv(L) @ [to_points; 0 0 0] -> [n+3, 2]."""
    from_points, to_points = np.asarray(from_points), np.asarray(to_points)
    ll = _make_L_matrix(from_points)
    v = np.resize(to_points, (len(to_points) + 3, 2))
    v[-3:, :] = 0
    return np.dot(np.linalg.pinv(ll), v)


def _mgrid_axis(lo, hi, num):
    """np.mgrid[lo:hi:num*1j]: int(num) points at i*step + lo, step = (hi-lo)/float(count-1) (1 if one point)."""
    cnt = int(abs(num))
    if cnt < 1:
        raise ValueError("tps: empty approximate grid (%r points)" % num)
    return cnt, ((hi - lo) / float(cnt - 1) if cnt != 1 else 1.0)


class InverseWarp:
    """tps._make_inverse_warp (tps.py:41-75) on the device: the TPS map to_points -> from_points evaluated on the
    approximate grid ([2, nx, ny] f64), plus the upsampling parameters of tps.py:55-74 (None when
    approximate_grid == 1)."""

    def __init__(self, from_points, to_points, output_region, approximate_grid, device="cuda", solved=None):
        """solved: (to_points, coefficients) already on the device (augmentation.augment_many uploads every
        sample's in one copy); else they are solved here and uploaded."""
        x_min, y_min, x_max, y_max = output_region
        if approximate_grid is None:
            approximate_grid = 1
        x_steps = (x_max - x_min) / approximate_grid
        y_steps = (y_max - y_min) / approximate_grid
        nx, xstep = _mgrid_axis(x_min, x_max, x_steps)
        ny, ystep = _mgrid_axis(y_min, y_max, y_steps)
        if solved is None:
            # the reverse transform (to -> from), because images are resampled backwards (tps.py:50-51)
            coeffs = _coefficients(to_points, from_points)
            pts = torch.from_numpy(np.ascontiguousarray(np.asarray(to_points, np.float64))).to(device)
            co = torch.from_numpy(np.ascontiguousarray(coeffs, np.float64)).to(device)
        else:
            pts, co = solved
        self.grid = ops.tps_grid(pts, co, nx, ny, x_min, xstep, y_min, ystep)
        self.upsample = None if approximate_grid == 1 else (x_steps, x_max - x_min, y_steps, y_max - y_min)
        self.shape = (nx, ny) if self.upsample is None else (x_max - x_min + 1, y_max - y_min + 1)

    def sample(self, img, order=1):
        """map_coordinates(img planes, this map, order) — img [ih, iw] or [ih, iw, cn] on the device."""
        return ops.tps_sample(self.grid, img, order, self.upsample)


def _device(a):
    if isinstance(a, torch.Tensor):
        return a if a.is_cuda else a.cuda()
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def warp_images(from_points, to_points, images, output_region, interpolation_order=1, approximate_grid=2):
    """tps.warp_images (tps.py:14-34): warp each 2-D image by the TPS that maps from_points onto to_points.

    Planes of equal dtype and shape are resampled in one launch (interleaved).  Returns a list in input order:
    numpy arrays for numpy inputs, device tensors for torch inputs."""
    if interpolation_order not in (0, 1):
        raise NotImplementedError("warp_images: interpolation_order %r (the reference uses 0 or 1)"
                                  % (interpolation_order,))
    images = list(images)
    if not images:
        return []
    as_numpy = not isinstance(images[0], torch.Tensor)
    dev = [_device(im) for im in images]
    for d in dev:
        if d.dim() != 2:
            raise ValueError("warp_images: every image must be 2-D, got %s" % (tuple(d.shape),))
    device = dev[0].device
    inv = InverseWarp(from_points, to_points, output_region, approximate_grid, device)
    out = [None] * len(dev)
    groups = {}
    for i, d in enumerate(dev):
        groups.setdefault((d.dtype, tuple(d.shape)), []).append(i)
    for idx in groups.values():
        stack = dev[idx[0]][:, :, None] if len(idx) == 1 else torch.stack([dev[i] for i in idx], dim=-1)
        res = inv.sample(stack, interpolation_order)
        for k, i in enumerate(idx):
            out[i] = res[:, :, k]
    if as_numpy:
        return [o.cpu().numpy() for o in out]
    return out


def deform_grid(h, w, n=5, fact=0.05):
    """The landmark draws of tps.deform (tps.py:127-143): a regular n x n grid and its perturbation, one
    np.random.uniform per interior coordinate, column before row (host RNG, the reference's order)."""
    bound = min(w, h) * fact
    vec1 = (h / (n - 1)) * np.arange(n)
    vec2 = (w / (n - 1)) * np.arange(n)
    grid = np.transpose([np.repeat(vec1, n), np.tile(vec2, n)])
    # the reference's loop draws one np.random.uniform(-bound, bound) per interior coordinate, point by point, x
    # before y; the legacy RandomState gives the same doubles drawn as one array in that order (off + scale * u
    # each), so the draws are made at once and scattered (~10x less host time per sample)
    inner = np.stack([(grid[:, 1] > 0.) & (grid[:, 1] < w), (grid[:, 0] > 0.) & (grid[:, 0] < h)], axis=1).ravel()
    d = np.zeros(2 * n * n)
    d[inner] = np.random.uniform(-bound, bound, size=int(inner.sum()))
    new_grid = grid.copy()
    new_grid[:, 1] += d[0::2]  # + 0.0 where no draw: the coordinate unchanged
    new_grid[:, 0] += d[1::2]
    return grid, new_grid


def deform(img):
    """tps.deform (tps.py:126-149): random TPS deformation of a BGR image -> (h+1, w+1, 3).  The reference's
    commented-out arrow drawing is not reproduced."""
    h, w = img.shape[:2]
    grid, new_grid = deform_grid(h, w)
    d = _device(img)
    inv = InverseWarp(grid, new_grid, (0, 0, h, w), 2, d.device)
    res = inv.sample(d, 1)
    return res.cpu().numpy() if not isinstance(img, torch.Tensor) else res
