"""Augmentation row on the GPU: measured deviation from the oracle (TPS map, warped planes) and 1080p timing."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import golden  # noqa: E402
from oracle import augment as oa  # noqa: E402
from vmatting import augmentation as va, tps  # noqa: E402

g = golden("tps")
for n in "abcd":
    reg = tuple(int(v) for v in g[n + "_region"]); ag = float(g[n + "_ag"]); ag = int(ag) if ag == int(ag) else ag
    planes = [g["img"][:, :, 0], g["img"][:, :, 1], g["img"][:, :, 2], g["alpha"], g[n + "_f32_in"]]
    r = tps.warp_images(g[n + "_from"], g[n + "_to"], planes, reg, int(g[n + "_order"]), ag)
    u8 = np.stack(r[:3], -1).astype(int) - g[n + "_u8"]
    print("tps %s: u8 differing %d, f64 max %.3g, f32 max %.3g" % (n, (u8 != 0).sum(), np.abs(r[3] - g[n + "_f64"]).max(),
                                                                  np.abs(r[4] - g[n + "_f32"]).max()))
a = golden("augment")
for i in range(2):
    np.random.seed(int(a["seed%d" % i]))
    f, b, al = va.augment(a["fg%d" % i], a["bg%d" % i], a["alpha%d" % i])
    print("augment %d: fg differing %d, bg equal %s, alpha max %.3g" % (
        i, (f != a["new_fg%d" % i]).sum(), np.array_equal(b, a["new_bg%d" % i]), np.abs(al - a["new_alpha%d" % i]).max()))

h, w = 1080, 1920
rs = np.random.RandomState(9)
yy, xx = np.mgrid[0:h, 0:w]
alpha = torch.from_numpy(np.clip(1.2 - np.sqrt(((yy - 500) / 300.) ** 2 + ((xx - 900) / 400.) ** 2), 0, 1)).cuda()
fg = torch.from_numpy((rs.rand(h, w, 3) * 255).astype(np.uint8)).cuda()
bg = torch.from_numpy((rs.rand(h, w, 3) * 255).astype(np.uint8)).cuda()
inv = tps.InverseWarp(*tps.deform_grid(h, w), (0, 0, h, w), 2)
print("grid", tuple(inv.grid.shape))
for _ in range(3):
    va.augment(fg, bg, alpha)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    va.augment(fg, bg, alpha)
torch.cuda.synchronize()
print("augment 1080p: %.3f ms/sample wall (host draws + pinv + 1 sync + kernels)" % (1e3 * (time.perf_counter() - t0) / n))
