"""The split-bf16 x6 forward (vmatting/split6.py, UNetVideo(dtype="bf16x6")): unet.py's forward (unet.py:86-217)
at f32 accuracy on the bf16 MFMA kernels.

  split kernel   vm_split6_nhwc bit-exact against the same three-part RNE split in torch (CPU), incl. the fused
                 2x2 SAME pool (odd sizes), channel padding and a segment of a concat buffer
  filter split   the three parts of every filter sum back to it exactly in float64 (CPU, test_host-style)
  goldens        the reference-generated goldens (tests/golden/unet_*_70x90.npz): alpha within 1e-4
  1080p          the bench's timed frame and weights: alpha within 1e-4 of the CPU oracle (numpy f32, the
                 reference's op sequence) — north_star's bound — and logits within the fp32 path's relative error
"""

import numpy as np
import pytest
import torch

from conftest import golden, gpu_available
from oracle import models as om

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"


def H(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _split_ref(x):
    """x f32 (CPU torch) -> the six slabs [l, m, h, m, h, h] as bf16 (torch's RNE conversion)."""
    h = x.bfloat16()
    r = x - h.float()
    m = r.bfloat16()
    lo = (r - m.float()).bfloat16()
    return [lo, m, h, m, h, h]


@pytest.mark.parametrize("n,h,w,c,S,off", [(2, 7, 9, 7, 8, 0), (1, 16, 33, 64, 64, 0), (1, 5, 6, 128, 256, 128),
                                           (2, 3, 5, 24, 40, 16)])
@pytest.mark.parametrize("pool", [False, True])
def test_split6_kernel_bit_exact(n, h, w, c, S, off, pool):
    from vmatting.split6 import split6
    torch.manual_seed(c + h)
    x = (torch.randn(n, h, w, c + 3) * torch.logspace(-6, 4, c + 3)).float()
    xd = x.to(DEV)[..., 1:1 + c]  # a channel-slice f32 view
    buf = torch.zeros((n, h, w, 6 * S), dtype=torch.bfloat16, device=DEV)
    cc = (c + 7) // 8 * 8
    pb = None
    if pool:
        pb = torch.zeros((n, (h + 1) // 2, (w + 1) // 2, 6 * S), dtype=torch.bfloat16, device=DEV)
    split6(xd, buf[..., off:off + cc], None if pb is None else pb[..., off:off + cc])
    torch.cuda.synchronize()
    xs = x[..., 1:1 + c]
    xp = torch.zeros((n, h, w, cc))
    xp[..., :c] = xs
    got = buf.cpu()
    for p, ref in enumerate(_split_ref(xp)):
        assert torch.equal(got[..., p * S + off:p * S + off + cc].view(torch.int16), ref.view(torch.int16)), p
    # h + m + l carries x's 24 bits (the last part's own rounding at most 2^-25 of x)
    parts = [got[..., p * S + off:p * S + off + c].double() for p in range(3)]
    assert ((parts[0] + parts[1] + parts[2] - xs.double()).abs() <= 2.0 ** -24 * xs.double().abs()).all()
    if pool:
        ph, pw = (h + 1) // 2, (w + 1) // 2
        xx = torch.full((n, 2 * ph, 2 * pw, cc), -float("inf"))
        xx[:, :h, :w] = xp
        mx = xx.view(n, ph, 2, pw, 2, cc).amax(dim=(2, 4))
        gp = pb.cpu()
        for p, ref in enumerate(_split_ref(mx)):
            assert torch.equal(gp[..., p * S + off:p * S + off + cc].view(torch.int16), ref.view(torch.int16)), p


@pytest.mark.parametrize("case", ["unet_video_70x90", "unet_video_64x96", "unet_image_70x90"])
def test_unet_bf16x6_matches_reference_golden(case, vgg0):
    from vmatting import unet
    g = golden(case)
    cls = unet.UNetVideo if int(g["video"]) else unet.UNetImage
    np.random.seed(int(g["weight_seed"]))
    m = cls(vgg0, dtype="bf16x6")
    m.build(g["x"])
    torch.cuda.synchronize()
    alpha, logits = H(m.output), H(m.conv1_3)
    err = np.abs(alpha - g["output"]).max()
    print("%s bf16x6 alpha max-abs %.3g, logits rel %.3g" % (case, err, np.abs(logits - g["logits"]).max()
                                                               / np.abs(g["logits"]).max()))
    assert err <= 1e-4
    assert np.all(np.abs(logits - g["logits"]) <= 1e-4 * np.abs(g["logits"]).max() + 1e-4)


def test_unet_bf16x6_graph_equals_eager(vgg0):
    from vmatting import unet
    np.random.seed(0)
    m = unet.UNetVideo(vgg0, dtype="bf16x6")
    m.prepare()
    x = torch.randn(2, 72, 100, 7, device=DEV) * 40
    a = m.forward(x).clone()
    g = m.capture(x)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(g.output, a)


@pytest.mark.slow
def test_unet_bf16x6_1080p_timed_frame_vs_oracle():
    """north_star's bound on the bench's own frame and weights: the bf16x6 alpha within 1e-4 max-abs of the CPU
    oracle's float32 forward (the reference's op sequence), where the bf16 path is 0.45 off."""
    from vmatting import unet, video
    from vmatting.weights import synthetic_vgg16
    np.random.seed(0)
    m = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16x6")
    m.prepare()
    x = video.synthetic_frames(1, 1080, 1920, first=0, device=DEV)
    alpha = H(m.forward(x))
    logits = H(m.conv1_3)
    r = om.unet_forward(x.cpu().numpy(), m.params, dtype=np.float32)
    err = np.abs(alpha - r["output"]).max()
    lrel = np.abs(logits - r["conv1_3"]).max() / np.abs(r["conv1_3"]).max()
    print("1080p bf16x6 alpha max-abs vs oracle %.3e, logits rel %.3e" % (err, lrel))
    assert err <= 1e-4
    assert lrel <= 1e-5
