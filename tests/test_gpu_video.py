"""BASELINE config 4 on the GPU: the product's frame-parallel path (video.py: shard -> chunked HIP-graph replay ->
all-gather) over synthetic 1080p frames, checked frame by frame.

* bf16: every gathered matte is bit-equal to a standalone single-frame forward() of that frame (the chunked,
  graph-replayed, batched path changes nothing about a frame's arithmetic);
* fp32: one sampled frame's alpha within 1e-4 max-abs of the numpy f32 oracle (north_star's bound), its logits
  within 1e-4 of their scale.
World 1 here (the box has one GPU); the world-2 sharding / gather arithmetic is covered with gloo in test_host.py.
"""

import numpy as np
import pytest
import torch

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

H, W = 1080, 1920


@pytest.fixture(scope="module")
def model_bf16(vgg0):
    from vmatting import unet
    np.random.seed(0)
    return unet.UNetVideo(vgg0, dtype="bf16", device="cuda").prepare()


@pytest.mark.parametrize("n_frames,rank,world,chunk", [(32, 0, 1, 8), (37, 1, 3, 8), (5, 2, 3, 4)])
def test_video_batch_bit_equal_to_single_frames(model_bf16, n_frames, rank, world, chunk):
    from vmatting import parallel, video
    a, b = video.shard(n_frames, rank, world)
    assert (a, b) == parallel.shard_range(n_frames, rank, world)
    frames = video.synthetic_frames(b - a, H, W, first=a)
    full, vm = video.matte_video(model_bf16, frames, n_frames if world == 1 else b - a, chunk=chunk)
    torch.cuda.synchronize()
    assert tuple(full.shape) == (b - a, H, W, 1)
    got = full.clone()
    for i in range(b - a):
        one = model_bf16.forward(frames[i:i + 1].clone()).clone()
        assert torch.equal(one[0], got[i]), "frame %d differs from its standalone forward" % (a + i)
    # a second replay of the same graphs reproduces the result (no stale state between chunks)
    vm.run()
    torch.cuda.synchronize()
    assert torch.equal(vm.alpha, got)
    assert float(got.min()) >= 0.0 and float(got.max()) <= 1.0


def test_video_batch_eager_equals_graph(model_bf16):
    from vmatting import video
    frames = video.synthetic_frames(3, 136, 250, first=7)
    g = video.VideoMatter(model_bf16, frames, chunk=2, graph=True).run().clone()
    e = video.VideoMatter(model_bf16, frames, chunk=2, graph=False).run().clone()
    assert torch.equal(g, e)


@pytest.mark.slow
def test_video_batch_fp32_frame_vs_oracle(vgg0):
    """One sampled 1080p frame of the config-4 path in fp32 against the oracle: alpha within 1e-4."""
    from oracle import models as om
    from vmatting import unet, video
    np.random.seed(0)
    m = unet.UNetVideo(vgg0, dtype="fp32", device="cuda").prepare()
    frames = video.synthetic_frames(2, H, W, first=100)
    full, _ = video.matte_video(m, frames, 2, chunk=2)
    torch.cuda.synchronize()
    x = frames[1:2].cpu().numpy()
    r = om.unet_forward(x, m.params, dtype=np.float32)
    err = float(np.abs(full[1].cpu().numpy() - r["output"][0]).max())
    print("config-4 sampled frame: fp32 alpha max-abs err vs oracle %.3e" % err)
    assert err <= 1e-4
    lg = m.conv1_3[1].cpu().numpy()  # logits of the last chunk's frames (the model's buffer)
    assert np.abs(lg - r["conv1_3"][0]).max() <= 1e-4 * np.abs(r["conv1_3"]).max() + 1e-4
