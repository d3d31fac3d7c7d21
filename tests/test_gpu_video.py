"""BASELINE config 4 on the GPU: the product's frame-parallel path (video.py: shard -> chunked HIP-graph replay ->
all-gather) over synthetic 1080p frames, checked frame by frame.

* bf16: every gathered matte is bit-equal to a standalone single-frame forward() of that frame (the chunked,
  graph-replayed, batched path changes nothing about a frame's arithmetic);
* fp32: one sampled frame's alpha within 1e-4 max-abs of the numpy f32 oracle (north_star's bound), its logits
  within 1e-4 of their scale.
World 1 here, plus world 2 as two processes sharing the one GPU over gloo (the real model, broadcast, graphs and
the uneven gather); the sharding / gather arithmetic alone is covered with gloo on CPU in test_host.py.
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


def test_shape_switch_after_dropped_graph(vgg0):
    """a captured forward's buffer set is allocated on the warm-up side stream and replayed on the
    caller's stream (GraphedForward records that use).  Capture at one shape, replay, drop the graph, switch the model
    to other shapes (the old set is freed and its memory handed out again) and back: every output equals a fresh
    model's eager forward bit for bit."""
    import gc
    from vmatting import unet, video
    np.random.seed(0)
    m = unet.UNetVideo(vgg0, dtype="bf16", device="cuda").prepare()
    np.random.seed(0)
    ref = unet.UNetVideo(vgg0, dtype="bf16", device="cuda").prepare()
    fa = video.synthetic_frames(2, 136, 250, first=3)
    fb = video.synthetic_frames(1, 70, 90, first=4)
    g = m.capture(fa)
    for _ in range(3):
        g.replay()
    got_a = g.output.clone()
    del g
    gc.collect()
    outs = [m.forward(fb).clone(), m.forward(video.synthetic_frames(3, 40, 64, first=5)).clone(), m.forward(fa).clone()]
    torch.cuda.synchronize()
    assert torch.equal(got_a, ref.forward(fa))
    assert torch.equal(outs[0], ref.forward(fb))
    assert torch.equal(outs[2], got_a)


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


def _world2_worker(rank, world, port, q, n_frames, h, w, chunk):
    """One rank of the real frame-parallel path on the shared cuda:0 (gloo moves the device tensors): its own
    init_conv draws, rank 0's packed weights broadcast into them, its uneven shard through video.matte_video (chunked
    graph replay), the all-gather of the mattes; then every gathered matte against a standalone forward() with the
    broadcast weights."""
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from vmatting import parallel, unet, video
        from vmatting.weights import synthetic_vgg16
        parallel.init_from_env(backend="gloo")
        torch.cuda.set_device(0)
        np.random.seed(100 + rank)  # each rank draws different init_conv filters: the broadcast must replace them
        model = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device="cuda:0").prepare()
        mine = torch.cat([t.reshape(-1).view(torch.uint8) for t in model.weights_flat()]).clone()
        parallel.broadcast_tensors(model.weights_flat(), src=0)
        flat = torch.cat([t.reshape(-1).view(torch.uint8) for t in model.weights_flat()])
        a, b = video.shard(n_frames)
        frames = video.synthetic_frames(b - a, h, w, first=a, device="cuda:0")
        full, vm = video.matte_video(model, frames, n_frames, chunk=chunk)
        torch.cuda.synchronize()
        got = full.clone()
        # replicas: identical weights after the broadcast (rank 1's own draws differed before it)
        sums = [torch.empty(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(sums, torch.tensor([float(flat.double().sum()), float(mine.double().sum())],
                                           dtype=torch.float64))
        ok_w = all(float(s[0]) == float(sums[0][0]) for s in sums) and float(sums[1][1]) != float(sums[0][1])
        ok_shape = tuple(got.shape) == (n_frames, h, w, 1)
        allf = video.synthetic_frames(n_frames, h, w, first=0, device="cuda:0")
        bad = []
        for i in range(n_frames):
            ref = model.forward(allf[i:i + 1].clone())[0]
            if not torch.equal(ref, got[i]):  # (frame, max |diff|, differing pixels, first one) for the report
                d = (ref.float() - got[i].float()).abs()
                bad.append((i, float(d.max()), int((d > 0).sum()), tuple(int(v) for v in (d > 0).nonzero()[0])))
        q.put((rank, ok_w, ok_shape, bad, len(vm.spans)))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, False, False, [repr(e), traceback.format_exc()[-800:]], 0))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_frame_parallel_world2_real_model():
    """Config 4's product path at world 2 on the one GPU (two processes on cuda:0, gloo): rank-0 weight broadcast
    into captured graphs, an uneven 4/3 split of 7 frames, graph replay on rank 1, the matte all-gather — every
    gathered matte bit-equal to rank 0's standalone forward() of that frame (train.py:318-332's frame loop)."""
    import multiprocessing as mp
    import os
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29200 + (os.getpid() % 500)
    procs = [ctx.Process(target=_world2_worker, args=(r, 2, port, q, 7, 270, 480, 2)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(30)
    assert [r[0] for r in res] == [0, 1], res
    for rank, ok_w, ok_shape, bad, spans in res:
        assert ok_w and ok_shape and bad == [], (rank, ok_w, ok_shape, bad)
    assert [r[4] for r in res] == [2, 2]  # 4 frames -> 2 chunks of 2; 3 frames -> 2 + 1


def _contention_worker(rank, q, seconds, h, w):
    """One of two processes sharing cuda:0: chunked graph replay (video.matte_video) vs standalone forward() of the
    same frames, over and over, with the 4 x 32-pixel patch tiling forced on every patch-kernel layer."""
    import time
    try:
        from vmatting import _lib, unet, video
        from vmatting.weights import synthetic_vgg16
        torch.cuda.set_device(0)
        _lib.set_option("patch_cfg", 25)
        np.random.seed(100)
        model = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device="cuda:0").prepare()
        frames = video.synthetic_frames(4, h, w, first=4 * rank, device="cuda:0")
        t0, it, bad = time.time(), 0, []
        while time.time() - t0 < seconds:
            full, _ = video.matte_video(model, frames, 4, chunk=2)
            torch.cuda.synchronize()
            got = full.clone()
            for i in range(4):
                ref = model.forward(frames[i:i + 1].clone())[0]
                if not torch.equal(ref, got[i]):
                    bad.append((it, i, float((ref - got[i]).abs().max())))
            it += 1
        q.put((rank, it, bad[:5], len(bad)))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, 0, [repr(e), traceback.format_exc()[-800:]], -1))


def test_graph_vs_eager_under_contention():
    """Two processes on the one GPU, each replaying chunked HIP graphs and the eager forward of the same frames for
    ~20 s: every matte bit-identical.  Regression test for the LDS race fixed in r03 (a ring slot's refill DMA could
    overtake a queued fragment read when the consuming MFMAs were scheduled past the slot-release barrier; with a
    second process on the GPU about 1 % of the frames differed, with the 4 x 32 tiling several per second)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_contention_worker, args=(r, q, 20.0, 270, 480)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=115) for _ in procs)
    for p in procs:
        p.join(30)
    for rank, iters, bad, nbad in res:
        assert nbad == 0 and iters > 50, (rank, iters, nbad, bad)
