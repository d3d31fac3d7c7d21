"""CPU checks of the config-5 training step's host side and its oracle (no GPU):
the torch-f64 restatement's forward equals the numpy oracle (pinned by the reference builders' goldens), its
gradients pass a finite-difference probe, the flat parameter layout covers the trainable variables, TF-Adam's
oracle behaves as ApplyAdam, and the DDP gradient all-reduce is correct at world size 2 (gloo)."""

import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from oracle import models as om
from oracle import ops as oops
from oracle import train_ref as tr
from vmatting.train import param_layout


def _case(n=1, h=20, w=24, seed=3):
    rs = np.random.RandomState(seed)
    mean = np.array([103.939, 116.779, 123.68])
    fg = rs.uniform(0, 255, (n, h, w, 3))
    bg = rs.uniform(0, 255, (n, h, w, 3))
    gt = rs.uniform(0, 1, (n, h, w, 1))
    cmp = gt * fg + (1 - gt) * bg - mean
    warped = np.repeat(gt, 3, -1)
    return cmp, bg - mean, warped, gt, fg


@pytest.fixture(scope="module")
def small_vgg():
    return om.synthetic_vgg16(0)


def test_restatement_forward_matches_numpy_oracle(small_vgg):
    cmp, bg, warped, gt, fg = _case()
    p = om.unet_simple_params(np.random.RandomState(1))
    terms, alpha, grads = tr.train_step_grads(cmp, bg, warped, gt, fg, small_vgg, p)
    ref = om.unet_simple_forward(cmp, bg, warped, True, small_vgg, p)
    assert np.abs(alpha - ref["output"]).max() <= 1e-10
    np.testing.assert_allclose(terms, oops.matting_loss(ref["output"], gt, fg, bg, cmp), rtol=1e-9)
    assert set(grads) == {(s, k) for s, k, _, _ in param_layout()[0]}


def test_restatement_gradient_finite_difference(small_vgg):
    """Central differences on a few filter/gamma entries of the deepest and shallowest layers."""
    cmp, bg, warped, gt, fg = _case(h=16, w=16, seed=4)
    p = om.unet_simple_params(np.random.RandomState(2))
    _, _, grads = tr.train_step_grads(cmp, bg, warped, gt, fg, small_vgg, p)
    for scope, idx in (("output", (1, 1, 3, 0)), ("conv2", (0, 2, 5, 7)), ("upconv3", (2, 1, 10, 4))):
        h = 1e-4
        w = p[scope][0].astype(np.float64)
        vals = []
        for s in (h, -h):
            q = dict(p)
            w2 = w.copy()
            w2[idx] += s
            q[scope] = (w2, p[scope][1])
            vals.append(tr.train_step_grads(cmp, bg, warped, gt, fg, small_vgg, q)[0][0])
        fd = (vals[0] - vals[1]) / (2 * h)
        assert abs(fd - grads[scope, "w"][idx]) <= 1e-5 * max(1.0, abs(fd)) + 1e-7, (scope, fd, grads[scope, "w"][idx])


def test_param_layout_is_the_trainable_set():
    from vmatting.train import param_layout
    from vmatting.unet_simple import NEW_CONVS
    lay, n = param_layout()
    conv = sum(9 * ci * co for _, ci, co in NEW_CONVS)
    bias = sum(co for s, _, co in NEW_CONVS if not s.startswith("upconv"))
    bnw = sum({"upconv4": 96, "upconv3": 48, "upconv2": 32, "upconv1": 30}.get(s, co) for s, _, co in NEW_CONVS)
    assert n == conv + bias + 2 * bnw
    assert 1.5e6 < n < 1.7e6  # ~1.62M trainable simple_unet parameters
    offs = [o for _, _, o, _ in lay]
    assert offs == sorted(offs) and len(set(offs)) == len(offs)
    assert not any(s.startswith("upconv") and k == "b" for s, k, _, _ in lay)


def test_adam_oracle_first_step_is_lr_sign():
    g = np.array([3.0, -0.5, 1e-3, -20.0], np.float32)
    var, m, v = tr.adam_tf(np.zeros(4, np.float32), np.zeros(4, np.float32), np.zeros(4, np.float32), g, 1)
    np.testing.assert_allclose(var, -1e-3 * np.sign(g), rtol=1e-3)  # eps costs 3e-4 at |g| = 1e-3
    np.testing.assert_allclose(m, 0.1 * g, rtol=1e-6)


def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from vmatting import parallel
    parallel.init_from_env(backend="gloo")
    try:
        g = torch.arange(10, dtype=torch.float32) * (rank + 1)
        scale = parallel.allreduce_grads(g)
        ok = scale == 0.5 and torch.equal(g * scale, torch.arange(10, dtype=torch.float32) * 1.5)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_gradient_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    assert sorted(r for r, _ in res) == [0, 1] and all(ok for _, ok in res), res


# ---------------------------------------------------------------------------- small_train.py (UNetSmall, all variables)

def _small_case(n=2, h=18, w=22, seed=6):
    rs = np.random.RandomState(seed)
    mean = np.array([103.939, 116.779, 123.68])
    fg = rs.uniform(0, 255, (n, h, w, 3))
    bg = rs.uniform(0, 255, (n, h, w, 3))
    gt = rs.uniform(0, 1, (n, h, w, 1))
    return gt * fg + (1 - gt) * bg - mean, bg - mean, gt, fg


def test_small_restatement_forward_and_layout():
    """small_step_grads' forward equals the numpy oracle (pinned by the small_70x90_train golden), and its gradient
    keys are exactly SmallTrainer's flat layout: every variable of small.py except the upconvs' unused biases."""
    from vmatting.small_train import param_layout as small_layout
    cmp, bg, gt, fg = _small_case()
    p = om.unet_small_params(np.random.RandomState(1), cin=6)
    terms, alpha, grads, _ = tr.small_step_grads(cmp, bg, gt, fg, p)
    ref = om.unet_small_forward(np.concatenate([cmp, bg], -1), True, p)
    assert np.abs(alpha - ref["output"]).max() <= 1e-10
    np.testing.assert_allclose(terms, oops.matting_loss(ref["output"], gt, fg, bg, cmp), rtol=1e-9)
    layout, total = small_layout(6)
    assert set(grads) == {(s, k) for s, k, _, _ in layout}
    assert total == sum(int(np.prod(g.shape)) for g in grads.values())


def test_small_restatement_gradient_finite_difference():
    """Central differences through the max-pools, the [skip, up] concats' BN and the first (6-channel) conv."""
    cmp, bg, gt, fg = _small_case(h=14, w=15, seed=8)
    p = om.unet_small_params(np.random.RandomState(2), cin=6)
    _, _, grads, _ = tr.small_step_grads(cmp, bg, gt, fg, p)
    for scope, idx in (("conv1_1", (0, 2, 5, 3)), ("conv2_1", (1, 1, 4, 9)), ("upconv1", (2, 0, 7, 5)),
                       ("conv1_3", (1, 2, 6, 0))):
        h = 1e-5
        w = p[scope][0].astype(np.float64)
        vals = []
        for s in (h, -h):
            q = dict(p)
            w2 = w.copy()
            w2[idx] += s
            q[scope] = (w2, p[scope][1])
            vals.append(tr.small_step_grads(cmp, bg, gt, fg, q)[0][0])
        fd = (vals[0] - vals[1]) / (2 * h)
        g = grads[scope, "w"][idx]
        assert abs(fd - g) <= 1e-5 * max(1e-6, abs(g)) + 1e-9, (scope, fd, g)


def test_image_step_oracle_forward_matches_numpy_oracle():
    """oracle/train_ref.image_step_grads (the UNetImage training step's autograd oracle, train.py:37-109) runs the
    same forward as oracle/models.unet_forward, which the reference's builders pin (unet_image_70x90 golden), and
    yields a gradient for every variable train.py:51-52 trains: 20 filters + 16 biases (no upconv biases)."""
    vgg = om.synthetic_vgg16(0)
    p = om.unet_params(vgg, np.random.RandomState(3), video=False)
    rs = np.random.RandomState(1)
    n, h, w = 1, 21, 27
    cmp, bg = rs.uniform(-100, 100, (n, h, w, 3)), rs.uniform(-100, 100, (n, h, w, 3))
    gt, fg = rs.uniform(0, 1, (n, h, w, 1)), rs.uniform(0, 255, (n, h, w, 3))
    terms, alpha, grads, fwd = tr.image_step_grads(cmp, bg, gt, fg, p)
    r = om.unet_forward(np.concatenate([cmp, bg], -1), p)
    for k in ("conv1_2", "pool2", "conv4_3", "conv5_2", "upconv1", "upconv4", "conv1_3", "output"):
        assert np.abs(r[k] - fwd[k]).max() <= 1e-12 * max(1.0, np.abs(r[k]).max()), k
    assert len(grads) == 36
    assert not any(s.startswith("upconv") for s, k in grads if k == "b")
    assert all(np.isfinite(g).all() for g in grads.values())


def test_split6_filter_parts_reconstruct_the_filter():
    """vmatting/split6.py: the filter's three bf16 parts (h, m, l) sum back to the f32 filter to within 2^-24 of
    each weight, each part is exactly representable in bf16, and the stack follows the slab order [h, m, l, h, m, h]
    with zero padding rows past cin."""
    from vmatting.split6 import split6_filter, W_PARTS
    rs = np.random.RandomState(0)
    w = (rs.normal(size=(3, 3, 5, 7)) * np.logspace(-3, 2, 7)).astype(np.float32)
    s = split6_filter(w, 8, 7).numpy().astype(np.float64)
    assert s.shape == (3, 3, 48, 7)
    parts = [s[:, :, p * 8:p * 8 + 5] for p in range(3)]
    assert np.all(np.abs(parts[0] + parts[1] + parts[2] - w) <= 2.0 ** -24 * np.abs(w))
    for p in range(6):
        blk = s[:, :, p * 8:(p + 1) * 8]
        assert not blk[:, :, 5:].any()
        assert np.array_equal(blk[:, :, :5], parts[W_PARTS[p]])
        t = torch.from_numpy(blk.astype(np.float32))
        assert torch.equal(t.bfloat16().float(), t)
