"""small_train.py's training step (vmatting/small_train.py SmallTrainer) against the float64 autograd restatement
(oracle/train_ref.py small_step_grads): UNetSmall(concat(cmp, bg), phase=True) (small.py:37-50), the loss of
small_train.py:39-44, Adam over every variable (small_train.py:47-48).  Plus the max-pool adjoint kernel on its own
(TF MaxPoolGrad's first-maximum tie rule), DDP replicas and SyncBN with unequal per-rank batches."""

import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from conftest import gpu_available
from oracle import models as om
from oracle import ops as oops
from oracle import train_ref as tr

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"


def T(a, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV, dtype)


def H(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _maxpool_bwd_ref(x, dy, add=None):
    """TF MaxPoolGrad for 2x2/2 SAME: each window's gradient to its first maximum in row-major order."""
    n, h, w, c = x.shape
    dx = np.zeros_like(x, dtype=np.float64) if add is None else np.array(add, np.float64)
    for oy in range(dy.shape[1]):
        for ox in range(dy.shape[2]):
            win = [(2 * oy + a, 2 * ox + b) for a in (0, 1) for b in (0, 1) if 2 * oy + a < h and 2 * ox + b < w]
            vals = np.stack([x[:, yy, xx] for yy, xx in win], 0)  # [k, n, c]
            first = np.argmax(vals, axis=0)  # argmax returns the first maximum
            for k, (yy, xx) in enumerate(win):
                dx[:, yy, xx] += np.where(first == k, dy[:, oy, ox], 0.0)
    return dx


@pytest.mark.parametrize("shape", [(2, 9, 13, 16), (1, 8, 8, 8), (1, 1, 1, 3), (2, 17, 6, 32), (1, 5, 5, 40)])
@pytest.mark.parametrize("xdtype", ["fp32", "bf16"])
@pytest.mark.parametrize("add", [None, "separate", "inplace"])
def test_maxpool_backward(shape, xdtype, add):
    """vm_maxpool2x2_backward_nhwc vs TF's rule, with many exact ties (values drawn from a few levels, relu zeros)
    and odd edges; the optional skip gradient added, also in place."""
    from vmatting import ops
    n, h, w, c = shape
    rs = np.random.RandomState(h * w + c)
    x = np.maximum(rs.randint(-2, 4, size=shape), 0).astype(np.float32) * 0.5  # ties everywhere
    dy = rs.normal(size=(n, (h + 1) // 2, (w + 1) // 2, c)).astype(np.float32)
    a = rs.normal(size=shape).astype(np.float32) if add else None
    tdt = torch.float32 if xdtype == "fp32" else torch.bfloat16
    xd = T(x, tdt)
    if add == "inplace":
        dx = T(a)
        ops.maxpool_backward(xd, T(dy), dx, add=dx)
    else:
        dx = torch.full(shape, 9.0, device=DEV)
        ops.maxpool_backward(xd, T(dy), dx, add=None if a is None else T(a))
    want = _maxpool_bwd_ref(x.astype(np.float64), dy.astype(np.float64), a)
    assert np.abs(H(dx) - want).max() <= 1e-6, np.abs(H(dx) - want).max()


def _small_batch(n, h, w, seed=3):
    rs = np.random.RandomState(seed)
    mean = np.array([103.939, 116.779, 123.68])
    fg = rs.uniform(0, 255, (n, h, w, 3))
    bg = rs.uniform(0, 255, (n, h, w, 3))
    yy, xx = np.mgrid[:h, :w]
    gt = np.clip(1.2 - np.hypot((yy - h / 2) / (h / 3), (xx - w / 2) / (w / 3)), 0, 1)[None, :, :, None]
    gt = np.clip(np.repeat(gt, n, 0) + rs.normal(0, 0.05, (n, h, w, 1)), 0, 1)
    cmp = gt * fg + (1 - gt) * bg - mean
    f = lambda a: a.astype(np.float32)  # noqa: E731
    return f(cmp), f(bg - mean), f(gt), f(fg)


def _bn_draw(params, seed=2):
    rs = np.random.RandomState(seed)
    width = {"upconv1": 32, "upconv2": 16}
    return {k: (rs.uniform(0.5, 1.5, width.get(k, w.shape[3])).astype(np.float32),
                rs.normal(0, 0.2, width.get(k, w.shape[3])).astype(np.float32)) for k, (w, _) in params.items()}


@pytest.fixture(scope="module", params=[(2, 64, 64), (2, 37, 45)], ids=["2x64x64", "2x37x45"])
def small_case(request):
    from vmatting.small_train import SmallTrainer
    n, h, w = request.param
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    bn = _bn_draw(params)
    cmp, bg, gt, fg = _small_batch(n, h, w)
    trn = SmallTrainer(6, "fp32", DEV, params=params, bn=bn)
    p0 = H(trn.flat).astype(np.float32)
    loss = H(trn.step(cmp, bg, gt, fg))
    torch.cuda.synchronize()
    terms, alpha, grads, _ = tr.small_step_grads(cmp, bg, gt, fg, params, bn)
    return dict(trn=trn, p0=p0, loss=loss, terms=terms, alpha=alpha, grads=grads, alpha_gpu=H(trn.output))


def test_small_oracle_forward_matches_numpy_oracle():
    """The autograd restatement's forward equals models.unet_small_forward (pinned by the reference builder's
    small_70x90_train golden) on the concat(cmp, bg) input."""
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    cmp, bg, gt, fg = _small_batch(2, 21, 30)
    _, alpha, _, fwd = tr.small_step_grads(cmp, bg, gt, fg, params)
    ref = om.unet_small_forward(np.concatenate([cmp, bg], -1), True, params)
    assert np.abs(alpha - ref["output"]).max() <= 1e-10
    assert np.abs(fwd["conv1_3"] - ref["conv1_3"]).max() <= 1e-8 * max(1.0, np.abs(ref["conv1_3"]).max())


def test_small_step_loss_and_alpha(small_case):
    c = small_case
    np.testing.assert_allclose(c["loss"], c["terms"], rtol=1e-5)
    assert np.abs(c["alpha_gpu"] - c["alpha"]).max() <= 1e-4


def test_small_step_gradients(small_case):
    """Every variable's gradient (all 9 convs' filters and biases, every BN gamma / beta): relative L2 <= 2e-3 and
    max-abs <= 1.5e-2 of the tensor's max-abs (conv biases are zero in exact arithmetic — BN removes them — so they
    are bounded by their filter gradient's scale)."""
    c = small_case
    trn, grads = c["trn"], c["grads"]
    assert set(grads) == {(s, k) for s, k, _, _ in trn.layout}
    bad, worst = [], 0.0
    for (scope, kind), g_ref in grads.items():
        g = H(trn.G[scope, kind])
        ref_n = grads[scope, "w"] if kind == "b" else g_ref
        l2 = np.linalg.norm(g - g_ref) / max(np.linalg.norm(ref_n), 1e-30)
        mx = np.abs(g - g_ref).max() / max(np.abs(ref_n).max(), 1e-30)
        worst = max(worst, l2)
        if not (mx <= 1.5e-2 and l2 <= 2e-3):
            bad.append((scope, kind, round(float(l2), 6), round(float(mx), 6)))
    print("small step: worst relative L2 gradient error %.2e" % worst)
    assert not bad, bad


def test_small_step_adam_update(small_case):
    c = small_case
    trn = c["trn"]
    g = H(trn.grad).astype(np.float32)
    want, _, _ = tr.adam_tf(c["p0"], np.zeros_like(g), np.zeros_like(g), g, 1, lr=1e-5)
    assert np.abs(H(trn.flat) - want).max() <= 1e-6 * max(1.0, np.abs(want).max())
    # the packed forward filters follow the updated flat buffer
    from vmatting import ops
    pc = trn.convs["conv2_2"]
    x = torch.randn((1, 6, 7, pc.cin), device=DEV)
    fresh = ops.PackedConv(trn.P["conv2_2", "w"].clone(), trn.P["conv2_2", "b"].clone(), "fp32", DEV)
    assert torch.equal(ops.conv3x3(x, pc, "none", affine=False), ops.conv3x3(x, fresh, "none", affine=False))


def test_small_steps_stay_finite_and_decrease():
    """A few fp32 steps at lr 1e-3 on one batch: finite, and the loss goes down."""
    from vmatting.small_train import SmallTrainer
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    cmp, bg, gt, fg = _small_batch(2, 48, 40, seed=9)
    trn = SmallTrainer(6, "fp32", DEV, params=params, lr=1e-3)
    losses = [H(trn.step(cmp, bg, gt, fg))[0] for _ in range(8)]
    assert np.all(np.isfinite(losses)) and np.all(np.isfinite(H(trn.flat)))
    assert losses[-1] < losses[0], losses


@pytest.mark.slow
def test_small_step_bf16_gradients_bench_shape():
    """The bf16 step (bf16 activations, f32 pre-BN buffers, MFMA filter gradients, bf16 data-gradient convs) at
    small_train.py's batch (params.py:8-9: 8 x 320^2) against float64 autograd.  Self-calibrated bound as the config-5
    bench-shape test: per tensor relative L2 <= 3x the f64 gradient's sensitivity to bf16-sized relative noise
    (2^-9) on the filters and the input + 1e-2; whole-gradient cosine >= 0.99."""
    from vmatting.small_train import SmallTrainer
    n, h, w = 8, 320, 320
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    cmp, bg, gt, fg = _small_batch(n, h, w, seed=17)
    trn = SmallTrainer(6, "bf16", DEV, params=params)
    trn.forward(cmp, bg)
    trn.grad.zero_()
    trn.backward(T(gt), T(fg), T(bg), T(cmp))
    torch.cuda.synchronize()
    _, _, grads, _ = tr.small_step_grads(cmp, bg, gt, fg, params, device=DEV)
    rs = np.random.RandomState(7)
    nz = lambda a: (a * (1 + 2.0 ** -9 * rs.normal(size=a.shape))).astype(np.float32)  # noqa: E731
    p2 = {k: (nz(w_), b_) for k, (w_, b_) in params.items()}
    _, _, g2, _ = tr.small_step_grads(nz(cmp), nz(bg), gt, fg, p2, device=DEV)
    bad, got_all, ref_all, rows = [], [], [], []
    for (scope, kind), g_ref in grads.items():
        if kind == "b":
            continue
        g = H(trn.G[scope, kind])
        nrm = max(np.linalg.norm(g_ref), 1e-30)
        l2 = np.linalg.norm(g - g_ref) / nrm
        sens = np.linalg.norm(g2[scope, kind] - g_ref) / nrm
        got_all.append(g.ravel())
        ref_all.append(g_ref.ravel())
        rows.append("%s/%s %.3e (sens %.3e)" % (scope, kind, l2, sens))
        if not l2 <= 3 * sens + 1e-2:
            bad.append((scope, kind, round(float(l2), 4), round(float(sens), 4)))
    a, b_ = np.concatenate(got_all), np.concatenate(ref_all)
    cos = float(a @ b_ / (np.linalg.norm(a) * np.linalg.norm(b_)))
    print("small bf16 step 8x320^2: gradient cosine %.5f\n  %s" % (cos, "\n  ".join(rows)))
    assert not bad, bad
    assert cos >= 0.99


def test_small_bf16_steps_run():
    from vmatting.small_train import SmallTrainer
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    cmp, bg, gt, fg = _small_batch(2, 64, 48)
    trn = SmallTrainer(6, "bf16", DEV, params=params)
    losses = [H(trn.step(cmp, bg, gt, fg))[0] for _ in range(3)]
    assert np.all(np.isfinite(losses)) and np.all(np.isfinite(H(trn.grad)))
    terms, _, _, _ = tr.small_step_grads(cmp, bg, gt, fg, params)
    assert abs(losses[0] - terms[0]) <= 0.02 * terms[0]


# ------------------------------------------------------------------------------------------- world 2 (gloo)

def _worker(rank, world, port, q, kind, sizes, sync_bn, seed_base, dtype="fp32", pre=()):
    """One forward + backward per rank on its slice of a batch split ``sizes``, then the DDP exchange + Adam.
    ``pre``: earlier splits run first (forward + backward, no update) — a batch size that changes between steps."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from vmatting import parallel
        parallel.init_from_env(backend="gloo")  # gloo moves the cuda tensors; both ranks share cuda:0
        torch.cuda.set_device(0)
        if kind == "small":
            from vmatting.small_train import SmallTrainer
            np.random.seed(seed_base + rank)  # different draws per rank: the broadcast must make them identical
            trn = SmallTrainer(6, dtype, "cuda:0", sync_bn=sync_bn)
        else:
            from vmatting.train import VideoTrainer
            from vmatting.weights import synthetic_vgg16
            params = om.unet_simple_params(np.random.RandomState(1))
            trn = VideoTrainer(synthetic_vgg16(0), dtype, "cuda:0", params=params, sync_bn=sync_bn)
        p0 = trn.flat.cpu().numpy()
        for sz in tuple(pre) + (sizes,):
            a, b = sum(sz[:rank]), sum(sz[:rank + 1])
            if kind == "small":
                cmp, bg, gt, fg = (x[a:b] for x in _small_batch(sum(sz), 32, 40, seed=13))
                trn.forward(cmp, bg)
            else:
                from test_gpu_train import _batch
                cmp, bg, warped, gt, fg = (x[a:b] for x in _batch(sum(sz), 48, 64, seed=13))
                trn.forward(cmp, bg, warped)
            trn.grad.zero_()
            trn.backward(T(gt), T(fg), T(bg), T(cmp))
        torch.cuda.synchronize()
        local = trn.grad.cpu().numpy().copy()
        trn.apply_gradients()  # DDP all-reduce (in place: trn.grad is the replicas' sum) + Adam
        torch.cuda.synchronize()
        q.put((rank, p0, local, trn.flat.cpu().numpy(), trn.grad.cpu().numpy().copy(), None))
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, None, None, traceback.format_exc()[-2000:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_world2(kind, sizes, sync_bn, seed_base=100, dtype="fp32", pre=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 97) + (7 if sync_bn else 0) + (3 if kind == "small" else 0) + \
        (11 if dtype == "bf16" else 0) + (17 if pre else 0)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, kind, sizes, sync_bn, seed_base, dtype, pre))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=110) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(30)
    assert all(r[5] is None for r in res), [r[5] for r in res]
    return res


def test_small_ddp_replicas_start_and_stay_identical():
    """Two replicas drawing different init_conv weights (small.py:5-10 uses the global RNG) start from rank 0's
    variables and stay bit-identical after the all-reduced Adam step."""
    res = _run_world2("small", (1, 1), False)
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][3], res[1][3])
    assert not np.array_equal(res[0][2], res[1][2])  # different data -> different local gradients


@pytest.mark.parametrize("kind,pre,sizes", [("small", (), (1, 2)), ("video", (), (1, 2)),
                                             ("small", ((2, 2),), (2, 1)), ("video", ((2, 2),), (2, 1))])
def test_syncbn_unequal_batches_match_single_device(kind, pre, sizes):
    """SyncBN with unequal per-rank batches (the backward must use the forward's global pixel count).
    The replicas jointly minimise the sum of their batch-mean losses, e.g. S = l_0 + (l_1 + l_2) / 2 for sizes (1, 2),
    with batch statistics over the whole batch; the all-reduced gradient must equal dS/dW of the float64 restatement
    on the whole batch with those per-sample weights (a wrong count in the BN backward moves every gradient upstream
    of a BN by O(1)).  ``pre``: a (2, 2) step first, then (2, 1) — an uneven last shard after full
    steps, where only rank 1's batch changes; every rank must still run the same collectives and use this step's
    global count."""
    res = _run_world2(kind, sizes, True, pre=pre)
    np.testing.assert_array_equal(res[0][4], res[1][4])  # the all-reduced gradient is the same on both ranks
    g = res[0][4].astype(np.float64)
    wts = [1.0 / sizes[0]] * sizes[0] + [1.0 / sizes[1]] * sizes[1]
    if kind == "small":
        from vmatting.small_train import param_layout as lay
        np.random.seed(100)  # rank 0's draws: the replicas run on them after the broadcast
        from vmatting.small import NEW_CONVS
        from vmatting.weights import init_conv
        params = {}
        for name, ci, co in NEW_CONVS:
            w, b = init_conv(6 if ci is None else ci, co)
            params[name] = (w, None if name.startswith("upconv") else b)
        cmp, bg, gt, fg = _small_batch(sum(sizes), 32, 40, seed=13)
        _, _, grads, _ = tr.small_step_grads(cmp, bg, gt, fg, params, sample_weights=wts)
        layout = lay(6)[0]
    else:
        from test_gpu_train import _batch
        from vmatting.train import param_layout as lay
        from vmatting.weights import synthetic_vgg16
        params = om.unet_simple_params(np.random.RandomState(1))
        cmp, bg, warped, gt, fg = _batch(sum(sizes), 48, 64, seed=13)
        _, _, grads = tr.train_step_grads(cmp, bg, warped, gt, fg, synthetic_vgg16(0), params, sample_weights=wts)
        layout = lay()[0]
    bad, worst = [], 0.0
    for scope, k, off, shape in layout:
        if k == "b":  # conv biases: zero in exact arithmetic (BN removes them)
            continue
        n = int(np.prod(shape))
        a, b = g[off:off + n], grads[scope, k].reshape(-1)
        l2 = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        worst = max(worst, l2)
        # BN gamma / beta gradients are whole-batch sums of a signed gradient (cancellation in f32): 5e-3
        if l2 > (5e-3 if k in ("gamma", "beta") else 2e-3):
            bad.append((scope, k, float(l2)))
    print("syncbn %s worst rel L2 %.3g" % (kind, worst))
    assert not bad, bad


def _small_params(seed):
    from vmatting.small import NEW_CONVS
    from vmatting.weights import init_conv
    np.random.seed(seed)
    params = {}
    for name, ci, co in NEW_CONVS:
        w, b = init_conv(6 if ci is None else ci, co)
        params[name] = (w, None if name.startswith("upconv") else b)
    return params


@pytest.mark.parametrize("kind", ["small", "video"])
def test_syncbn_bf16_two_replicas_match_one_device(kind):
    """SyncBN in bf16: two replicas with one sample each give the gradient of one bf16 trainer on both
    samples (the replicas' summed batch-mean gradients = 2x the single device's batch-mean gradient).  The f64
    objective is no reference here: at 32x40 the level-4 BN sums over 3 pixels' worth of rows cancel, so bf16
    rounding alone moves those gradients by tens of % against f64, while the same bf16 arithmetic on one device
    differs only where a statistic's last f32 bit flips a bf16 activation (a wrong count would be O(1) everywhere)."""
    sizes = (1, 1)
    res = _run_world2(kind, sizes, True, dtype="bf16")
    np.testing.assert_array_equal(res[0][4], res[1][4])
    g = res[0][4].astype(np.float64)
    if kind == "small":
        from vmatting.small_train import SmallTrainer
        ref = SmallTrainer(6, "bf16", DEV, params=_small_params(100))
        cmp, bg, gt, fg = _small_batch(2, 32, 40, seed=13)
        np.testing.assert_array_equal(H(ref.flat), res[0][1])  # same starting variables as the replicas
        ref.forward(cmp, bg)
    else:
        from test_gpu_train import _batch
        from vmatting.train import VideoTrainer
        from vmatting.weights import synthetic_vgg16
        ref = VideoTrainer(synthetic_vgg16(0), "bf16", DEV, params=om.unet_simple_params(np.random.RandomState(1)))
        cmp, bg, warped, gt, fg = _batch(2, 48, 64, seed=13)
        ref.forward(cmp, bg, warped)
    ref.grad.zero_()
    ref.backward(T(gt), T(fg), T(bg), T(cmp))
    torch.cuda.synchronize()
    g_ref = 2.0 * H(ref.grad).astype(np.float64)
    bad, worst = [], 0.0
    for scope, k, off, shape in ref.layout:
        if k == "b":
            continue
        n = int(np.prod(shape))
        a, b = g[off:off + n], g_ref[off:off + n]
        l2 = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        worst = max(worst, l2)
        if l2 > 3e-2:
            bad.append((scope, k, float(l2)))
    print("syncbn bf16 %s worst rel L2 vs one device %.3g" % (kind, worst))
    assert not bad, bad


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_small_graph_step_equals_eager(dtype):
    """SmallTrainer.capture: two steps replayed from the forward / backward HIP graphs (new batches copied in, Adam
    eager in between) leave bit-identical parameters and losses to two eager steps."""
    from vmatting.small_train import SmallTrainer
    params = om.unet_small_params(np.random.RandomState(1), cin=6)
    b1, b2 = _small_batch(2, 48, 64, seed=3), _small_batch(2, 48, 64, seed=4)
    eager = SmallTrainer(6, dtype, DEV, params=params, lr=1e-3)
    le = [H(eager.step(*b)) for b in (b1, b2)]
    graphed = SmallTrainer(6, dtype, DEV, params=params, lr=1e-3)
    g = graphed.capture(*b1)
    lg = [H(g.step(*b)) for b in (b1, b2)]
    torch.cuda.synchronize()
    assert all(np.array_equal(a, b) for a, b in zip(le, lg)), (le, lg)
    assert torch.equal(eager.flat, graphed.flat)
