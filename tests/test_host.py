"""CPU checks of the host logic: weight construction order, .flo I/O, sharding and the
frame-parallel collectives (gloo, world_size 2)."""

import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import golden
from oracle import flow as oflow
from oracle import models as om


def test_synthetic_vgg_matches_oracle_generator():
    from vmatting.weights import synthetic_vgg16
    a, b = synthetic_vgg16(0), om.synthetic_vgg16(0)
    for k in a:
        assert np.array_equal(a[k][0], b[k][0]) and np.array_equal(a[k][1], b[k][1])


@pytest.mark.parametrize("case", ["unet_video_70x90", "unet_image_70x90"])
def test_unet_weight_draw_order_matches_reference(case, vgg0):
    """vmatting.unet draws fresh filters from the global numpy RNG in the reference's order."""
    from vmatting import unet
    g = golden(case)
    cls = unet.UNetVideo if int(g["video"]) else unet.UNetImage
    m = cls.__new__(cls)
    m.data_dict = vgg0
    np.random.seed(int(g["weight_seed"]))
    p = m._make_params()
    ref = om.unet_params(vgg0, np.random.RandomState(int(g["weight_seed"])), video=bool(g["video"]))
    assert set(p) == set(ref)
    for k in ref:
        assert np.array_equal(p[k][0], ref[k][0]), k
        assert (p[k][1] is None) == (ref[k][1] is None), k
        if p[k][1] is not None:
            assert np.array_equal(p[k][1], ref[k][1]), k


def test_unet_flop_count_matches_survey():
    from vmatting import unet
    m = unet.UNetVideo.__new__(unet.UNetVideo)
    m.data_dict = om.synthetic_vgg16(0)
    np.random.seed(0)
    m.params = m._make_params()
    assert m.conv_flops(1, 1080, 1920) == 3_232_595_312_640  # SURVEY.md §8d / BASELINE.md


def test_read_flow_roundtrip_and_bad_magic(capsys):
    from vmatting import reader
    f = oflow.smooth_flow(37, 53, seed=3)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.flo")
        reader.write_flow(p, f)
        assert np.array_equal(reader.read_flow(p), f)
        assert np.array_equal(oflow.read_flow(p), f)
        raw = bytearray(open(p, "rb").read())
        raw[0:4] = np.array([1.0], np.float32).tobytes()
        open(p, "wb").write(bytes(raw))
        out = reader.read_flow(p)  # prints, continues (reader.py:25-26)
        assert "invalid key" in capsys.readouterr().out
        assert np.array_equal(out, f)


def test_composite_matches_reference_formula():
    from vmatting import reader
    rs = np.random.RandomState(0)
    fg = rs.randint(0, 256, (5, 7, 3)).astype(np.uint8)
    bg = rs.randint(0, 256, (5, 7, 3)).astype(np.uint8)
    a = rs.uniform(size=(5, 7))
    ref = a[..., None] * fg + (1 - a[..., None]) * bg
    assert np.allclose(reader.create_composite_image(fg, bg, a), ref, rtol=0, atol=1e-12)


def test_shard_ranges_cover_frames():
    from vmatting.parallel import shard_range
    for n in (1, 7, 256, 257):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from vmatting import parallel
    parallel.init_from_env(backend="gloo")
    try:
        # weights: rank 0's values win everywhere (one flattened collective)
        w = [torch.full((5,), float(rank)), torch.arange(6, dtype=torch.float32).reshape(2, 3) * (rank + 1),
             torch.tensor([rank], dtype=torch.int32)]
        parallel.broadcast_tensors(w, src=0)
        ok_b = bool(torch.all(w[0] == 0)) and bool(torch.equal(w[1], torch.arange(6.).reshape(2, 3))) and int(w[2]) == 0
        # frames: 7 frames sharded 3/4, each rank "computes" frame index * 10, all-gather in order
        n = 7
        a, b = parallel.shard_range(n, rank, world)
        local = torch.arange(a, b, dtype=torch.float32)[:, None, None, None].expand(b - a, 2, 3, 1) * 10
        full = parallel.gather_frames(local.contiguous(), n)
        ok_g = full.shape == (7, 2, 3, 1) and bool(torch.equal(full[:, 0, 0, 0], torch.arange(7.) * 10))
        # even split (config 4's 256 frames / P): gathered straight into the receive buffer
        a, b = parallel.shard_range(8, rank, world)
        local = torch.arange(a, b, dtype=torch.float32)[:, None, None, None].expand(b - a, 2, 3, 1) * 10
        full = parallel.gather_frames(local.contiguous(), 8)
        ok_g = ok_g and full.shape == (8, 2, 3, 1) and bool(torch.equal(full[:, 1, 2, 0], torch.arange(8.) * 10))
        q.put((rank, ok_b, ok_g))
    finally:
        dist.destroy_process_group()


def test_frame_parallel_collectives_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    assert sorted(r for r, _, _ in res) == [0, 1]
    assert all(b and g for _, b, g in res), res


# ---------------------------------------------------------------- loader host logic (no GPU)

@pytest.mark.parametrize("fg_hw,bg_hw", [((330, 340), (250, 300)), ((300, 700), (500, 375)), ((1080, 1920), (720, 1280)),
                                         ((200, 200), (640, 640)), ((700, 310), (90, 1300))])
def test_loader_plan_replays_reference_draws(fg_hw, bg_hw):
    """The product's host planning consumes np.random exactly like the oracle restatement of loader.py."""
    from oracle import loader as ol
    from vmatting import loader as vl
    for seed in range(12):
        np.random.seed(seed)
        want = ol.plan_crop(fg_hw, bg_hw)
        a = np.random.randint(0, 1 << 30)
        np.random.seed(seed)
        got = vl.plan_crop(fg_hw, bg_hw)
        b = np.random.randint(0, 1 << 30)
        assert a == b
        assert [tuple(x) for x in got] == [x.astuple() for x in want[1:]]


def test_loader_get_padded_img_matches_oracle_maps():
    from oracle import loader as ol
    from vmatting import loader as vl
    img = np.arange(7 * 9 * 2).reshape(7, 9, 2)
    for seed in range(6):
        for crop in ((5, 12), (9, 4), (7, 9)):
            np.random.seed(seed)
            got = vl.get_padded_img(img, *crop)
            np.random.seed(seed)
            rows, cols = ol.pad_axis(7, crop[0]), ol.pad_axis(9, crop[1])
            want = ol.Axis(rows[0], 0, *rows[1:]).gather(ol.Axis(cols[0], 0, *cols[1:]).gather(img, 1), 0)
            assert np.array_equal(got, want)


def test_loader_struct_layout():
    import ctypes
    from vmatting import _lib
    assert ctypes.sizeof(_lib.VmCropAxis) == 20
    assert ctypes.sizeof(_lib.VmLoaderSample) == 144
    assert ctypes.sizeof(_lib.VmLoaderOutputs) == 64


def test_loader_file_helpers(tmp_path):
    from vmatting import loader as vl
    lst = tmp_path / "list.txt"
    lst.write_text("a/fg.png a/tr.png b/bg.jpg\nc/fg.png c/tr.png d/bg.jpg\n")
    files = vl.get_file_list("/data", str(lst))
    assert files[1] == ["/data/c/fg.png", "/data/c/tr.png", "/data/d/bg.jpg"]
    assert not vl.epoch_is_over(files, 2)
    assert vl.get_batch_list(files, 1) == [["/data/c/fg.png", "/data/c/tr.png", "/data/d/bg.jpg"]]
    assert vl.epoch_is_over(files, 2)


def test_load_vgg16_explicit_npy_is_not_redirected(tmp_path):
    """an explicitly named .npy is loaded as named (here: refused as a pickle) even when a sibling .npz
    exists; only the default location prefers its converted .npz."""
    from vmatting import weights
    d = weights.synthetic_vgg16(0)
    np.save(tmp_path / "vgg16.npy", np.array(d, dtype=object), allow_pickle=True)
    weights.save_vgg16_npz({"conv1_1": d["conv1_1"]}, str(tmp_path / "vgg16.npz"))
    with pytest.raises(ValueError, match="pickled"):
        weights.load_vgg16(str(tmp_path / "vgg16.npy"))
    got = weights.load_vgg16(str(tmp_path / "vgg16.npz"))
    assert list(got) == ["conv1_1"] and np.array_equal(got["conv1_1"][0], d["conv1_1"][0])


def _bench(*args, env=None):
    import json
    import subprocess
    import sys
    from conftest import REPO
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + list(args), env=e, capture_output=True,
                       text=True, timeout=150)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, [json.loads(ln) for ln in lines], r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_its_own_ranks(n):
    """`bench.py --gpus N` without torchrun starts N ranks itself (the same launcher the GPU run
    uses) — here with --dist-selftest: gloo on the CPU, rank 0's broadcast and the uneven matte all-gather."""
    rc, recs, err = _bench("--gpus", str(n), "--dist-selftest")
    assert rc == 0, err[-2000:]
    assert len(recs) == 1, recs  # only rank 0 prints
    r = recs[0]
    assert r["n_gpus"] == n and r["backend"] == "gloo" and r["ok"] and r["broadcast_ok"] and r["gather_ok"]
    assert r["frames"] == 2 * n + 1 and r["split"][-1][1] == 2 * n + 1


@pytest.mark.parametrize("selftest", [True, False])
def test_bench_launcher_parent_stays_gpu_free(selftest):
    """the `--gpus N` launcher parent makes no torch.cuda / HIP call before (or after) it starts
    its ranks.  The parent runs with every device query patched to raise; the ranks are ordinary children.  With
    --dist-selftest the run succeeds; without it (no GPU here) each rank reports the missing GPUs itself and the
    launcher returns that non-zero code — the parent never raised."""
    import subprocess
    import sys
    from conftest import REPO
    bench = os.path.join(REPO, "bench.py")
    argv = ["--gpus", "2"] + (["--dist-selftest"] if selftest else [])
    code = ("import sys, runpy, torch\n"
            "def boom(*a, **k):\n"
            "    raise SystemExit('PARENT TOUCHED THE GPU')\n"
            "torch.cuda.device_count = boom\n"
            "torch.cuda.is_available = boom\n"
            "torch.cuda.init = boom\n"
            "torch._C._cuda_getDeviceCount = boom\n"
            "sys.argv = [%r] + %r\n"
            "runpy.run_path(%r, run_name='__main__')\n" % (bench, argv, bench))
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=150)
    assert "PARENT TOUCHED THE GPU" not in r.stderr + r.stdout
    if selftest:
        assert r.returncode == 0, r.stderr[-2000:]
        assert '"ok": true' in r.stdout
    else:
        assert r.returncode == 2, r.stderr[-2000:]
        assert "need 2 GPU(s)" in r.stderr


def test_bench_refuses_a_world_other_than_gpus():
    """A run whose initialised world differs from --gpus (here: a torchrun-style env of world 1) exits non-zero
    instead of reporting a one-GPU number as N GPUs."""
    rc, recs, err = _bench("--gpus", "2", "--dist-selftest", env={"WORLD_SIZE": "1", "RANK": "0"})
    assert rc != 0 and not recs
    assert "initialised world" in err


@pytest.mark.parametrize("h,w,n,fact", [(1080, 1920, 5, 0.05), (37, 51, 5, 0.05), (64, 64, 4, 0.1), (9, 300, 6, 0.2)])
def test_deform_grid_draws_match_the_reference_loop(h, w, n, fact):
    """tps.deform_grid draws its landmark offsets as one array; the reference (tps.py:127-143, restated in
    oracle/augment.py) draws one scalar per interior coordinate, x before y: same grids, bit for bit, and the
    same global RNG state after."""
    from oracle import augment as oa
    from vmatting import tps
    for seed in range(5):
        np.random.seed(seed)
        g1, d1 = tps.deform_grid(h, w, n, fact)
        after1 = np.random.rand()
        np.random.seed(seed)
        g2, d2 = oa.deform_grid(h, w, n, fact)
        after2 = np.random.rand()
        assert np.array_equal(g1, g2) and np.array_equal(d1, d2) and after1 == after2


def test_training_procedures_follow_the_reference_loop(tmp_path):
    """vmatting.procedures: per epoch the lists are copied and shuffled (train first), batches popped off the end
    until fewer than a batch remain, each fed to one step; training_procedure's validation over the test list."""
    import random
    from vmatting import procedures
    seen = []

    class FakeTrainer:
        device = "cpu"

        def step(self, *batch):
            seen.append(batch[0])
            return len(seen)

    made = []

    def make(batch_list):
        made.append(list(batch_list))
        return (tuple(batch_list),)

    files = ["f%d" % i for i in range(11)]
    random.seed(3)
    steps = []
    procedures._loop(FakeTrainer(), files, files[:5], make, 2, 4, False,
                     lambda e, it, loss: steps.append((e, it, loss)), None)
    random.seed(3)
    want = []
    for _ in range(2):
        tl, vl = list(files), list(files[:5])
        random.shuffle(tl)
        random.shuffle(vl)
        while len(tl) >= 4:
            want.append([tl.pop() for _ in range(4)])
    assert made == want and [s[1] for s in steps] == list(range(4)) and files == ["f%d" % i for i in range(11)]


def test_training_procedures_example_draws_and_graph_shape_guard():
    """the loops make the reference's example-summary draws (train.py:102-104: 5 np.random.randint picks
    of the test list + the loader call, every epoch; small_train.py:78-82: every 1000 iterations), so np.random stays
    on the reference's stream after epoch 1; and a HIP-graph loop refuses a batch of another shape instead of an
    eager step under the captured graph's buffers."""
    from vmatting import procedures

    class FakeTrainer:
        device = "cpu"

        def step(self, *batch):
            return 0

        def capture(self, *batch):
            return self

    made = []

    def make(batch_list):
        made.append(list(batch_list))
        np.random.rand()  # stands for the loader's own draws
        return (np.zeros((len(batch_list), 2)),)

    files = ["f%d" % i for i in range(9)]
    np.random.seed(4)
    procedures._loop(FakeTrainer(), files, files[:5], make, 2, 4, False, None, None, examples=make)
    after = np.random.rand()
    np.random.seed(4)
    for _ in range(2):
        for _ in range(2):
            np.random.rand()  # two training batches of 4 per epoch
        [np.random.randint(0, 5) for _ in range(5)]
        np.random.rand()
    assert after == np.random.rand()
    assert [len(m) for m in made] == [4, 4, 5, 4, 4, 5]
    # small_train.py's cadence: draws whenever (iteration + 1) % every == 0
    made.clear()
    procedures._loop(FakeTrainer(), files, files[:5], make, 1, 1, False, None, None, examples=make, example_every=3)
    assert [len(m) for m in made] == [1, 1, 5, 1, 1, 1, 5, 1, 1, 1, 5, 1]
    # graph loop: one batch shape
    st = procedures._Stepper(FakeTrainer(), True)
    st(np.zeros((4, 2)))
    st(np.zeros((4, 2)))
    with pytest.raises(ValueError, match="one batch shape"):
        st(np.zeros((3, 2)))


def test_entry_points_without_arguments_name_what_is_missing(tmp_path, monkeypatch):
    """train(), simple_train(), video_train() and small_train.train() take no arguments, like the
    reference (train.py:112,241,346; small_train.py:91); without the reference's dataset (params.py:3-6, 12-15) they
    raise a ValueError naming it instead of a TypeError / open(None)."""
    from vmatting import params, procedures
    monkeypatch.chdir(tmp_path)
    monkeypatch.setattr(params, "SYNTHETIC_DATASET", None)
    for fn, what in ((procedures.train, "SYNTHETIC_DATASET"), (procedures.simple_train, "SYNTHETIC_DATASET"),
                     (procedures.small_train, "SYNTHETIC_DATASET"), (procedures.video_train, "TRAIN_AUGMENTED")):
        with pytest.raises(ValueError, match=what):
            fn()
    monkeypatch.setattr(params, "SYNTHETIC_DATASET", str(tmp_path))
    with pytest.raises(ValueError, match="dataset/train.txt"):
        procedures.train()
    (tmp_path / "dataset").mkdir()
    (tmp_path / "dataset" / "train.txt").write_text("a b c\n")
    with pytest.raises(ValueError, match="dataset/valid.txt"):
        procedures.small_train()


def test_split3_filter_parts_carry_the_scaled_filter():
    """vmatting.split3: the fp16 filter parts of w * 2^t (t from filter_scale: max |w * 2^t| in (2^11, 2^12]) sum back
    to it within 2^-22 relative (the two-part fp16 residual) and sit in slab order [Wh, Wl, Wh]; the scale is an
    exact power of two, so the epilogue's 2^-t undoes it exactly."""
    import torch
    from vmatting.split3 import filter_scale, split3_filter
    rs = np.random.RandomState(5)
    for cin, cout, std in ((7, 64, 0.2), (64, 128, 0.06), (512, 8, 0.02)):
        w = (rs.randn(3, 3, cin, cout) * std).astype(np.float32)
        t = filter_scale(w)
        assert t == 2.0 ** round(np.log2(t)) and 2 ** 11 < np.abs(w).max() * t <= 2 ** 12
        f = split3_filter(w, cin, cout, t).double().numpy()
        wh, wl, wh2 = f[:, :, :cin], f[:, :, cin:2 * cin], f[:, :, 2 * cin:]
        assert np.array_equal(wh, wh2)
        assert np.array_equal(wh, wh.astype(np.float16).astype(np.float64))  # exact fp16 values
        assert np.array_equal(wl, wl.astype(np.float16).astype(np.float64))
        ws = w.astype(np.float64) * t
        assert np.all(np.abs(wh + wl - ws) <= 2.0 ** -22 * np.abs(ws) + 2.0 ** -24)
        # wider slabs: zero rows past the filter's channels
        f2 = split3_filter(w, cin + 8, cout, t).numpy()
        assert not f2[:, :, cin:cin + 8].any() and np.array_equal(f2[:, :, cin + 8:2 * cin + 8], f[:, :, cin:2 * cin])
    assert torch.float16 is not None


def test_split3_fold_up2x_is_resize_then_conv_inside_the_frame():
    """vmatting.split3.fold_up2x: the phase filters of conv3x3(resize2x(x), W) (TF-1 legacy bilinear, unet.py:58-60)
    reproduce it exactly away from the frame border, with the low-res frame replicated past its bottom / right edge
    (the folded kernel's loads); the border rows / columns are the border pass's (tests/test_gpu_split3.py)."""
    from oracle import ops as oo
    from vmatting.split3 import fold_up2x
    rs = np.random.RandomState(0)
    for h, w, ci, co in ((6, 7, 5, 4), (9, 4, 3, 2)):
        wt, x = rs.randn(3, 3, ci, co), rs.randn(2, h, w, ci)
        ref = oo.conv3x3_same(oo.resize_bilinear_tf1(x, 2 * h, 2 * w), wt)
        xp = np.pad(x, ((0, 0), (0, 1), (0, 1), (0, 0)), mode="edge")
        y = oo.conv3x3_same(xp, fold_up2x(wt))[:, :h, :w]
        got = np.zeros_like(ref)
        for p in range(4):
            got[:, p >> 1::2, p & 1::2] = y[..., p * co:(p + 1) * co]
        assert np.abs(got - ref)[:, 1:-1, 1:-1].max() <= 1e-12 * np.abs(ref).max()
