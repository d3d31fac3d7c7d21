"""GPU parity of the training-sample loader (vmatting.loader / csrc/loader.hip) — bit-exact.

The loader's arithmetic is float64 with OpenCV's float32 resize coefficients, so the bar is identity:
  * dtype=float64 outputs == oracle/loader.py (itself pinned to the reference's loader.py by
    tests/golden/loader_calls.npz) bit for bit, and == the golden samples;
  * dtype=float32 outputs == the float64 values rounded once (numpy astype).
"""

import os

import numpy as np
import pytest
import torch

from conftest import golden, gpu_available
from oracle import loader as ol
from test_oracle_golden import check_loader_call, loader_call_outputs

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]


def _write_entry(d, idx, ent):
    from PIL import Image
    from oracle.flow import write_flow
    p = lambda s: os.path.join(d, "e%d_%s" % (idx, s))  # noqa: E731
    Image.fromarray(np.ascontiguousarray(ent[0][:, :, [2, 1, 0, 3]])).save(p("fg.png"))
    Image.fromarray(np.ascontiguousarray(ent[1][:, :, ::-1])).save(p("bg.png"))
    if len(ent) > 2:
        Image.fromarray(np.ascontiguousarray(ent[2][:, :, [2, 1, 0, 3]])).save(p("prev.png"))
        write_flow(p("flow.flo"), ent[3])
        return (p("fg.png"), p("bg.png"), p("prev.png"), p("flow.flo"))
    Image.fromarray(ent[0][:, :, 3]).save(p("trimap.png"))
    return (p("fg.png"), p("trimap.png"), p("bg.png"))


def H(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("ci", range(11))
def test_loader_file_api_matches_reference_golden(ci, tmp_path):
    """vmatting.loader's reference-named functions, fed PNG/.flo files, reproduce the reference loader's
    sampled outputs bit for bit (float64) and consume the same np.random draws."""
    from vmatting import loader as vl
    g = golden("loader_calls")
    ents = {}

    def run(idx, size, mirror, fn):
        paths = []
        for e in idx:
            if e not in ents:
                s, fh, fw, bh, bw, v = (int(x) for x in g["entries"][e])
                ents[e] = _write_entry(str(tmp_path), e, ol.synthetic_entry(s, (fh, fw), (bh, bw), bool(v)))
            paths.append(ents[e])
        f64 = torch.float64
        if fn == "video_load_crop":
            r = vl.video_load_crop(paths[0], size, dtype=f64)
            return {k: H(t)[None] for k, t in zip(("cmp", "bg", "label", "warped", "fg"), r)}
        if fn == "simple_load_crop":
            r = vl.simple_load_crop(paths[0], size, dtype=f64)
            return {k: H(t)[None] for k, t in zip(("cmp", "bg", "label", "fg"), r)}
        if fn == "get_batch":
            r = vl.get_batch(paths, size, rd_mirror=mirror, dtype=f64)
            return {k: H(t) for k, t in zip(("input", "label", "fg"), r)}
        r = vl.video_batch(paths, size, dtype=f64)
        return {k: H(t) for k, t in zip(("cmp", "bg", "label", "warped", "fg"), r)}

    out, nxt = loader_call_outputs(g, ci, run)
    torch.cuda.synchronize()
    check_loader_call(g, ci, out, nxt)


def _oracle_batch(samples, size, mirror):
    outs = []
    for s, m in zip(samples, mirror):
        fr, fc, br, bc = (ol.Axis(*a) for a in s["plan"])
        fg_c, a_c, w_c, bg_c = ol.crop_sources(s["fg"], s["bg"], fr, fc, br, bc, s.get("prev"), s.get("flow"))
        o = ol.compose(fg_c, a_c, bg_c, size, w_c)
        outs.append({k: (np.flip(v, axis=1) if m else v) for k, v in o.items()})
    return {k: np.stack([o[k] for o in outs]) for k in outs[0]}


@pytest.mark.parametrize("size", [(320, 320), (288, 288), (160, 160)])
def test_loader_batch_1080p_sources_bit_exact(size):
    """A batch of 6 video samples from 1080p sources (every crop type, padding, mirroring) through
    compose_batch: f64 == oracle exactly, f32 == oracle rounded once."""
    from vmatting import loader as vl
    np.random.seed(17)
    samples, mirror = [], []
    for i in range(6):
        hw = [(1080, 1920), (400, 600), (1080, 1920), (500, 300), (1080, 1920), (640, 640)][i]
        fg, bg, prev, flow = ol.synthetic_entry(500 + i, hw, [(720, 1280), (640, 640), (1080, 1920)][i % 3])
        s = {"fg": fg, "bg": bg, "prev": prev, "flow": flow}
        s["plan"] = vl.plan_crop(fg.shape[:2], bg.shape[:2])
        samples.append(s)
        mirror.append(i % 2 == 1)
    want = _oracle_batch(samples, size, mirror)
    names = ("cmp", "bg", "label", "warped", "fg")
    got = vl.compose_batch(samples, size, names, mirror, dtype=torch.float64)
    got32 = vl.compose_batch(samples, size, names, mirror, dtype=torch.float32)
    torch.cuda.synchronize()
    for k in names:
        g64 = H(got[k])
        assert np.array_equal(g64, want[k]), "%s: max diff %g" % (k, np.abs(g64 - want[k]).max())
        assert np.array_equal(H(got32[k]), want[k].astype(np.float32)), k


def test_loader_batch_beyond_kernarg_descriptors():
    """Batches of up to 8 samples pass their descriptors in the kernel arguments, larger ones upload them to the
    workspace: a 10-sample batch equals the oracle exactly, and its first 5 samples equal a 5-sample batch."""
    from vmatting import loader as vl
    np.random.seed(23)
    samples, mirror = [], []
    for i in range(10):
        fg, bg, prev, flow = ol.synthetic_entry(700 + i, (120 + 8 * i, 150), (140, 170 + 4 * i))
        s = {"fg": fg, "bg": bg, "prev": prev, "flow": flow, "plan": vl.plan_crop(fg.shape[:2], bg.shape[:2])}
        samples.append(s)
        mirror.append(i % 3 == 0)
    names = ("cmp", "bg", "label", "warped")
    want = _oracle_batch(samples, (64, 64), mirror)
    got = vl.compose_batch(samples, (64, 64), names, mirror, dtype=torch.float64)
    part = vl.compose_batch(samples[:5], (64, 64), names, mirror[:5], dtype=torch.float64)
    torch.cuda.synchronize()
    for k in names:
        assert np.array_equal(H(got[k]), want[k]), k
        assert torch.equal(got[k][:5], part[k]), k


def test_loader_device_resident_inputs_and_input_layout():
    """Inputs already in HBM (device tensors) and get_batch's 6-channel input layout."""
    from vmatting import loader as vl
    fg, bg = ol.synthetic_entry(7, (700, 900), (480, 640), video=False)
    np.random.seed(3)
    plan = vl.plan_crop(fg.shape[:2], bg.shape[:2])
    s = {"fg": torch.from_numpy(fg).cuda(), "bg": torch.from_numpy(bg).cuda(), "plan": plan}
    r = vl.compose_batch([s], (96, 96), ("input", "label", "fg"), dtype=torch.float64)
    r2 = vl.compose_batch([s], (96, 96), ("cmp", "bg"), dtype=torch.float64)
    torch.cuda.synchronize()
    want = _oracle_batch([{"fg": fg, "bg": bg, "plan": plan}], (96, 96), [False])
    assert np.array_equal(H(r["input"]), np.concatenate([want["cmp"], want["bg"]], axis=3))
    assert np.array_equal(H(r["label"]), want["label"]) and np.array_equal(H(r["fg"]), want["fg"])
    assert np.array_equal(H(r2["cmp"]), want["cmp"]) and np.array_equal(H(r2["bg"]), want["bg"])
    with pytest.raises(ValueError):
        vl.compose_batch([s], (96, 96), ("input", "cmp"))


def test_loader_rejects_bad_windows():
    from vmatting import loader as vl
    fg, bg = ol.synthetic_entry(8, (100, 120), (80, 90), video=False)
    bad = {"fg": fg, "bg": bg, "plan": ((50, 60, 0, 100, 10), (120, 0, 0, 120, 0), (80, 0, 0, 80, 0), (90, 0, 0, 90, 0))}
    with pytest.raises(ValueError):  # rows 60..109 + shift 10 run past the 100-row image
        vl.compose_batch([bad], (32, 32))
    ok = dict(bad, plan=((50, 0, 0, 100, 0),) + bad["plan"][1:])
    with pytest.raises(ValueError):  # warped output needs the previous frame and flow
        vl.compose_batch([ok], (32, 32), ("cmp", "warped"))
    with pytest.raises(ValueError):  # batch loaders need a square input_size, as the reference's arrays do
        vl.simple_batch([], (64, 32))
