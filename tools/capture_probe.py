"""Which stream fork / join pattern breaks a HIP graph capture (the `capture_end` segfault of
gpurun_out/c17t.log, from a VideoTrainer variant that forked each pass onto its own high-priority stream).

    python tools/capture_probe.py            # every case, each in its own child process, stop at the first crash
    python tools/capture_probe.py CASE       # one case in this process

Each case captures a few kernels into a torch.cuda.CUDAGraph, replays it and checks the result against eager
execution.  A child that dies by a signal (segfault in capture_end) ends the run: nothing more is started on the
GPU after a crash.  Output: one line per case, `CASE rc=... ok|error ...`.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]

import torch  # noqa: E402

N = 1 << 20


def _bufs():
    x = torch.arange(N, dtype=torch.float32, device="cuda") / N
    return x, [torch.zeros_like(x) for _ in range(4)]


def _work(x, outs, streams):
    """out[i] = x * (i + 2) + i on streams[i] (forked from the current stream, joined back)."""
    cur = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(cur)
    for i, (s, o) in enumerate(zip(streams, outs)):
        with torch.cuda.stream(s):
            torch.add(torch.mul(x, i + 2, out=o), i, out=o)
    for s in streams:
        cur.wait_stream(s)


def _expect(x, outs, n):
    return all(torch.equal(outs[i], x * (i + 2) + i) for i in range(n))


def _capture(fn):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def case_fork_default():
    """fork onto default-priority streams made before the capture, joined back: the pattern VideoTrainer uses."""
    x, outs = _bufs()
    ss = [torch.cuda.Stream() for _ in range(3)]
    g = _capture(lambda: _work(x, outs, ss))
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    return _expect(x, outs, 3)


def case_fork_prio():
    """the same onto a high-priority stream."""
    x, outs = _bufs()
    hp = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    g = _capture(lambda: _work(x, outs, [hp]))
    outs[0].zero_()
    g.replay()
    torch.cuda.synchronize()
    return _expect(x, outs, 1)


def case_fork_prio_nested():
    """capture stream -> high-priority stream -> 3 default-priority side streams -> joined back in reverse."""
    x, outs = _bufs()
    hp = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    ss = [torch.cuda.Stream() for _ in range(3)]

    def fn():
        cur = torch.cuda.current_stream()
        hp.wait_stream(cur)
        with torch.cuda.stream(hp):
            _work(x, outs, ss)
            torch.add(outs[0], 1, out=outs[3])
        cur.wait_stream(hp)
    g = _capture(fn)
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    return _expect(x, outs, 3) and torch.equal(outs[3], outs[0] + 1)


def _nested(mid, inner):
    x, outs = _bufs()

    def fn():
        cur = torch.cuda.current_stream()
        mid.wait_stream(cur)
        with torch.cuda.stream(mid):
            _work(x, outs, inner)
            torch.add(outs[0], 1, out=outs[3])
        cur.wait_stream(mid)
    g = _capture(fn)
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    return _expect(x, outs, len(inner)) and torch.equal(outs[3], outs[0] + 1)


def case_nested_default():
    """capture stream -> default-priority stream -> 3 default-priority side streams -> joined back: the nested fork
    alone, no stream priority."""
    return _nested(torch.cuda.Stream(), [torch.cuda.Stream() for _ in range(3)])


def case_nested_default_single():
    """capture stream -> default-priority stream -> ONE default-priority stream -> joined back."""
    return _nested(torch.cuda.Stream(), [torch.cuda.Stream()])


def case_prio_nested_single():
    """capture stream -> high-priority stream -> ONE default-priority stream -> joined back."""
    return _nested(torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1]), [torch.cuda.Stream()])


def case_capture_on_prio_stream():
    """the capture itself begun while a high-priority stream is current (caller-level priority)."""
    x, outs = _bufs()
    hp = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    ss = [torch.cuda.Stream() for _ in range(3)]
    with torch.cuda.stream(hp):
        g = _capture(lambda: _work(x, outs, ss))
        for o in outs:
            o.zero_()
        g.replay()
    torch.cuda.synchronize()
    return _expect(x, outs, 3)


def case_side_wait_only():
    """a side stream waits on the capture (joins it) but nothing joins it back before capture_end: HIP must report
    hipErrorStreamCaptureUnjoined, CUDA's contract."""
    x, outs = _bufs()
    s = torch.cuda.Stream()

    def fn():
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            torch.mul(x, 2, out=outs[0])
    try:
        _capture(fn)
    except RuntimeError as e:
        print("  raised:", str(e).splitlines()[0][:200], flush=True)
        return True
    return False


def _trainer_hp(fork_on="pass"):
    """VideoTrainer at the bench's shape class with each pass forked onto a trainer-owned high-priority stream (the
    dropped r04 variant), then TrainGraph's capture; the graph step must equal the eager step."""
    import numpy as np
    from vmatting import train as vt
    from vmatting.weights import synthetic_vgg16
    from oracle import models as om

    class HPTrainer(vt.VideoTrainer):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self._hp = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])

        def _fork(self, fn, *a):
            cur = torch.cuda.current_stream()
            self._hp.wait_stream(cur)
            with torch.cuda.stream(self._hp):
                r = fn(*a)
            cur.wait_stream(self._hp)
            return r

        def forward(self, *a):
            return self._fork(super().forward, *a)

        def backward(self, *a):
            return self._fork(super().backward, *a)

    rs = np.random.RandomState(5)
    n, h, w = 2, 64, 80
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()  # noqa: E731
    batch = [T(rs.uniform(-100, 100, (n, h, w, 3))), T(rs.uniform(-100, 100, (n, h, w, 3))),
             T(rs.uniform(0, 1, (n, h, w, 3))), T(rs.uniform(0, 1, (n, h, w, 1))), T(rs.uniform(0, 255, (n, h, w, 3)))]
    params = om.unet_simple_params(np.random.RandomState(1))
    eager = vt.VideoTrainer(synthetic_vgg16(0), "bf16", "cuda", params=params, lr=1e-3)
    le = eager.step(*batch).cpu()
    trn = HPTrainer(synthetic_vgg16(0), "bf16", "cuda", params=params, lr=1e-3)
    g = trn.capture(*batch)
    lg = g.step().cpu()
    torch.cuda.synchronize()
    return torch.equal(le, lg) and torch.equal(eager.flat, trn.flat)


def case_trainer_hp_fork():
    return _trainer_hp()


CASES = ["fork_default", "fork_prio", "fork_prio_nested", "capture_on_prio_stream", "trainer_hp_fork",
         "side_wait_only"]


def main():
    cases = CASES
    if len(sys.argv) > 2 and sys.argv[1] == "--cases":
        cases = sys.argv[2].split(",")
    elif len(sys.argv) > 1:
        ok = globals()["case_" + sys.argv[1]]()
        print("%s %s" % (sys.argv[1], "ok" if ok else "MISMATCH"), flush=True)
        return 0 if ok else 1
    for c in cases:
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), c], timeout=240)
            rc = r.returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
        print("CASE %s rc=%s" % (c, rc), flush=True)
        if rc != 0 and rc != 1:  # a signal, an abort or a hang: start nothing more on the GPU
            print("stopping after %s" % c, flush=True)
            return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
