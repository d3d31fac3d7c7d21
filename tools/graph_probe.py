"""Eager vs HIP-graph replay of the UNetVideo 1080p forward (is the launch gap worth a graph?)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "video-matting_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmatting import unet  # noqa: E402
from vmatting.weights import synthetic_vgg16  # noqa: E402

np.random.seed(0)
m = unet.UNetVideo(synthetic_vgg16(0), dtype="bf16", device="cuda").prepare()
x = torch.randn(1, 1080, 1920, 7, device="cuda") * 50
for _ in range(3):
    m.forward(x)
torch.cuda.synchronize()
N = 50
t0 = time.perf_counter()
for _ in range(N):
    m.forward(x)
torch.cuda.synchronize()
te = (time.perf_counter() - t0) / N
ref = m.output.clone()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    m.forward(x)
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    m.forward(x)
g.replay()
torch.cuda.synchronize()
print("graph output matches eager:", bool(torch.equal(m.output, ref)))
t0 = time.perf_counter()
for _ in range(N):
    g.replay()
torch.cuda.synchronize()
tg = (time.perf_counter() - t0) / N
print("eager %.3f ms  graph %.3f ms" % (te * 1e3, tg * 1e3))
# events inside a capture?
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g2 = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g2):
        e0.record()
        m.forward(x)
        e1.record()
    g2.replay()
    torch.cuda.synchronize()
    print("events in graph: %.3f ms" % e0.elapsed_time(e1))
except Exception as ex:  # noqa: BLE001
    print("events in graph failed:", repr(ex)[:200])
