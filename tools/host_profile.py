import os, sys, cProfile, pstats, io
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [REPO, os.path.join(REPO, "video-matting_amd")]
import torch
import bench
from vmatting.train import VideoTrainer
from vmatting.weights import synthetic_vgg16
import numpy as np
dev = torch.device("cuda:0")
n, size = 8, 320
rs = np.random.RandomState(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
cmp, bg, warped, gt, fg = [T(rs.uniform(0, 1, (n, size, size, c))) for c in (3, 3, 3, 1, 3)]
np.random.seed(1)
trn = VideoTrainer(synthetic_vgg16(0), "bf16", dev)
for _ in range(3):
    trn.step(cmp, bg, warped, gt, fg)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    trn.forward(cmp, bg, warped)
    trn.grad.zero_()
    trn.backward(gt, fg, bg, cmp)
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
