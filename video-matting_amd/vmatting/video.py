"""Frame-parallel matting of a video batch (BASELINE config 4) — the product path that bench.py times.

The reference evaluates its per-frame forward inside sess.run over batches drawn from a frame list
(train.py:318-332); frames never interact at inference (UNetVideo has no BN), so a video batch of F frames is
cut into contiguous per-rank blocks (parallel.shard_range), each rank runs its block through UNetVideo in
chunks of ``chunk`` frames, and one all-gather (RCCL ring over xGMI) hands every rank the whole matte batch.

Chunks are recorded as HIP graphs whose input IS the caller's frame slice and whose alpha output IS the
result slice (UNet.capture(static=True, out=...)): no per-frame staging copies, one host call per chunk, and a
chunk of 8 frames gives the small L4/L5 convs 8x the tiles of a single frame.  All chunks share the model's
activation buffers (they run in order on one stream).
"""

import torch

from . import parallel

VGG_MEAN = (103.939, 116.779, 123.68)  # params.py:10


def synthetic_frames(n, h, w, first=0, device="cuda"):
    """SURVEY.md §8d synthetic 7-channel frames, generated on the device: frame f (seed 1234+f): composite and
    background BGR U{0..255} - VGG_MEAN; trimap {0, .5, 1} - .5 from a random ellipse with an 8-px unknown band
    (loader.py:76-78 layout).  -> [n, h, w, 7] f32."""
    out = torch.empty((n, h, w, 7), dtype=torch.float32, device=device)
    mean = torch.tensor(VGG_MEAN, device=device)
    yy = torch.arange(h, device=device, dtype=torch.float32)[:, None]
    xx = torch.arange(w, device=device, dtype=torch.float32)[None, :]
    for i in range(n):
        g = torch.Generator(device=device)
        g.manual_seed(1234 + first + i)
        out[i, :, :, 0:3] = torch.randint(0, 256, (h, w, 3), generator=g, device=device).float() - mean
        out[i, :, :, 3:6] = torch.randint(0, 256, (h, w, 3), generator=g, device=device).float() - mean
        c = torch.rand(4, generator=g, device=device)
        cy, cx = (0.3 + 0.4 * c[0]) * h, (0.3 + 0.4 * c[1]) * w
        ry, rx = (0.15 + 0.15 * c[2]) * h, (0.15 + 0.15 * c[3]) * w
        d = torch.sqrt(((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2)
        band = 8.0 / float(min(ry, rx))
        tri = torch.where(d < 1 - band, 1.0, torch.where(d < 1 + band, 0.5, 0.0))
        out[i, :, :, 6] = tri - 0.5
    return out


class VideoMatter:
    """Mattes for frames[a:b] of a video batch resident on the device: ``run()`` replays the chunk graphs into
    ``alpha`` ([b-a, H, W, 1] f32).  ``frames`` is this rank's [b-a, H, W, 7] f32 block (kept alive by the
    object: the graphs read it in place)."""

    def __init__(self, model, frames, chunk=8, graph=True, alpha=None):
        if frames.dim() != 4 or not frames.is_cuda or frames.dtype != torch.float32 or not frames.is_contiguous():
            raise ValueError("frames must be a contiguous [F,H,W,C] f32 device tensor")
        model.prepare()
        self.model, self.frames, self.chunk = model, frames, max(1, int(chunk))
        f, h, w, _ = frames.shape
        self.alpha = alpha if alpha is not None else torch.empty((f, h, w, 1), dtype=torch.float32,
                                                                 device=frames.device)
        if tuple(self.alpha.shape) != (f, h, w, 1) or not self.alpha.is_contiguous():
            raise ValueError("alpha must be a contiguous [F,H,W,1] f32 tensor")
        self.spans = [(i, min(f, i + self.chunk)) for i in range(0, f, self.chunk)]
        self.graphs = None
        if graph and f > 0:
            self.graphs = [model.capture(frames[a:b], static=True, out=self.alpha[a:b]) for a, b in self.spans]

    def run(self):
        if self.graphs is not None:
            for g in self.graphs:
                g.replay()
        else:
            for a, b in self.spans:
                self.model.forward(self.frames[a:b], out=self.alpha[a:b])
        return self.alpha


def shard(n_frames, rank=None, world=None):
    """This rank's contiguous [start, stop) block of an n_frames video batch."""
    if world is None:
        world = parallel.world_size()
    if rank is None:
        rank = torch.distributed.get_rank() if world > 1 else 0
    return parallel.shard_range(n_frames, rank, world)


def matte_video(model, frames, n_frames, chunk=8, graph=True, recv=None):
    """Config 4 in one call: ``frames`` is this rank's block (shard(n_frames)) as [b-a, H, W, 7] f32 on the
    device; returns (the all-gathered [n_frames, H, W, 1] matte batch, the VideoMatter, so a caller can replay
    it).  ``recv`` optionally preallocates the [world * max_block, H, W, 1] all-gather buffer."""
    vm = VideoMatter(model, frames, chunk, graph)
    vm.run()
    return parallel.gather_frames(vm.alpha, n_frames, out=recv), vm
