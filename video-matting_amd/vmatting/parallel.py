"""Frame-parallel execution across the GPUs of a node (one process per GPU, RCCL over xGMI).

Frames are independent at inference (UNetVideo has no BN; BN in inference mode is a
per-frame affine), so a video batch is split into contiguous per-rank blocks and every
rank runs the whole network on its block with no communication in the data path.
Collectives exist only at the edges: one broadcast of the packed weights from rank 0
(so every replica computes with bit-identical weights) and an optional all-gather of
the mattes.  backend 'nccl' is RCCL on ROCm; 'gloo' runs the same code on CPU tensors.
"""

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*) if present."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, world, local


def world_size():
    """Number of ranks of the default process group (1 when torch.distributed is not initialised)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def shard_range(n_frames, rank, world):
    """Contiguous block of frames for ``rank``: [start, stop)."""
    start = (n_frames * rank) // world
    stop = (n_frames * (rank + 1)) // world
    return start, stop


def broadcast_tensors(tensors, src=0):
    """Broadcast a list of same-device tensors from ``src`` with ONE collective (flattened byte buffer)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return tensors
    flat = torch.cat([t.contiguous().view(-1).view(torch.uint8) for t in tensors])
    dist.broadcast(flat, src)
    off = 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        t.view(-1).view(torch.uint8).copy_(flat[off:off + nb])
        off += nb
    return tensors


def gather_frames(local, n_frames, out=None):
    """All-gather per-rank frame blocks (contiguous, possibly uneven) into the full [n_frames, ...] batch.

    One ``all_gather_into_tensor`` (RCCL ring over xGMI) into a [world * max_block, ...] buffer; with an even
    split the result is that buffer itself (no extra copy), otherwise the padded rows are squeezed out.
    ``out`` may pass a preallocated [world * max_block, ...] receive buffer."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    sizes = [shard_range(n_frames, r, world) for r in range(world)]
    mx = max(b - a for a, b in sizes)
    if local.shape[0] != mx:
        pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
    else:
        pad = local.contiguous()
    if out is None:
        out = torch.empty((world * mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "gloo":  # gloo's collective is the list form (host-staged for device tensors)
        recv = out if out.is_contiguous() else torch.empty(out.shape, dtype=out.dtype, device=out.device)
        dist.all_gather(list(recv.view((world, mx) + tuple(local.shape[1:])).unbind(0)), pad)
        if recv is not out:
            out.copy_(recv)
    else:
        dist.all_gather_into_tensor(out, pad)
    if all(b - a == mx for a, b in sizes):
        return out
    return torch.cat([out[r * mx:r * mx + (b - a)] for r, (a, b) in enumerate(sizes)], dim=0)


def allreduce_grads(flat):
    """Data-parallel gradient exchange of the training step (train.py:302-304 under DDP): ONE all-reduce (sum) of
    the flat f32 gradient buffer (≈6.5 MB for UNetSimple).  Returns the scale (1/world) the optimizer applies, so
    the averaging costs no extra pass over the buffer."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 1.0
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    return 1.0 / dist.get_world_size()


def allreduce_sum(t):
    """In-place sum over the ranks (SyncBN's per-channel moments and gradient sums: a few KB per BN layer)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t

