"""The reference's training loops (vmatting/procedures.py: train.py training_procedure / simple_procedure /
video_procedure, small_train.py small_training) on real PNG / .flo entries: each runs the same batches in the same
order as a hand-written loop of the reference's form (copy + random.shuffle per epoch, get_batch_list pops from the
end, loader call, one step) and its per-step losses are bit-identical to that loop's; graph=True (HIP-graph step
replays) matches too; training_procedure's validation loss equals the forward loss over the test batches."""

import random

import numpy as np
import pytest
import torch

from conftest import gpu_available
from oracle import loader as ol
from test_gpu_loader import _write_entry

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a ROCm GPU")]

DEV = "cuda"
SIZE = (32, 32)


def _files(tmp_path, video, n=5):
    out = []
    for i in range(n):
        ent = ol.synthetic_entry(40 + i, (36 + 2 * i, 44), (40, 40 + 3 * i), video)
        out.append(_write_entry(str(tmp_path), i, ent))
    return out


def _reference_loop(trainer, files, tests, make, epochs, bs, validate=False, examples=False):
    """train.py:64-109 as the reference writes it (summaries aside); validate: training_procedure's validation
    batches (their loader draws; the forward leaves the model as it is); examples: the epoch-end example summary's
    draws (train.py:102-104: 5 np.random.randint picks of the test list, then the loader call over them)."""
    from vmatting import loader
    losses = []
    for _ in range(epochs):
        training_list, test_list = files.copy(), tests.copy()
        random.shuffle(training_list)
        random.shuffle(test_list)
        while not loader.epoch_is_over(training_list, bs):
            losses.append(trainer.step(*make(loader.get_batch_list(training_list, bs))).cpu().numpy())
        while validate and not loader.epoch_is_over(test_list, bs):
            make(loader.get_batch_list(test_list, bs))
        if examples:
            make([tests[np.random.randint(0, len(tests))] for _ in range(5)])
    return losses


def _run(kind, tmp_path, graph):
    from vmatting import loader, procedures
    from vmatting.weights import synthetic_vgg16
    video = kind == "video"
    files = _files(tmp_path, video)
    tests = files[:3]

    def trainer():
        np.random.seed(11)
        if kind == "image":
            from vmatting.image_train import ImageTrainer
            return ImageTrainer(synthetic_vgg16(0), "fp32", DEV)
        if kind == "small":
            from vmatting.small_train import SmallTrainer
            return SmallTrainer(6, "fp32", DEV)
        from vmatting.train import VideoTrainer
        return VideoTrainer(synthetic_vgg16(0), "fp32", DEV, lr=1e-4 if kind == "simple" else 1e-3)

    def make(bl):
        if kind == "image":
            inp, lab, rfg = loader.get_batch(bl, SIZE, rd_mirror=True)
            return inp[..., :3].contiguous(), inp[..., 3:].contiguous(), lab, rfg
        if kind == "video":
            cmp, bg, lab, warped, rfg = loader.video_batch(bl, SIZE)
            return cmp, bg, warped, lab, rfg
        cmp, bg, lab, rfg = loader.simple_batch(bl, SIZE)
        return (cmp, bg, cmp - bg, lab, rfg) if kind == "simple" else (cmp, bg, lab, rfg)

    proc = {"image": procedures.training_procedure, "simple": procedures.simple_procedure,
            "video": procedures.video_procedure, "small": procedures.small_training}[kind]
    got, vals = [], []
    t = trainer()
    random.seed(5)
    np.random.seed(6)
    proc(t, files, tests, n_epochs=2, batch_size=2, input_size=SIZE, graph=graph,
         on_step=lambda e, i, loss: got.append(loss.cpu().numpy()), on_epoch=lambda e, i, v: vals.append(v))
    t2 = trainer()
    random.seed(5)
    np.random.seed(6)
    # the epoch-end example draws of train.py (small_train.py makes them every 1000 iterations: none here)
    want = _reference_loop(t2, files, tests, make, 2, 2, validate=kind == "image", examples=kind != "small")
    return got, want, vals


@pytest.mark.parametrize("kind", ["image", "simple", "video", "small"])
def test_procedure_matches_reference_loop(kind, tmp_path):
    got, want, vals = _run(kind, tmp_path, False)
    assert len(got) == len(want) == 4  # 2 epochs x (5 entries // batch 2)
    for a, b in zip(got, want):
        assert np.array_equal(a, b), (a, b)
    if kind == "image":
        assert len(vals) == 2 and all(np.isfinite(v) and v > 0 for v in vals)
    else:
        assert vals == [None, None]


@pytest.mark.parametrize("kind", ["video", "small"])
def test_procedure_graph_replay_matches_eager(kind, tmp_path):
    got, want, _ = _run(kind, tmp_path, True)
    for a, b in zip(got, want):
        assert np.array_equal(a, b), (a, b)


def test_image_validation_loss_is_the_forward_loss(tmp_path):
    """training_procedure's validation (train.py:82-95): mean over the test list's batches of the forward loss."""
    from vmatting import loader, ops, procedures
    from vmatting.image_train import ImageTrainer
    from vmatting.weights import synthetic_vgg16
    files = _files(tmp_path, False)
    np.random.seed(11)
    t = ImageTrainer(synthetic_vgg16(0), "fp32", DEV)
    vals = []
    random.seed(2)
    np.random.seed(3)
    procedures.training_procedure(t, files[:2], files, n_epochs=1, batch_size=2, input_size=SIZE,
                                  on_epoch=lambda e, i, v: vals.append(v))
    # replay: the same shuffles, the training batch's draws, then the validation batches on the updated model
    random.seed(2)
    np.random.seed(3)
    tl, vl = files[:2], list(files)
    random.shuffle(tl)
    random.shuffle(vl)
    loader.get_batch([tl.pop() for _ in range(2)], SIZE, rd_mirror=True)
    acc = []
    while len(vl) >= 2:
        inp, lab, rfg = loader.get_batch([vl.pop() for _ in range(2)], SIZE, rd_mirror=True)
        cmp, bg = inp[..., :3].contiguous(), inp[..., 3:].contiguous()
        acc.append(float(ops.matting_loss(t.forward(cmp, bg), lab, rfg, bg, cmp)[0]))
    torch.cuda.synchronize()
    assert vals == [sum(acc) / len(acc)]
