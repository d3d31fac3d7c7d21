"""The reference's training entry points and their epoch loops, over the device trainers.

    train.py        training_procedure (train.py:37-109)  + train()        (train.py:112-135)  UNetImage, ImageTrainer
                    simple_procedure   (train.py:156-238) + simple_train() (train.py:241-262)  UNetSimple(cmp, bg, cmp-bg)
                    video_procedure    (train.py:288-343) + video_train()  (train.py:346-366)  UNetSimple(cmp, bg, warped)
    small_train.py  small_training     (small_train.py:34-88) + train(lr)  (small_train.py:91-112)  UNetSmall

Each loop is the reference's: per epoch (params.N_EPOCHS) the train and test lists are copied and shuffled with
Python's ``random`` (train list first), batches are popped off the END of the shuffled list by
loader.get_batch_list until loader.epoch_is_over, made by the loader call the reference uses (get_batch with
rd_mirror=True / simple_batch / video_batch: the gfx950 loader of vmatting.loader) and fed to one training step
(the trainer's fused forward + loss + backward + TF-Adam; a HIP-graph replay of it with ``graph=True``).
training_procedure then computes the validation loss over the test list (forward + loss only, train.py:82-95).

Out of scope, as SURVEY.md §2 has it: tf.summary writers, tf.train.Saver checkpoints and the timestamped log
directories.  The example-image summaries are not written either, but their draws are made (5 np.random.randint
picks of the test list and the loader call over them, results discarded: train.py:102-104,230-233,335-338,
small_train.py:78-82), so a seeded run keeps the reference's np.random stream in every epoch.  In their place every loop takes ``on_step(epoch, iteration, loss)`` (loss =
the device tensor [loss, alpha_loss, compositional_loss] of that step, before the update) and ``on_epoch(epoch,
iteration, val_loss)`` callbacks; ``trainer.params_numpy()`` gives the variables for a checkpoint.  Returns the
trainer.
"""

import os
import random

import numpy as np

from . import loader, ops, params


def _shuffled(file_list):
    out = list(file_list)  # train.py:66: file_list.copy()
    random.shuffle(out)
    return out


def _epoch_batches(file_list, batch_size):
    """train.py:70-72: pop batch_size entries off the end until fewer than batch_size are left."""
    while not loader.epoch_is_over(file_list, batch_size):
        yield loader.get_batch_list(file_list, batch_size)


class _Stepper:
    """trainer.step(*batch), or the same step replayed from a HIP graph captured on the first batch (the graph's
    static inputs are re-loaded per batch).  The reference's loops only make full batches of one input size
    (loader.epoch_is_over), so a graph loop takes one shape: a batch of another shape raises instead of running an
    eager step, which would rebuild the trainer's buffers under the captured graph."""

    def __init__(self, trainer, graph):
        self.trainer, self.graph, self.g, self.shapes = trainer, bool(graph), None, None

    def __call__(self, *batch):
        if not self.graph:
            return self.trainer.step(*batch)
        shapes = tuple(tuple(t.shape) for t in batch)
        if self.g is None:
            self.g, self.shapes = self.trainer.capture(*batch), shapes
        if shapes != self.shapes:
            raise ValueError("graph=True loop: batch shapes %s differ from the captured %s (one batch shape per "
                             "HIP-graph loop; run with graph=False)" % (shapes, self.shapes))
        return self.g.step(*batch)


def _example_draws(test_file_list, make_batch, n_ex=5):
    """The example summary's draws (train.py:102-104): 5 np.random.randint picks of the test list, then the loader
    call over them (its own crop / mirror draws); the batch itself is discarded (no summary writers here)."""
    ex_list = [test_file_list[np.random.randint(0, len(test_file_list))] for _ in range(n_ex)]
    make_batch(ex_list)


def _loop(trainer, train_file_list, test_file_list, make_batch, n_epochs, batch_size, graph, on_step, on_epoch,
          validate=None, examples=None, example_every=None):
    """examples: the loader call of the example summary (None = no draws); made after each epoch, or, with
    example_every (small_train.py:78), whenever (iteration + 1) % example_every == 0 after a step."""
    step = _Stepper(trainer, graph)
    iteration = 0
    for epoch in range(n_epochs):
        training_list = _shuffled(train_file_list)
        test_list = _shuffled(test_file_list)
        for batch_list in _epoch_batches(training_list, batch_size):
            loss = step(*make_batch(batch_list))
            if on_step is not None:
                on_step(epoch, iteration, loss)
            iteration += 1
            if examples is not None and example_every and (iteration + 1) % example_every == 0:
                _example_draws(test_file_list, examples)
        val_loss = validate(test_list) if validate is not None else None
        if examples is not None and not example_every:
            _example_draws(test_file_list, examples)
        if on_epoch is not None:
            on_epoch(epoch, iteration, val_loss)
    return trainer


# ------------------------------------------------------------------------------------------------ train.py

def training_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                       batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                       on_epoch=None, examples=True):
    """train.py:37-109 on an ImageTrainer (UNetImage, Adam lr 1e-5 over every variable): loader.get_batch with
    random mirroring -> step; after each epoch the validation loss = mean over the test list's batches of the
    forward loss (train.py:82-95: a test list shorter than one batch divides 0. by 0 and raises ZeroDivisionError,
    as the reference's Python float division does), then the example draws (``examples``)."""

    def make(batch_list):
        inp, lab, rfg = loader.get_batch(batch_list, input_size, rd_scale=False, rd_mirror=True,
                                         device=trainer.device)
        return inp[..., :3], inp[..., 3:], lab, rfg  # train.py:41: tf.split(x, [3, 3])

    def validate(test_list):
        val, n = 0.0, 0
        for batch_list in _epoch_batches(test_list, batch_size):
            cmp, bg, lab, rfg = [t.contiguous() for t in make(batch_list)]
            alpha = trainer.forward(cmp, bg)
            val += float(ops.matting_loss(alpha, lab, rfg, bg, cmp)[0])
            n += 1
        return val / n  # train.py:96 (n == 0: ZeroDivisionError, like the reference)

    return _loop(trainer, train_file_list, test_file_list,
                 lambda bl: tuple(t.contiguous() for t in make(bl)), n_epochs, batch_size, graph, on_step, on_epoch,
                 validate, make if examples else None)


def simple_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                     batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                     on_epoch=None, examples=True):
    """train.py:156-238 on a VideoTrainer(lr=1e-4) (UNetSimple over (cmp, bg, diff = cmp - bg), Adam over
    simple_unet's variables): loader.simple_batch -> step.  Its validation is commented out in the reference."""

    def make(batch_list):
        cmp, bg, lab, rfg = loader.simple_batch(batch_list, input_size, device=trainer.device)
        return cmp, bg, cmp - bg, lab, rfg  # train.py:245: diff = tf.subtract(in_cmp, in_bg)

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch,
                 examples=make if examples else None)


def video_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                    batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                    on_epoch=None, examples=True):
    """train.py:288-343 on a VideoTrainer (lr 1e-3): loader.video_batch -> (cmp, bg, label, warped, raw_fg) ->
    step(cmp, bg, warped, label, raw_fg)."""

    def make(batch_list):
        cmp, bg, lab, warped, rfg = loader.video_batch(batch_list, input_size, device=trainer.device)
        return cmp, bg, warped, lab, rfg

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch,
                 examples=make if examples else None)


def _dataset_files(dataset, list_path, who):
    """loader.get_file_list(dataset, list_path) with the reference's params defaults (params.py:3,5-6: the author's
    SYNTHETIC_DATASET root and ./dataset/*.txt lists), or a ValueError naming what is missing."""
    dataset = params.SYNTHETIC_DATASET if dataset is None else dataset
    if dataset is None:
        raise ValueError("%s: no dataset root — pass dataset=... or set vmatting.params.SYNTHETIC_DATASET (env "
                         "VM_SYNTHETIC_DATASET); the reference's params.py:3 names a directory on its author's "
                         "machine" % who)
    if not os.path.isfile(list_path):
        raise ValueError("%s: list file %r not found (the reference's %s, params.py:5-6; pass it explicitly)"
                         % (who, list_path, "TEST_LIST" if list_path == params.TEST_LIST else "TRAINING_LIST"))
    return loader.get_file_list(dataset, list_path)


def train(dataset=None, training_list=None, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:112-135: a fresh UNetImage (VGG16 encoder from vgg16_npy_path, halved conv1_1) trained by
    training_procedure on loader.get_file_list(dataset, training_list) — the reference passes its TRAINING_LIST
    as the test list too (train.py:123-124), and so does this.  Called with no arguments, like the reference, it
    reads params.SYNTHETIC_DATASET / params.TRAINING_LIST and raises ValueError when they are not there."""
    from .image_train import ImageTrainer
    files = _dataset_files(dataset, params.TRAINING_LIST if training_list is None else training_list, "train()")
    trainer = ImageTrainer(vgg16_npy_path, dtype, device, lr=1e-5)
    return training_procedure(trainer, files, files, **kw)


def simple_train(dataset=None, training_list=None, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:241-262: UNetSimple over the three VGG16 towers, trained by simple_procedure (TRAINING_LIST as
    the test list too, train.py:254-255); no arguments: params' dataset and list, as train()."""
    from .train import VideoTrainer
    files = _dataset_files(dataset, params.TRAINING_LIST if training_list is None else training_list,
                           "simple_train()")
    trainer = VideoTrainer(vgg16_npy_path, dtype, device, lr=1e-4)
    return simple_procedure(trainer, files, files, **kw)


def video_train(train_list=None, test_list=None, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:346-366: UNetSimple(cmp, bg, warped) trained by video_procedure.  The reference lists its
    (fg, bg, previous, flo) entries with loader.video_file_list() (a directory walk of its dataset layout under the
    working directory, loader.py:240-282, split by params' name lists); with no lists given, video_file_list below
    does that walk with vmatting.params' lists, and a walk that finds nothing raises ValueError."""
    from .train import VideoTrainer
    if train_list is None or test_list is None:
        tr, te = video_file_list(".", params.TRAIN_AUGMENTED, params.TEST_AUGMENTED, params.TRAIN_SYNTHETIC,
                                 params.TEST_SYNTHETIC)
        train_list = tr if train_list is None else train_list
        test_list = te if test_list is None else test_list
        if not train_list:
            raise ValueError("video_train(): no training entries — the walk of ./flow/{augmented,synthetic} and "
                             "./SYNTHETIC (loader.py:240-282) found none under %r for the name lists "
                             "vmatting.params.TRAIN_AUGMENTED / TRAIN_SYNTHETIC (%d / %d names); pass train_list / "
                             "test_list" % (os.getcwd(), len(params.TRAIN_AUGMENTED), len(params.TRAIN_SYNTHETIC)))
    trainer = VideoTrainer(vgg16_npy_path, dtype, device, lr=1e-3)
    return video_procedure(trainer, train_list, test_list, **kw)


# ------------------------------------------------------------------------------------------------ small_train.py

def small_training(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                   batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                   on_epoch=None, examples=True):
    """small_train.py:34-88 on a SmallTrainer (UNetSmall(concat(cmp, bg)), Adam over every variable at the
    trainer's lr): loader.simple_batch -> step(cmp, bg, label, raw_fg); the example draws whenever
    (iteration + 1) % 1000 == 0 (small_train.py:78-82)."""

    def make(batch_list):
        return loader.simple_batch(batch_list, input_size, device=trainer.device)

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch,
                 examples=make if examples else None, example_every=1000)


def small_train(learning_rate=1e-5, dataset=None, training_list=None, test_list=None, dtype="fp32",
                device="cuda", **kw):
    """small_train.train(learning_rate) (small_train.py:91-112): a fresh UNetSmall on 6 input channels trained
    by small_training on get_file_list(dataset, TRAINING_LIST) / get_file_list(dataset, TEST_LIST) (params'
    defaults when not given, as train())."""
    from .small_train import SmallTrainer
    train_files = _dataset_files(dataset, params.TRAINING_LIST if training_list is None else training_list,
                                 "small_train.train()")
    test_files = _dataset_files(dataset, params.TEST_LIST if test_list is None else test_list, "small_train.train()")
    trainer = SmallTrainer(6, dtype, device, lr=learning_rate)
    return small_training(trainer, train_files, test_files, **kw)


# ------------------------------------------------------------------------------------------------ file lists

def video_file_list(root=".", train_augmented=(), test_augmented=(), train_synthetic=(), test_synthetic=()):
    """loader.video_file_list (loader.py:240-282): (fg, bg, previous, flo) path tuples of the augmented set
    (flow/augmented/{fg,bg,flow}) and of the synthetic videos (flow/synthetic/<video>/*.flo over
    SYNTHETIC/{fg,bg}/<video>/in%04d.png), split into train / test by the name lists of the reference's params.py
    (TRAIN_AUGMENTED, TEST_AUGMENTED, TRAIN_SYNTHETIC, TEST_SYNTHETIC; passed in here).  Entries with a missing
    previous frame are skipped, as in the reference; names in neither list are reported and skipped."""
    import os
    join = os.path.join
    aug_train, aug_test, syn_train, syn_test = [], [], [], []
    aug = join(root, "flow", "augmented")
    for filename in sorted(os.listdir(join(aug, "flow"))) if os.path.isdir(join(aug, "flow")) else []:
        stem = filename.split(".")[0]
        basename, id_ = "_".join(stem.split("_")[:-1]), int(stem.split("_")[-1])
        prev = join(aug, "fg", "{}_fg_ref.png".format(basename))
        fg = join(aug, "fg", "{}_fg_{:04d}.png".format(basename, id_))
        bg = join(aug, "bg", "{}_bg_{:04d}.png".format(basename, id_))
        if not (os.path.isfile(prev) and os.path.isfile(fg) and os.path.isfile(bg)):
            print("ERROR LOADING FILE {} FOR ID {}".format(basename, id_))
            continue
        entry = (fg, bg, prev, join(aug, "flow", filename))
        if basename in train_augmented:
            aug_train.append(entry)
        elif basename in test_augmented:
            aug_test.append(entry)
        else:
            print("ERROR, CANT FIND {}".format(basename))
    syn = join(root, "flow", "synthetic")
    for title in sorted(os.listdir(syn)) if os.path.isdir(syn) else []:
        for filename in sorted(os.listdir(join(syn, title))):
            id_ = int(filename.split(".")[0][2:])
            fg = join(root, "SYNTHETIC", "fg", title, "in{:04d}.png".format(id_ + 1))
            bg = join(root, "SYNTHETIC", "bg", title, "in{:04d}.png".format(id_ + 1))
            prev = join(root, "SYNTHETIC", "fg", title, "in{:04d}.png".format(id_))
            if not os.path.isfile(prev):
                continue
            entry = (fg, bg, prev, join(syn, title, filename))
            if title in train_synthetic:
                syn_train.append(entry)
            elif title in test_synthetic:
                syn_test.append(entry)
    return aug_train + syn_train, aug_test + syn_test


__all__ = ["training_procedure", "simple_procedure", "video_procedure", "small_training", "train", "simple_train",
           "video_train", "small_train", "video_file_list"]
