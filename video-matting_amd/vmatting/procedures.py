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

Out of scope, as SURVEY.md §2 has it: tf.summary writers and the example-image summaries, tf.train.Saver checkpoints
and the timestamped log directories.  In their place every loop takes ``on_step(epoch, iteration, loss)`` (loss =
the device tensor [loss, alpha_loss, compositional_loss] of that step, before the update) and ``on_epoch(epoch,
iteration, val_loss)`` callbacks; ``trainer.params_numpy()`` gives the variables for a checkpoint.  Returns the
trainer.
"""

import random

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
    static inputs are re-loaded per batch; a batch of another shape falls back to the eager step)."""

    def __init__(self, trainer, graph):
        self.trainer, self.graph, self.g, self.shapes = trainer, bool(graph), None, None

    def __call__(self, *batch):
        if not self.graph:
            return self.trainer.step(*batch)
        shapes = tuple(tuple(t.shape) for t in batch)
        if self.g is None:
            self.g, self.shapes = self.trainer.capture(*batch), shapes
        if shapes != self.shapes:
            return self.trainer.step(*batch)
        return self.g.step(*batch)


def _loop(trainer, train_file_list, test_file_list, make_batch, n_epochs, batch_size, graph, on_step, on_epoch,
          validate=None):
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
        val_loss = validate(test_list) if validate is not None else None
        if on_epoch is not None:
            on_epoch(epoch, iteration, val_loss)
    return trainer


# ------------------------------------------------------------------------------------------------ train.py

def training_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                       batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                       on_epoch=None):
    """train.py:37-109 on an ImageTrainer (UNetImage, Adam lr 1e-5 over every variable): loader.get_batch with
    random mirroring -> step; after each epoch the validation loss = mean over the test list's batches of the
    forward loss (train.py:82-95; 0/0 -> nan on a test list shorter than a batch, as np does)."""

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
        return val / n if n else float("nan")

    return _loop(trainer, train_file_list, test_file_list,
                 lambda bl: tuple(t.contiguous() for t in make(bl)), n_epochs, batch_size, graph, on_step, on_epoch,
                 validate)


def simple_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                     batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                     on_epoch=None):
    """train.py:156-238 on a VideoTrainer(lr=1e-4) (UNetSimple over (cmp, bg, diff = cmp - bg), Adam over
    simple_unet's variables): loader.simple_batch -> step.  Its validation is commented out in the reference."""

    def make(batch_list):
        cmp, bg, lab, rfg = loader.simple_batch(batch_list, input_size, device=trainer.device)
        return cmp, bg, cmp - bg, lab, rfg  # train.py:245: diff = tf.subtract(in_cmp, in_bg)

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch)


def video_procedure(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                    batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                    on_epoch=None):
    """train.py:288-343 on a VideoTrainer (lr 1e-3): loader.video_batch -> (cmp, bg, label, warped, raw_fg) ->
    step(cmp, bg, warped, label, raw_fg)."""

    def make(batch_list):
        cmp, bg, lab, warped, rfg = loader.video_batch(batch_list, input_size, device=trainer.device)
        return cmp, bg, warped, lab, rfg

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch)


def train(dataset=None, training_list=None, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:112-135: a fresh UNetImage (VGG16 encoder from vgg16_npy_path, halved conv1_1) trained by
    training_procedure on loader.get_file_list(dataset, training_list) — the reference passes its TRAINING_LIST
    as the test list too (train.py:123-124), and so does this."""
    from .image_train import ImageTrainer
    files = loader.get_file_list(dataset, training_list)
    trainer = ImageTrainer(vgg16_npy_path, dtype, device, lr=1e-5)
    return training_procedure(trainer, files, files, **kw)


def simple_train(dataset=None, training_list=None, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:241-262: UNetSimple over the three VGG16 towers, trained by simple_procedure (TRAINING_LIST as
    the test list too, train.py:254-255)."""
    from .train import VideoTrainer
    files = loader.get_file_list(dataset, training_list)
    trainer = VideoTrainer(vgg16_npy_path, dtype, device, lr=1e-4)
    return simple_procedure(trainer, files, files, **kw)


def video_train(train_list, test_list, vgg16_npy_path=None, dtype="fp32", device="cuda", **kw):
    """train.py:346-366: UNetSimple(cmp, bg, warped) trained by video_procedure.  The reference lists its
    (fg, bg, previous, flo) entries with loader.video_file_list() (a directory walk of its dataset layout,
    loader.py:240-282); video_file_list below does that walk, or pass the lists directly."""
    from .train import VideoTrainer
    trainer = VideoTrainer(vgg16_npy_path, dtype, device, lr=1e-3)
    return video_procedure(trainer, train_list, test_list, **kw)


# ------------------------------------------------------------------------------------------------ small_train.py

def small_training(trainer, train_file_list, test_file_list, n_epochs=params.N_EPOCHS,
                   batch_size=params.BATCH_SIZE, input_size=params.INPUT_SIZE, graph=False, on_step=None,
                   on_epoch=None):
    """small_train.py:34-88 on a SmallTrainer (UNetSmall(concat(cmp, bg)), Adam over every variable at the
    trainer's lr): loader.simple_batch -> step(cmp, bg, label, raw_fg)."""

    def make(batch_list):
        return loader.simple_batch(batch_list, input_size, device=trainer.device)

    return _loop(trainer, train_file_list, test_file_list, make, n_epochs, batch_size, graph, on_step, on_epoch)


def small_train(learning_rate=1e-5, dataset=None, training_list=None, test_list=None, dtype="fp32",
                device="cuda", **kw):
    """small_train.train(learning_rate) (small_train.py:91-112): a fresh UNetSmall on 6 input channels trained
    by small_training on get_file_list(dataset, TRAINING_LIST) / get_file_list(dataset, TEST_LIST)."""
    from .small_train import SmallTrainer
    trainer = SmallTrainer(6, dtype, device, lr=learning_rate)
    return small_training(trainer, loader.get_file_list(dataset, training_list),
                          loader.get_file_list(dataset, test_list), **kw)


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
