"""Reference-named entry point: `import train` as the reference's scripts do (train.py:1-366).

Re-exports the training entry points and epoch loops (vmatting.procedures) and the device trainers they drive
(vmatting.train.VideoTrainer for simple_procedure / video_procedure, vmatting.image_train.ImageTrainer for
training_procedure).  Summaries, Saver checkpoints and log directories are out of scope.
"""
from vmatting.image_train import ImageTrainer  # noqa: F401
from vmatting.procedures import (simple_procedure, simple_train, train, training_procedure,  # noqa: F401
                                 video_file_list, video_procedure, video_train)
from vmatting.train import TrainGraph, VideoTrainer  # noqa: F401
