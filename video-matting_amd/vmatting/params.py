"""The constants of reference params.py (params.py:1-15).

The hot path uses N_EPOCHS, BATCH_SIZE, INPUT_SIZE and VGG_MEAN (params.py:7-10).  The dataset locations are the
reference's entry-point defaults (train.py:121-124, small_train.py:95-96, loader.py:240-282): its absolute paths
name directories on the author's machine, so here the dataset root comes from the environment (VM_SYNTHETIC_DATASET;
unset = None, and the argument-free entry points then raise a ValueError naming it), the list files keep the
reference's relative paths, and the video name lists (params.py:12-15: which augmented / synthetic clips are train
or test) are empty unless VM_VIDEO_SPLIT names a JSON file {"TRAIN_AUGMENTED": [...], "TEST_AUGMENTED": [...],
"TRAIN_SYNTHETIC": [...], "TEST_SYNTHETIC": [...]} — the split is dataset metadata, not part of the hot path.
"""

import json
import os

SYNTHETIC_DATASET = os.environ.get("VM_SYNTHETIC_DATASET") or None  # params.py:3
TRAINING_LIST = "./dataset/train.txt"  # params.py:5
TEST_LIST = "./dataset/valid.txt"      # params.py:6
N_EPOCHS = 3
BATCH_SIZE = 8
INPUT_SIZE = (320, 320)
VGG_MEAN = [103.939, 116.779, 123.68]  # BGR order (cv2)
LOG_DIR = "./log/"                     # params.py:11 (no summary writers here)


def _video_split():
    path = os.environ.get("VM_VIDEO_SPLIT")
    if not path:
        return {}
    with open(path) as f:
        return json.load(f)


_split = _video_split()
TRAIN_AUGMENTED = tuple(_split.get("TRAIN_AUGMENTED", ()))  # params.py:12
TEST_AUGMENTED = tuple(_split.get("TEST_AUGMENTED", ()))    # params.py:13
TRAIN_SYNTHETIC = tuple(_split.get("TRAIN_SYNTHETIC", ()))  # params.py:14
TEST_SYNTHETIC = tuple(_split.get("TEST_SYNTHETIC", ()))    # params.py:15
