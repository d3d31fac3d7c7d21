"""The constants of reference params.py that the hot path uses (params.py:7-10)."""

N_EPOCHS = 3
BATCH_SIZE = 8
INPUT_SIZE = (320, 320)
VGG_MEAN = [103.939, 116.779, 123.68]  # BGR order (cv2)
