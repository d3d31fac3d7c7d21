"""Convert a trusted, pickled vgg16.npy data_dict (the file unet.py:29 loads) into a weights-only .npz.

    python tools/vgg_npy_to_npz.py weights/vgg16.npy [weights/vgg16.npz]

Run once on a file you trust; afterwards vmatting.weights.load_vgg16 reads the .npz with allow_pickle=False.
"""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "video-matting_amd"))

from vmatting.weights import load_vgg16, save_vgg16_npz  # noqa: E402


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else os.path.splitext(src)[0] + ".npz"
    save_vgg16_npz(load_vgg16(src, allow_pickle=True), dst)
    print("wrote", dst)


if __name__ == "__main__":
    main()
