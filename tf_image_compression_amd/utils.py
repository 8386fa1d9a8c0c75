"""Host-side helpers mirroring /root/reference/utils/utils.py (same names, same behaviour).

crop_image_input_patches / concat_patches are host numpy glue exactly as in the
reference (utils/utils.py:96-167); read_image_list as :74-81; restore_params loads the
TF-named weights (utils/utils.py:84-93 restores a TF checkpoint; here an .npz with the
same variable names, see weights.py).
"""
from __future__ import annotations

import os

import numpy as np


def read_image_list(data_list):
    with open(data_list) as f:
        return [line.strip("\n") for line in f if line.strip("\n")]


def crop_image_input_patches(image, patch_size):
    """Reflect-pad bottom/right to a multiple of patch_size (np.pad 'reflect' excludes the
    edge pixel, utils/utils.py:109) and cut row-major patches."""
    height, width, _ = image.shape
    ph = (patch_size - height % patch_size) % patch_size
    pw = (patch_size - width % patch_size) % patch_size
    padded = np.pad(image, ((0, ph), (0, pw), (0, 0)), "reflect")
    H, W, _ = padded.shape
    return [padded[i * patch_size:(i + 1) * patch_size, j * patch_size:(j + 1) * patch_size]
            for i in range(H // patch_size) for j in range(W // patch_size)]


def concat_patches(patches, height, width, patch_size):
    """Stitch row-major patches and crop to (height, width) (utils/utils.py:136-167)."""
    hn = -(-height // patch_size)
    wn = -(-width // patch_size)
    rows = [np.concatenate(list(patches[i * wn:(i + 1) * wn]), axis=1) for i in range(hn)]
    return np.concatenate(rows, axis=0)[:height, :width]


def default_params_file(model_num):
    """utils/utils.py:86: model_N/params_for_test/params (a TF checkpoint prefix, or + '.npz')."""
    return os.path.join(f"model_{model_num}", "params_for_test", "params")


def restore_params(args_or_path, model_num=None):
    """Load weights for a codec: ``args.params_file`` (or the default path), a TF V2
    checkpoint prefix (tf_checkpoint.py) or an .npz of the same variable names."""
    from .weights import load_params
    if isinstance(args_or_path, str):
        path = args_or_path
    else:
        path = args_or_path.params_file or default_params_file(args_or_path.model_num)
        model_num = int(args_or_path.model_num)
    params = load_params(path, model_num)
    print(f"Params in {path} restored complete")
    return params


def imread(path):
    from PIL import Image
    img = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)
    return img


def imsave(path, image):
    from PIL import Image
    Image.fromarray(np.asarray(image, dtype=np.uint8)).save(path)
