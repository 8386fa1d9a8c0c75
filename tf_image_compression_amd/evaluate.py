"""Rate / distortion evaluation, mirroring processing_utils/evaluate.py (same names and
formulas) with the per-image squared error optionally computed on the GPU.

* ``mse(a, b)``          evaluate.py:10-11 — the SUM of squared differences (the reference
                          names it mse; the division by the pixel count happens later).
* ``mse2psnr(m)``        :14-15 — 20 log10(255) - 10 log10(m).
* ``evaluate(pairs)``    :18-32 — dataset PSNR = mse2psnr(sum of SSE / sum of dims).
* ``get_code_size`` / ``calc_bpp`` / ``calc_psnr``  :35-66.

``sse_device(codec, d_a, d_b, n)`` is the GPU form of ``mse`` for uint8 images already in
HBM (exact integer sum, tic_sse_u8_device); the sharded dataset run and the benchmark
reduce it over ranks with the one stats all-gather.
"""
from __future__ import annotations

import os
from os.path import getsize, isfile, join

import numpy as np


def mse(image0, image1):
    return np.sum(np.square(np.asarray(image1, np.float32) - np.asarray(image0, np.float32)))


def mse2psnr(m):
    return 20.0 * np.log10(255.0) - 10.0 * np.log10(m)


def _read(path):
    from PIL import Image
    return np.asarray(Image.open(path), dtype=np.float32)


def evaluate(image_files):
    """image_files: iterable of (original, reconstruction) — paths or arrays."""
    num_dims = 0
    sq = []
    for a, b in image_files:
        img = _read(a) if isinstance(a, str) else np.asarray(a, np.float32)
        rec = _read(b) if isinstance(b, str) else np.asarray(b, np.float32)
        num_dims += img.size
        sq.append(mse(img, rec))
    return mse2psnr(np.sum(sq) / num_dims)


def get_code_size(folder):
    return sum(getsize(join(folder, f)) for f in os.listdir(folder)
               if isfile(join(folder, f)) and ".png" not in f)


def calc_bpp(code_dir, pixel_num):
    return get_code_size(code_dir) * 8.0 / pixel_num


def calc_psnr(ori_images_dir, recons_images_dir):
    pairs = [(join(ori_images_dir, f), join(recons_images_dir, f)) for f in os.listdir(ori_images_dir)]
    return evaluate(pairs)


def sse_device(codec, d_a, d_b, n: int, d_acc=None) -> int:
    """Exact sum of squared differences of two uint8 device buffers of n bytes."""
    own = d_acc is None
    if own:
        d_acc = codec.alloc(8)
    codec.memset_device(d_acc, 0, 8)
    codec.sse_u8_device(d_a, d_b, n, d_acc)
    v = int(d_acc.download((1,), np.uint64)[0])
    if own:
        d_acc.free()
    return v
