"""Block-effect post-filter of the CLIC submission 2 (submit/2/rmbe/rmbe.py:15-111,
network submit/2/rmbe/model.py:113-197), on the gfx950 path.

``rmbe(image)``: 128x128 windows at column offset 64 over all full rows of windows are
filtered and written back, then 128x128 windows at row offset 64 over all full columns;
edge strips that do not fill a window stay untouched.  The reference rebuilds a TF graph
and session and restores the weights on every call (run_rmbe_model :28-44); here the
network lives in one libtic handle and each pass is one batched launch sequence.
"""
from __future__ import annotations

import numpy as np

from .topology import RMBE_ID

PATCH, OFFSET = 128, 64  # submit/2/rmbe/rmbe.py:12,16


class RmbeFilter:
    def __init__(self, params, mean, std, device=0):
        from .codec import Codec
        self.codec = Codec(RMBE_ID, params, mean, std, patch_size=PATCH, device=device)

    @classmethod
    def from_files(cls, weights_npz, norm_npz=None, device=0):
        import os
        from .weights import load_params, load_normalization
        mean, std = load_normalization(norm_npz if norm_npz and os.path.exists(norm_npz) else None)
        return cls(load_params(weights_npz), mean, std, device)

    def _pass(self, img, r0, c0, hn, wn):
        if hn <= 0 or wn <= 0:
            return img
        P = PATCH
        wins = np.stack([img[r0 + i * P:r0 + (i + 1) * P, c0 + j * P:c0 + (j + 1) * P]
                         for i in range(hn) for j in range(wn)])
        out = self.codec.rmbe_windows(wins)
        for i in range(hn):
            for j in range(wn):
                img[r0 + i * P:r0 + (i + 1) * P, c0 + j * P:c0 + (j + 1) * P] = out[i * wn + j]
        return img

    def apply(self, image):
        img = np.array(image, dtype=np.float32, copy=True)
        h, w, _ = img.shape
        img = self._pass(img, 0, OFFSET, h // PATCH, (w - OFFSET) // PATCH)      # rmbe_height :70-89
        img = self._pass(img, OFFSET, 0, (h - OFFSET) // PATCH, w // PATCH)      # rmbe_width :92-111
        return img

    def close(self):
        self.codec.close()
