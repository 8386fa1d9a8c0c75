"""Block-effect post-filter of the CLIC submission 2 (submit/2/rmbe/rmbe.py:15-111,
network submit/2/rmbe/model.py:113-197), on the gfx950 path.

``rmbe(image)``: 128x128 windows at column offset 64 over all full rows of windows are
filtered and written back, then 128x128 windows at row offset 64 over all full columns;
edge strips that do not fill a window stay untouched.  The reference rebuilds a TF graph
and session and restores the weights on every call (run_rmbe_model :28-44); here the
network lives in one libtic handle, the window gather / write-back are kernels
(image_ops.hip) and each pass is one batched launch sequence (tic_rmbe_image_device).
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
        return cls(load_params(weights_npz, RMBE_ID), mean, std, device)

    def apply(self, image):
        """rmbe.rmbe(image) (submit/2/rmbe/rmbe.py:15-24): float32 HxWx3 in [0,255] -> filtered
        copy; both window passes run on the GPU (tic_rmbe_image_device)."""
        img = np.ascontiguousarray(image, dtype=np.float32)
        h, w, _ = img.shape
        d = self.codec.alloc(img.nbytes)
        try:
            d.upload(img)
            self.codec.rmbe_image_device(d, h, w)
            self.codec.synchronize()
            return d.download(img.shape, np.float32)
        finally:
            d.free()

    def close(self):
        self.codec.close()
