"""Reference-shaped model modules: ``tf_image_compression_amd.model_N.model`` exposes
``encoder(input, patch_size, quan_scale)`` and ``decoder(input, quan_scale)`` like
model_N/model.py:34 and :147, backed by one libtic handle per (patch_size, quan_scale).

Differences from the TF graph functions, by design: inputs/outputs are numpy arrays,
``encoder`` returns uint8 symbols (the reference returns float32 values in {0..Q-1} and
casts them with astype(int) at encode.py:182), ``decoder`` returns the float32
reconstruction clipped to [0,255] exactly like the reference graph (np.around is the
caller's, decode.py:249), and ``decoder_u8`` returns the already-rounded uint8 image.
Weights / statistics are bound with ``restore(params, mean, std)`` (utils.restore_params
+ the import-time npz load of model_0/model.py:26-28).
"""
from __future__ import annotations

import os

import numpy as np

from .weights import load_normalization

NORM_FILE = os.path.join("data_info", "channel_normalization_params.npz")


class ModelModule:
    def __init__(self, model_id: int):
        self.model_id = model_id
        self.params = None
        self.mean = self.std = None
        self.device = int(os.environ.get("TIC_DEVICE", "0"))
        self._codecs = {}

    def restore(self, params, mean=None, std=None, device=None):
        if mean is None or std is None:
            mean, std = load_normalization(NORM_FILE if os.path.exists(NORM_FILE) else None)
        self.params, self.mean, self.std = params, np.asarray(mean, np.float32), np.asarray(std, np.float32)
        if device is not None:
            self.device = int(device)
        self.close()

    def codec(self, patch_size, quan_scale):
        if self.params is None:
            raise RuntimeError(f"model_{self.model_id}: weights not restored (call restore / utils.restore_params)")
        key = (int(patch_size), int(quan_scale))
        if key not in self._codecs:
            from .codec import Codec
            self._codecs[key] = Codec(self.model_id, self.params, self.mean, self.std, patch_size=key[0],
                                      quan_scale=key[1], device=self.device)
        return self._codecs[key]

    def encoder(self, input, patch_size, quan_scale):
        x = np.asarray(input)
        if x.dtype != np.uint8:
            x = np.clip(np.rint(x), 0, 255).astype(np.uint8)
        return self.codec(patch_size, quan_scale).encode(x.reshape(-1, patch_size, patch_size, 3))

    def _patch_for(self, input, quan_scale):
        for (p, q), c in self._codecs.items():
            if q == quan_scale and tuple(c.code_shape) == tuple(np.shape(input)[1:]):
                return c
        from .config import load_config
        return self.codec(load_config(self.model_id)["patch_size"], quan_scale)

    def decoder(self, input, quan_scale):
        _, f = self._patch_for(input, quan_scale).decode(np.asarray(input), return_float=True)
        return f

    def decoder_u8(self, input, quan_scale):
        return self._patch_for(input, quan_scale).decode(np.asarray(input))

    def close(self):
        for c in self._codecs.values():
            c.close()
        self._codecs = {}
