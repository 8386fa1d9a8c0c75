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
        """The reference feeds skimage's uint8 pixels cast to float32 (encode.py:154-157,
        model_0/model.py:39-44).  The device path reads uint8, so float input is accepted
        only when every value is an integer in [0, 255] (exactly what the reference sees);
        anything else raises instead of being silently rounded."""
        x = np.asarray(input)
        if x.dtype != np.uint8:
            if not np.issubdtype(x.dtype, np.number):
                raise ValueError(f"encoder input must be numeric, got {x.dtype}")
            xf = x.astype(np.float64)
            if not np.all(np.isfinite(xf)) or np.any(xf != np.rint(xf)) or np.any(xf < 0) or np.any(xf > 255):
                raise ValueError("encoder input must hold integer pixel values in [0, 255] "
                                 "(the device path reads uint8 pixels)")
            x = xf.astype(np.uint8)
        if x.size % (patch_size * patch_size * 3):
            raise ValueError(f"input of {x.size} values is not a whole number of {patch_size}x{patch_size}x3 patches")
        return self.codec(patch_size, quan_scale).encode(x.reshape(-1, patch_size, patch_size, 3))

    def _patch_for(self, input, quan_scale):
        """The decoder graph takes [N, h, w, C] and returns [N, P, P, 3] (decode.py:159-167):
        P follows from the code's spatial size and the model's stride-2 layers."""
        shape = tuple(np.shape(input)[1:])
        if len(shape) != 3 or shape[0] != shape[1]:
            raise ValueError(f"decoder input must be [N, h, h, C], got {np.shape(input)}")
        for (p, q), c in self._codecs.items():
            if q == quan_scale and tuple(c.code_shape) == shape:
                return c
        from .topology import bottleneck_shape, layer_table
        n_s2 = sum(1 for lay in layer_table(self.model_id) if lay.stage == "enc" and lay.kind == "conv_s2")
        P = shape[0] << n_s2
        if tuple(bottleneck_shape(self.model_id, P)) != shape:
            raise ValueError(f"model_{self.model_id}: no patch size produces a code of shape {shape}")
        return self.codec(P, quan_scale)

    def decoder(self, input, quan_scale):
        _, f = self._patch_for(input, quan_scale).decode(np.asarray(input), return_float=True)
        return f

    def decoder_u8(self, input, quan_scale):
        return self._patch_for(input, quan_scale).decode(np.asarray(input))

    def close(self):
        for c in self._codecs.values():
            c.close()
        self._codecs = {}
