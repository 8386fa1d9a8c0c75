"""tf_image_compression_amd — MI355X-native encode/decode hot path of
bolin-chen/tf_image_compression (conv/deconv autoencoder codec).

Host side is Python over a ctypes C-ABI (libtic.so, include/tic.h); the compute is
hand-written gfx950 HIP.  No PyTorch, no CPU fallback.
"""
from .topology import layer_table, param_shapes, bottleneck_shape, RMBE_ID  # noqa: F401

__version__ = "0.1.0"


def Codec(*args, **kwargs):  # lazy: importing the package must not load the GPU runtime
    from .codec import Codec as _C
    return _C(*args, **kwargs)
