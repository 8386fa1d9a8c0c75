"""``from tf_image_compression_amd.model_0 import model`` — drop-in for ``from model_0 import model``
(encode.py:225-232): encoder / decoder over the gfx950 libtic path (see model_module.py)."""
from ..model_module import ModelModule

_module = ModelModule(0)
encoder = _module.encoder
decoder = _module.decoder
decoder_u8 = _module.decoder_u8
restore = _module.restore
codec = _module.codec
