"""``from tf_image_compression_amd.base_model.ch_128 import model`` — drop-in for the reference's
base_model/ch_128/model.py encoder / decoder (:34, :123): the 128-channel trunk
(TIC_MODEL_CH128) over the gfx950 libtic path (see model_module.py)."""
from ...model_module import ModelModule
from ...topology import CH128_ID

_module = ModelModule(CH128_ID)
encoder = _module.encoder
decoder = _module.decoder
decoder_u8 = _module.decoder_u8
restore = _module.restore
codec = _module.codec
