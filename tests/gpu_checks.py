"""Shared GPU parity checks (imported by the -m gpu test modules; not a test module).

The bars are DESIGN.md §4's: pre-activations within 1e-4 relative of the oracle, symbols
bit-exact outside the 1e-5 decision band, decoder float within 1e-2 on the [0,255]
scale when fed the same symbols, uint8 within 1 and only on .5 rounding edges, dataset
PSNR within 0.02 dB (north_star tolerance)."""
import numpy as np

from oracle import tic_oracle as o


def check_codec(codec, params, model_id, P, patches, Q=2):
    idx, pre = codec.encode(patches, return_preact=True)
    ref_pre, ref_idx = o.encoder(params, codec_mean(), codec_std(), patches, P, Q, model_id)
    scale = max(1.0, float(np.max(np.abs(ref_pre))))
    assert pre.shape == ref_pre.shape and idx.shape == ref_idx.shape
    assert float(np.max(np.abs(pre - ref_pre))) <= 1e-4 * scale
    margin = o.decision_margin(ref_pre, Q)
    safe = margin > 1e-5 * scale
    mism = int(np.count_nonzero((idx != ref_idx) & safe))
    assert mism == 0, f"{mism} symbol mismatches outside the tie band"
    # decoder on the GPU's own symbols, oracle on the same symbols
    rgb, f = codec.decode(idx, return_float=True)
    ref_f, ref_u8 = o.decoder(params, codec_mean(), codec_std(), idx, Q, model_id)
    assert float(np.max(np.abs(f - ref_f))) <= 1e-2
    du = np.abs(rgb.astype(np.int16) - ref_u8.astype(np.int16))
    assert int(du.max()) <= 1
    edge = np.abs((ref_f - np.floor(ref_f)) - 0.5) < 1e-2
    assert int(np.count_nonzero((du > 0) & ~edge)) == 0
    p_gpu = o.dataset_psnr([(patches[i], rgb[i]) for i in range(len(patches))])
    p_ref = o.dataset_psnr([(patches[i], ref_u8[i]) for i in range(len(patches))])
    assert abs(p_gpu - p_ref) <= 0.02, (p_gpu, p_ref)
    return idx, rgb


def check_codec_subset(codec, params, model_id, P, patches, k, Q=2):
    """Encode + decode ALL patches in one call each (the launch sequence of that batch
    size), check the first k against the oracle with check_codec's bars; returns the full
    symbols and bytes."""
    idx, pre = codec.encode(patches, return_preact=True)
    rgb, f = codec.decode(idx, return_float=True)
    sub = patches[:k]
    ref_pre, ref_idx = o.encoder(params, codec_mean(), codec_std(), sub, P, Q, model_id)
    scale = max(1.0, float(np.max(np.abs(ref_pre))))
    assert float(np.max(np.abs(pre[:k] - ref_pre))) <= 1e-4 * scale
    safe = o.decision_margin(ref_pre, Q) > 1e-5 * scale
    mism = int(np.count_nonzero((idx[:k] != ref_idx) & safe))
    assert mism == 0, f"{mism} symbol mismatches outside the tie band"
    ref_f, ref_u8 = o.decoder(params, codec_mean(), codec_std(), idx[:k], Q, model_id)
    assert float(np.max(np.abs(f[:k] - ref_f))) <= 1e-2
    du = np.abs(rgb[:k].astype(np.int16) - ref_u8.astype(np.int16))
    assert int(du.max()) <= 1
    edge = np.abs((ref_f - np.floor(ref_f)) - 0.5) < 1e-2
    assert int(np.count_nonzero((du > 0) & ~edge)) == 0
    p_gpu = o.dataset_psnr([(sub[i], rgb[i]) for i in range(k)])
    p_ref = o.dataset_psnr([(sub[i], ref_u8[i]) for i in range(k)])
    assert abs(p_gpu - p_ref) <= 0.02, (p_gpu, p_ref)
    return idx, rgb


def codec_mean():
    from tf_image_compression_amd.weights import SYNTH_MEAN
    return SYNTH_MEAN


def codec_std():
    from tf_image_compression_amd.weights import SYNTH_STD
    return SYNTH_STD
