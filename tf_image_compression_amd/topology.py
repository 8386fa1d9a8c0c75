"""Layer tables of the reference models, expanded to one entry per convolution.

The executing copy of these tables lives in the native runtime
(``csrc/tic_runtime.cpp``, exported through ``tic_model_layer``); this module is the
host-side mirror used for weight names/shapes and roofline accounting, and
``tests/test_abi.py`` checks the two agree (and agree with the oracle's own,
independently written tables).

Sources: model_0/model.py:50-246, model_1/model.py (widths 16 at :52/:226),
model_2/model.py:50-193, model_3/model.py:50-300, base_model/ch_128/model.py:50-200,
submit/2/rmbe/model.py:118-189.
``res_block`` (basic_block/basic_block.py:74-93) expands into ``<scope>/conv_0`` and
``<scope>/conv_1`` (both ReLU); the block input is added after conv_1 (no activation).
"""
from __future__ import annotations

from dataclasses import dataclass

RMBE_ID = 100  # pseudo model id for the submit/2 block-effect post-filter
CH128_ID = 128  # base_model/ch_128: the 128-channel trunk (include/tic.h TIC_MODEL_CH128)
MODEL_IDS = (0, 1, 2, 3, CH128_ID, RMBE_ID)


@dataclass(frozen=True)
class Layer:
    name: str        # TF variable scope, e.g. 'encode_res_1/conv_1'
    kind: str        # 'conv_s2' | 'conv_s1' | 'convT'
    cin: int
    cout: int
    act: str         # 'relu' | 'identity'
    stage: str       # 'enc' | 'dec'
    residual: bool   # add the enclosing res_block's input after the activation


def _blocks(model_id):
    r = "relu"
    i = "identity"
    if model_id in (0, 1):
        w0 = 32 if model_id == 0 else 16
        w1 = 32 if model_id == 0 else 16
        enc = [("encode_0", "conv_s2", 3, w0, r), ("encode_1", "conv_s2", w0, 32, r),
               ("encode_2", "conv_s2", 32, 64, r), ("encode_3", "conv_s2", 64, 64, r),
               ("encode_res_1", "res", 64, 64, r), ("encode_res_2", "res", 64, 64, r),
               ("encode_4", "conv_s1", 64, 64, i)]
        dec = [("decode_4", "conv_s1", 64, 64, i),
               ("decode_res_1", "res", 64, 64, r), ("decode_res_2", "res", 64, 64, r),
               ("decode_3", "convT", 64, 64, r), ("decode_2", "convT", 64, 32, r),
               ("decode_1", "convT", 32, w1, r), ("decode_0", "convT", w1, 3, i)]
        return enc, dec
    if model_id == 2:
        enc = [("encode_1", "conv_s2", 3, 32, r), ("encode_2", "conv_s2", 32, 64, r),
               ("encode_3", "conv_s2", 64, 64, r),
               ("encode_res_1", "res", 64, 64, r), ("encode_res_2", "res", 64, 64, r),
               ("encode_4", "conv_s2", 64, 64, i)]
        dec = [("decode_4", "convT", 64, 64, i),
               ("decode_res_1", "res", 64, 64, r), ("decode_res_2", "res", 64, 64, r),
               ("decode_3", "convT", 64, 64, r), ("decode_2", "convT", 64, 32, r),
               ("decode_1", "convT", 32, 3, i)]
        return enc, dec
    if model_id == 3:
        enc = [("encode_1", "conv_s2", 3, 32, r), ("encode_2", "conv_s2", 32, 64, r),
               ("encode_res_m1", "res", 64, 64, r), ("encode_res_0", "res", 64, 64, r),
               ("encode_3", "conv_s2", 64, 64, r),
               ("encode_res_1", "res", 64, 64, r), ("encode_res_2", "res", 64, 64, r),
               ("encode_res_3", "res", 64, 64, r),
               ("encode_4", "conv_s2", 64, 80, i)]
        dec = [("decode_4", "convT", 80, 64, i),
               ("decode_res_1", "res", 64, 64, r), ("decode_res_2", "res", 64, 64, r),
               ("decode_res_3", "res", 64, 64, r),
               ("decode_3", "convT", 64, 64, r),
               ("decode_res_4", "res", 64, 64, r), ("decode_res_5", "res", 64, 64, r),
               ("decode_2", "convT", 64, 32, r), ("decode_1", "convT", 32, 3, i)]
        return enc, dec
    if model_id == CH128_ID:
        enc = [("encode_1", "conv_s2", 3, 64, r), ("encode_2", "conv_s2", 64, 128, r),
               ("encode_res_1", "res", 128, 128, r), ("encode_res_2", "res", 128, 128, r),
               ("encode_3", "conv_s1", 128, 64, i)]
        dec = [("decode_3", "conv_s1", 64, 128, i),
               ("decode_res_1", "res", 128, 128, r), ("decode_res_2", "res", 128, 128, r),
               ("decode_2", "convT", 128, 64, r), ("decode_1", "convT", 64, 3, i)]
        return enc, dec
    if model_id == RMBE_ID:
        enc = [("conv_1", "conv_s2", 3, 32, r), ("conv_2", "conv_s2", 32, 64, r),
               ("conv_3", "conv_s1", 64, 64, r), ("conv_4", "conv_s1", 64, 64, r)]
        dec = [("conv_5", "convT", 64, 32, r), ("conv6", "convT", 32, 3, i)]
        return enc, dec
    raise ValueError(f"unknown model id {model_id}")


def layer_table(model_id: int) -> list[Layer]:
    out = []
    enc, dec = _blocks(model_id)
    for stage, blocks in (("enc", enc), ("dec", dec)):
        for name, kind, cin, cout, act in blocks:
            if kind == "res":
                out.append(Layer(f"{name}/conv_0", "conv_s1", cin, cout, "relu", stage, False))
                out.append(Layer(f"{name}/conv_1", "conv_s1", cout, cout, "relu", stage, True))
            else:
                out.append(Layer(name, kind, cin, cout, act, stage, False))
    return out


def param_shapes(model_id: int) -> dict[str, tuple]:
    shapes = {}
    for lay in layer_table(model_id):
        shapes[f"{lay.name}/kernel"] = ((3, 3, lay.cout, lay.cin) if lay.kind == "convT"
                                        else (3, 3, lay.cin, lay.cout))
        shapes[f"{lay.name}/bias"] = (lay.cout,)
    return shapes


def bottleneck_shape(model_id: int, patch_size: int) -> tuple[int, int, int]:
    """(h, w, C) of the quantised code for one patch."""
    h = patch_size
    for lay in layer_table(model_id):
        if lay.stage != "enc":
            break
        if lay.kind == "conv_s2":
            h = -(-h // 2)
        c = lay.cout
    return h, h, c


def layer_work(model_id: int, patch_size: int):
    """Per-layer algorithmic work for ONE patch: list of (layer, flops, bytes, out_hw).

    FLOPs = 2 x MACs of the 3x3 convolution (transpose: 9 x Cin MACs per *input*
    position, i.e. 9/4 taps per output on average).  Bytes = the layer's activations
    read once and written once at their HBM dtype: f32 inside the network, u8 RGB patch
    in (f32 for the rmbe post-filter), u8 indices out of the encoder and into the
    decoder, u8 RGB out (f32 for rmbe); plus the residual read.  Weights are per
    launch, not per patch: see ``weight_bytes``."""
    rows = []
    layers = layer_table(model_id)
    rmbe = model_id == RMBE_ID
    h = patch_size
    for i, lay in enumerate(layers):
        ho = -(-h // 2) if lay.kind == "conv_s2" else (2 * h if lay.kind == "convT" else h)
        macs = (h * h if lay.kind == "convT" else ho * ho) * 9 * lay.cin * lay.cout
        first = i == 0
        last = i == len(layers) - 1
        first_dec = (not rmbe) and lay.stage == "dec" and layers[i - 1].stage == "enc"
        last_enc = (not rmbe) and lay.stage == "enc" and layers[i + 1].stage == "dec"
        if first:
            in_b = h * h * 3 * (4 if rmbe else 1)
        elif first_dec:
            in_b = h * h * lay.cin
        else:
            in_b = h * h * lay.cin * 4
        if last_enc:
            out_b = ho * ho * lay.cout
        elif last:
            out_b = ho * ho * 3 * (4 if rmbe else 1)
        else:
            out_b = ho * ho * lay.cout * 4
        res_b = ho * ho * lay.cout * 4 if lay.residual else 0
        rows.append((lay, 2.0 * macs, float(in_b + out_b + res_b), ho))
        h = ho
    return rows


def weight_bytes(lay: Layer) -> int:
    return (9 * lay.cin * lay.cout + lay.cout) * 4
