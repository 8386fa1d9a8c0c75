"""CPU oracle for the tf_image_compression encode/decode hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``tf_image_compression_amd``)
never imports it and has no CPU fallback.

What it restates (NumPy, float64 accumulation by default):

* ``basic_block.my_conv2d``           /root/reference/basic_block/basic_block.py:27-47
  (HWIO kernel :30, ``tf.nn.conv2d`` SAME :33, ``bias_add`` :36, activation :43)
* ``basic_block.my_conv2d_transpose``  basic_block/basic_block.py:50-71
  (kernel ``[kh,kw,Cout,Cin]`` :53, output hard-coded to ``2H x 2W`` :54, op :57)
* ``basic_block.res_block``            basic_block/basic_block.py:74-93 (add, no act, :91)
* ``basic_block.reverse_sigmoid``      basic_block/basic_block.py:152-155
* normalise / quantise / dequantise / denormalise+clip of
  model_0/model.py:38-46,136-144,148-155,250-259 (same in model_1..3)
* layer tables of model_{0,1,2,3}/model.py encoder/decoder and
  submit/2/rmbe/model.py:113-197
* tiling utils/utils.py:96-167, rmbe driver submit/2/rmbe/rmbe.py:15-111,
  dataset PSNR processing_utils/evaluate.py:10-32.

Numerics policy.  Every TF op boundary is rounded to float32 exactly as the
TF-1 graph does (conv result -> f32, then ``bias_add`` in f32, ``relu``, residual
add in f32, ``(x-mean)/std`` in f32, ``y*std+mean`` in f32, clip, half-even
round).  Inside a convolution the sum is accumulated in float64 (``acc``) and
rounded once: the exact value an ideal fp32 convolution approximates.

Parity status: **parity unpinned at the TensorFlow boundary.**  The reference
ships no golden vectors for the network; TensorFlow-1.x is
not installed here (ordinary ModuleNotFoundError, not a permission denial), so
the reference cannot be executed.  The TF semantics restated here (SAME padding
``pad_before = pad_total // 2``; conv2d_transpose = adjoint of the SAME stride-2
conv cropped to 2H; ``tf.round`` half-to-even) are cross-validated against an
independent brute-force scatter definition (tests/test_oracle.py) and, at
fixture-generation time, against torch-CPU ``F.conv2d``/``F.conv_transpose2d``
(tools/make_golden.py).  The committed fixtures in tests/golden/ pin this oracle.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32

# ---------------------------------------------------------------------------
# Layer tables.  Each entry: (scope name, kind, cin, cout, activation).
# kind: 'conv_s2' | 'conv_s1' | 'res' (two relu conv_s1 + add) | 'convT'
# ---------------------------------------------------------------------------

# model_0/model.py:50-134 (encoder) and :159-246 (decoder)
_M0_ENC = [
    ("encode_0", "conv_s2", 3, 32, "relu"),
    ("encode_1", "conv_s2", 32, 32, "relu"),
    ("encode_2", "conv_s2", 32, 64, "relu"),
    ("encode_3", "conv_s2", 64, 64, "relu"),
    ("encode_res_1", "res", 64, 64, "relu"),
    ("encode_res_2", "res", 64, 64, "relu"),
    ("encode_4", "conv_s1", 64, 64, "identity"),
]
_M0_DEC = [
    ("decode_4", "conv_s1", 64, 64, "identity"),
    ("decode_res_1", "res", 64, 64, "relu"),
    ("decode_res_2", "res", 64, 64, "relu"),
    ("decode_3", "convT", 64, 64, "relu"),
    ("decode_2", "convT", 64, 32, "relu"),
    ("decode_1", "convT", 32, 32, "relu"),
    ("decode_0", "convT", 32, 3, "identity"),
]
# model_1/model.py: as model_0 but widths 16 at the ends (:52 filters=16, :226 filters=16)
_M1_ENC = [
    ("encode_0", "conv_s2", 3, 16, "relu"),
    ("encode_1", "conv_s2", 16, 32, "relu"),
    ("encode_2", "conv_s2", 32, 64, "relu"),
    ("encode_3", "conv_s2", 64, 64, "relu"),
    ("encode_res_1", "res", 64, 64, "relu"),
    ("encode_res_2", "res", 64, 64, "relu"),
    ("encode_4", "conv_s1", 64, 64, "identity"),
]
_M1_DEC = [
    ("decode_4", "conv_s1", 64, 64, "identity"),
    ("decode_res_1", "res", 64, 64, "relu"),
    ("decode_res_2", "res", 64, 64, "relu"),
    ("decode_3", "convT", 64, 64, "relu"),
    ("decode_2", "convT", 64, 32, "relu"),
    ("decode_1", "convT", 32, 16, "relu"),
    ("decode_0", "convT", 16, 3, "identity"),
]
# model_2/model.py:50-122 (encoder), :118-193 (decoder)
_M2_ENC = [
    ("encode_1", "conv_s2", 3, 32, "relu"),
    ("encode_2", "conv_s2", 32, 64, "relu"),
    ("encode_3", "conv_s2", 64, 64, "relu"),
    ("encode_res_1", "res", 64, 64, "relu"),
    ("encode_res_2", "res", 64, 64, "relu"),
    ("encode_4", "conv_s2", 64, 64, "identity"),
]
_M2_DEC = [
    ("decode_4", "convT", 64, 64, "identity"),
    ("decode_res_1", "res", 64, 64, "relu"),
    ("decode_res_2", "res", 64, 64, "relu"),
    ("decode_3", "convT", 64, 64, "relu"),
    ("decode_2", "convT", 64, 32, "relu"),
    ("decode_1", "convT", 32, 3, "identity"),
]
# model_3/model.py:50-161 (encoder), :157-300 (decoder)
_M3_ENC = [
    ("encode_1", "conv_s2", 3, 32, "relu"),
    ("encode_2", "conv_s2", 32, 64, "relu"),
    ("encode_res_m1", "res", 64, 64, "relu"),
    ("encode_res_0", "res", 64, 64, "relu"),
    ("encode_3", "conv_s2", 64, 64, "relu"),
    ("encode_res_1", "res", 64, 64, "relu"),
    ("encode_res_2", "res", 64, 64, "relu"),
    ("encode_res_3", "res", 64, 64, "relu"),
    ("encode_4", "conv_s2", 64, 80, "identity"),
]
_M3_DEC = [
    ("decode_4", "convT", 80, 64, "identity"),
    ("decode_res_1", "res", 64, 64, "relu"),
    ("decode_res_2", "res", 64, 64, "relu"),
    ("decode_res_3", "res", 64, 64, "relu"),
    ("decode_3", "convT", 64, 64, "relu"),
    ("decode_res_4", "res", 64, 64, "relu"),
    ("decode_res_5", "res", 64, 64, "relu"),
    ("decode_2", "convT", 64, 32, "relu"),
    ("decode_1", "convT", 32, 3, "identity"),
]
# base_model/ch_128/model.py:50-110 (encoder), :135-200 (decoder): the 128-channel trunk
_CH128_ENC = [
    ("encode_1", "conv_s2", 3, 64, "relu"),
    ("encode_2", "conv_s2", 64, 128, "relu"),
    ("encode_res_1", "res", 128, 128, "relu"),
    ("encode_res_2", "res", 128, 128, "relu"),
    ("encode_3", "conv_s1", 128, 64, "identity"),
]
_CH128_DEC = [
    ("decode_3", "conv_s1", 64, 128, "identity"),
    ("decode_res_1", "res", 128, 128, "relu"),
    ("decode_res_2", "res", 128, 128, "relu"),
    ("decode_2", "convT", 128, 64, "relu"),
    ("decode_1", "convT", 64, 3, "identity"),
]
# submit/2/rmbe/model.py:118-189 (block-effect post-filter)
RMBE = [
    ("conv_1", "conv_s2", 3, 32, "relu"),
    ("conv_2", "conv_s2", 32, 64, "relu"),
    ("conv_3", "conv_s1", 64, 64, "relu"),
    ("conv_4", "conv_s1", 64, 64, "relu"),
    ("conv_5", "convT", 64, 32, "relu"),
    ("conv6", "convT", 32, 3, "identity"),
]

MODELS = {
    0: (_M0_ENC, _M0_DEC),
    1: (_M1_ENC, _M1_DEC),
    2: (_M2_ENC, _M2_DEC),
    3: (_M3_ENC, _M3_DEC),
    128: (_CH128_ENC, _CH128_DEC),  # base_model/ch_128
}

# model_N/config.json (patch_size, quan_scale); model_2/3 use 128 (model_3/config.json:5)
DEFAULT_PATCH = {0: 256, 1: 256, 2: 128, 3: 128}


def expand(layers):
    """Expand res blocks into their two convs (basic_block.py:78-89: scopes conv_0, conv_1)."""
    out = []
    for name, kind, cin, cout, act in layers:
        if kind == "res":
            out.append((f"{name}/conv_0", "conv_s1", cin, cout, "relu"))
            out.append((f"{name}/conv_1", "conv_s1", cout, cout, "relu"))
        else:
            out.append((name, kind, cin, cout, act))
    return out


def param_shapes(layers):
    """TF variable names/shapes: '<scope>/kernel' HWIO (conv) or [3,3,Cout,Cin] (convT), '<scope>/bias'."""
    shapes = {}
    for name, kind, cin, cout, _ in expand(layers):
        shapes[f"{name}/kernel"] = (3, 3, cout, cin) if kind == "convT" else (3, 3, cin, cout)
        shapes[f"{name}/bias"] = (cout,)
    return shapes


# ---------------------------------------------------------------------------
# Primitive ops
# ---------------------------------------------------------------------------

def tf_same_pads(in_size: int, stride: int, k: int = 3):
    """TF 'SAME': out = ceil(in/s); pad_total = max((out-1)s + k - in, 0); before = total//2."""
    out = -(-in_size // stride)
    total = max((out - 1) * stride + k - in_size, 0)
    return out, total // 2, total - total // 2


def conv2d_same(x, kernel, stride, acc=np.float64):
    """tf.nn.conv2d(x, W[3,3,Cin,Cout], strides=[1,s,s,1], 'SAME') (basic_block.py:33).

    Returns the raw convolution (before bias) rounded once to float32."""
    n, h, w, c = x.shape
    ho, pt, pb = tf_same_pads(h, stride)
    wo, pl, pr = tf_same_pads(w, stride)
    xp = np.pad(np.asarray(x, acc), ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    s0, s1, s2, s3 = xp.strides
    cols = np.lib.stride_tricks.as_strided(
        xp, shape=(n, ho, wo, 3, 3, c), strides=(s0, s1 * stride, s2 * stride, s1, s2, s3))
    out = cols.reshape(n * ho * wo, 9 * c) @ np.asarray(kernel, acc).reshape(9 * c, -1)
    return out.reshape(n, ho, wo, -1).astype(F32)


# phase -> [(kernel tap, input offset)] for the stride-2 SAME transpose with pad_before = 0
_T_TAPS = {0: ((0, 0), (2, -1)), 1: ((1, 0),)}


def conv2d_transpose_x2(x, kernel, acc=np.float64):
    """tf.nn.conv2d_transpose(x, W[3,3,Cout,Cin], [N,2H,2W,Cout], stride 2, 'SAME')
    (basic_block.py:53-57): y[2m+py] = sum_{(k,d) in taps(py)} x[m+d] W[k]; result rounded to f32."""
    n, h, w, c = x.shape
    co = kernel.shape[2]
    k = np.asarray(kernel, acc)
    xp = np.pad(np.asarray(x, acc), ((0, 0), (1, 0), (1, 0), (0, 0)))
    y = np.empty((n, 2 * h, 2 * w, co), F32)
    for py in (0, 1):
        for px in (0, 1):
            s = np.zeros((n * h * w, co), acc)
            for ky, dy in _T_TAPS[py]:
                for kx, dx in _T_TAPS[px]:
                    xs = xp[:, 1 + dy:1 + dy + h, 1 + dx:1 + dx + w, :].reshape(-1, c)
                    s += xs @ k[ky, kx].T
            y[:, py::2, px::2, :] = s.reshape(n, h, w, co).astype(F32)
    return y


def _act(y, act):
    return np.maximum(y, F32(0)) if act == "relu" else y


def my_conv2d(x, params, name, stride, act, acc=np.float64):
    """basic_block.my_conv2d (basic_block.py:27-47): conv -> bias_add (f32) -> act."""
    y = conv2d_same(x, params[f"{name}/kernel"], stride, acc)
    y = y + np.asarray(params[f"{name}/bias"], F32)
    return _act(y, act)


def my_conv2d_transpose(x, params, name, act, acc=np.float64):
    """basic_block.my_conv2d_transpose (basic_block.py:50-71)."""
    y = conv2d_transpose_x2(x, params[f"{name}/kernel"], acc)
    y = y + np.asarray(params[f"{name}/bias"], F32)
    return _act(y, act)


def res_block(x, params, name, acc=np.float64):
    """basic_block.res_block (basic_block.py:74-93), layer_num=2, relu, no act after add."""
    y = my_conv2d(x, params, f"{name}/conv_0", 1, "relu", acc)
    y = my_conv2d(y, params, f"{name}/conv_1", 1, "relu", acc)
    return x + y


def run_layers(x, params, layers, acc=np.float64, trace=None):
    for name, kind, cin, cout, act in layers:
        if kind == "res":
            x = res_block(x, params, name, acc)
        elif kind == "conv_s2":
            x = my_conv2d(x, params, name, 2, act, acc)
        elif kind == "conv_s1":
            x = my_conv2d(x, params, name, 1, act, acc)
        elif kind == "convT":
            x = my_conv2d_transpose(x, params, name, act, acc)
        else:
            raise ValueError(kind)
        if trace is not None:
            trace[name] = x
    return x


def normalize(patches, mean, std, patch_size):
    """model_0/model.py:38-46: reshape [-1,P,P,3]; (x - mean) / std in float32."""
    x = np.asarray(patches, F32).reshape(-1, patch_size, patch_size, 3)
    return (x - np.asarray(mean, F32)) / np.asarray(std, F32)


def quantize(preact, quan_scale):
    """model_0/model.py:136-138: round(sigmoid(x) * (Q-1)), tf.round = half-to-even.
    Evaluated in float64; ties are excluded by the decision-margin band in tests."""
    s = 1.0 / (1.0 + np.exp(-np.asarray(preact, np.float64))) * (quan_scale - 1)
    return np.rint(s).astype(np.uint8)


def decision_margin(preact, quan_scale):
    """Distance of each pre-activation to the nearest quantiser decision threshold
    x_k = logit((k + 0.5) / (Q-1)); for Q=2 that is |x|."""
    x = np.asarray(preact, np.float64)
    q1 = quan_scale - 1
    th = np.array([np.log((k + 0.5) / (q1 - k - 0.5)) for k in range(q1)], np.float64)
    return np.min(np.abs(x[..., None] - th), axis=-1)


def dequant_lut(quan_scale):
    """reverse_sigmoid((q + 1e-6) / (Q - 1 + 1e-5)) in float32 (model_0/model.py:153,
    basic_block.py:152-155).  Q=2 -> [-13.815519, 11.611643]."""
    q = np.arange(quan_scale, dtype=F32)
    a = (q + F32(1e-6)) / F32(quan_scale - 1 + 1e-5)
    return np.log(a / (F32(1) - a)).astype(F32)


def denormalize(y, mean, std):
    """model_0/model.py:250-259: y*std + mean (two f32 ops), clip [0,255]."""
    out = (np.asarray(y, F32) * np.asarray(std, F32)) + np.asarray(mean, F32)
    return np.clip(out, F32(0), F32(255)).astype(F32)


def around_u8(y):
    """decode.py:249: np.around (half-to-even) -> uint8."""
    return np.around(y).astype(np.uint8)


# ---------------------------------------------------------------------------
# Model-level entry points (mirror model_N.encoder / model_N.decoder)
# ---------------------------------------------------------------------------

def encoder(params, mean, std, patches, patch_size, quan_scale, model_id, acc=np.float64, trace=None):
    """model_N.encoder(input, patch_size, quan_scale) -> (preact f32 [N,h,w,C], idx u8)."""
    enc, _ = MODELS[model_id]
    x = normalize(patches, mean, std, patch_size)
    pre = run_layers(x, params, enc, acc, trace)
    return pre, quantize(pre, quan_scale)


def decoder(params, mean, std, idx, quan_scale, model_id, acc=np.float64, trace=None):
    """model_N.decoder(input, quan_scale) -> (f32 recon in [0,255], uint8 via np.around)."""
    _, dec = MODELS[model_id]
    x = dequant_lut(quan_scale)[np.asarray(idx, np.int64)]
    y = run_layers(x, params, dec, acc, trace)
    f = denormalize(y, mean, std)
    return f, around_u8(f)


def rmbe_model(params, mean, std, patches_f32, acc=np.float64):
    """submit/2/rmbe/model.py:113-197: normalise -> 6 layers -> denorm + clip (float out)."""
    x = normalize(patches_f32, mean, std, patches_f32.shape[1])
    y = run_layers(x, params, RMBE, acc)
    return denormalize(y, mean, std)


RMBE_PATCH, RMBE_OFFSET = 128, 64  # submit/2/rmbe/rmbe.py:12,16


def rmbe(image, params, mean, std, acc=np.float64):
    """submit/2/rmbe/rmbe.py:15-111: filter 128^2 windows at column offset 64 (all rows),
    write back, then at row offset 64 (all columns); partial edge windows untouched."""
    img = np.array(image, F32, copy=True)
    h, w, _ = img.shape
    P, o = RMBE_PATCH, RMBE_OFFSET
    # rmbe_height (:70-89)
    hn, wn = h // P, (w - o) // P
    if hn > 0 and wn > 0:
        wins = [img[i * P:(i + 1) * P, o + j * P:o + (j + 1) * P] for i in range(hn) for j in range(wn)]
        out = rmbe_model(params, mean, std, np.stack(wins), acc)
        for i in range(hn):
            for j in range(wn):
                img[i * P:(i + 1) * P, o + j * P:o + (j + 1) * P] = out[i * wn + j]
    # rmbe_width (:92-111)
    hn, wn = (h - o) // P, w // P
    if hn > 0 and wn > 0:
        wins = [img[o + i * P:o + (i + 1) * P, j * P:(j + 1) * P] for i in range(hn) for j in range(wn)]
        out = rmbe_model(params, mean, std, np.stack(wins), acc)
        for i in range(hn):
            for j in range(wn):
                img[o + i * P:o + (i + 1) * P, j * P:(j + 1) * P] = out[i * wn + j]
    return img


# ---------------------------------------------------------------------------
# Host-side tiling + metrics
# ---------------------------------------------------------------------------

def crop_image_input_patches(image, patch_size):
    """utils/utils.py:96-133: reflect-pad bottom/right to a multiple of P, row-major patches."""
    h, w, _ = image.shape
    ph = (patch_size - h % patch_size) % patch_size
    pw = (patch_size - w % patch_size) % patch_size
    padded = np.pad(image, ((0, ph), (0, pw), (0, 0)), "reflect")
    H, W, _ = padded.shape
    return [padded[i * patch_size:(i + 1) * patch_size, j * patch_size:(j + 1) * patch_size]
            for i in range(H // patch_size) for j in range(W // patch_size)]


def concat_patches(patches, height, width, patch_size):
    """utils/utils.py:136-167: stitch row-major patches, crop to (height, width)."""
    hn = -(-height // patch_size)
    wn = -(-width // patch_size)
    rows = [np.concatenate(list(patches[i * wn:(i + 1) * wn]), axis=1) for i in range(hn)]
    return np.concatenate(rows, axis=0)[:height, :width]


def dataset_psnr(pairs):
    """processing_utils/evaluate.py:10-32: 20log10(255) - 10log10(sum SSE / sum dims)."""
    sse, dims = 0.0, 0
    for a, b in pairs:
        a = np.asarray(a, np.float32)
        b = np.asarray(b, np.float32)
        sse += float(np.sum(np.square(b - a), dtype=np.float64))
        dims += a.size
    if sse == 0:
        return float("inf")
    return 20.0 * np.log10(255.0) - 10.0 * np.log10(sse / dims)
