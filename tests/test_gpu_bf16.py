"""The bf16x6 form of the stride-2 / transposed convolutions (csrc/conv3x3_bf.h, option
"mma" = 1): f32 operands split exactly into three bf16 parts, the six leading part products
summed in f32 on the bf16 matrix path.  Bars: every layer within the f32 form's per-layer bar
(3e-5 of the output scale) against the f64 oracle, with an error of the same size as the f32
MFMA form's on the same inputs (the error ratio is asserted, so a reduced-precision product
would fail here); every tiling of the form bit-identical; end to end the codec bars of
DESIGN.md §4 (tests/gpu_checks.py).  Reference layers: basic_block/basic_block.py:27-71
(my_conv2d stride 2, my_conv2d_transpose), model_0/model.py:62-96,198-234,
model_3/model.py:62-161,157-286."""
import os

import numpy as np
import pytest

from conftest import structured_patches
from gpu_checks import check_codec
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu

K_S1, K_S2, K_T2 = 0, 1, 2

# (kind, cin, cout, act, in/out size) of the compiled bf16x6 signatures (f32 in / out)
BF_LAYERS = [
    (K_S2, 32, 64, 1, 32, 32),
    (K_S2, 32, 64, 1, 30, 22),
    (K_S2, 64, 64, 1, 17, 15),
    (K_S2, 64, 64, 1, 32, 32),
    (K_T2, 64, 64, 1, 16, 16),
    (K_T2, 64, 64, 1, 9, 13),
    (K_T2, 64, 32, 1, 32, 32),
    (K_T2, 64, 32, 1, 5, 21),
]
BF_TILES = [(2, 1), (2, 2), (4, 1), (4, 2)]


@pytest.fixture(scope="module")
def codec64():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    c = Codec(0, synthetic_params(0, seed=0), SYNTH_MEAN, SYNTH_STD, patch_size=64)
    yield c
    c.close()


def _run_layer(codec, kind, act, x, k, b, tile):
    from tf_image_compression_amd._lib import TicError
    n, H, W, cin = x.shape
    cout = b.shape[0]
    Ho = 2 * H if kind == K_T2 else (H + 1) // 2
    Wo = 2 * W if kind == K_T2 else (W + 1) // 2
    d_in = codec.alloc(x.nbytes)
    d_in.upload(x)
    d_out = codec.alloc(n * Ho * Wo * cout * 4)
    try:
        os.environ["TIC_FORCE_TILE"] = f"{tile[0]},{tile[1]},{tile[2]}"
        try:
            codec.conv3x3_device(kind, act, d_in, n, H, W, cin, cout, k, b, None, d_out)
        except TicError as e:
            assert "no compiled" in str(e)
            return None
        return d_out.download((n, Ho, Wo, cout), np.float32)
    finally:
        os.environ.pop("TIC_FORCE_TILE", None)
        d_in.free()
        d_out.free()


@pytest.mark.parametrize("kind,cin,cout,act,H,W", BF_LAYERS)
def test_bf16x6_layer(codec64, kind, cin, cout, act, H, W):
    r = np.random.default_rng(np.random.PCG64(7000 + kind * 100 + cin + cout + H))
    n = 2
    x = r.standard_normal((n, H, W, cin)).astype(np.float32)
    kshape = (3, 3, cout, cin) if kind == K_T2 else (3, 3, cin, cout)
    k = (r.standard_normal(kshape) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    b = (r.standard_normal(cout) * 0.1).astype(np.float32)
    params = {"l/kernel": k, "l/bias": b}
    a = "relu" if act else "identity"
    ref = o.my_conv2d_transpose(x, params, "l", a) if kind == K_T2 else o.my_conv2d(x, params, "l", 2, a)
    scale = max(1.0, float(np.max(np.abs(ref))))
    f32 = _run_layer(codec64, kind, act, x, k, b, (4, 1, 0))
    assert f32 is not None
    err_f32 = float(np.max(np.abs(f32 - ref)))
    outs = []
    for th, ns in BF_TILES:
        got = _run_layer(codec64, kind, act, x, k, b, (th, ns, 6))
        if got is not None:
            outs.append(((th, ns), got))
    assert outs, "no bf16x6 tiling compiled for this layer"
    for tile, got in outs:
        err = float(np.max(np.abs(got - ref)))
        assert err <= 3e-5 * scale, (tile, err, scale)
        # an f32-accurate form: the same error class as the f32 MFMA form (a product kept to
        # bf16 or to 16 bits would be ~100x / ~10x above it)
        assert err <= 4.0 * max(err_f32, 1e-7 * scale), (tile, err, err_f32)
        assert np.array_equal(got, outs[0][1]), tile


@pytest.mark.parametrize("model_id,P", [(0, 64), (0, 256), (3, 64), (2, 128)])
def test_bf16x6_codec_parity(model_id, P):
    """The whole codec with its stride-2 / transposed layers in the bf16x6 form (option
    mma = 1; the quantiser and dequantiser layers included where compiled) meets the
    end-to-end bars, and its symbols / bytes equal the f32 form's except inside the tie band."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(model_id, seed=0)
    patches = structured_patches(3, P, seed=900 + model_id + P)
    with Codec(model_id, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, tuning="none") as c:
        c.set_option("mma", 1)
        kern = c.layer_kernels(3)
        assert any(k.startswith("conv3x3_bf_kernel<") for k in kern), kern
        check_codec(c, params, model_id, P, patches)
        c.set_option("mma", 0)
        assert not any(k.startswith("conv3x3_bf_kernel<") for k in c.layer_kernels(3))
        check_codec(c, params, model_id, P, patches)


def test_bf16x6_tuning_flag_roundtrip():
    """flag mma travels with the tuning text; the tuned per-layer choices are keyed by form,
    so an f32-form choice never runs a bf16x6 layer or the reverse."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(0, seed=0)
    x = structured_patches(4, 64, seed=910)
    with Codec(0, params, SYNTH_MEAN, SYNTH_STD, patch_size=64, tuning="none") as c:
        c.set_option("mma", 1)
        d_in = c.alloc(x.nbytes)
        d_in.upload(x)
        c.autotune(d_in, 2, reps=1)
        text = c.tuning_export()
        assert "flag mma 1" in text
        ref = c.encode(x)
        with Codec(0, params, SYNTH_MEAN, SYNTH_STD, patch_size=64, tuning="none") as c2:
            c2.tuning_import(text)
            assert c2.tuning_export() == text
            assert c2.layer_kernels(2) == c.layer_kernels(2)
            assert np.array_equal(c2.encode(x), ref)
