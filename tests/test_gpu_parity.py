"""GPU parity: libtic (gfx950 HIP) vs the CPU oracle on identical inputs and weights.

Bars:
* per layer: max |gpu - oracle| <= 3e-5 * max(1, max|oracle|) (fp32 MFMA vs f64-accumulated);
* quantised symbols: bit-exact wherever the oracle's pre-activation is farther than
  1e-5 * max|preact| from a quantiser decision threshold (SURVEY §7 "hard parts" 1);
* reconstruction (decoder fed the SAME symbols): float max |diff| <= 1e-2 on the [0,255]
  scale (4e-5 of full scale; model_3's 28 layers of fp32 reach ~3e-3), uint8 differs by at most 1 and only where the float sits on a .5 rounding edge,
  dataset-PSNR difference <= 0.02 dB (north_star tolerance).
"""
import numpy as np
import pytest

from conftest import structured_patches
from gpu_checks import check_codec as _check_codec, codec_mean, codec_std  # noqa: F401
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu

K_S1, K_S2, K_T2 = 0, 1, 2


@pytest.fixture(scope="module")
def lib_codec():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    cache = {}

    def get(model_id, P, Q=2):
        key = (model_id, P, Q)
        if key not in cache:
            params = synthetic_params(model_id, seed=0)
            cache[key] = (Codec(model_id, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, quan_scale=Q), params)
        return cache[key]

    yield get
    for c, _ in cache.values():
        c.close()


TILES = [(th, ns, wl) for th, ns in [(4, 1), (4, 2), (8, 1), (2, 1), (2, 2), (4, 4), (1, 1)] for wl in (0, 1, 2)]

LAYER_CASES = [
    (K_S1, 64, 64, 1, False, 16, 16),
    (K_S1, 64, 64, 1, True, 20, 13),
    (K_S1, 64, 64, 0, False, 33, 17),
    (K_S2, 16, 32, 1, False, 64, 64),
    (K_S2, 32, 32, 1, False, 30, 22),
    (K_S2, 32, 64, 1, False, 32, 32),
    (K_S2, 64, 64, 1, False, 17, 15),
    (K_T2, 64, 64, 1, False, 16, 16),
    (K_T2, 64, 32, 1, False, 9, 13),
    (K_T2, 32, 32, 1, False, 32, 32),
    (K_T2, 32, 16, 1, False, 8, 8),
    (K_T2, 64, 64, 0, False, 5, 21),
]


@pytest.mark.parametrize("kind,cin,cout,act,res,H,W", LAYER_CASES)
def test_conv3x3_layer(lib_codec, kind, cin, cout, act, res, H, W):
    codec, _ = lib_codec(0, 64)
    r = np.random.default_rng(np.random.PCG64(kind * 1000 + cin + cout + H))
    n = 2
    x = r.standard_normal((n, H, W, cin)).astype(np.float32)
    kshape = (3, 3, cout, cin) if kind == K_T2 else (3, 3, cin, cout)
    k = (r.standard_normal(kshape) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    b = (r.standard_normal(cout) * 0.1).astype(np.float32)
    params = {"l/kernel": k, "l/bias": b}
    a = "relu" if act else "identity"
    if kind == K_T2:
        ref = o.my_conv2d_transpose(x, params, "l", a)
    else:
        ref = o.my_conv2d(x, params, "l", 1 if kind == K_S1 else 2, a)
    resid = r.standard_normal(ref.shape).astype(np.float32) if res else None
    if res:
        ref = ref + resid
    d_in = codec.alloc(x.nbytes)
    d_in.upload(x)
    d_out = codec.alloc(ref.nbytes)
    d_res = None
    if res:
        d_res = codec.alloc(resid.nbytes)
        d_res.upload(resid)
    import os
    from tf_image_compression_amd._lib import TicError
    outs = []
    try:
        for th, ns, wl in TILES:
            os.environ["TIC_FORCE_TILE"] = f"{th},{ns},{wl}"
            try:
                codec.conv3x3_device(kind, act, d_in, n, H, W, cin, cout, k, b, d_res, d_out)
            except TicError as e:
                assert "no compiled" in str(e)
                continue
            outs.append(((th, ns, wl), d_out.download(ref.shape, np.float32)))
    finally:
        os.environ.pop("TIC_FORCE_TILE", None)
    for buf in (d_in, d_out, d_res):
        if buf is not None:
            buf.free()
    assert outs, "no compiled tiling for this layer"
    scale = max(1.0, float(np.max(np.abs(ref))))
    for tile, got in outs:
        err = float(np.max(np.abs(got - ref)))
        assert err <= 3e-5 * scale, (tile, err, scale)
        # every tiling runs the same per-output fma order: results are bit-identical
        assert np.array_equal(got, outs[0][1]), tile


# Winograd F(2x2,3x3) tilings of the stride-1 layers: (th = 2 TTY, nsplit, NN)
WINO_TILES = [(2, 1, 1), (4, 1, 1), (4, 2, 1), (4, 4, 1), (2, 4, 1), (4, 1, 2), (8, 1, 2)]


@pytest.mark.parametrize("act,res,H,W", [(1, False, 16, 16), (1, True, 20, 13), (0, False, 33, 17),
                                         (1, True, 64, 64), (1, False, 7, 40)])
def test_conv3x3_winograd(lib_codec, act, res, H, W):
    """Winograd form of the stride-1 layers: within the per-layer bar of the oracle (same
    3e-5 relative bound as the direct form), every Winograd tiling bit-identical to every
    other, partial tiles at odd sizes included."""
    import os
    codec, _ = lib_codec(0, 64)
    cin = cout = 64
    r = np.random.default_rng(np.random.PCG64(777 + H * 100 + W))
    n = 2
    x = r.standard_normal((n, H, W, cin)).astype(np.float32)
    k = (r.standard_normal((3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    b = (r.standard_normal(cout) * 0.1).astype(np.float32)
    ref = o.my_conv2d(x, {"l/kernel": k, "l/bias": b}, "l", 1, "relu" if act else "identity")
    resid = r.standard_normal(ref.shape).astype(np.float32) if res else None
    if res:
        ref = ref + resid
    d_in, d_out = codec.alloc(x.nbytes), codec.alloc(ref.nbytes)
    d_in.upload(x)
    d_res = None
    if res:
        d_res = codec.alloc(resid.nbytes)
        d_res.upload(resid)
    outs = []
    try:
        for th, ns, nn in WINO_TILES:
            os.environ["TIC_FORCE_TILE"] = f"{th},{ns},4,{nn}"
            d_out.upload(np.full(ref.shape, np.nan, np.float32))
            codec.conv3x3_device(0, act, d_in, n, H, W, cin, cout, k, b, d_res, d_out)
            outs.append(((th, ns, nn), d_out.download(ref.shape, np.float32)))
    finally:
        os.environ.pop("TIC_FORCE_TILE", None)
    for buf in (d_in, d_out, d_res):
        if buf is not None:
            buf.free()
    scale = max(1.0, float(np.max(np.abs(ref))))
    for tile, got in outs:
        err = float(np.max(np.abs(got - ref)))
        assert err <= 3e-5 * scale, (tile, err, scale)
        assert np.array_equal(got, outs[0][1]), tile


# Winograd F(4x4,3x3) tilings (th = 4 TTY: 4x64, 8x32, 16x16 output pixels per workgroup)
WINO4_TILES = [4, 8, 16]


@pytest.mark.parametrize("act,res,H,W", [(1, False, 16, 16), (1, True, 20, 13), (1, True, 64, 64),
                                         (1, False, 7, 40), (1, False, 33, 17), (1, True, 32, 32)])
def test_conv3x3_winograd4(lib_codec, act, res, H, W):
    """Winograd F(4x4,3x3) form (conv3x3_wino4.h): within the per-layer bar of the oracle,
    every tiling bit-identical to every other, partial tiles at odd sizes included, no
    output left unwritten."""
    import os
    codec, _ = lib_codec(0, 64)
    cin = cout = 64
    r = np.random.default_rng(np.random.PCG64(4777 + H * 100 + W))
    n = 3
    x = r.standard_normal((n, H, W, cin)).astype(np.float32)
    k = (r.standard_normal((3, 3, cin, cout)) * np.sqrt(2.0 / (9 * cin))).astype(np.float32)
    b = (r.standard_normal(cout) * 0.1).astype(np.float32)
    ref = o.my_conv2d(x, {"l/kernel": k, "l/bias": b}, "l", 1, "relu" if act else "identity")
    resid = r.standard_normal(ref.shape).astype(np.float32) if res else None
    if res:
        ref = ref + resid
    d_in, d_out = codec.alloc(x.nbytes), codec.alloc(ref.nbytes)
    d_in.upload(x)
    d_res = None
    if res:
        d_res = codec.alloc(resid.nbytes)
        d_res.upload(resid)
    outs = []
    try:
        for th in WINO4_TILES:
            os.environ["TIC_FORCE_TILE"] = f"{th},1,5,1"
            d_out.upload(np.full(ref.shape, np.nan, np.float32))
            codec.conv3x3_device(0, act, d_in, n, H, W, cin, cout, k, b, d_res, d_out)
            outs.append((th, d_out.download(ref.shape, np.float32)))
    finally:
        os.environ.pop("TIC_FORCE_TILE", None)
    for buf in (d_in, d_out, d_res):
        if buf is not None:
            buf.free()
    assert len(outs) == len(WINO4_TILES)
    scale = max(1.0, float(np.max(np.abs(ref))))
    for tile, got in outs:
        assert not np.isnan(got).any(), tile
        err = float(np.max(np.abs(got - ref)))
        assert err <= 3e-5 * scale, (tile, err, scale)
        assert np.array_equal(got, outs[0][1]), tile


@pytest.mark.parametrize("model_id,P", [(0, 64), (3, 64), (1, 32), (3, 128)])
def test_codec_s1_forms(lib_codec, model_id, P):
    """Every stride-1 form (direct, Winograd F(2x2,3x3), Winograd F(4x4,3x3) — layers with
    no F(4x4,3x3) instance fall back to F(2x2,3x3)) meets the end-to-end parity bar."""
    codec, params = lib_codec(model_id, P)
    patches = structured_patches(2, P, seed=61 + model_id)
    try:
        for form in (0, 1, 2):
            codec.set_option("s1_form", form)
            _check_codec(codec, params, model_id, P, patches)
    finally:
        codec.set_option("s1_form", -1)


@pytest.mark.parametrize("form", ["scatter", "dense"])
def test_last_layer_mfma_forms(lib_codec, monkeypatch, form):
    """The MFMA forms of the last layer (col2im, dense sub-pixel) meet the same parity bar
    as the default VALU form."""
    monkeypatch.setenv("TIC_RGB_OUT_FORM", form)
    P = 64
    codec, params = lib_codec(0, P)
    _check_codec(codec, params, 0, P, structured_patches(3, P, seed=41))


@pytest.mark.parametrize("model_id,P", [(0, 256), (3, 64), (0, 48)])
def test_last_layer_valu_tilings_bit_identical(lib_codec, monkeypatch, model_id, P):
    """Every tiling of the VALU last layer (TW 64/32/16, one-shot and persistent; the
    persistent ones also with a grid capped at 7 so each workgroup walks several tiles) gives
    identical bytes and floats, including partial edge tiles (P = 48: 24-wide decode_0
    input) and the unaligned path."""
    codec, _ = lib_codec(model_id, P)
    idx = codec.encode(structured_patches(3, P, seed=43))
    outs = []
    for t in range(6):
        monkeypatch.setenv("TIC_RGB_OUT_TILE", str(t))
        outs.append(codec.decode(idx, return_float=True))
        if t >= 3:
            codec.set_option("persist_grid", 7)
            outs.append(codec.decode(idx, return_float=True))
            codec.set_option("persist_grid", 0)
    for u8, f in outs[1:]:
        assert np.array_equal(u8, outs[0][0]) and np.array_equal(f, outs[0][1])


@pytest.mark.parametrize("model_id", [0, 1, 2, 3])
def test_codec_small_patches(lib_codec, model_id):
    P = 64
    codec, params = lib_codec(model_id, P)
    patches = structured_patches(3, P, seed=model_id)
    _check_codec(codec, params, model_id, P, patches)


def test_codec_model3_native_128(lib_codec):
    codec, params = lib_codec(3, 128)
    patches = structured_patches(2, 128, seed=7)
    _check_codec(codec, params, 3, 128, patches)


def test_codec_model0_full_size(lib_codec):
    """configs[1] geometry (256x256): oracle on 4 patches, batch invariance at n=64."""
    P = 256
    codec, params = lib_codec(0, P)
    patches = structured_patches(4, P, seed=11)
    idx4, rgb4 = _check_codec(codec, params, 0, P, patches)
    big = np.concatenate([patches, structured_patches(60, P, seed=12)])
    idx64 = codec.encode(big)
    rgb64 = codec.decode(idx64)
    assert np.array_equal(idx64[:4], idx4)
    assert np.array_equal(rgb64[:4], rgb4)
    # determinism
    assert np.array_equal(codec.encode(big), idx64)


def test_autotuned_equals_default(lib_codec):
    """Autotuning only changes tilings, never results (bit-exact)."""
    P, n = 256, 16
    codec, params = lib_codec(0, P)
    x = structured_patches(n, P, seed=31)
    ref_idx, ref_pre = codec.encode(x, return_preact=True)
    ref_rgb = codec.decode(ref_idx)
    d_in = codec.alloc(x.nbytes)
    d_in.upload(x)
    codec.autotune(d_in, n, reps=2)
    d_idx = codec.alloc(ref_idx.nbytes)
    d_pre = codec.alloc(ref_pre.nbytes)
    d_rgb = codec.alloc(x.nbytes)
    codec.encode_device(d_in, n, d_idx, d_pre)
    codec.decode_device(d_idx, n, d_rgb)
    codec.synchronize()
    assert np.array_equal(d_idx.download(ref_idx.shape, np.uint8), ref_idx)
    assert np.array_equal(d_pre.download(ref_pre.shape, np.float32), ref_pre)
    assert np.array_equal(d_rgb.download(x.shape, np.uint8), ref_rgb)
    for b in (d_in, d_idx, d_pre, d_rgb):
        b.free()


ENC01_VARIANTS = range(5)  # conv_rgb.hip enc01_variants(): TH1 2/4 padded, 2/4/8 compact


@pytest.mark.parametrize("model_id,P", [(0, 256), (0, 48), (1, 64), (3, 128), (2, 64)])
def test_fused_first_layers_bit_identical(lib_codec, monkeypatch, model_id, P):
    """enc01_kernel (layers 0+1 through LDS), every variant == the two separate kernels, bit
    for bit (P = 48: partial edge tiles)."""
    codec, params = lib_codec(model_id, P)
    x = structured_patches(5, P, seed=50 + model_id)
    try:
        codec.set_option("fuse01", 0)
        idx0, pre0 = codec.encode(x, return_preact=True)
        codec.set_option("fuse01", 1)
        for v in ENC01_VARIANTS:
            monkeypatch.setenv("TIC_ENC01_VARIANT", str(v))
            idx1, pre1 = codec.encode(x, return_preact=True)
            assert np.array_equal(pre0, pre1) and np.array_equal(idx0, idx1), v
    finally:
        codec.set_option("fuse01", -1)


def test_fused_rmbe_first_layers_bit_identical(monkeypatch):
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import RMBE_ID
    r = np.random.default_rng(4)
    win = np.clip(r.normal(120, 50, (3, 128, 128, 3)), 0, 255).astype(np.float32)
    with Codec(RMBE_ID, synthetic_params(RMBE_ID), SYNTH_MEAN, SYNTH_STD, patch_size=128) as c:
        c.set_option("fuse01", 0)
        a = c.rmbe_windows(win)
        c.set_option("fuse01", 1)
        for v in ENC01_VARIANTS:
            monkeypatch.setenv("TIC_ENC01_VARIANT", str(v))
            assert np.array_equal(a, c.rmbe_windows(win)), v


def test_quan_scale_256(lib_codec):
    """Q = 256 (base_model/1/config.json:6): multi-level quantiser + 256-entry LUT."""
    P = 64
    codec, params = lib_codec(0, P, Q=256)
    patches = structured_patches(2, P, seed=5)
    _check_codec(codec, params, 0, P, patches, Q=256)


def test_rmbe_network(lib_codec):
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import RMBE_ID
    params = synthetic_params(RMBE_ID)
    r = np.random.default_rng(3)
    win = np.clip(r.normal(120, 50, (3, 128, 128, 3)), 0, 255).astype(np.float32)
    with Codec(RMBE_ID, params, SYNTH_MEAN, SYNTH_STD, patch_size=128) as c:
        got = c.rmbe_windows(win)
    ref = o.rmbe_model(params, SYNTH_MEAN, SYNTH_STD, win)
    assert float(np.max(np.abs(got - ref))) <= 2e-3


@pytest.mark.parametrize("name", ["model0_p64.npz", "model3_p64.npz", "model1_p32.npz", "model2_p32.npz",
                                  "model0_p256.npz"])
def test_codec_vs_golden_fixture(name):
    """The HIP path against the committed fixtures (no live oracle in the loop)."""
    import os
    from conftest import GOLDEN
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params
    z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    m, P = int(z["model_id"]), int(z["patch"])
    with Codec(m, synthetic_params(m, seed=0), z["mean"], z["std"], patch_size=P) as c:
        idx, pre = c.encode(z["patches"], return_preact=True)
        rgb = c.decode(z["idx"])
    ref = z["preact"]
    scale = max(1.0, float(np.abs(ref).max()))
    assert float(np.abs(pre - ref).max()) <= 1e-4 * scale
    safe = o.decision_margin(ref, 2) > 1e-5 * scale
    assert int(np.count_nonzero((idx != z["idx"]) & safe)) == 0
    du = np.abs(rgb.astype(np.int16) - z["recon_u8"].astype(np.int16))
    assert int(du.max()) <= 1 and float(np.mean(du > 0)) < 1e-3


def test_lanes_bit_identical(lib_codec):
    """Splitting a chunk over 1..4 lanes (HIP streams) changes nothing in the results."""
    codec, _ = lib_codec(0, 64)
    x = structured_patches(7, 64, seed=71)
    outs = []
    try:
        for k in (1, 2, 3, 4):
            codec.set_option("streams", k)
            idx = codec.encode(x)
            outs.append((idx, codec.decode(idx)))
    finally:
        codec.set_option("streams", 2)
    for idx, rgb in outs[1:]:
        assert np.array_equal(idx, outs[0][0]) and np.array_equal(rgb, outs[0][1])


@pytest.mark.parametrize("model_id,P", [(0, 256), (0, 48), (1, 64), (3, 64), (2, 32)])
def test_fused_tail_bit_identical(lib_codec, monkeypatch, model_id, P):
    """dec10_kernel (decode_1 + decode_0 through LDS, halo recomputed on the VALU) == the two
    separate kernels (decode_1 by conv3x3_kernel, decode_0 in the VALU form), bit for bit,
    bytes and floats, partial edge tiles included (P = 48)."""
    codec, _ = lib_codec(model_id, P)
    idx = codec.encode(structured_patches(3, P, seed=81 + model_id))
    try:
        codec.set_option("fuse_tail", 0)
        u0, f0 = codec.decode(idx, return_float=True)
        codec.set_option("fuse_tail", 1)
        outs = []
        for v in range(16):  # conv_rgb.hip dec10_variants(): PK x PF x TA x CMP
            monkeypatch.setenv("TIC_DEC10_VARIANT", str(v))
            outs.append(codec.decode(idx, return_float=True))
    finally:
        codec.set_option("fuse_tail", -1)
    for u1, f1 in outs:
        assert np.array_equal(u0, u1) and np.array_equal(f0, f1)


def test_fused_tail_rmbe_bit_identical():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import RMBE_ID
    r = np.random.default_rng(5)
    win = np.clip(r.normal(120, 50, (3, 128, 128, 3)), 0, 255).astype(np.float32)
    with Codec(RMBE_ID, synthetic_params(RMBE_ID), SYNTH_MEAN, SYNTH_STD, patch_size=128) as c:
        c.set_option("fuse_tail", 0)
        a = c.rmbe_windows(win)
        c.set_option("fuse_tail", 1)
        b = c.rmbe_windows(win)
    assert np.array_equal(a, b)
