"""The product default IS the benchmarked configuration.

A ``Codec`` made the way the reference's callers make it — through the drop-in module
``model_N.model`` (model_0/model.py:34,147) as encode.py:225-232 / decode.py:280-287 load
it, or directly — applies the shipped tuning database (tf_image_compression_amd/tune/),
so it launches exactly the kernel sequence bench.py times: enc01_kernel, the tuned
per-layer tilings, wino_chain_kernel (model_0) and dec10_kernel.  These tests run THAT
sequence (batch 64 = the tuned per-lane batch of 32 on two lanes; model_3 batch 256 = 128
per lane) against the oracle and the committed golden fixture, and bit for bit against the
unfused, heuristically tiled path.  Plus the lane-ordering contract of successive device
calls with different batch splits.
Bars: tests/gpu_checks.py."""
import importlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, structured_patches
from gpu_checks import check_codec_subset
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu


def _kernels_of(codec, n):
    return " ".join(codec.layer_kernels(n))


def _plain_codec(model_id, params, P):
    """The same weights with no tuning and every fusion off: conv3x3 / Winograd launches
    per layer with the heuristic tilings (the round-1 path)."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import SYNTH_MEAN, SYNTH_STD
    c = Codec(model_id, params, SYNTH_MEAN, SYNTH_STD, patch_size=P, tuning="none")
    for k in ("fuse01", "fuse_tail", "chain"):
        c.set_option(k, 0)
    return c


@pytest.fixture
def m0_module():
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    mod = importlib.import_module("tf_image_compression_amd.model_0.model")
    params = synthetic_params(0, seed=0)
    mod.restore(params, SYNTH_MEAN, SYNTH_STD)
    yield mod, params
    mod.restore(params, SYNTH_MEAN, SYNTH_STD)  # releases the handles


def test_module_codec_runs_the_benchmarked_kernels(m0_module):
    """model_0.model's codec at the config's P = 256 applies the shipped tuning: the fused
    head, the two chains and the fused tail, with the tuned tilings of the other layers."""
    mod, _ = m0_module
    c = mod.codec(256, 2)
    assert c.tuning_source.startswith("shipped tuning:"), c.tuning_source
    k = _kernels_of(c, 32)
    assert "enc01_kernel" in k and "dec10_kernel" in k and k.count("wino_chain_kernel") == 2, k
    exported = c.tuning_export()
    from tf_image_compression_amd import tuning
    shipped = tuning.entries(0, 256, 2)[0][2]["tuning"]
    assert sorted(exported.splitlines()) == sorted(shipped.splitlines())


def test_encode_py_load_model_runs_the_benchmarked_kernels(tmp_path):
    """encode.py's own load_model (the CLI path) ends on the same tuned launch sequence."""
    import encode
    args = encode.my_parse_args(["-m", "0", "-g", "0", "--synthetic-weights", "--norm", "/nonexistent",
                                 "-o", str(tmp_path)])
    cfg = encode.load_config("0")
    model = encode.load_model(args, cfg)
    try:
        c = model.codec(cfg["patch_size"], cfg["quan_scale"])
        k = _kernels_of(c, 32)
        assert "enc01_kernel" in k and "dec10_kernel" in k and "wino_chain_kernel" in k, k
    finally:
        model._module.close()


def test_tuned_model0_p256_batch64_vs_oracle_and_plain(m0_module):
    """configs[1] exactly as timed (batch 64, two lanes of 32, shipped tuning): oracle on
    four patches, and every symbol / byte of all 64 equal to the unfused default path."""
    mod, params = m0_module
    c = mod.codec(256, 2)
    x = np.concatenate([structured_patches(4, 256, seed=1101),
                        np.random.default_rng(1102).integers(0, 256, (60, 256, 256, 3), dtype=np.uint8)])
    idx, rgb = check_codec_subset(c, params, 0, 256, x, k=4)
    plain = _plain_codec(0, params, 256)
    try:
        assert "enc01" not in _kernels_of(plain, 32) and "wino_chain" not in _kernels_of(plain, 32)
        assert np.array_equal(plain.encode(x), idx)
        assert np.array_equal(plain.decode(idx), rgb)
    finally:
        plain.close()


def test_tuned_model0_p256_vs_golden_fixture(m0_module):
    """The committed golden patch (tests/golden/model0_p256.npz) as patch 0 of a batch of 64
    on the tuned sequence: pre-activations, symbols and bytes at the fixture's bars."""
    mod, _ = m0_module
    z = np.load(os.path.join(GOLDEN, "model0_p256.npz"), allow_pickle=False)
    c = mod.codec(256, 2)
    x = np.concatenate([z["patches"], structured_patches(63, 256, seed=1103)])
    idx, pre = c.encode(x, return_preact=True)
    ref = z["preact"]
    scale = max(1.0, float(np.abs(ref).max()))
    assert float(np.abs(pre[:1] - ref).max()) <= 1e-4 * scale
    safe = o.decision_margin(ref, 2) > 1e-5 * scale
    assert int(np.count_nonzero((idx[:1] != z["idx"]) & safe)) == 0
    sym = idx.copy()
    sym[:1] = z["idx"]  # the fixture's reconstruction is of its own symbols
    rgb = c.decode(sym)
    du = np.abs(rgb[:1].astype(np.int16) - z["recon_u8"].astype(np.int16))
    assert int(du.max()) <= 1 and float(np.mean(du > 0)) < 1e-3


def test_tuned_model3_p256_batch256_vs_oracle_and_plain():
    """configs[2] exactly as timed (model_3, P = 256, batch 256 = two lanes of 128, shipped
    tuning): oracle on two patches, all 256 equal to the unfused default path."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(3, seed=0)
    with Codec(3, params, SYNTH_MEAN, SYNTH_STD, patch_size=256) as c:
        assert c.tuning_source.startswith("shipped tuning:"), c.tuning_source
        k = _kernels_of(c, 128)
        assert "enc01_kernel" in k and "dec10_kernel" in k, k
        x = np.concatenate([structured_patches(2, 256, seed=1111),
                            np.random.default_rng(1112).integers(0, 256, (254, 256, 256, 3), dtype=np.uint8)])
        idx, rgb = check_codec_subset(c, params, 3, 256, x, k=2)
    plain = _plain_codec(3, params, 256)
    try:
        assert np.array_equal(plain.encode(x), idx)
        assert np.array_equal(plain.decode(idx), rgb)
    finally:
        plain.close()


class _View:
    """A device pointer into a DeviceBuffer at a byte offset (what a C caller passes)."""

    def __init__(self, buf, offset):
        import ctypes as C
        self.ptr = C.c_void_p(buf.ptr.value + int(offset))


@pytest.mark.parametrize("decouple", [1, 0])
def test_device_calls_with_different_splits_are_ordered(decouple):
    """encode_device(n = 100) then decode_device of 50 + 50 patches on the
    same symbol buffer — the lanes split the calls differently (lane 1 of the first decode
    reads symbols lane 0 of the encode wrote), and an offset view makes the second decode's
    lanes read the other half; results must equal the host path's, every round."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P, n = 128, 100
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        c.set_option("decouple", decouple)
        x = structured_patches(n, P, seed=1201)
        ref_idx = c.encode(x)
        ref_rgb = c.decode(ref_idx)
        eh, ew, ec = c.code_shape
        ce, pp = eh * ew * ec, P * P * 3
        d_in, d_idx, d_rgb = c.alloc(x.nbytes), c.alloc(n * ce), c.alloc(x.nbytes)
        d_in.upload(x)
        for r in range(3):
            c.memset_device(d_idx, 0xFF, n * ce)
            c.memset_device(d_rgb, 0, x.nbytes)
            c.synchronize()
            c.encode_device(d_in, n, d_idx)
            c.decode_device(d_idx, 50, d_rgb)
            c.decode_device(_View(d_idx, 50 * ce), 50, _View(d_rgb, 50 * pp))
            c.encode_device(d_in, 60, d_idx)  # rewrites 0..60 with the same symbols (WAW)
            c.synchronize()
            assert np.array_equal(d_idx.download(ref_idx.shape, np.uint8), ref_idx), r
            assert np.array_equal(d_rgb.download(x.shape, np.uint8), ref_rgb), r


def test_chain_declined_where_geometry_cannot_run():
    """a chain whose regions cannot all be resident (rw + 2 per lane
    beyond the CU slots) or whose hand-off offsets would overflow 32 bits falls back to the
    per-layer launches: model_0 at P = 8192 (16x16-region rows of 64 per 512x512 stage)
    needs 2 x (2 x 64 + 2) slots > 256."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=8192, tuning="none") as c:
        assert "wino_chain_kernel" not in _kernels_of(c, 1)
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=256, tuning="none") as c:
        assert "wino_chain_kernel" in _kernels_of(c, 32)
        c.set_option("chunk", 100_000)  # n * R * 8 KB > 2^31 - 1 for the largest launch
        assert "wino_chain_kernel" not in _kernels_of(c, 32)


def test_chain_shortened_where_a_long_run_cannot_be_resident():
    """a region keeps its workgroup for all nl layers and publishing
    layer k of region t waits on region t + rw + 1 (and so on), so min(R, (nl - 1)(rw + 1) + 1)
    workgroups of a patch must be resident in every lane.  model_0 at P = 4096 (a 256x256
    stage, rw = 32) fits two-layer runs (2 lanes x 34 regions) but not the 5-layer ones the
    old rw + 2 guard accepted (2 x 133 > 256 slots): every chain launch covers at most two
    layers, and the shortened chains run to the unfused launches' exact results."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P = 4096
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P, tuning="none") as c:
        c.set_option("s1_form", 1)
        c.set_option("chain", 1)
        # at most 8 patches per launch: the default chunk (256) of 4096x4096 patches would put
        # the hand-off buffer's byte offsets past 2^31 and decline every chain (the other guard)
        c.set_option("chunk", 8)
        kern = c.layer_kernels(1)
        starts = [i for i, k in enumerate(kern) if k.startswith("wino_chain_kernel")]
        assert starts, kern
        for i in starts:  # a run = the chain launch + the '' entries of the layers inside it
            j = i + 1
            while j < len(kern) and kern[j] == "":
                j += 1
            assert j - i <= 2, (i, kern)
        x = np.random.default_rng(4096).integers(0, 256, (1, P, P, 3), dtype=np.uint8)
        idx, pre = c.encode(x, return_preact=True)
        rgb = c.decode(idx)
        c.set_option("chain", 0)
        idx0, pre0 = c.encode(x, return_preact=True)
        rgb0 = c.decode(idx0)
        assert np.array_equal(pre, pre0) and np.array_equal(idx, idx0) and np.array_equal(rgb, rgb0)
        c.set_option("chain", -1)
        c.set_option("s1_form", -1)
