"""GPU coverage of the BASELINE.json configurations beyond configs[1], of the RCCL binding
and of the reference-shaped Python plugin point, all through the C-ABI:

* configs[2]: model_3 at 256x256 (patch_size overridden, bottleneck 16x16x80) against the
  oracle, and batch invariance + determinism at the configuration's batch of 256;
* configs[4]: model_3 at P = 256 + the rmbe post-filter on a whole image against the
  oracle chain crop -> encoder -> decoder -> concat -> rmbe -> np.around
  (utils/utils.py:96-167, submit/2/rmbe/rmbe.py:15-111, decode.py:249), and a
  3840x2160 property run (determinism, untouched edge strips, symbol count);
* configs[3]: sharded.run_shard at world size 1 (dataset PSNR vs the oracle on the same
  images, processing_utils/evaluate.py:18-32) and the RCCL communicator (dist.RcclComm)
  built directly at world size 1, so the ctypes signatures run before any 8-GPU job;
* the plugin point model_N.model.encoder / decoder (model_0/model.py:34,147) called the
  way encode.py:147 and decode.py:167 call it;
* HIP-graph replay after the lane workspaces were reallocated by a larger batch.
Bars: tests/gpu_checks.py."""
import importlib

import numpy as np
import pytest

from conftest import structured_patches
from gpu_checks import check_codec
from oracle import tic_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m3_256():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(3, seed=0)
    c = Codec(3, params, SYNTH_MEAN, SYNTH_STD, patch_size=256)
    yield c, params
    c.close()


@pytest.fixture(scope="module")
def rmbe_codec():
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    from tf_image_compression_amd.topology import RMBE_ID
    params = synthetic_params(RMBE_ID, seed=0)
    c = Codec(RMBE_ID, params, SYNTH_MEAN, SYNTH_STD, patch_size=128)
    yield c, params
    c.close()


def _image(H, W, seed):
    r = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    base = 128 + 60 * np.sin(xx / 17.0)[..., None] * np.cos(yy / 23.0)[..., None] + r.normal(0, 12, (H, W, 3))
    return np.clip(base, 0, 255).astype(np.uint8)


def test_codec_model3_256(m3_256):
    """configs[2] geometry: the 64x64 and 32x32 residual stages, 16x16x80 code."""
    codec, params = m3_256
    assert codec.code_shape == (16, 16, 80)
    check_codec(codec, params, 3, 256, structured_patches(2, 256, seed=301))


@pytest.mark.parametrize("form", [1, 2])
def test_codec_model3_256_s1_form(m3_256, form):
    """configs[2] geometry in each Winograd form of the residual stages (F(2x2,3x3) and
    F(4x4,3x3)) against the oracle, 4 patches."""
    codec, params = m3_256
    try:
        codec.set_option("s1_form", form)
        check_codec(codec, params, 3, 256, structured_patches(4, 256, seed=307))
    finally:
        codec.set_option("s1_form", -1)


def test_model3_256_batch_256_invariance(m3_256):
    """configs[2] batch: 256 patches in one call equal the same patches run 2 at a time
    (bit for bit, symbols and uint8), and a second run is identical (determinism)."""
    codec, _ = m3_256
    x = np.concatenate([structured_patches(2, 256, seed=302), structured_patches(254, 256, seed=303)])
    idx = codec.encode(x)
    rgb = codec.decode(idx)
    idx2 = codec.encode(x[:2])
    assert np.array_equal(idx[:2], idx2)
    assert np.array_equal(rgb[:2], codec.decode(idx2))
    assert np.array_equal(rgb[-3:], codec.decode(idx[-3:]))
    assert np.array_equal(codec.encode(x), idx)
    assert np.array_equal(codec.decode(idx), rgb)


def test_image_model3_rmbe_256(m3_256, rmbe_codec):
    """configs[4] chain on a 600x900 image (3 x 4 patches of 256, 4 + 4 rmbe windows)."""
    from tf_image_compression_amd.image_codec import ImageCodec
    from tf_image_compression_amd.weights import SYNTH_MEAN, SYNTH_STD
    c3, p3 = m3_256
    cr, pr = rmbe_codec
    H, W, P = 600, 900, 256
    img = _image(H, W, 17)
    ic = ImageCodec(c3, cr)
    try:
        sym = ic.encode_image(img)
        patches = np.stack(o.crop_image_input_patches(img, P))
        pre, ref_sym = o.encoder(p3, SYNTH_MEAN, SYNTH_STD, patches, P, 2, 3)
        scale = max(1.0, float(np.abs(pre).max()))
        safe = o.decision_margin(pre, 2) > 1e-5 * scale
        assert sym.shape == ref_sym.shape == (12, 16, 16, 80)
        assert int(np.count_nonzero((sym != ref_sym) & safe)) == 0
        rec = ic.decode_image(sym, H, W, post_filter=True)
    finally:
        ic.close()
    f, _ = o.decoder(p3, SYNTH_MEAN, SYNTH_STD, sym, 2, 3)  # decoder fed the SAME symbols
    fimg = o.rmbe(o.concat_patches(f, H, W, P), pr, SYNTH_MEAN, SYNTH_STD)
    ref = o.around_u8(fimg)
    du = np.abs(rec.astype(np.int16) - ref.astype(np.int16))
    assert int(du.max()) <= 1
    edge = np.abs(np.abs(fimg - np.floor(fimg)) - 0.5) < 1e-2
    assert not np.any((du > 0) & ~edge)
    p_gpu = o.dataset_psnr([(img, rec)])
    p_ref = o.dataset_psnr([(img, ref)])
    assert abs(p_gpu - p_ref) <= 0.02


def test_image_4k_properties(m3_256, rmbe_codec):
    """configs[4] at full size (3840x2160 -> 9 x 15 = 135 patches, 944 rmbe windows):
    symbol count, determinism, and the strips no rmbe window covers equal the unfiltered
    reconstruction (submit/2/rmbe/rmbe.py:70-111: rows >= 64 + 128 * 16 = 2112 and the
    top-left 64x64 corner)."""
    from tf_image_compression_amd.image_codec import ImageCodec
    c3, _ = m3_256
    cr, _ = rmbe_codec
    H, W = 2160, 3840
    img = np.random.default_rng(4).integers(0, 256, (H, W, 3), dtype=np.uint8)
    ic = ImageCodec(c3, cr)
    try:
        sym = ic.encode_image(img)
        assert sym.shape == (135, 16, 16, 80) and int(sym.max()) <= 1
        rec = ic.decode_image(sym, H, W, post_filter=True)
        plain = ic.decode_image(sym, H, W, post_filter=False)
        assert np.array_equal(ic.encode_image(img), sym)
        assert np.array_equal(ic.decode_image(sym, H, W, post_filter=True), rec)
    finally:
        ic.close()
    assert np.array_equal(rec[2112:], plain[2112:])
    assert np.array_equal(rec[:64, :64], plain[:64, :64])
    assert not np.array_equal(rec[:2112], plain[:2112])  # the filter did run elsewhere


def test_sharded_world1_gpu():
    """configs[3] orchestration at world size 1 on the GPU, device-resident
    (sharded.run_device_shard: the shard uploaded once, tic_codec_device per batch of 64 at
    buffer offsets, the exact SSE kernel, one all-gather): 70 synthetic images (a full and a
    partial batch), dataset PSNR within 0.02 dB of the oracle's on the same images, counts
    exact, and the device SSE equal to the host path's."""
    from tf_image_compression_amd import dist, sharded
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.topology import bottleneck_shape
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    n, P = 70, 256
    params = synthetic_params(0, seed=0)
    eh, ew, ec = bottleneck_shape(0, P)
    with Codec(0, params, SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        comm = dist.make_comm(c)
        summary, st = sharded.run_device_shard(c, comm, 0, 1, n, batch=64, passes=2)
        host = sharded.run_shard(lambda x: c.decode(c.encode(x)), 0, 1, n, P, 64, eh * ew * ec)
        comm.close()
    assert summary["images"] == 2 * n and st.dims == 2 * n * P * P * 3 and st.bits == 2 * n * eh * ew * ec
    assert st.sse == 2 * host.sse
    x = sharded.image_batch(0, n, P)
    _, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, P, 2, 0, acc=np.float32)
    _, rec = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, 0, acc=np.float32)
    p_ref = o.dataset_psnr(list(zip(x, rec)))
    assert abs(summary["psnr_db"] - p_ref) <= 0.02, (summary["psnr_db"], p_ref)
    assert abs(summary["bpp"] - eh * ew * ec / (P * P)) < 1e-12


def test_rccl_comm_world1():
    """dist.RcclComm over librccl.so at world size 1: ncclGetUniqueId / ncclCommInitRank
    (128-byte id by value), ncclAllReduce(max) and ncclAllGather of the 48-byte stats
    record on the codec's HIP stream, then ncclCommDestroy."""
    from tf_image_compression_amd import dist
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=64) as c:
        comm = dist.RcclComm(c, 0, 1)
        try:
            assert comm.allreduce_max(3.25) == 3.25
            comm.barrier()
            st = dist.RankStats(sse=12.5, dims=300, bits=64, images=2, t_start=1.0, t_end=2.5)
            got = comm.allgather_stats(st)
            assert len(got) == 1 and got[0] == st
        finally:
            comm.close()
        assert comm.comm is None


@pytest.mark.parametrize("model_id,P", [(0, 256), (3, 256)])
def test_plugin_module_encoder_decoder(model_id, P):
    """model_N.model.encoder(input, patch_size, quan_scale) / decoder(input, quan_scale) as
    encode.py:147 / decode.py:167 call them: float32 pixel input, float32 reconstruction in
    [0,255]; the decoder derives the patch size from the code shape (model_3 at a
    non-default P = 256); non-integer pixels are rejected."""
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    mod = importlib.import_module(f"tf_image_compression_amd.model_{model_id}.model")
    params = synthetic_params(model_id, seed=0)
    x = structured_patches(2, P, seed=400 + model_id)
    try:
        mod.restore(params, SYNTH_MEAN, SYNTH_STD)
        sym = mod.encoder(x.astype(np.float32), P, 2)
        pre, ref_sym = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, P, 2, model_id)
        scale = max(1.0, float(np.abs(pre).max()))
        safe = o.decision_margin(pre, 2) > 1e-5 * scale
        assert sym.dtype == np.uint8 and sym.shape == ref_sym.shape
        assert int(np.count_nonzero((sym != ref_sym) & safe)) == 0
        mod.restore(params, SYNTH_MEAN, SYNTH_STD)  # fresh handles: decoder must infer P
        rec = mod.decoder(sym.astype(np.float32), 2)
        ref_f, _ = o.decoder(params, SYNTH_MEAN, SYNTH_STD, sym, 2, model_id)
        assert rec.dtype == np.float32 and rec.shape == (2, P, P, 3)
        assert float(np.abs(rec - ref_f).max()) <= 1e-2
        with pytest.raises(ValueError):
            mod.encoder(x.astype(np.float32) + 0.25, P, 2)
        with pytest.raises(ValueError):
            mod.decoder(sym[:, :-1], 2)
    finally:
        mod.restore(params, SYNTH_MEAN, SYNTH_STD)  # releases the handles


def test_graph_replay_after_workspace_growth():
    """a captured graph holds the lane workspaces; a larger batch on the same
    handle reallocates them, and the next replay must not use the freed memory."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P = 64
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        x8 = structured_patches(8, P, seed=501)
        ref_idx = c.encode(x8)
        ref_rgb = c.decode(ref_idx)
        eh, ew, ec = c.code_shape
        d_in, d_idx, d_rgb = c.alloc(x8.nbytes), c.alloc(8 * eh * ew * ec), c.alloc(x8.nbytes)
        d_in.upload(x8)
        c.set_option("graph", 1)
        for _ in range(2):  # capture, then replay
            c.codec_device(d_in, 8, d_idx, d_rgb)
        c.synchronize()
        assert np.array_equal(d_idx.download(ref_idx.shape, np.uint8), ref_idx)
        big = structured_patches(48, P, seed=502)
        d_big, d_bidx = c.alloc(big.nbytes), c.alloc(48 * eh * ew * ec)
        d_big.upload(big)
        c.encode_device(d_big, 48, d_bidx)  # grows (reallocates) the lane workspaces
        c.synchronize()
        d_rgb.upload(np.zeros_like(x8))
        c.codec_device(d_in, 8, d_idx, d_rgb)
        c.synchronize()
        assert np.array_equal(d_idx.download(ref_idx.shape, np.uint8), ref_idx)
        assert np.array_equal(d_rgb.download(x8.shape, np.uint8), ref_rgb)
        c.set_option("graph", 0)


@pytest.mark.parametrize("mark,chain_x", [("encode_0", 1), ("encode_res_1/conv_0", 0), ("decode_1", 1),
                                          ("encode_3", 0), ("encode_3", 1)])
def test_mark_layer_in_step_timing(mark, chain_x):
    """bench.py's in-step launch timing (option mark_layer + tic_mark_durations): one event
    pair per lane per call around the launch that starts at the marked layer — a fused
    pair, a chain run, a chain run with its stride-2 head (chain_x: the launch starts at
    encode_3) or a plain layer — and the results stay bit-identical."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.topology import layer_table
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P, n, calls = 64, 8, 5
    names = [lay.name for lay in layer_table(0)]
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        c.set_option("fuse01", 1)
        c.set_option("fuse_tail", 1)
        c.set_option("chain", 1)
        c.set_option("chain_x", chain_x)
        x = structured_patches(n, P, seed=520)
        eh, ew, ec = c.code_shape
        d_in, d_idx, d_rgb = c.alloc(x.nbytes), c.alloc(n * eh * ew * ec), c.alloc(x.nbytes)
        d_in.upload(x)
        c.codec_device(d_in, n, d_idx, d_rgb)
        c.synchronize()
        ref = d_idx.download((n, eh, ew, ec), np.uint8), d_rgb.download(x.shape, np.uint8)
        c.set_option("mark_layer", names.index(mark))
        for _ in range(calls):
            c.codec_device(d_in, n, d_idx, d_rgb)
        ms = c.mark_durations()
        assert len(ms) == calls * 2 and np.all(ms > 0) and np.all(ms < 50), ms  # two lanes
        assert len(c.mark_durations()) == 0  # cleared
        assert np.array_equal(d_idx.download((n, eh, ew, ec), np.uint8), ref[0])
        assert np.array_equal(d_rgb.download(x.shape, np.uint8), ref[1])
        c.set_option("mark_layer", -1)
        c.codec_device(d_in, n, d_idx, d_rgb)
        assert len(c.mark_durations()) == 0


@pytest.mark.parametrize("decouple", [0, 1])
def test_lane_decoupling_orders_stream_work(decouple):
    """Lanes fork from the handle stream only when it has new work (option "decouple"):
    glue work enqueued on the handle stream between two codec calls must still see the
    first call's results (the histogram reads d_idx before the second call overwrites it)
    and the second call must see the caller's new input."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.image_codec import symbol_histogram
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    P, n = 64, 12
    x1, x2 = structured_patches(n, P, seed=801), structured_patches(n, P, seed=802)
    with Codec(0, synthetic_params(0), SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        c.set_option("decouple", decouple)
        c.set_option("streams", 3)
        ref1, ref2 = c.encode(x1), c.encode(x2)
        eh, ew, ec = c.code_shape
        d_in, d_idx, d_rgb = c.alloc(x1.nbytes), c.alloc(n * eh * ew * ec), c.alloc(x1.nbytes)
        d_cnt = c.alloc(16)
        for _ in range(3):
            d_in.upload(x1)
            c.codec_device(d_in, n, d_idx, d_rgb)
            c.memset_device(d_cnt, 0, 16)
            c.histogram_device(d_idx, n * eh * ew * ec, 2, d_cnt)  # reads call 1's symbols
            d_in.upload(x2)
            c.codec_device(d_in, n, d_idx, d_rgb)
            got1 = d_cnt.download((2,), np.uint64)
            c.synchronize()
            assert np.array_equal(got1.astype(np.int64), np.histogram(ref1, [0, 1, 2])[0])
            assert np.array_equal(d_idx.download(ref2.shape, np.uint8), ref2)
        c.set_option("streams", 2)


@pytest.mark.parametrize("P", [64, 128])
def test_codec_ch128(P):
    """base_model/ch_128 (channel width 128): the 64 -> 128 stride-2
    layer, the 128-wide residual stages (direct and Winograd forms), the 128 -> 64
    quantiser layer, the 64 -> 128 dequantiser layer and the 128 -> 64 / 64 -> 3 transposed
    convs, against the oracle; code P/4 x P/4 x 64 (base_model/ch_128/model.py:34-215)."""
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.topology import CH128_ID
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(CH128_ID, seed=0)
    with Codec(CH128_ID, params, SYNTH_MEAN, SYNTH_STD, patch_size=P) as c:
        assert c.code_shape == (P // 4, P // 4, 64)
        x = structured_patches(2, P, seed=900 + P)
        idx, rgb = check_codec(c, params, CH128_ID, P, x)
        c.set_option("s1_form", 0)  # the direct form of the 128-wide stride-1 layers
        check_codec(c, params, CH128_ID, P, x)


def test_ch128_model_module():
    """The drop-in module path of base_model/ch_128: encoder / decoder as the reference's
    (base_model/ch_128/model.py:34,123), patch size recovered from the code shape."""
    from tf_image_compression_amd.base_model.ch_128 import model
    from tf_image_compression_amd.topology import CH128_ID
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(CH128_ID, seed=0)
    model.restore(params, SYNTH_MEAN, SYNTH_STD)
    try:
        x = structured_patches(2, 128, seed=910)
        sym = model.encoder(x, 128, 2)
        assert sym.shape == (2, 32, 32, 64)
        ref_pre, ref_idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, 128, 2, CH128_ID)
        safe = o.decision_margin(ref_pre, 2) > 1e-5 * max(1.0, float(np.max(np.abs(ref_pre))))
        assert int(np.count_nonzero((sym != ref_idx) & safe)) == 0
        f = model.decoder(sym, 2)
        ref_f, _ = o.decoder(params, SYNTH_MEAN, SYNTH_STD, sym, 2, CH128_ID)
        assert f.shape == (2, 128, 128, 3) and float(np.max(np.abs(f - ref_f))) <= 1e-2
    finally:
        model._module.close()
