"""wino_chain_kernel (csrc/wino_chain.h): every run of stride-1 64->64 layers in one launch,
8x8 regions per workgroup with the region borders handed between workgroups.  It
reproduces the unfused Winograd launches operation for operation, so the bar is bit
identity with them (pre-activations, symbols, decoder floats and bytes), on every model
and at patch sizes whose bottleneck is a single partial region (P = 48, 64), 2x2 regions
(model_0 at 256), 4x4 and 8x8 regions (model_3 at 256: 32x32 and 64x64 stages), and at
batches whose grid exceeds what the GPU holds at once (the ticket order must keep every
patch's regions co-resident).  Reference layers: model_0/model.py:98-196,
model_3/model.py:66-281, submit/2/rmbe/model.py:140-160."""
import re

import numpy as np
import pytest

from conftest import structured_patches

pytestmark = pytest.mark.gpu


def _codec(model_id, P):
    from tf_image_compression_amd.codec import Codec
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    return Codec(model_id, synthetic_params(model_id, seed=0), SYNTH_MEAN, SYNTH_STD, patch_size=P)


def _run(c, x):
    idx, pre = c.encode(x, return_preact=True)
    u8, f = c.decode(idx, return_float=True)
    return idx, pre, u8, f


@pytest.mark.parametrize("model_id,P,n", [(0, 256, 6), (0, 64, 5), (0, 48, 3), (1, 64, 4), (2, 128, 3),
                                          (3, 128, 3), (3, 256, 3)])
def test_wino_chain_bit_identical(model_id, P, n):
    with _codec(model_id, P) as c:
        x = structured_patches(n, P, seed=600 + model_id + P)
        c.set_option("s1_form", 1)
        c.set_option("chain", 0)
        ref = _run(c, x)
        assert not any("wino_chain" in k for k in c.layer_kernels(n))
        c.set_option("chain", 1)
        c.set_option("chain_x", 0)
        for wh in (1, 2):  # 256- / 512-thread workgroups
            c.set_option("chain_wh", wh)
            c.set_option("streams", 1)
            kern = c.layer_kernels(n)
            assert any(re.fullmatch(rf"wino_chain_kernel<\d,\d,{wh},\d>", k) for k in kern), kern
            got = _run(c, x)
            for a, b in zip(ref, got):
                assert np.array_equal(a, b)
            # lanes split the batch: chain launches on two streams at once
            c.set_option("streams", 2)
            assert all(np.array_equal(a, b) for a, b in zip(ref, _run(c, x)))
        c.set_option("chain", 0)


def test_wino_chain_oversubscribed_grid():
    """model_0 at 256 with 256 patches per launch: 1024 region workgroups on one stream and
    another 1024 on the second lane, more than are resident at once — the ticket order must
    still complete every launch, and repeated launches (epochs) stay correct."""
    with _codec(0, 256) as c:
        x = structured_patches(8, 256, seed=700)
        big = np.concatenate([x] * 64)  # 512 patches, 2 lanes x 256
        c.set_option("chain", 0)
        ref_idx = c.encode(x)
        ref_u8 = c.decode(ref_idx)
        c.set_option("chain", 1)
        c.set_option("chunk", 512)
        for wh in (2, 1):
            c.set_option("chain_wh", wh)
            for _ in range(3):
                idx = c.encode(big)
                assert all(np.array_equal(idx[i * 8:(i + 1) * 8], ref_idx) for i in range(64))
            u8 = c.decode(idx)
            assert all(np.array_equal(u8[i * 8:(i + 1) * 8], ref_u8) for i in range(64))
        c.set_option("chain", 0)


def test_wino_chain_rmbe_bit_identical():
    """The chain on the rmbe net's 32x32 stage, in the F(2x2,3x3) form it computes (the net's
    default stride-1 form is F(4x4,3x3), which the chain does not run)."""
    from tf_image_compression_amd.topology import RMBE_ID
    r = np.random.default_rng(8)
    win = np.clip(r.normal(120, 50, (5, 128, 128, 3)), 0, 255).astype(np.float32)
    with _codec(RMBE_ID, 128) as c:
        c.set_option("s1_form", 1)
        c.set_option("chain", 0)
        a = c.rmbe_windows(win)
        c.set_option("chain", 1)
        outs = []
        for wh in (2, 1):
            c.set_option("chain_wh", wh)
            assert any(k.startswith("wino_chain") for k in c.layer_kernels(5))
            outs.append(c.rmbe_windows(win))
    assert all(np.array_equal(a, b) for b in outs)


def test_wino_chain_device_path_and_tuning_replay():
    """codec_device with the chain on equals the host path; tic_tuning_export / import
    carries the chain flag and every tuned choice to a second handle (bit-identical run)."""
    P, n = 256, 16
    x = structured_patches(n, P, seed=710)
    with _codec(0, P) as c:
        c.set_option("chain", 1)
        idx, u8 = c.encode(x), None
        u8 = c.decode(idx)
        d_in, d_idx, d_rgb = c.alloc(x.nbytes), c.alloc(idx.nbytes), c.alloc(x.nbytes)
        d_in.upload(x)
        c.autotune(d_in, n // 2, reps=1)
        c.codec_device(d_in, n, d_idx, d_rgb)
        c.synchronize()
        assert np.array_equal(d_idx.download(idx.shape, np.uint8), idx)
        assert np.array_equal(d_rgb.download(x.shape, np.uint8), u8)
        text = c.tuning_export()
        assert "flag chain 1" in text and "flag chain_wh " in text
        with _codec(0, P) as c2:
            c2.tuning_import(text)
            assert c2.tuning_export() == text
            assert c2.layer_kernels(n // 2) == c.layer_kernels(n // 2)
            assert np.array_equal(c2.encode(x), idx)
            with pytest.raises(ValueError):
                c2.tuning_import("tic-tuning 1\nconv 0 8 2 0\n")  # a T2 kernel for the first layer
            # variants are validated against the layer role's variant set
            for bad in ("var 5 32 1", "var 0 -32 5", "var 0 32 3", "var 16 32 16", "var 17 32 12", "var 16 -32 1"):
                with pytest.raises(ValueError):
                    c2.tuning_import("tic-tuning 1\n" + bad + "\n")
            assert c2.tuning_export() == text  # nothing applied by the rejected imports


def test_chain_cut_inside_res_block_fails_loudly(monkeypatch):
    """a chain run that ends inside a res_block keeps the block input in
    LDS only, so the block's residual conv that follows unfused has no block input in a
    workspace.  The planner never makes such a run (round 4's P = 4096 page fault was one);
    forced through the test hook, the call must fail with TIC_EINVAL ("residual input not in
    a workspace") instead of launching that conv on workspace -1.  Reference:
    basic_block/basic_block.py:74-93 (the residual add of res_block)."""
    x = structured_patches(2, 256, seed=720)
    with _codec(0, 256) as c:
        c.set_option("s1_form", 1)
        c.set_option("chain", 1)
        c.set_option("streams", 1)
        ref = c.encode(x)
        # model_0 encoder run: res_1/conv_0, res_1/conv_1, res_2/conv_0 | res_2/conv_1 ...
        monkeypatch.setenv("TIC_TEST_CHAIN_CUT", "3")
        with pytest.raises(ValueError, match=r"\[EINVAL\].*residual input not in a workspace"):
            c.encode(x)
        monkeypatch.delenv("TIC_TEST_CHAIN_CUT")
        c.synchronize()
        assert np.array_equal(c.encode(x), ref)  # the handle stays usable


@pytest.mark.parametrize("model_id,P,n", [(0, 256, 9), (3, 128, 3)])
def test_wino_chain_region_orders_bit_identical(model_id, P, n):
    """The chain's region orders (option chain_order: 0 atomic ticket, 1 blockIdx, 2 blockIdx
    with a patch's regions on one XCD, -1 auto) only place the workgroups: the outputs are
    identical (n = 9 at model_0: one full group of eight patches plus a tail patch that keeps
    the identity order)."""
    with _codec(model_id, P) as c:
        x = structured_patches(n, P, seed=730 + model_id)
        c.set_option("s1_form", 1)
        c.set_option("chain", 1)
        outs = []
        for order in (0, 1, 2, -1):
            c.set_option("chain_order", order)
            for streams in (1, 2):
                c.set_option("streams", streams)
                outs.append(_run(c, x))
        for got in outs[1:]:
            assert all(np.array_equal(a, b) for a, b in zip(outs[0], got))


@pytest.mark.parametrize("model_id,P,n", [(0, 256, 6), (0, 64, 5), (0, 48, 3), (1, 64, 4), (2, 128, 3)])
def test_wino_chain_stride2_neighbours_bit_identical(model_id, P, n):
    """Option chain_x: the encoder's stride-2 layer in front of a run (encode_3) as the chain
    launch's head and the decoder's transposed layer behind it (decode_3) as its tail
    (wino_chain.h HT).  They replay conv3x3_kernel's MODE_S2 / MODE_T2 step order, so the
    whole codec stays bit-identical to the unfused launches: at 2x2 regions (model_0 at 256,
    model_2 at 128), a single region with its halo outside the image (P = 64) and a single
    partial region (P = 48), one lane and two.  Reference layers: model_0/model.py:90-96
    (encode_3), 198-206 (decode_3); model_2/model.py."""
    with _codec(model_id, P) as c:
        x = structured_patches(n, P, seed=740 + model_id + P)
        c.set_option("s1_form", 1)
        c.set_option("chain", 0)
        ref = _run(c, x)
        c.set_option("chain", 1)
        c.set_option("chain_wh", 2)
        c.set_option("chain_x", 1)
        for streams in (1, 2):
            c.set_option("streams", streams)
            kern = c.layer_kernels(n)
            heads = [k for k in kern if re.fullmatch(r"wino_chain_kernel<\d,\d,2,[13]>", k)]
            tails = [k for k in kern if re.fullmatch(r"wino_chain_kernel<\d,\d,2,[23]>", k)]
            assert heads and tails, kern
            # the head's launch starts at encode_3 and carries the run; decode_3 has no launch
            names = [lay[0] for lay in c.layers()]
            assert kern[names.index("encode_3")] in heads and kern[names.index("encode_3") + 1] == "", kern
            assert kern[names.index("decode_3")] == "", kern
            got = _run(c, x)
            for a, b in zip(ref, got):
                assert np.array_equal(a, b)
        c.set_option("chain_x", 0)
        assert not any(re.fullmatch(r"wino_chain_kernel<\d,\d,2,[123]>", k) for k in c.layer_kernels(n))


def test_wino_chain_stride2_neighbours_oversubscribed():
    """The head / tail launches with 2 x 256 patches (2048 region workgroups, more than are
    resident): the ticket order still completes them, epoch after epoch."""
    with _codec(0, 256) as c:
        x = structured_patches(8, 256, seed=760)
        big = np.concatenate([x] * 64)
        c.set_option("chain", 0)
        ref_idx = c.encode(x)
        ref_u8 = c.decode(ref_idx)
        c.set_option("chain", 1)
        c.set_option("chain_wh", 2)
        c.set_option("chain_x", 1)
        c.set_option("chunk", 512)
        for _ in range(3):
            idx = c.encode(big)
            assert all(np.array_equal(idx[i * 8:(i + 1) * 8], ref_idx) for i in range(64))
        u8 = c.decode(idx)
        assert all(np.array_equal(u8[i * 8:(i + 1) * 8], ref_u8) for i in range(64))


@pytest.mark.parametrize("model_id,P,n,fuse_tail", [(0, 256, 6, None), (0, 64, 5, None), (0, 48, 3, None),
                                                    (1, 64, 4, None), (0, 288, 2, None), (2, 128, 4, 0)])
def test_wino_chain_decode2_behind_tail_bit_identical(model_id, P, n, fuse_tail):
    """chain_x 2: decode_2 (transposed 64 -> 32) runs in the decoder chain's launch as well,
    on decode_3's output kept in LDS; decode_3's outputs just above / left of a region are
    recomputed from the run's halo ring in conv3x3_kernel's order (as dec10 does for decode_1),
    so everything stays bit-identical to the unfused launches: 2x2 regions (P = 256), one
    region (P = 64), one partial region (P = 48), 3x3 regions with partial ones at the bottom
    and right (P = 288).  model_2 with the decoder-tail fusion off: its decode_2 is
    the layer before the network's last, so the chain's tail2 output feeds decode_1 (32 -> 3,
    denorm, u8) running standalone.  Reference layers: model_0/model.py:198-222 (decode_3,
    decode_2), model_2/model.py:190-235."""
    with _codec(model_id, P) as c:
        x = structured_patches(n, P, seed=770 + model_id + P)
        if fuse_tail is not None:
            c.set_option("fuse_tail", fuse_tail)
        c.set_option("s1_form", 1)
        c.set_option("s2_form", 0)  # decode_2's direct form (the polyphase one: test_gpu_pwino.py)
        c.set_option("chain", 0)
        ref = _run(c, x)
        c.set_option("chain", 1)
        c.set_option("chain_wh", 2)
        c.set_option("chain_x", 2)
        names = [lay[0] for lay in c.layers()]
        for streams in (1, 2):
            c.set_option("streams", streams)
            kern = c.layer_kernels(n)
            assert any(re.fullmatch(r"wino_chain_kernel<\d,\d,2,6>", k) for k in kern), kern
            assert kern[names.index("decode_3")] == "" and kern[names.index("decode_2")] == "", kern
            got = _run(c, x)
            for a, b in zip(ref, got):
                assert np.array_equal(a, b)
        c.set_option("chain_x", 1)
        assert not any(re.fullmatch(r"wino_chain_kernel<\d,\d,2,6>", k) for k in c.layer_kernels(n))


def test_wino_chain_exact_fill_with_fewer_cus(monkeypatch):
    """the automatic region order is the blockIdx-based, XCD-aware one (2) when
    nlanes x n x R workgroups fit num_cus — model_0's shipped configuration sits exactly on that
    line (2 lanes x 32 patches x 4 regions = 256).  A region under order 2 waits only on regions
    of its own patch, dispatched to the same XCD right after it (blocks b, b+8, b+16, b+24), so
    in-order dispatch per XCD needs R free slots per lane and XCD, not a slot for every
    workgroup.  Checked here with the lane streams restricted to 248 of the CUs by a CU mask
    (the grid of 256 chain workgroups cannot be resident at once): orders 2, 1 and 0 finish
    without a hand-off timeout and bit-identical to the unfused path."""
    monkeypatch.setenv("TIC_TEST_LANE_CU_OFF", "8")
    P, n = 256, 64
    x = structured_patches(n, P, seed=740)
    with _codec(0, P) as c:
        c.set_option("s1_form", 1)
        c.set_option("streams", 2)
        c.set_option("chain", 0)
        ref = _run(c, x)
        c.set_option("chain", 1)
        c.set_option("chain_wh", 2)
        for order in (-1, 2, 1, 0):
            c.set_option("chain_order", order)
            assert any("wino_chain" in k for k in c.layer_kernels(n // 2))
            for _ in range(3):
                got = _run(c, x)
                assert all(np.array_equal(a, b) for a, b in zip(ref, got)), order
