"""TF V2 checkpoint reader (tf_checkpoint.py) — the stand-in for tf.train.Saver.restore
(utils/utils.py:84-93).  Parity unpinned against real TF files (none in the reference, no
TF here); pinned by CRC-32C known answers (RFC 3720 / LevelDB test vectors) and by reading
back checkpoints from the independent writer in tests/tf_bundle_writer.py."""
import os

import numpy as np
import pytest

from tf_bundle_writer import crc32c_py, mask, write_checkpoint

from tf_image_compression_amd import tf_checkpoint as tc


def test_crc32c_known_answers():
    assert tc.crc32c(b"123456789") == 0xE3069283
    assert tc.crc32c(bytes(32)) == 0x8A9136AA              # leveldb crc32c_test
    assert tc.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert tc.crc32c(bytes(range(32))) == 0x46DD794E
    assert tc.crc32c(b"") == 0
    data = np.random.default_rng(0).integers(0, 256, 1003, dtype=np.uint8).tobytes()
    assert tc.crc32c(data) == crc32c_py(data)
    assert tc.crc32c(data[500:], tc.crc32c(data[:500])) == tc.crc32c(data)   # continuation
    assert tc.mask_crc(0x12345678) == mask(0x12345678)


@pytest.mark.parametrize("block_size", [64, 256, 1 << 16])
def test_round_trip_model_checkpoint(tmp_path, block_size):
    from tf_image_compression_amd.weights import synthetic_params
    params = synthetic_params(0, seed=3)
    extra = {"global_step": np.array(123456, np.int64),
             "encode_0/kernel/Adam": np.ones((3, 3, 3, 32), np.float32),
             "beta1_power": np.array(0.9, np.float32)}
    prefix = str(tmp_path / "params")
    write_checkpoint(prefix, {**params, **extra}, block_size=block_size)
    allt = tc.read_checkpoint(prefix)
    assert set(allt) == set(params) | set(extra)
    assert allt["global_step"].shape == () and allt["global_step"].dtype == np.int64
    assert int(allt["global_step"]) == 123456
    got = tc.load_model_params(prefix, 0)
    assert set(got) == set(params)
    for k in params:
        assert got[k].dtype == np.float32 and np.array_equal(got[k], params[k])


def test_restore_params_reads_checkpoint_prefix(tmp_path):
    from types import SimpleNamespace
    from tf_image_compression_amd import utils
    from tf_image_compression_amd.weights import synthetic_params
    params = synthetic_params(3, seed=1)
    prefix = str(tmp_path / "params")
    write_checkpoint(prefix, params)
    got = utils.restore_params(SimpleNamespace(params_file=prefix, model_num="3"))
    assert all(np.array_equal(got[k], params[k]) for k in params)


def test_corruption_and_unsupported_are_errors(tmp_path):
    from tf_image_compression_amd.weights import synthetic_params
    params = synthetic_params(0, seed=3)
    prefix = str(tmp_path / "p")
    write_checkpoint(prefix, params)
    data = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    data[100] ^= 0x40
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(ValueError, match="checksum"):
        tc.read_checkpoint(prefix)
    assert tc.read_checkpoint(prefix, verify=False)["decode_0/bias"].shape == (3,)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[5] ^= 1
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(ValueError, match="checksum"):
        tc.read_checkpoint(prefix)
    idx[-1] ^= 1  # magic
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(ValueError, match="magic"):
        tc.read_checkpoint(prefix)
    write_checkpoint(prefix, {"encode_0/kernel": np.zeros((3, 3, 3, 32), np.float32)})
    with pytest.raises(KeyError):
        tc.load_model_params(prefix, 0)
    p2 = dict(params)
    p2["encode_1/bias"] = np.zeros(31, np.float32)
    write_checkpoint(prefix, p2)
    with pytest.raises(ValueError, match="shape"):
        tc.load_model_params(prefix, 0)
    assert not tc.is_checkpoint(str(tmp_path / "missing"))
    assert os.path.exists(prefix + ".index")
