"""CPU tests of the native range coder against the contract of the reference's own
range-coder suite (other/test_range_coder.py): the 17-byte known-answer stream, error
classes, multi-table round trips, fuzzing, and prob_to_cum_freq properties."""
import os
import random

import numpy as np
import pytest

from tf_image_compression_amd.range_coder import (RangeDecoder, RangeEncoder, cum_freq_to_prob,
                                                  prob_to_cum_freq, symbol_table)


def test_known_answer_stream(tmp_path):
    """other/test_range_coder.py:37-68: [0,0,0,0,1,2] x 17 with cumFreq [0,4,6,8] is 17 bytes,
    bytes 4..16 are 0x0b (each 6-symbol sequence carries exactly 8 bits)."""
    path = str(tmp_path / "kat")
    enc = RangeEncoder(path)
    enc.encode([0, 0, 0, 0, 1, 2] * 17, [0, 4, 6, 8])
    enc.close()
    with pytest.raises(RuntimeError):
        enc.encode([0, 0, 0, 0, 1, 2], [0, 4, 6, 8])
    data = open(path, "rb").read()
    assert len(data) == 17
    assert data[4:] == b"\x0b" * 13
    dec = RangeDecoder(path)
    assert dec.decode(102, [0, 4, 6, 8]) == [0, 0, 0, 0, 1, 2] * 17


def test_error_contract(tmp_path):
    path = str(tmp_path / "err")
    data = [0, 0, 0, 0, 1, 2] * 17
    enc = RangeEncoder(path)
    with pytest.raises(OverflowError):
        enc.encode(data, [-1, 1])
    with pytest.raises(ValueError):
        enc.encode(data, [1, 2, 3])
    with pytest.raises(ValueError):
        enc.encode(data, [0, 1])
    with pytest.raises(ValueError):
        enc.encode(data, [0, 8, 8, 8])
    with pytest.raises(ValueError):
        enc.encode(data, [])
    with pytest.raises(ValueError):
        enc.encode(data, [0])
    cum = prob_to_cum_freq(np.array([4, 6, 8]) / 18.0, 128)
    cum[-1] = 2 ** 32
    with pytest.raises(OverflowError):
        enc.encode([2, 2] * 17, cum)
    enc.close()
    dec = RangeDecoder(path)
    with pytest.raises(ValueError):
        dec.decode(3, [])
    with pytest.raises(ValueError):
        dec.decode(3, [0])
    assert dec.decode(0, [0, 4, 6, 8]) == []


def test_two_tables_round_trip(tmp_path):
    random.seed(558)
    path = str(tmp_path / "rt")
    c0, c1 = [0, 4, 6, 8], [0, 2, 5, 7, 10, 14]
    d0 = [random.randint(0, len(c0) - 2) for _ in range(10)]
    d1 = [random.randint(0, len(c1) - 2) for _ in range(17)]
    enc = RangeEncoder(path)
    enc.encode(d0, c0)
    enc.encode(d1, c1)
    enc.close()
    dec = RangeDecoder(path)
    assert dec.decode(len(d0), c0) == d0
    assert dec.decode(len(d1), c1) == d1
    dec.close()


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_round_trip(tmp_path, seed):
    r = np.random.RandomState(seed)
    nsym = r.randint(1, 300)
    cum = [0] + [int(v) for v in np.cumsum(r.randint(1, 5000, size=nsym))]
    if cum[-1] > 2 ** 24:
        cum = [int(v * (2 ** 24) // cum[-1]) for v in cum]
        cum = [0] + [max(cum[i + 1], cum[i] + 1) for i in range(len(cum) - 1)]
    freq = np.diff(cum)
    syms = np.flatnonzero(freq > 0)
    data = r.choice(syms, size=r.randint(0, 5000))
    path = str(tmp_path / f"f{seed}")
    enc = RangeEncoder(path)
    enc.encode(data, cum)
    enc.close()
    assert RangeDecoder(path).decode(len(data), cum) == data.tolist()


def test_decoder_survives_random_bytes(tmp_path):
    path = str(tmp_path / "rand")
    with open(path, "wb") as f:
        f.write(os.urandom(64))
    r = np.random.RandomState(827)
    for _ in range(10):
        cum = [0] + [int(v) for v in np.cumsum(r.randint(1, 100, size=r.randint(1, 20)))]
        out = RangeDecoder(path).decode(100, cum)
        assert len(out) == 100 and all(0 <= s < len(cum) - 1 for s in out)


def test_binary_code_rate(tmp_path):
    """Q=2 symbols at p(1)=0.1: the coded size is close to the entropy."""
    r = np.random.RandomState(5)
    data = (r.rand(200000) < 0.1).astype(np.int64)
    cum = symbol_table(np.array([0.9, 0.1]), resolution=4096)
    path = str(tmp_path / "rate")
    enc = RangeEncoder(path)
    enc.encode(data, cum)
    enc.close()
    h = -(0.9 * np.log2(0.9) + 0.1 * np.log2(0.1))
    assert os.path.getsize(path) * 8 / data.size < h * 1.01 + 1e-3
    assert RangeDecoder(path).decode_array(data.size, cum).tolist() == data.tolist()


def test_prob_to_cum_freq_properties():
    rs = np.random.RandomState(190)
    p0 = rs.dirichlet([.1] * 50)
    c0 = prob_to_cum_freq(p0, 1024)
    p1 = cum_freq_to_prob(c0)
    c1 = prob_to_cum_freq(p1, 1024)
    assert c0[-1] == 1024 and len(c0) == len(p0) + 1
    assert np.all(np.diff(c0)[p0 > 0.] > 0)
    assert np.isclose(np.sum(p1), 1.)
    assert c0 == c1


def _greedy_reference(prob, resolution):
    """The published allocation of the range_coder package, written as the plain loop:
    `resolution` times, freq[nanargmax(prob / freq)] += 1."""
    prob = np.asarray(prob, dtype=np.float64)
    freq = np.zeros(prob.size, dtype=np.int64)
    with np.errstate(divide="ignore", invalid="ignore"):
        for _ in range(resolution):
            freq[np.nanargmax(prob / freq)] += 1
    return [0] + np.cumsum(freq).tolist()


@pytest.mark.parametrize("seed,n,res", [(0, 2, 4096), (1, 3, 8), (2, 50, 1024), (3, 256, 4096), (4, 7, 7),
                                        (5, 16, 100)])
def test_prob_to_cum_freq_matches_greedy_loop(seed, n, res):
    rs = np.random.RandomState(seed)
    p = rs.dirichlet([0.3] * n)
    p[rs.rand(n) < 0.2] = 0.0
    if p.sum() == 0:
        p[0] = 1.0
    assert prob_to_cum_freq(p, res) == _greedy_reference(p, res)
    # the reference CLI's construction (encode.py:81-86) too
    m = p * 4096 + 1
    assert symbol_table(p, 4096) == _greedy_reference(m / m.sum(), 4096)


def test_prob_to_cum_freq_zero_prob():
    c1 = prob_to_cum_freq([0.5, 0.25, 0.25], resolution=8)
    c0 = prob_to_cum_freq([0.5, 0., 0.25, 0.25, 0., 0.], resolution=8)
    assert c1 == [0, 4, 6, 8]
    assert [c0[0]] + [c0[i + 1] for i, p in enumerate([0.5, 0., 0.25, 0.25, 0., 0.]) if p > 0.] == c1
