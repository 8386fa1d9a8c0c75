"""Drop-in for the third-party ``range_coder`` package the reference CLIs import
(encode.py:9,76-97; decode.py:9,79-101): ``RangeEncoder``, ``RangeDecoder``,
``prob_to_cum_freq``, ``cum_freq_to_prob`` with the same call signatures and error
classes that other/test_range_coder.py pins (RuntimeError after close, OverflowError for
frequencies that do not fit 32 bits, ValueError for malformed tables / zero-probability
symbols).  The coder itself is native (csrc/range_coder.cpp, C-ABI tic_rc_*); this module
is only the binding.  Byte-level compatibility with the unvendored package is not claimed
(SURVEY.md §8f): streams round-trip through this implementation.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import lib

_EINVAL, _ESTATE, _EOVERFLOW, _EIO = -1, -3, -7, -8


def _L():
    return lib()  # signatures bound in _lib.SIGNATURES


def _raise(rc, what):
    msg = f"{what}: {_L().tic_rc_last_error().decode(errors='replace')}"
    if rc == _EOVERFLOW:
        raise OverflowError(msg)
    if rc == _EINVAL:
        raise ValueError(msg)
    if rc == _EIO:
        raise IOError(msg)
    raise RuntimeError(msg)


def _table(cum_freq):
    """Integer cumulative table as int64 (values beyond int64 -> OverflowError)."""
    try:
        vals = [int(v) for v in cum_freq]
    except (TypeError, ValueError) as e:
        raise ValueError(f"invalid frequency table: {e}")
    for v in vals:
        if v < 0 or v >= 2 ** 32:
            raise OverflowError("cumulative frequencies must fit in an unsigned 32-bit integer")
    return np.ascontiguousarray(np.array(vals, dtype=np.int64).reshape(-1))


class RangeEncoder:
    """``RangeEncoder(filepath)``; ``encode(data, cum_freq)``; ``close()``."""

    def __init__(self, filepath):
        h = C.c_void_p()
        rc = _L().tic_rc_encoder_open(os.fsencode(filepath), C.byref(h))
        if rc:
            _raise(rc, "RangeEncoder")
        self._h = h
        self._closed = False

    def encode(self, data, cum_freq):
        if self._closed:
            raise RuntimeError("RangeEncoder is closed")
        table = _table(cum_freq)
        d = np.ascontiguousarray(np.asarray(data, dtype=np.int64).reshape(-1))
        rc = _L().tic_rc_encode(self._h, d.ctypes.data_as(C.POINTER(C.c_int64)), d.size,
                                table.ctypes.data_as(C.POINTER(C.c_int64)), table.size)
        if rc:
            _raise(rc, "RangeEncoder.encode")

    def close(self):
        if not self._closed:
            self._closed = True
            rc = _L().tic_rc_encoder_close(self._h)
            if rc:
                _raise(rc, "RangeEncoder.close")

    def __del__(self):
        try:
            self.close()
            _L().tic_rc_encoder_free(self._h)
        except Exception:
            pass


class RangeDecoder:
    """``RangeDecoder(filepath)``; ``decode(num_symbols, cum_freq) -> list``; ``close()``."""

    def __init__(self, filepath):
        h = C.c_void_p()
        rc = _L().tic_rc_decoder_open(os.fsencode(filepath), C.byref(h))
        if rc:
            _raise(rc, "RangeDecoder")
        self._h = h
        self._closed = False

    def decode(self, num_symbols, cum_freq):
        return self.decode_array(num_symbols, cum_freq).tolist()

    def decode_array(self, num_symbols, cum_freq) -> np.ndarray:
        if self._closed:
            raise RuntimeError("RangeDecoder is closed")
        table = _table(cum_freq)
        n = int(num_symbols)
        out = np.empty(max(n, 0), np.int64)
        rc = _L().tic_rc_decode(self._h, n, table.ctypes.data_as(C.POINTER(C.c_int64)), table.size,
                                out.ctypes.data_as(C.POINTER(C.c_int64)))
        if rc:
            _raise(rc, "RangeDecoder.decode")
        return out

    def close(self):
        if not self._closed:
            self._closed = True
            _L().tic_rc_decoder_close(self._h)

    def __del__(self):
        try:
            self.close()
            _L().tic_rc_decoder_free(self._h)
        except Exception:
            pass


def prob_to_cum_freq(prob, resolution=1024):
    """Probability vector -> cumulative frequency table [0, ..., resolution] in which every
    non-zero probability gets a non-zero frequency and zero probabilities get none
    (properties pinned by other/test_range_coder.py:186-229).  Frequencies are
    floor(p * resolution), raised to 1 for every non-zero p; missing counts go to the
    largest fractional remainders (ties to the lower index), surplus counts are taken from
    the entries rounded up the most.  The package's exact rounding is unvendored."""
    p = np.asarray(prob, dtype=np.float64).reshape(-1)
    if p.size == 0 or np.any(p < 0) or not np.all(np.isfinite(p)) or p.sum() <= 0:
        raise ValueError("invalid probability vector")
    nz = p > 0
    if int(nz.sum()) > resolution:
        raise ValueError("more non-zero probabilities than the resolution")
    p = p / p.sum()
    exact = p * resolution
    freq = np.floor(exact + 1e-9).astype(np.int64)
    freq[nz & (freq == 0)] = 1
    diff = int(resolution - freq.sum())
    if diff > 0:
        order = sorted(np.flatnonzero(nz), key=lambda i: (-(exact[i] - np.floor(exact[i])), i))
        for k in range(diff):
            freq[order[k % len(order)]] += 1
    elif diff < 0:
        order = sorted(np.flatnonzero(freq > 1), key=lambda i: ((exact[i] - freq[i]), i))
        k = 0
        while diff < 0:
            i = order[k % len(order)]
            if freq[i] > 1:
                freq[i] -= 1
                diff += 1
            k += 1
    return [0] + [int(v) for v in np.cumsum(freq)]


def cum_freq_to_prob(cum_freq):
    c = np.asarray(cum_freq, dtype=np.float64)
    return np.diff(c) / c[-1]


def symbol_table(prob, resolution=4096):
    """The reference's table construction (encode.py:77-86, decode.py:80-89):
    freq = prob * resolution + 1 (no zero probability), renormalised, then
    prob_to_cum_freq(..., resolution)."""
    modified_freq = np.asarray(prob, np.float64) * resolution + 1
    return prob_to_cum_freq(modified_freq / np.sum(modified_freq), resolution=resolution)
