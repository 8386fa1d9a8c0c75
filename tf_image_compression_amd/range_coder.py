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
    """Probability vector -> cumulative frequency table [0, ..., resolution].

    The budget is handed out one count at a time, each to the entry with the largest
    prob / freq (the first such index on ties; a zero frequency counts as infinitely far
    behind, a zero probability never receives a count), which is the published allocation
    of the third-party ``range_coder`` package (unvendored; greedy descent of the KL
    divergence).  So every non-zero probability gets a non-zero frequency whenever
    len(prob) <= resolution, the properties other/test_range_coder.py:186-229 pins.  The
    heap reproduces the sequential argmax exactly: keys are the same float64 quotients and
    ties resolve to the lower index.  Byte compatibility with the package stays unpinned
    (no fixture exists), see SURVEY.md §8f."""
    import heapq
    p = np.asarray(prob, dtype=np.float64).reshape(-1)
    if p.size == 0 or np.any(p < 0) or not np.all(np.isfinite(p)) or p.sum() <= 0:
        raise ValueError("invalid probability vector")
    nz = np.flatnonzero(p > 0)
    if nz.size > resolution:
        raise ValueError("more non-zero probabilities than the resolution")
    freq = np.zeros(p.size, np.int64)
    # first pass: freq == 0 -> prob / freq = inf for every non-zero entry, lowest index first
    k = min(int(resolution), nz.size)
    freq[nz[:k]] = 1
    heap = [(-(p[i] / 1.0), int(i)) for i in nz[:k]]
    heapq.heapify(heap)
    for _ in range(int(resolution) - k):
        _, i = heapq.heappop(heap)
        freq[i] += 1
        heapq.heappush(heap, (-(p[i] / float(freq[i])), i))
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
