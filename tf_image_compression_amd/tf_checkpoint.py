"""Reader for TensorFlow V2 checkpoints (tensor bundles), so ``-p model_N/params_for_test/params``
works as in the reference (utils/utils.py:84-93: ``tf.train.Saver().restore(sess, path)``)
without TensorFlow.

Format (TF's tensor_bundle, as written by ``Saver`` in TF 1.x; restated from its published
layout — TensorFlow is not installed here and the reference ships no checkpoint, so this
reader is **parity unpinned** against real files; tests pin it with an independent writer
and CRC-32C known answers):

* ``<prefix>.index`` — an immutable sorted string table (LevelDB table format):
  data blocks of prefix-compressed entries (varint32 shared, varint32 non_shared,
  varint32 value_len, key suffix, value) followed by a restart array (uint32 offsets,
  uint32 count); every block carries a 5-byte trailer (compression type: 0 = none,
  masked CRC-32C of block + type byte); an index block maps the last key of each data
  block to its BlockHandle (varint64 offset, varint64 size); a 48-byte footer holds the
  metaindex and index handles and the magic 0xdb4775248b80fb57.
* Entry "" — BundleHeaderProto {num_shards = 1, endianness = 2, version = 3}.
* Every other entry — the tensor name -> BundleEntryProto {dtype = 1, shape = 2
  (TensorShapeProto: repeated dim = 2 {size = 1}), shard_id = 3, offset = 4, size = 5,
  crc32c = 6 (fixed32, masked CRC-32C of the tensor bytes), slices = 7}.
* ``<prefix>.data-SSSSS-of-NNNNN`` — raw little-endian tensor bytes at (offset, size).

Only what a model checkpoint holds is supported: DT_FLOAT / DT_DOUBLE / DT_INT32 /
DT_INT64 (global_step) tensors, unpartitioned; anything else raises ValueError.
"""
from __future__ import annotations

import os
import struct

import numpy as np

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_LEN = 48
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64}  # types.proto DataType
_MASK_DELTA = 0xA282EAD8

# ---------------------------------------------------------------- CRC-32C (Castagnoli)
def crc32c(data: bytes, crc: int = 0) -> int:
    """CRC-32C (Castagnoli) of ``data`` continuing ``crc`` (libtic tic_crc32c, host code)."""
    import ctypes as C
    from ._lib import lib
    buf = bytes(data)
    return int(lib().tic_crc32c(buf, len(buf), C.c_uint32(crc)))


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


# ---------------------------------------------------------------- varints / protobuf
def _varint(buf: bytes, pos: int) -> tuple[int, int]:
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise ValueError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _proto_fields(buf: bytes):
    """Yield (field_number, wire_type, value) of a serialized protobuf message."""
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _parse_shape(buf: bytes) -> tuple[int, ...]:
    dims = []
    for fn, wt, v in _proto_fields(buf):
        if fn == 2 and wt == 2:  # Dim
            size = 0
            for f2, w2, v2 in _proto_fields(v):
                if f2 == 1 and w2 == 0:
                    size = v2 if v2 < 1 << 63 else v2 - (1 << 64)
            dims.append(size)
        elif fn == 3 and wt == 0 and v:
            raise ValueError("unknown-rank tensor shape")
    return tuple(dims)


def parse_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": (), "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "slices": 0}
    for fn, wt, v in _proto_fields(buf):
        if fn == 1 and wt == 0:
            e["dtype"] = v
        elif fn == 2 and wt == 2:
            e["shape"] = _parse_shape(v)
        elif fn == 3 and wt == 0:
            e["shard_id"] = v
        elif fn == 4 and wt == 0:
            e["offset"] = v
        elif fn == 5 and wt == 0:
            e["size"] = v
        elif fn == 6 and wt == 5:
            e["crc32c"] = v
        elif fn == 7:
            e["slices"] += 1
    return e


def parse_header(buf: bytes) -> dict:
    h = {"num_shards": 1, "endianness": 0}
    for fn, wt, v in _proto_fields(buf):
        if fn == 1 and wt == 0:
            h["num_shards"] = v
        elif fn == 2 and wt == 0:
            h["endianness"] = v
    return h


# ---------------------------------------------------------------- SSTable
def _read_block(data: bytes, offset: int, size: int, verify: bool) -> bytes:
    end = offset + size
    if end + 5 > len(data):
        raise ValueError("block handle out of range")
    block = data[offset:end]
    ctype = data[end]
    if verify:
        (stored,) = struct.unpack_from("<I", data, end + 1)
        if mask_crc(crc32c(data[offset:end + 1])) != stored:
            raise ValueError(f"block checksum mismatch at offset {offset}")
    if ctype != 0:
        raise ValueError(f"compressed table block (type {ctype}) not supported")
    return block


def _block_entries(block: bytes):
    if len(block) < 4:
        raise ValueError("block too short")
    (nrestart,) = struct.unpack_from("<I", block, len(block) - 4)
    limit = len(block) - 4 - 4 * nrestart
    if limit < 0:
        raise ValueError("bad restart count")
    pos, key = 0, b""
    while pos < limit:
        shared, pos = _varint(block, pos)
        non_shared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        if shared > len(key):
            raise ValueError("bad key prefix")
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        yield key, block[pos:pos + vlen]
        pos += vlen


def read_table(path: str, verify: bool = True) -> list[tuple[bytes, bytes]]:
    data = open(path, "rb").read()
    if len(data) < FOOTER_LEN:
        raise ValueError(f"{path}: too short for a table")
    (magic,) = struct.unpack_from("<Q", data, len(data) - 8)
    if magic != TABLE_MAGIC:
        raise ValueError(f"{path}: bad table magic {magic:#x}")
    footer = data[len(data) - FOOTER_LEN:]
    _, p = _varint(footer, 0)  # metaindex offset
    _, p = _varint(footer, p)  # metaindex size
    idx_off, p = _varint(footer, p)
    idx_size, p = _varint(footer, p)
    out = []
    for _, handle in _block_entries(_read_block(data, idx_off, idx_size, verify)):
        off, q = _varint(handle, 0)
        size, _ = _varint(handle, q)
        out.extend(_block_entries(_read_block(data, off, size, verify)))
    return out


# ---------------------------------------------------------------- bundle
def is_checkpoint(prefix: str) -> bool:
    return os.path.exists(prefix + ".index")


def read_checkpoint(prefix: str, names=None, verify: bool = True) -> dict[str, np.ndarray]:
    """All (or the named) tensors of the checkpoint ``prefix`` as numpy arrays."""
    entries = read_table(prefix + ".index", verify)
    header = None
    tensors = {}
    for key, val in entries:
        if key == b"":
            header = parse_header(val)
            continue
        tensors[key.decode()] = parse_entry(val)
    if header is None:
        raise ValueError(f"{prefix}.index: no bundle header")
    if header["endianness"] != 0:
        raise ValueError("big-endian bundle not supported")
    nshards = header["num_shards"]
    want = list(tensors) if names is None else list(names)
    shards = {}
    out = {}
    for name in want:
        if name not in tensors:
            raise KeyError(f"{name} not found in checkpoint {prefix}")
        e = tensors[name]
        if e["slices"]:
            raise ValueError(f"{name}: partitioned variables not supported")
        if e["dtype"] not in _DTYPES:
            raise ValueError(f"{name}: dtype {e['dtype']} not supported")
        sid = e["shard_id"]
        if sid not in shards:
            shards[sid] = open(f"{prefix}.data-{sid:05d}-of-{nshards:05d}", "rb").read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(raw) != e["size"]:
            raise ValueError(f"{name}: data shard truncated")
        if verify and e["crc32c"] is not None:
            c = crc32c(raw)
            if mask_crc(c) != e["crc32c"] and c != e["crc32c"]:
                raise ValueError(f"{name}: tensor checksum mismatch")
        dt = np.dtype(_DTYPES[e["dtype"]]).newbyteorder("<")
        arr = np.frombuffer(raw, dt).astype(dt.newbyteorder("="))
        shape = e["shape"]
        if int(np.prod(shape, dtype=np.int64)) != arr.size:
            raise ValueError(f"{name}: {arr.size} values for shape {shape}")
        out[name] = arr.reshape(shape)
    return out


def load_model_params(prefix: str, model_id: int) -> dict[str, np.ndarray]:
    """The model's TF variables (utils/utils.py:84-93 restores exactly the graph's
    variables; optimizer slots / global_step in the file are ignored)."""
    from .topology import param_shapes
    shapes = param_shapes(model_id)
    params = read_checkpoint(prefix, names=list(shapes))
    for k, s in shapes.items():
        if tuple(params[k].shape) != tuple(s):
            raise ValueError(f"{k}: checkpoint shape {params[k].shape}, model expects {tuple(s)}")
        params[k] = np.ascontiguousarray(params[k], np.float32)
    return params
