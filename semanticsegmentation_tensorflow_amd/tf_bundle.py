"""TF1 V2 checkpoint ("tensor bundle") files, written and read without
TensorFlow: what `tf.train.Saver.save` / `restore` put on disk for the
reference's save-and-resume flow (Network/model/FCN.py:370-378,
Network/main.py:143-153, :190).

A checkpoint `<prefix>` is two files:

* `<prefix>.data-00000-of-00001`: the tensors' raw little-endian bytes,
  back to back;
* `<prefix>.index`: a LevelDB-format SSTable whose keys are the tensor names
  in sorted order, plus the empty key first.  The empty key's value is a
  serialized `BundleHeaderProto` (num_shards, endianness, version); every
  other value a `BundleEntryProto` (dtype, shape, shard_id, offset, size,
  masked CRC-32C of the bytes).

SSTable layout (LevelDB table format): data blocks of prefix-compressed
entries with restart points, each followed by a 5-byte trailer (compression
type 0 = none, masked CRC-32C of block + type), a meta-index block, an index
block mapping a separator key >= each data block's last key to the block's
(offset, size) handle, and a 48-byte footer (the two handles as varints,
zero-padded, then the magic 0xdb4775248b80fb57).  Protobuf messages are
encoded by hand (field tags + varints), so no generated code is needed.

The writer emits uncompressed blocks (what TF writes); the reader accepts
any block size / restart interval and refuses compressed blocks.  Parity is
pinned by the format's published constants (CRC-32C check value, SSTable
magic, field numbers) and by round trips; no TF-written file exists here to
read (TensorFlow is not installed), which DESIGN.md records.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from . import _lib

MAGIC = 0xDB4775248B80FB57
_MASK_DELTA = 0xA282EAD8
# tensorflow/core/framework/types.proto
DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
      np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
      np.dtype(np.float16): 19}
DT_INV = {v: k for k, v in DT.items()}
DT_BFLOAT16 = 14


# --------------------------------------------------------------- checksums
def crc32c(data, crc=0):
    """CRC-32C (Castagnoli) of a bytes-like object (host C code in libsegkern)."""
    if not isinstance(data, bytes):
        data = bytes(data)
    if not data:
        return crc
    return int(_lib.lib().seg_crc32c(ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p), len(data), crc))


def mask_crc(c):
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(m):
    r = (m - _MASK_DELTA) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# --------------------------------------------------------------- varints / protobuf
def _varint(v):
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("malformed varint")


def _field_varint(num, v):
    return _varint(num << 3) + _varint(v)


def _field_bytes(num, b):
    return _varint((num << 3) | 2) + _varint(len(b)) + b


def _field_fixed32(num, v):
    return _varint((num << 3) | 5) + struct.pack("<I", v)


def _parse_fields(buf):
    """protobuf wire format -> {field: [values]} (varint ints, bytes, fixed32/64 ints)."""
    out = {}
    pos = 0
    while pos < len(buf):
        tag, pos = _read_varint(buf, pos)
        num, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.setdefault(num, []).append(v)
    return out


def _header_proto():
    # BundleHeaderProto{num_shards=1, endianness=LITTLE(0), version=VersionDef{producer=1}}
    return _field_varint(1, 1) + _field_varint(2, 0) + _field_bytes(3, _field_varint(1, 1))


def _shape_proto(shape):
    # TensorShapeProto{repeated Dim dim = 2 {int64 size = 1}}
    return b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)


def _entry_proto(dtype, shape, offset, size, crc):
    # BundleEntryProto{dtype=1, shape=2, shard_id=3, offset=4, size=5, crc32c=6 (fixed32)}
    out = _field_varint(1, dtype) + _field_bytes(2, _shape_proto(shape))
    out += _field_varint(4, offset) if offset else b""
    out += _field_varint(5, size) + _field_fixed32(6, crc)
    return out


def _parse_entry(buf):
    f = _parse_fields(buf)
    shape = []
    for sp in f.get(2, []):
        for dim in _parse_fields(sp).get(2, []):
            d = _parse_fields(dim)
            size = d.get(1, [0])[0]
            shape.append(size - (1 << 64) if size >= 1 << 63 else size)
    if f.get(7):
        raise NotImplementedError("partitioned (sliced) variables are not on the hot path")
    return {"dtype": f.get(1, [0])[0], "shape": tuple(shape), "shard_id": f.get(3, [0])[0],
            "offset": f.get(4, [0])[0], "size": f.get(5, [0])[0], "crc32c": f.get(6, [None])[0]}


# --------------------------------------------------------------- SSTable
def _block(entries, restart_interval=16):
    """One LevelDB block (prefix-compressed, restart points)."""
    out = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _block_entries(block):
    n_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * n_restarts
    pos, key, out = 0, b"", []
    while pos < limit:
        shared, pos = _read_varint(block, pos)
        nonshared, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        key = key[:shared] + bytes(block[pos:pos + nonshared])
        pos += nonshared
        out.append((key, bytes(block[pos:pos + vlen])))
        pos += vlen
    return out


def _handle(offset, size):
    return _varint(offset) + _varint(size)


def _write_block(f, data):
    offset = f.tell()
    f.write(data)
    f.write(bytes([0]) + struct.pack("<I", mask_crc(crc32c(data + bytes([0])))))
    return offset, len(data)


def _read_block(raw, offset, size, verify=True):
    data = raw[offset:offset + size]
    ctype = raw[offset + size]
    if ctype != 0:
        raise NotImplementedError("compressed SSTable blocks (TF writes them uncompressed)")
    if verify:
        want = struct.unpack_from("<I", raw, offset + size + 1)[0]
        if unmask_crc(want) != crc32c(bytes(data) + bytes([ctype])):
            raise ValueError("checkpoint index block checksum mismatch")
    return data


def _write_sstable(path, items, block_size=256 * 1024):
    items = sorted(items, key=lambda kv: kv[0])
    with open(path, "wb") as f:
        index = []
        cur, cur_bytes = [], 0
        for k, v in items:
            cur.append((k, v))
            cur_bytes += len(k) + len(v)
            if cur_bytes >= block_size:
                index.append((cur[-1][0], _write_block(f, _block(cur))))
                cur, cur_bytes = [], 0
        if cur or not index:
            index.append((cur[-1][0] if cur else b"", _write_block(f, _block(cur))))
        meta = _write_block(f, _block([]))
        idx = _write_block(f, _block([(k, _handle(*h)) for k, h in index], restart_interval=1))
        footer = _handle(*meta) + _handle(*idx)
        footer += b"\0" * (40 - len(footer)) + struct.pack("<Q", MAGIC)
        f.write(footer)


def _read_sstable(path):
    raw = memoryview(open(path, "rb").read())
    if len(raw) < 48 or struct.unpack_from("<Q", raw, len(raw) - 8)[0] != MAGIC:
        raise ValueError(f"{path}: not a TF checkpoint index (bad SSTable magic)")
    foot = raw[len(raw) - 48:]
    _, pos = _read_varint(foot, 0)              # meta-index handle (unused)
    _, pos = _read_varint(foot, pos)
    io, pos = _read_varint(foot, pos)
    isz, pos = _read_varint(foot, pos)
    out = []
    for _, h in _block_entries(_read_block(raw, io, isz)):
        bo, p2 = _read_varint(h, 0)
        bs, _ = _read_varint(h, p2)
        out += _block_entries(_read_block(raw, bo, bs))
    return out


# --------------------------------------------------------------- bundle API
def data_path(prefix):
    return f"{prefix}.data-00000-of-00001"


def write_bundle(prefix, tensors):
    """tensors: {name: numpy array} -> <prefix>.index + <prefix>.data-00000-of-00001."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    entries = []
    offset = 0
    with open(data_path(prefix), "wb") as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            a = np.ascontiguousarray(a) if a.ndim else a.copy()      # (ascontiguousarray makes scalars 1-d)
            if a.dtype.byteorder == ">":
                a = a.astype(a.dtype.newbyteorder("<"))
            if np.dtype(a.dtype) not in DT:
                raise TypeError(f"{name}: dtype {a.dtype} has no TF checkpoint type here")
            b = a.tobytes()
            f.write(b)
            entries.append((name.encode(), _entry_proto(DT[np.dtype(a.dtype)], a.shape, offset, len(b),
                                                        mask_crc(crc32c(b)))))
            offset += len(b)
    _write_sstable(f"{prefix}.index", [(b"", _header_proto())] + entries)


def read_index(prefix):
    """{name: entry dict} of a bundle's index (header checked)."""
    items = _read_sstable(f"{prefix}.index")
    if not items or items[0][0] != b"":
        raise ValueError("checkpoint index lacks its header entry")
    hdr = _parse_fields(items[0][1])
    if hdr.get(1, [1])[0] != 1:
        raise NotImplementedError("multi-shard checkpoints")
    if hdr.get(2, [0])[0] != 0:
        raise NotImplementedError("big-endian checkpoints")
    return {k.decode(): _parse_entry(v) for k, v in items[1:]}


def read_bundle(prefix, names=None, verify=True):
    """{name: numpy array} for `names` (default: every tensor)."""
    index = read_index(prefix)
    out = {}
    with open(data_path(prefix), "rb") as f:
        for name in (names if names is not None else sorted(index)):
            e = index[name]
            f.seek(e["offset"])
            b = f.read(e["size"])
            if len(b) != e["size"]:
                raise ValueError(f"{name}: truncated checkpoint data")
            if verify and e["crc32c"] is not None and unmask_crc(e["crc32c"]) != crc32c(b):
                raise ValueError(f"{name}: checkpoint data checksum mismatch")
            if e["dtype"] == DT_BFLOAT16:
                u = np.frombuffer(b, np.uint16).astype(np.uint32) << 16
                out[name] = u.view(np.float32).reshape(e["shape"])
            else:
                out[name] = np.frombuffer(b, DT_INV[e["dtype"]]).reshape(e["shape"]).copy()
    return out


def is_bundle(prefix):
    return os.path.exists(f"{prefix}.index") and os.path.exists(data_path(prefix))
