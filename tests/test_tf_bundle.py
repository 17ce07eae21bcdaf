"""TF V2 checkpoint (tensor bundle) format, host-only: known answers of the
format's building blocks and writer/reader round trips (tf_bundle.py).
TensorFlow is not installed, so no TF-written file can be read here: the
pins are the published CRC-32C check value, the LevelDB table magic and
block layout, and the protobuf field numbers of BundleHeaderProto /
BundleEntryProto (parity beyond these is unpinned)."""
import struct

import numpy as np
import pytest

from semanticsegmentation_tensorflow_amd import tf_bundle as B


def test_crc32c_known_answers():
    assert B.crc32c(b"123456789") == 0xE3069283            # CRC-32C check value
    assert B.crc32c(b"\x00" * 32) == 0x8A9136AA              # RFC 3720 B.4 test vectors
    assert B.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert B.crc32c(bytes(range(32))) == 0x46DD794E
    data = np.random.default_rng(0).integers(0, 256, 100_003, dtype=np.uint8).tobytes()
    assert B.crc32c(data[50_000:], B.crc32c(data[:50_000])) == B.crc32c(data)     # incremental
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert B.unmask_crc(B.mask_crc(c)) == c


def test_varint_and_entry_proto():
    for v in (0, 1, 127, 128, 300, 2 ** 31, 2 ** 40 + 5):
        enc = B._varint(v)
        assert B._read_varint(enc, 0) == (v, len(enc))
    assert B._varint(300) == b"\xac\x02"
    e = B._parse_entry(B._entry_proto(1, (7, 7, 512, 4096), 123456789, 411041792, 0xDEADBEEF))
    assert e == {"dtype": 1, "shape": (7, 7, 512, 4096), "shard_id": 0, "offset": 123456789,
                 "size": 411041792, "crc32c": 0xDEADBEEF}


def test_sstable_multi_block_round_trip(tmp_path):
    items = [(f"layer{i:04d}/weights".encode(), bytes([i % 251]) * (i % 37)) for i in range(2000)]
    p = str(tmp_path / "t.index")
    B._write_sstable(p, items, block_size=4096)            # many data blocks + index entries
    raw = open(p, "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57
    assert B._read_sstable(p) == sorted(items)
    bad = bytearray(raw)
    bad[10] ^= 0xFF                                         # corrupt the first data block
    open(p, "wb").write(bytes(bad))
    with pytest.raises(ValueError, match="checksum"):
        B._read_sstable(p)


def test_bundle_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    t = {"conv1_1/weights": rng.standard_normal((3, 3, 3, 64)).astype(np.float32),
         "conv1_1/weights/Adam": rng.standard_normal((3, 3, 3, 64)).astype(np.float32),
         "global_step": np.int64(123456789012),
         "beta1_power": np.float32(0.9 ** 5),
         "scalar_f64": np.float64(1.5), "flags": np.array([True, False]),
         "half": rng.standard_normal(17).astype(np.float16)}
    prefix = str(tmp_path / "model.ckpt-5")
    B.write_bundle(prefix, t)
    assert B.is_bundle(prefix)
    idx = B.read_index(prefix)
    assert sorted(idx) == sorted(t)
    assert idx["global_step"]["dtype"] == 9 and idx["global_step"]["shape"] == ()
    back = B.read_bundle(prefix)
    for k, v in t.items():
        assert back[k].dtype == np.asarray(v).dtype and np.array_equal(back[k], np.asarray(v)), k
    # data corruption is caught by the per-tensor checksum
    d = bytearray(open(B.data_path(prefix), "rb").read())
    d[idx["conv1_1/weights"]["offset"] + 5] ^= 0x10
    open(B.data_path(prefix), "wb").write(bytes(d))
    with pytest.raises(ValueError, match="checksum"):
        B.read_bundle(prefix, ["conv1_1/weights"])
    assert np.array_equal(B.read_bundle(prefix, ["global_step"])["global_step"], t["global_step"])
