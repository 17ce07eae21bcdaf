"""seg_png_decode (host, no GPU) against PIL: PIL-encoded PNGs of every
8-bit colour type and hand-filtered PNGs with each row filter (PNG spec 9.2)."""
import io
import struct
import zlib

import numpy as np
import pytest

from semanticsegmentation_tensorflow_amd import data

Image = pytest.importorskip("PIL.Image")


def _pil_png(a, mode):
    b = io.BytesIO()
    Image.fromarray(a, mode).save(b, "PNG")
    return b.getvalue()


@pytest.mark.parametrize("mode,c", [("RGB", 3), ("RGBA", 4), ("L", 1), ("LA", 2)])
def test_decode_matches_pil(mode, c):
    rng = np.random.default_rng(c)
    yy, xx = np.mgrid[0:37, 0:91]
    a = ((xx * 3 + yy * 5)[..., None] + rng.integers(0, 20, (37, 91, c))).astype(np.uint8)
    a = a[..., 0] if c == 1 else a
    png = _pil_png(a, mode)
    got = data.png_decode(png)
    want = np.asarray(Image.open(io.BytesIO(png)))
    assert np.array_equal(got.reshape(want.shape), want)


def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _filter_row(f, cur, prev, bpp):
    out = bytearray(len(cur))
    for i in range(len(cur)):
        a = cur[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        if f == 0:
            p = 0
        elif f == 1:
            p = a
        elif f == 2:
            p = b
        elif f == 3:
            p = (a + b) >> 1
        else:
            pp = a + b - c
            pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (cur[i] - p) & 0xFF
    return bytes([f]) + bytes(out)


def test_every_row_filter():
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (11, 9, 4), dtype=np.uint8)
    rows = [a[y].tobytes() for y in range(11)]
    raw = b"".join(_filter_row(y % 5, rows[y], rows[y - 1] if y else None, 4) for y in range(11))
    z = zlib.compress(raw, 9)
    png = (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", 9, 11, 8, 6, 0, 0, 0))
           + _chunk(b"IDAT", z[:7]) + _chunk(b"IDAT", z[7:]) + _chunk(b"IEND", b""))
    assert np.array_equal(data.png_decode(png), a)
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(png))), a)


def test_unsupported_falls_back(tmp_path):
    pal = Image.fromarray(np.arange(60, dtype=np.uint8).reshape(6, 10), "L").convert("P")
    p = tmp_path / "p.png"
    pal.save(p)
    assert data.png_decode(p.read_bytes()) is None          # palette: not the native path
    got = data.imread(str(p))
    assert np.array_equal(got, np.asarray(pal.convert("RGB")))
    assert data.png_decode(b"not a png") is None
