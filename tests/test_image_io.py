"""rt_write_image (bmp.rs:8-19 / main.rs:71-74 output step): the files decode back to the
exact RGB8 pixels.  Host code, runs on CPU."""
import struct
import zlib

import numpy as np
import pytest

from rust_tracer_amd import write_image


def frame(w, h, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype = ihdr[:4]
    assert (depth, ctype) == (8, 2)
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 3 * w)
    assert not rows[:, 0].any()   # filter type 0
    return rows[:, 1:].reshape(h, w, 3)


@pytest.mark.parametrize("w,h", [(1, 1), (17, 9), (512, 300)])
def test_png_roundtrip(tmp_path, w, h):
    img = frame(w, h)
    p = tmp_path / "x.png"
    write_image(p, img)
    assert np.array_equal(read_png(p), img)


def test_bmp_and_ppm_roundtrip(tmp_path):
    img = frame(13, 7, 1)
    write_image(tmp_path / "x.ppm", img)
    d = open(tmp_path / "x.ppm", "rb").read()
    head = b"P6\n13 7\n255\n"
    assert d.startswith(head) and np.array_equal(np.frombuffer(d[len(head):], np.uint8).reshape(7, 13, 3), img)
    write_image(tmp_path / "x.bmp", img)
    b = open(tmp_path / "x.bmp", "rb").read()
    assert b[:2] == b"BM" and struct.unpack("<ii", b[18:26]) == (13, 7)
    row = (13 * 3 + 3) & ~3
    px = np.frombuffer(b[54:], np.uint8).reshape(7, row)[::-1, :39].reshape(7, 13, 3)[..., ::-1]
    assert np.array_equal(px, img)
