"""pupil_image_save: EXR / HDR / PFM writers (util::BitmapTexture::Save,
framework/util/texture.cpp:12-85) read back with independent minimal parsers."""
import ctypes as C
import os
import struct

import numpy as np

from pupiloptixlab_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = os.path.join(ROOT, "gpurun_out", "test_images")


def _image(w=13, h=7, seed=0):
    rng = np.random.default_rng(seed)
    img = rng.uniform(0.0, 4.0, (h * w, 4)).astype(np.float32)
    img[:, 3] = 1.0
    img[3] = 0.0  # a black pixel
    return img


def _save(path, img, w, h, fmt=0):
    lib = abi.load_library()
    return lib.pupil_image_save(path.encode(), w, h, np.ascontiguousarray(img).ctypes.data_as(abi.f32p), fmt)


def read_exr(path):
    """Uncompressed scanline EXR reader (just enough for our writer)."""
    b = open(path, "rb").read()
    assert b[:4] == bytes([0x76, 0x2F, 0x31, 0x01]) and struct.unpack_from("<i", b, 4)[0] == 2
    pos, attrs = 8, {}
    while b[pos] != 0:
        name_end = b.index(b"\0", pos)
        name = b[pos:name_end].decode()
        type_end = b.index(b"\0", name_end + 1)
        typ = b[name_end + 1:type_end].decode()
        size = struct.unpack_from("<i", b, type_end + 1)[0]
        attrs[name] = (typ, b[type_end + 5:type_end + 5 + size])
        pos = type_end + 5 + size
    pos += 1
    chans, p = [], 0
    raw = attrs["channels"][1]
    while raw[p] != 0:
        e = raw.index(b"\0", p)
        chans.append((raw[p:e].decode(), struct.unpack_from("<i", raw, e + 1)[0]))
        p = e + 1 + 16
    assert attrs["compression"][1] == b"\0"
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    offsets = struct.unpack_from(f"<{h}Q", b, pos)
    out = {c: np.zeros((h, w), np.float32) for c, _ in chans}
    for r, off in enumerate(offsets):
        y, n = struct.unpack_from("<ii", b, off)
        assert n == 4 * w * len(chans)
        data = np.frombuffer(b, "<f4", w * len(chans), off + 8).reshape(len(chans), w)
        for k, (c, t) in enumerate(chans):
            assert t == 2  # FLOAT
            out[c][y] = data[k]
    return [c for c, _ in chans], out


def test_exr_roundtrip_bgr_and_top_row_first():
    os.makedirs(TMP, exist_ok=True)
    w, h = 13, 7
    img = _image(w, h)
    path = os.path.join(TMP, "t.exr")
    assert _save(path, img, w, h) == abi.OK
    names, ch = read_exr(path)
    assert names == ["B", "G", "R"]  # texture.cpp:57-63
    rgb = img.reshape(h, w, 4)[::-1]  # file line 0 = image top = buffer row h-1
    for k, c in enumerate("RGB"):
        assert np.array_equal(ch[c], rgb[..., k])


def test_pfm_and_hdr():
    w, h = 13, 7
    img = _image(w, h, 1)
    p = os.path.join(TMP, "t.pfm")
    assert _save(p, img, w, h) == abi.OK
    with open(p, "rb") as f:
        assert f.readline() == b"PF\n" and f.readline().split() == [b"13", b"7"] and float(f.readline()) < 0
        data = np.frombuffer(f.read(), "<f4").reshape(h * w, 3)
    assert np.array_equal(data, img[:, :3])
    p = os.path.join(TMP, "t.hdr")
    assert _save(p, img, w, h) == abi.OK
    b = open(p, "rb").read()
    head = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 7 +X 13\n"
    assert b.startswith(head)
    rgbe = np.frombuffer(b[len(head):], np.uint8).reshape(h, w, 4).astype(np.float64)
    dec = rgbe[..., :3] * np.ldexp(1.0, (rgbe[..., 3:4] - 136).astype(int))
    dec[rgbe[..., 3] == 0] = 0.0
    ref = img.reshape(h, w, 4)[::-1, :, :3]
    # RGBE keeps 8 bits relative to the pixel's largest component
    tol = ref.max(axis=2, keepdims=True) / 128.0 + 1e-6
    assert (np.abs(dec - ref) <= tol).all()


def test_bad_format_and_args():
    img = _image()
    assert _save(os.path.join(TMP, "t.png"), img, 13, 7) == abi.ERR_UNSUPPORTED
    lib = abi.load_library()
    assert lib.pupil_image_save(None, 1, 1, None, 0) == abi.ERR_INVALID
