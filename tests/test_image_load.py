"""Bitmap input formats (util::BitmapTexture::Load, framework/util/texture.cpp:87-174)
through pupil_image_load (C ABI, CPU only).

Files are written here (PIL for PNG / JPEG, small writers below for EXR, Radiance
HDR and interlaced PNG) and decoded by the engine's loader; the expected values
restate the reference's mapping: stb 8-bit samples -> pow(v / 255, 2.2) RGB, v / 255
alpha for 4-channel files, 1 otherwise; tinyexr floats as stored; stbi_loadf's
RGBE -> float.  PNG / EXR / HDR are lossless, so they are checked bit for bit.
JPEG: the loader restates stb_image's integer IDCT, fixed-point YCbCr and triangle
upsampling; PIL decodes with libjpeg (other rounding), so the decoded 8-bit samples
are compared with a tolerance -- parity with stb itself is unpinned (stb is absent
from the reference tree).
"""
import ctypes as C
import struct
import zlib

import numpy as np
import pytest

from pupiloptixlab_amd import abi

PIL = pytest.importorskip("PIL.Image")


def load(path):
    lib = abi.load_library()
    w, h = C.c_uint32(), C.c_uint32()
    rc = lib.pupil_image_load(str(path).encode(), C.byref(w), C.byref(h), None)
    if rc != 0:
        return rc, None
    out = np.zeros((h.value, w.value, 4), np.float32)
    assert lib.pupil_image_load(str(path).encode(), C.byref(w), C.byref(h), out.ctypes.data_as(abi.f32p)) == 0
    return 0, out


_libm = C.CDLL("libm.so.6")
_libm.powf.restype = C.c_float
_libm.powf.argtypes = [C.c_float, C.c_float]
_POW = np.array([_libm.powf(np.float32(v) * np.float32(1.0) / np.float32(255.0), np.float32(2.2)) for v in range(256)],
                np.float32)  # std::pow(float, float) of the loader, per 8-bit value


def stb_map(samples, c):
    """texture.cpp:107-117 over stb's interleaved 8-bit samples with c channels."""
    flat = np.asarray(samples, np.uint8).reshape(-1)
    n = flat.size
    out = np.zeros((n // c, 4), np.float32)
    at = lambda i: np.where(i < n, flat[np.minimum(i, n - 1)], 0).astype(np.float32)
    base = np.arange(0, n, c)
    for k in range(3):
        out[:, k] = _POW[at(base + k).astype(np.int64)]
    out[:, 3] = at(base + 3) / np.float32(255.0) if c == 4 else np.float32(1.0)
    return out


def test_png_every_colour_type(tmp_path):
    rng = np.random.default_rng(1)
    rgba = rng.integers(0, 256, (13, 17, 4), dtype=np.uint8)
    cases = {"RGB": rgba[..., :3], "RGBA": rgba, "L": rgba[..., 0], "LA": rgba[..., :2]}
    for mode, arr in cases.items():
        p = tmp_path / f"{mode}.png"
        PIL.fromarray(arr, mode).save(p)
        rc, img = load(p)
        assert rc == 0, mode
        c = 1 if arr.ndim == 2 else arr.shape[2]
        exp = stb_map(arr.reshape(-1), c).reshape(13, 17, 4)
        assert np.array_equal(img, exp), mode  # 1/2-channel files: the reference's G/B read-ahead


def test_png_palette_transparency_16bit_and_low_depth(tmp_path):
    rng = np.random.default_rng(2)
    idx = rng.integers(0, 16, (9, 11), dtype=np.uint8)
    pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
    im = PIL.fromarray(idx, "P")
    im.putpalette(pal.reshape(-1).tolist())
    im.save(tmp_path / "p.png")
    _, img = load(tmp_path / "p.png")
    assert np.array_equal(img, stb_map(pal[idx].reshape(-1), 3).reshape(9, 11, 4))
    alpha = rng.integers(0, 256, 16, dtype=np.uint8)
    im.info["transparency"] = bytes(alpha)
    im.save(tmp_path / "pt.png", transparency=bytes(alpha))
    _, img = load(tmp_path / "pt.png")
    exp = np.concatenate([pal[idx], alpha[idx][..., None]], -1)
    assert np.array_equal(img, stb_map(exp.reshape(-1), 4).reshape(9, 11, 4))
    g16 = rng.integers(0, 65536, (7, 5), dtype=np.uint16)
    PIL.fromarray(g16).save(tmp_path / "g16.png")  # uint16 -> mode I;16
    _, img = load(tmp_path / "g16.png")
    assert np.array_equal(img, stb_map((g16 >> 8).astype(np.uint8).reshape(-1), 1).reshape(7, 5, 4))
    bits = rng.integers(0, 2, (6, 21), dtype=np.uint8).astype(bool)
    PIL.fromarray(bits).save(tmp_path / "b1.png")
    _, img = load(tmp_path / "b1.png")
    assert np.array_equal(img, stb_map((bits * 255).astype(np.uint8).reshape(-1), 1).reshape(6, 21, 4))


def _png_chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def write_png_adam7_rgba(path, arr):
    """RGBA8 PNG with Adam7 interlacing (filter type chosen per row, all five used)."""
    h, w, _ = arr.shape
    raw = bytearray()
    passes = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
    row_no = 0
    for xo, yo, xs, ys in passes:
        sub = arr[yo::ys, xo::xs]
        if sub.size == 0:
            continue
        prev = np.zeros(sub.shape[1] * 4, np.int32)
        for y in range(sub.shape[0]):
            cur = sub[y].reshape(-1).astype(np.int32)
            ft = row_no % 5
            row_no += 1
            a = np.concatenate([np.zeros(4, np.int32), cur[:-4]])
            c = np.concatenate([np.zeros(4, np.int32), prev[:-4]])
            if ft == 0:
                enc = cur
            elif ft == 1:
                enc = cur - a
            elif ft == 2:
                enc = cur - prev
            elif ft == 3:
                enc = cur - ((a + prev) >> 1)
            else:
                p = a + prev - c
                pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - c)
                pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, c))
                enc = cur - pred
            raw += bytes([ft]) + bytes((enc & 0xFF).astype(np.uint8))
            prev = cur
    data = b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 1))
    data += _png_chunk(b"IDAT", zlib.compress(bytes(raw))) + _png_chunk(b"IEND", b"")
    path.write_bytes(data)


def test_png_adam7_and_all_filters(tmp_path):
    arr = np.random.default_rng(3).integers(0, 256, (19, 23, 4), dtype=np.uint8)
    write_png_adam7_rgba(tmp_path / "i.png", arr)
    rc, img = load(tmp_path / "i.png")
    assert rc == 0
    assert np.array_equal(img, stb_map(arr.reshape(-1), 4).reshape(19, 23, 4))


def half(x):
    return np.asarray(x, np.float16)


def write_exr(path, channels, w, h, compression=0, extra_header=b""):
    """Single-part scanline EXR; channels: {name: array (h, w) float16 or float32}."""
    names = sorted(channels)
    hdr = bytearray(b"\x76\x2f\x31\x01" + struct.pack("<I", 2))

    def attr(name, typ, payload):
        hdr.extend(name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(payload)) + payload)

    chl = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", 1 if channels[n].dtype == np.float16 else 2, 0, 1, 1)
                   for n in names) + b"\0"
    attr("channels", "chlist", chl)
    attr("compression", "compression", bytes([compression]))
    attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    attr("lineOrder", "lineOrder", b"\0")
    attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0))
    attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    hdr.extend(extra_header)
    hdr.extend(b"\0")
    lines = 16 if compression == 3 else 1
    chunks = []
    for y0 in range(0, h, lines):
        raw = b"".join(channels[n][y].astype(channels[n].dtype).tobytes() for y in range(y0, min(h, y0 + lines))
                       for n in names)
        if compression in (1, 2, 3):
            b = np.frombuffer(raw, np.uint8)
            inter = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
            pred = inter.copy()
            pred[1:] = (inter[1:] - inter[:-1] + 128) & 0xFF
            pred = pred.astype(np.uint8).tobytes()
            if compression == 1:
                enc = bytearray()
                i = 0
                while i < len(pred):  # OpenEXR RLE: runs of 3+ equal bytes, else literals
                    j = i
                    while j + 1 < len(pred) and pred[j + 1] == pred[i] and j - i < 126:
                        j += 1
                    if j - i >= 2:
                        enc += bytes([j - i, pred[i]])
                        i = j + 1
                    else:
                        k = i
                        while k < len(pred) and k - i < 127 and not (k + 2 < len(pred) and pred[k] == pred[k + 1] == pred[k + 2]):
                            k += 1
                        k = max(k, i + 1)
                        enc += bytes([(256 - (k - i)) & 0xFF]) + pred[i:k]
                        i = k
                payload = bytes(enc)
            else:
                payload = zlib.compress(pred)
            if len(payload) >= len(raw):
                payload = raw
        else:
            payload = raw
        chunks.append(struct.pack("<ii", y0, len(payload)) + payload)
    off = len(hdr) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    path.write_bytes(bytes(hdr) + table + b"".join(chunks))


@pytest.mark.parametrize("compression", [0, 1, 2, 3])
def test_exr_channels_types_and_compressions(tmp_path, compression):
    rng = np.random.default_rng(4 + compression)
    w, h = 37, 21
    r = rng.normal(size=(h, w)).astype(np.float32) * 10
    g = half(rng.uniform(0, 4, (h, w)))
    b = half(np.round(rng.uniform(0, 3, (h, w))))  # runs for RLE
    a = rng.uniform(0, 1, (h, w)).astype(np.float32)
    write_exr(tmp_path / "rgba.exr", {"R": r, "G": g, "B": b, "A": a}, w, h, compression)
    rc, img = load(tmp_path / "rgba.exr")
    assert rc == 0
    exp = np.stack([r, g.astype(np.float32), b.astype(np.float32), a], -1)
    assert np.array_equal(img.view(np.uint32), exp.view(np.uint32))
    write_exr(tmp_path / "rgb.exr", {"R": r, "G": g, "B": b}, w, h, compression)
    _, img = load(tmp_path / "rgb.exr")
    assert np.array_equal(img[..., 3], np.ones((h, w), np.float32))
    write_exr(tmp_path / "y.exr", {"Y": g}, w, h, compression)  # tinyexr: one channel -> R = G = B = A
    _, img = load(tmp_path / "y.exr")
    assert np.array_equal(img, np.repeat(g.astype(np.float32)[..., None], 4, -1))


def test_exr_rejections(tmp_path):
    w, h = 4, 4
    z = np.zeros((h, w), np.float32)
    write_exr(tmp_path / "piz.exr", {"R": z, "G": z, "B": z}, w, h, compression=4)
    assert load(tmp_path / "piz.exr")[0] == abi.ERR_IO
    write_exr(tmp_path / "noR.exr", {"X": z, "G": z, "B": z}, w, h)
    assert load(tmp_path / "noR.exr")[0] == abi.ERR_IO
    # the extension decides (texture.cpp:166-170): an EXR named .png is not decoded as EXR
    (tmp_path / "x.png").write_bytes((tmp_path / "noR.exr").read_bytes())
    assert load(tmp_path / "x.png")[0] == abi.ERR_IO


def test_exr_corrupt_files_fail_cleanly(tmp_path):
    """Untrusted texture files (scene XML names them): a chunk offset near 2^64, a chunk
    size running past the end, an attribute name without its terminator and a data
    window that overflows 32 bits are rejected with PUPIL_ERR_IO, never read past the
    buffer (the offset arithmetic used to wrap, and names were read up to any NUL)."""
    w, h = 4, 3
    z = np.zeros((h, w), np.float32)
    write_exr(tmp_path / "ok.exr", {"R": z, "G": z, "B": z}, w, h)
    good = bytearray((tmp_path / "ok.exr").read_bytes())
    assert load(tmp_path / "ok.exr")[0] == 0
    # the offset table follows the header's terminating NUL: find the first chunk offset
    first_off = len(good) - h * (8 + 3 * 4 * w)
    at = good.index(struct.pack("<Q", first_off))
    for bad_off in (2 ** 64 - 4, 2 ** 64 - 16, len(good) - 4):
        b = bytearray(good)
        b[at:at + 8] = struct.pack("<Q", bad_off)
        (tmp_path / "off.exr").write_bytes(bytes(b))
        assert load(tmp_path / "off.exr")[0] == abi.ERR_IO, bad_off
    b = bytearray(good)  # chunk size field: 2^31 - 1 bytes
    b[first_off + 4:first_off + 8] = struct.pack("<i", 2 ** 31 - 1)
    (tmp_path / "size.exr").write_bytes(bytes(b))
    assert load(tmp_path / "size.exr")[0] == abi.ERR_IO
    # header cut inside an attribute name (no NUL before the end of the file)
    (tmp_path / "name.exr").write_bytes(bytes(good[:8]) + b"channelsXXXXXXXXXXXXXXXXXXXXXXXXXXXX")
    assert load(tmp_path / "name.exr")[0] == abi.ERR_IO
    # data window spanning more than 2^31 columns
    b = bytearray(good)
    dwa = b.index(b"dataWindow\0box2i\0") + len(b"dataWindow\0box2i\0") + 4
    b[dwa:dwa + 16] = struct.pack("<iiii", -2 ** 31, 0, 2 ** 31 - 1, h - 1)
    (tmp_path / "dw.exr").write_bytes(bytes(b))
    assert load(tmp_path / "dw.exr")[0] == abi.ERR_IO
    for n in range(8, len(good), 7):  # every truncation fails cleanly
        (tmp_path / "cut.exr").write_bytes(bytes(good[:n]))
        assert load(tmp_path / "cut.exr")[0] == abi.ERR_IO, n


def test_jpeg_sampling_factors_must_divide_the_maxima(tmp_path):
    """stb_image rejects a component whose sampling factor does not divide the largest
    one ("bad H" / "bad V"); the decoder must too (its resampler would read past the
    component's rows)."""
    arr = np.random.default_rng(3).integers(0, 256, (32, 32, 3), dtype=np.uint8)
    PIL.fromarray(arr, "RGB").save(tmp_path / "a.jpg", quality=90, subsampling=2)
    data = bytearray((tmp_path / "a.jpg").read_bytes())
    assert load(tmp_path / "a.jpg")[0] == 0
    sof = data.index(b"\xff\xc0")
    comps = sof + 2 + 2 + 1 + 2 + 2 + 1  # marker, length, precision, height, width, count
    for y_hv, c_hv in ((0x41, 0x31), (0x14, 0x13), (0x44, 0x33)):
        b = bytearray(data)
        b[comps + 1] = y_hv      # Y: h, v
        b[comps + 3 + 1] = c_hv  # Cb: a factor that does not divide Y's
        (tmp_path / "bad.jpg").write_bytes(bytes(b))
        assert load(tmp_path / "bad.jpg")[0] == abi.ERR_IO, hex(c_hv)


def write_hdr(path, rgbe, rle=True):
    h, w, _ = rgbe.shape
    out = bytearray(b"#?RADIANCE\n# made by the test\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode())
    for y in range(h):
        if not rle:
            out += rgbe[y].tobytes()
            continue
        out += bytes([2, 2, w >> 8, w & 0xFF])
        for k in range(4):
            row = rgbe[y, :, k]
            i = 0
            while i < w:
                j = i
                while j + 1 < w and row[j + 1] == row[i] and j - i < 126:
                    j += 1
                if j - i >= 2:
                    out += bytes([128 + j - i + 1, row[i]])
                    i = j + 1
                else:
                    k2 = min(w, i + 128)
                    n = min(k2 - i, 2) if j > i else 1
                    n = max(1, min(128, n))
                    out += bytes([n]) + bytes(row[i:i + n])
                    i += n
    path.write_bytes(bytes(out))


@pytest.mark.parametrize("rle", [True, False])
def test_radiance_hdr(tmp_path, rle):
    rng = np.random.default_rng(7)
    h, w = 9, 40
    rgbe = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    rgbe[..., 3] = rng.integers(100, 160, (h, w))
    rgbe[2, :, :] = [200, 10, 10, 130]  # runs
    rgbe[3, 5:9, 3] = 0  # exponent 0 -> black
    write_hdr(tmp_path / "e.hdr", rgbe, rle)
    rc, img = load(tmp_path / "e.hdr")
    assert rc == 0
    f1 = np.ldexp(np.float32(1.0), rgbe[..., 3].astype(np.int32) - 136).astype(np.float32)
    exp = np.where(rgbe[..., 3:4] != 0, rgbe[..., :3].astype(np.float32) * f1[..., None], 0).astype(np.float32)
    assert np.array_equal(img[..., :3], exp)
    assert np.all(img[..., 3] == 1.0)


@pytest.mark.parametrize("subsampling", [0, 1, 2])
def test_jpeg_baseline_close_to_libjpeg(tmp_path, subsampling):
    """4:4:4 / 4:2:2 / 4:2:0 baseline JPEG: within 3 levels of libjpeg (PIL) everywhere,
    and a flat-colour image decodes to its exact value."""
    y, x = np.mgrid[0:48, 0:64]
    arr = np.stack([x * 4, y * 5, (x + y) * 2], -1).clip(0, 255).astype(np.uint8)
    PIL.fromarray(arr, "RGB").save(tmp_path / "a.jpg", quality=92, subsampling=subsampling)
    rc, img = load(tmp_path / "a.jpg")
    assert rc == 0
    ref = np.asarray(PIL.open(tmp_path / "a.jpg").convert("RGB")).astype(np.float32)
    ours = np.round(np.power(img[..., :3].astype(np.float64), 1 / 2.2) * 255)
    assert np.abs(ours - ref).max() <= 3
    flat = np.full((16, 24, 3), (90, 150, 30), np.uint8)
    PIL.fromarray(flat, "RGB").save(tmp_path / "f.jpg", quality=100, subsampling=0)
    _, img = load(tmp_path / "f.jpg")
    ref = np.asarray(PIL.open(tmp_path / "f.jpg").convert("RGB"))
    assert np.array_equal(img, stb_map(ref.reshape(-1), 3).reshape(16, 24, 4))


def test_jpeg_grayscale_restart_and_progressive(tmp_path):
    g = (np.add.outer(np.arange(40), np.arange(56)) * 2).clip(0, 255).astype(np.uint8)
    PIL.fromarray(g, "L").save(tmp_path / "g.jpg", quality=90)
    rc, img = load(tmp_path / "g.jpg")
    assert rc == 0
    ref = np.asarray(PIL.open(tmp_path / "g.jpg")).astype(np.float64)
    ours = np.round(np.power(img[..., 0].astype(np.float64), 1 / 2.2) * 255)
    assert np.abs(ours - ref).max() <= 2
    arr = np.random.default_rng(5).integers(0, 256, (32, 48, 3), dtype=np.uint8)
    PIL.fromarray(arr, "RGB").save(tmp_path / "r.jpg", quality=85, restart_marker_blocks=1)
    rc, img = load(tmp_path / "r.jpg")
    assert rc == 0
    ref = np.asarray(PIL.open(tmp_path / "r.jpg").convert("RGB")).astype(np.float64)
    ours = np.round(np.power(img[..., :3].astype(np.float64), 1 / 2.2) * 255)
    assert np.abs(ours - ref).max() <= 4
    PIL.fromarray(arr, "RGB").save(tmp_path / "p.jpg", progressive=True)
    assert load(tmp_path / "p.jpg")[0] == abi.ERR_IO


def test_bitmap_and_envmap_scene_use_the_loaders(tmp_path):
    """A scene's <texture type="bitmap"> (PNG) and <emitter type="envmap"> (EXR) are
    decoded by these loaders into the scene description."""
    from pupiloptixlab_amd import World

    tex = np.random.default_rng(8).integers(0, 256, (8, 8, 3), dtype=np.uint8)
    PIL.fromarray(tex, "RGB").save(tmp_path / "t.png")
    env = np.random.default_rng(9).uniform(0, 2, (6, 12)).astype(np.float32)
    write_exr(tmp_path / "env.exr", {"R": env, "G": env * 0.5, "B": env * 0.25}, 12, 6, 3)
    (tmp_path / "s.xml").write_text(
        '<scene><integrator type="path"><integer name="max_depth" value="3"/></integrator>'
        '<sensor type="perspective"><float name="fov" value="45"/><film type="hdrfilm">'
        '<integer name="width" value="16"/><integer name="height" value="16"/></film></sensor>'
        '<shape type="rectangle"><bsdf type="diffuse"><texture type="bitmap" name="reflectance">'
        '<string name="filename" value="t.png"/></texture></bsdf></shape>'
        '<emitter type="envmap"><string name="filename" value="env.exr"/></emitter></scene>')
    d = World().load_scene(str(tmp_path / "s.xml")).desc()
    m = d.materials[d.instances[0].material]
    t = m.tex[0]
    assert t.type == abi.TEX_BITMAP and (t.width, t.height) == (8, 8)
    got = np.ctypeslib.as_array(t.rgba, (8 * 8 * 4,)).reshape(8, 8, 4)
    assert np.array_equal(got, stb_map(tex.reshape(-1), 3).reshape(8, 8, 4))
    e = d.env.contents.radiance
    assert e.type == abi.TEX_BITMAP and (e.width, e.height) == (12, 6)
    got = np.ctypeslib.as_array(e.rgba, (12 * 6 * 4,)).reshape(6, 12, 4)
    assert np.array_equal(got[..., 0], env) and np.array_equal(got[..., 2], env * np.float32(0.25))
