"""Tiny image writers (PNG via zlib, PFM) for debugging and result dumps."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def tonemap(img, exposure=1.0):
    """ACES fit + gamma 2.2 (framework/system/gui/output.hlsl:58-73 display path)."""
    c = np.clip(img[..., :3] * exposure, 0, None)
    a, b, cc, d, e = 2.51, 0.03, 2.43, 0.59, 0.14
    c = (c * (a * c + b)) / (c * (cc * c + d) + e)
    return (np.clip(c, 0, 1) ** (1 / 2.2) * 255 + 0.5).astype(np.uint8)


def write_png(path, rgb8):
    """rgb8: (h, w, 3) uint8, row 0 = top."""
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def save_render(path, img_bottom_up, exposure=1.0):
    """img: (h, w, >=3) float, row 0 = image bottom (the tracer's pixel order)."""
    write_png(path, tonemap(np.asarray(img_bottom_up)[::-1], exposure))


def write_pfm(path, img_bottom_up):
    img = np.ascontiguousarray(np.asarray(img_bottom_up, np.float32)[..., :3])
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(img.astype("<f4").tobytes())  # PFM rows are bottom-to-top
