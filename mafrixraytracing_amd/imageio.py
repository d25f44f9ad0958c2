"""Minimal PNG writer for RGBA8 frames (y-major, as Scene.Render's buffer, Scene.fs:326-329)."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def write_png(path: str, rgba_ymajor: np.ndarray, width: int, height: int) -> None:
    img = np.asarray(rgba_ymajor, dtype=np.uint8).reshape(height, width, 4)
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(height))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", width, height, 8, 6, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))
