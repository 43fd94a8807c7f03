"""Framebuffer writers.  The reference presents frames on screen and
never reads them back (src/raytracer.cpp:502); these write the returned framebuffer.

Frames from ``Renderer.render`` are GL-ordered (row 0 = bottom).  PPM/PNG are top-down, so
they are flipped; PFM is bottom-up by definition and is written as is.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np


def to_srgb8(rgb: np.ndarray) -> np.ndarray:
    """Quantise the shader's output (already gamma-corrected, glsl:661) to 8 bits, as the
    default framebuffer would (clamp to [0,1], round)."""
    return (np.clip(np.nan_to_num(rgb, nan=0.0), 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)


def write_ppm(path, rgb: np.ndarray):
    img = to_srgb8(rgb)[::-1]
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(f"P6\n{w} {h}\n255\n".encode())
        f.write(np.ascontiguousarray(img).tobytes())


def write_pfm(path, rgb: np.ndarray):
    img = np.ascontiguousarray(rgb, np.float32)
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())  # negative scale = little endian
        f.write(img.astype("<f4").tobytes())


def read_pfm(path) -> np.ndarray:
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3).astype(np.float32)


def write_png(path, rgb: np.ndarray):
    img = to_srgb8(rgb)[::-1]
    h, w = img.shape[:2]
    raw = b"".join(b"\x00" + np.ascontiguousarray(img[y]).tobytes() for y in range(h))

    def chunk(tag, data):
        c = struct.pack(">I", len(data)) + tag + data
        return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))
