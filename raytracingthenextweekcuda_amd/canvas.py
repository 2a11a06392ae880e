"""Canvas output surface (Canvas.h): gamma quantisation, running-mean
accumulation for progressive rendering, and PPM/PNG writers.

Row convention: buffers are (height, width, 3) with row 0 = the BOTTOM image
row, as the reference stores them; writers flip vertically like
Canvas::writeToPNG (Canvas.h:141-154) and writeToPPM (:116-139).
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

from .renderer import gamma_u8


class Canvas:
    """Canvas(width, height) (Canvas.h:27-40) with float accumulation."""

    def __init__(self, width: int, height: int):
        self.width, self.height = int(width), int(height)
        self.accumulation = np.zeros((self.height, self.width, 3), np.float32)
        self.sampleCount = 0
        self.renderingTime = 0.0

    def clearAccumulationBuffer(self):
        # The reference memsets bytes to 1 (Canvas.h:163, a bug); this clears to 0.
        self.accumulation[...] = 0.0

    def resetSampleCount(self):
        self.sampleCount = 0

    def accumulate(self, mean_radiance: np.ndarray, samples: int):
        """Fold a batch rendered with `samples` spp into the running mean
        (accumulatePixel, Canvas.h:73-98, generalised to spp > 1)."""
        self.accumulation += mean_radiance.astype(np.float32) * np.float32(samples)
        self.sampleCount += samples

    def mean(self) -> np.ndarray:
        return self.accumulation / np.float32(max(self.sampleCount, 1))

    def pixels(self, radiance: np.ndarray | None = None) -> np.ndarray:
        return gamma_u8(self.mean() if radiance is None else radiance)

    def writeToPPM(self, path: str, radiance: np.ndarray | None = None):
        px = self.pixels(radiance)[::-1]
        with open(path, "w") as fh:
            fh.write(f"P3\n{self.width} {self.height}\n255\n")
            for row in px:
                for r, g, b in row:
                    fh.write(f"{r} {g} {b}\n")

    def writeToPNG(self, path: str, radiance: np.ndarray | None = None):
        write_png(path, self.pixels(radiance)[::-1])


def write_png(path: str, rgb_u8_top_down: np.ndarray):
    h, w, _ = rgb_u8_top_down.shape
    raw = b"".join(b"\x00" + np.ascontiguousarray(rgb_u8_top_down[y]).tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n")
        fh.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        fh.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        fh.write(chunk(b"IEND", b""))
