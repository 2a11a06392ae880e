"""Canvas output surface (Canvas.h): gamma quantisation, running-mean
accumulation for progressive rendering, and PPM/PNG writers.

Row convention: buffers are (height, width, 3) with row 0 = the BOTTOM image
row, as the reference stores them; writers flip vertically like
Canvas::writeToPNG (Canvas.h:141-154) and writeToPPM (:116-139).
"""
from __future__ import annotations

import json
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

    # ---- checkpoint / resume of a progressive render (an accumulation dump; the
    # reference keeps its accumulation only in device memory and loses it on exit) ----
    def save(self, path: str, rows=None):
        """The accumulation sums as a PFM (float32 RGB, bottom row first - the buffer's own row
        order) plus `<path>.json` with the sample count and rendering time; `rows` (the global
        row ids of a rank's tile) is recorded for per-rank dumps."""
        write_pfm(path, self.accumulation)
        meta = {"sampleCount": int(self.sampleCount), "renderingTime": float(self.renderingTime),
                "width": self.width, "height": self.height}
        if rows is not None:
            meta["rows"] = [int(r) for r in rows]
        with open(path + ".json", "w") as fh:
            json.dump(meta, fh)

    @classmethod
    def load(cls, path: str) -> "Canvas":
        with open(path + ".json") as fh:
            meta = json.load(fh)
        acc = read_pfm(path)
        cv = cls(acc.shape[1], acc.shape[0])
        cv.accumulation[...] = acc
        cv.sampleCount = int(meta["sampleCount"])
        cv.renderingTime = float(meta["renderingTime"])
        cv.rows = meta.get("rows")
        return cv


def write_pfm(path: str, rgb: np.ndarray):
    """Portable float map, little endian (scale -1), rows bottom to top as stored."""
    rgb = np.ascontiguousarray(rgb, "<f4")
    h, w, _ = rgb.shape
    with open(path, "wb") as fh:
        fh.write(f"PF\n{w} {h}\n-1.0\n".encode())
        fh.write(rgb.tobytes())


def read_pfm(path: str) -> np.ndarray:
    with open(path, "rb") as fh:
        if fh.readline().strip() != b"PF":
            raise ValueError(f"{path}: not an RGB PFM")
        w, h = (int(v) for v in fh.readline().split())
        scale = float(fh.readline())
        data = np.frombuffer(fh.read(), "<f4" if scale < 0 else ">f4", count=w * h * 3)
    return data.reshape(h, w, 3).astype(np.float32)


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
