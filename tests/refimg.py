"""Comparison against images the reference itself rendered (tests/golden/ref_images/).

The reference writes `Canvas::gamma(color / spp)` as 8-bit RGB (R/Canvas.h:198-200,
`uint8(255.99 * clamp(sqrt(c), 0, 0.999))`) and `writeToPNG` flips the rows so that the
top image row is y = H-1 (R/Canvas.h:141-154). Its RNG (cuRAND XORWOW) is not the one of
this build, so pixels cannot agree bit for bit; what must agree is the expectation. The
statistic is therefore:

* the global mean per channel, in 8-bit levels, and
* the per-channel means of 16x16 pixel tiles (1,024 tiles x 3 channels), whose absolute
  differences are summarised by their median, 95th percentile and max.

Both images are Monte Carlo estimates, so the tile differences have a noise floor set by
the two sample counts; DESIGN.md §2 derives the thresholds the tests use from it.

Provenance of the fixtures (sha256 of the reference files, copied unmodified):
* cornellbox0_512x512_10bounces_1024spp.png =
  R/images/cornellbox0_512x512_10bounces_1024spp_AABB_texture_memory.png
  (2be38479b21fc0b76f9e6e33a21c9ce3f6c8f333829096d62d0dc0a63b26e8ba): rayColor over
  resources/scenes/cornellbox0.yaml, 512x512, 1024 spp, BOUNCES 10 (R/main.cu:23).
* materialball_pathtrace_512x512_32spp_5bounces.png = R/render.png
  (3defa8c1d61b25b908b2daa4733dfe94ed59887433d97c2bb0303f46cbac6d35): the committed
  main() output (R/main.cu:948), pathTrace (R/main.cu:187) with samplesPerPixel 32 and
  maxDepth 5 (R/main.cu:168-171) over materialball.ply seen by cornellbox2.yaml's camera.
"""
from __future__ import annotations

import os

import numpy as np

REF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_images")
CORNELLBOX0 = os.path.join(REF_DIR, "cornellbox0_512x512_10bounces_1024spp.png")
MATERIALBALL = os.path.join(REF_DIR, "materialball_pathtrace_512x512_32spp_5bounces.png")


def load_png(path: str) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def to_png_rows(u8_bottom_up: np.ndarray) -> np.ndarray:
    """Rows of a renderer frame (y = 0 at the bottom, the reference's convention) in
    the order writeToPNG stores them (R/Canvas.h:143-146)."""
    return np.ascontiguousarray(u8_bottom_up[::-1])


def tile_means(img: np.ndarray, tile: int = 16) -> np.ndarray:
    h, w, c = img.shape
    assert h % tile == 0 and w % tile == 0, (img.shape, tile)
    return img.astype(np.float64).reshape(h // tile, tile, w // tile, tile, c).mean(axis=(1, 3))


def compare(ours_png_rows: np.ndarray, ref: np.ndarray, tile: int = 16) -> dict:
    assert ours_png_rows.shape == ref.shape, (ours_png_rows.shape, ref.shape)
    a = ours_png_rows.astype(np.float64)
    b = ref.astype(np.float64)
    g = a.reshape(-1, 3).mean(0) - b.reshape(-1, 3).mean(0)
    d = np.abs(tile_means(a, tile) - tile_means(b, tile))
    return {
        "global_delta": [float(x) for x in g],
        "global_abs_max": float(np.max(np.abs(g))),
        "tile_median": float(np.median(d)),
        "tile_p95": float(np.percentile(d, 95)),
        "tile_max": float(d.max()),
    }
