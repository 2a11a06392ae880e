"""Regenerates the radiance regression fixtures in tests/golden/radiance/ from
the CPU restatement (oracle/). They freeze the restatement's output so that any
change to it (or to the product, which must match it bit for bit) is visible;
they are NOT reference-binary outputs (the reference is unbuildable here,
DESIGN.md §2). Run from the repo root:  python tests/golden/make_radiance_fixtures.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from oracle import oracle as orc  # noqa: E402
from tests import scenes as S  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "radiance")

# name -> (builder, width, height, spp, depth)
FIXTURES = {
    # BASELINE config 1's scene at 64x64 (cb1_64x64_spp4_d4.f32)
    "cb1_64x64_spp4_d4": ("cornellbox1", 64, 64, 4, 4),
    # the committed pathTrace configuration (materialball_32x32_spp2.f32)
    "materialball_32x32_spp2_d5": ("materialball", 32, 32, 2, 5),
    # config 5's media scene
    "media_32x32_spp4_d16": ("media", 32, 32, 4, 16),
}


def render(kind, w, h, spp, depth):
    if kind == "materialball":
        cam = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox2.yaml"), S.MODELS, w, h)
        pt, _ = S.build_pathtrace_oracle("materialball")
        img, _ = pt.render(cam, w, h, spp, depth, threads=8)
        return img
    yaml_name = {"cornellbox1": "cornellbox1.yaml", "media": "cornellbox_media.yaml"}[kind]
    sc = orc.yaml_scene(os.path.join(S.SCENES, yaml_name), S.MODELS, w, h)
    img, _ = sc.render(w, h, spp, depth, threads=8)
    return img


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, args in FIXTURES.items():
        img = render(*args)
        img.astype("<f4").tofile(os.path.join(OUT, name + ".f32"))
        print(name, img.shape, float(img.mean()))


if __name__ == "__main__":
    main()
