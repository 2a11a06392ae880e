"""Diagnostic: section cycle shares and lane utilisation from an RT_STAMPS build
(tools/variants.sh stamps -DRT_STAMPS). Usage: python tools/stamps.py [cb1|bunny] [row_world] [lanes]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RTMI_LIB", "raytracingthenextweekcuda_amd/librtmi_stamps.so")
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

r = rtmi.Renderer(0)
scene = sys.argv[1] if len(sys.argv) > 1 else "cb1"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lanes = int(sys.argv[3]) if len(sys.argv) > 3 else 1
W = H = 512
(rtmi.cornell_box1 if scene == "cb1" else rtmi.bunny_cornell_box)(r, W, H)
spp = 128 if scene == "cb1" else 16
r.render(W, H, spp, 8, row_block=2, row_rank=0, row_world=world, lanes_per_pixel=lanes)
st = r.stats()
d = st["debug"]
tot = d[0] + d[1] + d[2]
names = ["regen", "closest_hit", "shade", "mesh_compact(in closest_hit)"]
print(scene, "world", world, "S", st["lanes_per_pixel"], {n: round(d[i] / tot, 4) for i, n in enumerate(names)},
      "trips", d[4], "live lane fraction", round(d[5] / (64 * d[4]), 4),
      "valid lane fraction", round(d[6] / (64 * d[4]), 4),
      "segments", st["segments"], "ms", round(st["kernel_ms"], 3), flush=True)
