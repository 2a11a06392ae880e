"""Diagnostic: section cycle shares from an RT_STAMPS build (tools/variants.sh stamps -DRT_STAMPS)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("RTMI_LIB", "raytracingthenextweekcuda_amd/librtmi_stamps.so")
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

r = rtmi.Renderer(0)
scene = sys.argv[1] if len(sys.argv) > 1 else "cb1"
W = H = 512
(rtmi.cornell_box1 if scene == "cb1" else rtmi.bunny_cornell_box)(r, W, H)
r.render(W, H, 16, 8, lanes_per_pixel=1)
st = r.stats()
d = st["debug"]
tot = d[0] + d[1] + d[2]
names = ["regen", "closest_hit", "shade", "mesh_compact(in closest_hit)"]
print({n: round(d[i] / tot, 4) for i, n in enumerate(names)}, "segments", st["segments"], "ms", st["kernel_ms"])
