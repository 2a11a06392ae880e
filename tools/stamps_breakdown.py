"""Section breakdown of the megakernel from the RT_STAMPS diagnostic build (wave-uniform
s_memtime stamps summed per wave; never a shipped build: rt_build_flags reports it).
  RTMI_LIB=raytracingthenextweekcuda_amd/librtmi_stamps.so python tools/stamps_breakdown.py [scene ...]
Sections (rt_kernel.hip): 7 queue refill + tail stealing, 0 camera / sample regeneration,
1 closest hit (incl. 3 = brute-force mesh compaction), 2 shading; 4 = loop trips,
5 = lanes tracing a segment, 6 = lanes owning a pixel (static grid only)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import bench  # noqa: E402
import raytracingthenextweekcuda_amd as rtmi  # noqa: E402
from raytracingthenextweekcuda_amd import _lib  # noqa: E402

assert _lib.build_flags() & _lib.BUILD_STAMPS, "needs the RT_STAMPS build (RTMI_LIB=...librtmi_stamps.so)"
for scene in sys.argv[1:] or ["cornellbox1"]:
    loader, W, H, spp, depth, _ = bench.SCENES[scene]
    with rtmi.Renderer(0) as r:
        getattr(rtmi, loader)(r, W, H)
        integ = bench.INTEGRATOR.get(scene, "rayColor")
        r.render(W, H, spp, depth, lanes_per_pixel=0, integrator=integ)
        st = r.stats()
    d = st["debug"]
    tot = d[7] + d[0] + d[1] + d[2]
    trips = max(d[4], 1)
    print(f"{scene}: kernel {st['kernel_ms']:.3f} ms, {st['segments']} segments, {d[4]} wave-trips, "
          f"{d[5] / (64 * trips):.3f} of lane-trips live")
    bvh = st["variant"] in (4, 5, 6, 7, 11)  # RT_VARIANT_BVH_*: slots 3 and 6 count the traversal loop
    for k, name in ((7, "queue+steal"), (0, "camera"), (1, "closest hit"), (3, "  of which mesh compaction"),
                    (2, "shading")):
        if bvh and k == 3:
            continue
        print(f"  {name:28s} {d[k] / tot:6.3f} of stamped cycles, {d[k] / trips:8.1f} cycles per wave-trip")
    if bvh and d[3]:
        print(f"  BVH traversal: {d[3] / trips:.1f} loop trips per wave-trip, lane utilisation "
              f"{d[6] / (64 * d[3]):.3f} (lanes with a subtree or stack entry per trip)")
