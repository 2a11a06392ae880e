"""Per-segment traversal counters and kernel time of the BVH scenes (bunny, spheres,
suzanne) at a reduced spp: node visits, triangle / sphere tests per segment.
Usage: python tools/traversal_stats.py [spp]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
for name, make, w, h, depth in [("bunny", rtmi.bunny_cornell_box, 1024, 1024, 8),
                                ("spheres", rtmi.random_spheres, 1280, 720, 10),
                                ("suzanne", rtmi.suzanne_cornell_box, 512, 512, 10)]:
    with rtmi.Renderer(0) as r:
        make(r, w, h)
        best = None
        for _ in range(2):
            r.render(w, h, spp, depth, lanes_per_pixel=0)
            st = r.stats()
            best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
        seg = best["segments"]
        print(f"{name} {w}x{h} spp {spp}: {best['kernel_ms']:.2f} ms, {seg / best['kernel_ms'] / 1e6:.2f} Gseg/s, "
              f"per segment: nodes {best['node_visits'] / seg:.2f} tris {best['tri_tests'] / seg:.2f} "
              f"mesh boxes {best['box_tests'] / seg:.2f} grp spheres "
              f"{(best['group_sphere_tests'] + best['group_moving_sphere_tests']) / seg:.2f}", flush=True)

# pathTrace (the reference's committed integrator): materialball through its exact BVH decisions
with rtmi.Renderer(0) as r:
    rtmi.materialball(r, 512, 512)
    best = None
    for _ in range(2):
        r.render(512, 512, spp, 5, lanes_per_pixel=0, integrator="pathTrace")
        st = r.stats()
        best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
    seg = best["segments"]
    print(f"materialball pathTrace 512x512 spp {spp}: {best['kernel_ms']:.2f} ms, "
          f"{seg / best['kernel_ms'] / 1e6:.2f} Gseg/s, per segment: nodes {best['node_visits'] / seg:.2f} "
          f"tris {best['tri_tests'] / seg:.2f}", flush=True)
