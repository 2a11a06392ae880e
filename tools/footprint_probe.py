"""L2-footprint probe for the rayColor mesh BVH: the same Cornell box with
bun_zipper.ply (69,451 triangles, tables > 4 MiB per-XCD L2) and with the
reference's bunny.ply (smaller tables), same placement. Prints time per node visit and
per triangle test.  Usage: python tools/footprint_probe.py [spp]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402
from raytracingthenextweekcuda_amd.scene import SCENES_DIR  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
w = h = 1024
for name in ("bunny_small_cornellbox.yaml", "bunny_cornellbox.yaml"):
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, os.path.join(SCENES_DIR, name), w, h)
        c = r.object_counts()
        best = None
        for _ in range(3):
            r.render(w, h, spp, 8, lanes_per_pixel=0)
            st = r.stats()
            best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
        seg, ms = best["segments"], best["kernel_ms"]
        print(f"{name}: {c['triangle']} tris, {c['bvh_node']} nodes, tables ~{(48 * c['triangle'] + 32 * c['bvh_node'] + 8 * c['triangle']) / 2**20:.2f} MiB; "
              f"{ms:.2f} ms, {seg / ms / 1e6:.2f} Gseg/s, nodes/seg {best['node_visits'] / seg:.2f}, "
              f"tris/seg {best['tri_tests'] / seg:.2f}, ns per node visit (chip) {ms * 1e6 / best['node_visits']:.4f}",
              flush=True)
