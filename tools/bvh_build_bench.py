"""BVH build time, host Recurse restatement vs the GPU builder (rt_bvh_gpu.hip), on
the BASELINE config-4 bunny (bun_zipper, 69,451 triangles, rt_commit) and the
pathTrace materialball / suzanne scenes (rt_process_triangle_data). Prints one
JSON line per scene: build-only wall ms (median of 5) and whether the trees match.
Usage: python tools/bvh_build_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402
from tests import scenes as S  # noqa: E402


def run(scene, builder):
    with rtmi.Renderer(0) as r:
        r.set_bvh_builder(builder)
        if scene == "bunny":
            rtmi.bunny_cornell_box(r, 64, 64)
            tree = r.object_counts()["bvh_node"]
        else:
            S.build_pathtrace_product(r, scene)
            tree = r.pathtrace_bvh_image()
        return r.bvh_build_stats(), tree


for scene in ("bunny", "materialball", "suzanne"):
    res = {}
    for builder in ("host", "gpu"):
        run(scene, builder)  # warm-up (page-in, HIP module load)
        ms, trees = [], []
        for _ in range(5):
            st, tree = run(scene, builder)
            assert builder == "host" or st["gpu_builds"] >= 1, st
            ms.append(st["build_ms"])
            trees.append(tree)
        res[builder] = (sorted(ms)[2], trees[0])
    print(json.dumps({"scene": scene, "host_ms": round(res["host"][0], 2), "gpu_ms": round(res["gpu"][0], 2),
                      "speedup": round(res["host"][0] / res["gpu"][0], 1),
                      "identical": res["host"][1] == res["gpu"][1]}), flush=True)
