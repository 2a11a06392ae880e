"""rocprofv3 target: four GPU builds of the config-4 bunny BVH (rt_commit with the GPU builder)."""
import os, sys
sys.path.insert(0, '/root/repo')
import torch
import raytracingthenextweekcuda_amd as rtmi
for i in range(4):
    with rtmi.Renderer(0) as r:
        r.set_bvh_builder("gpu")
        rtmi.bunny_cornell_box(r, 64, 64)
        print(r.bvh_build_stats())
