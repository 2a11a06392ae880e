"""Offline renderer CLI: the reference's main() (main.cu:945) for one scene file.

main() reads the scene (initialize(), main.cu:623-786: YAML with the reference's
rules, or the object-list JSON of the random-spheres scene), renders one frame
with renderKernel (rayColor, or the committed pathTrace setup), and writes the
gamma-corrected image with Canvas::writeToPNG (Canvas.h:141-154, rows flipped).

    python -m raytracingthenextweekcuda_amd SCENE [--width W] [--height H] [--spp S]
        [--depth D] [--out render.png] [--devices 0,1,...] [--integrator rayColor|pathTrace]
        [--bvh host|gpu] [--seed 1984]

SCENE is a path (.yaml / .json) or one of the built-in names: cornellbox1,
spheres, bunny, media, suzanne, materialball (materialball = the committed
pathTrace configuration). Several --devices render the row tiles of one frame
in this process (rt_render_multi); the multi-process RCCL path is bench.py /
distributed.py. Prints one line with the frame time and Mrays/s.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

BUILTIN = {
    # name: (scene loader, integrator, default depth)
    "cornellbox1": ("cornell_box1", "rayColor", 8),
    "spheres": ("random_spheres", "rayColor", 10),
    "bunny": ("bunny_cornell_box", "rayColor", 8),
    "media": ("cornell_box_media", "rayColor", 16),
    "suzanne": ("suzanne_cornell_box", "rayColor", 10),
    "materialball": ("materialball", "pathTrace", 5),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="python -m raytracingthenextweekcuda_amd", description=__doc__.split("\n")[0])
    ap.add_argument("scene", help="scene file (.yaml/.json) or built-in name: " + ", ".join(sorted(BUILTIN)))
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--depth", type=int, default=None, help="bounces (default: the scene's; reference BOUNCES 10)")
    ap.add_argument("--seed", type=int, default=1984)
    ap.add_argument("--integrator", choices=["rayColor", "pathTrace"], default=None)
    ap.add_argument("--devices", default="0", help="comma-separated GPU ids; several = row tiles in one process")
    ap.add_argument("--bvh", choices=["host", "gpu"], default="gpu", help="BVH builder")
    ap.add_argument("--out", default="render.png", help=".png or .ppm")
    a = ap.parse_args(argv)
    a.devices = [int(d) for d in a.devices.split(",") if d != ""]
    if not a.devices:
        ap.error("--devices needs at least one GPU id")
    if a.width < 1 or a.height < 1 or a.spp < 1:
        ap.error("width, height and spp must be >= 1")
    if not (a.out.endswith(".png") or a.out.endswith(".ppm")):
        ap.error("--out must end in .png or .ppm")
    return a


def load(r, a):
    """Builds the scene on renderer r; returns (integrator, depth)."""
    import raytracingthenextweekcuda_amd as rtmi

    if a.scene in BUILTIN:
        loader, integrator, depth = BUILTIN[a.scene]
        getattr(rtmi, loader)(r, a.width, a.height)
    elif a.scene.endswith(".json"):
        rtmi.load_json_scene(r, a.scene, a.width, a.height)
        integrator, depth = "rayColor", 10
    else:
        rtmi.load_yaml_scene(r, a.scene, a.width, a.height)
        integrator, depth = "rayColor", 10
    return a.integrator or integrator, a.depth if a.depth is not None else depth


def main(argv=None) -> int:
    a = parse(argv)
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.canvas import Canvas

    rs = []
    try:
        for d in a.devices:
            r = rtmi.Renderer(d)
            r.set_bvh_builder(a.bvh)
            rs.append(r)
            integrator, depth = load(r, a)
        t0 = time.perf_counter()
        if len(rs) == 1:
            img = rs[0].render(a.width, a.height, a.spp, depth, seed=a.seed, lanes_per_pixel=0,
                               integrator=integrator)
        else:
            img = rtmi.render_multi(rs, a.width, a.height, a.spp, depth, seed=a.seed, row_block=2,
                                    integrator=integrator)
        dt = time.perf_counter() - t0
        segs = sum(r.stats()["segments"] for r in rs)
        canvas = Canvas(a.width, a.height)
        (canvas.writeToPNG if a.out.endswith(".png") else canvas.writeToPPM)(a.out, img)
        print(f"{a.scene}: {a.width}x{a.height}, {a.spp} spp, depth {depth}, {integrator}, "
              f"{len(rs)} device(s): {dt * 1e3:.1f} ms, {segs / dt / 1e6:.1f} Mrays/s -> {os.path.abspath(a.out)}")
        return 0
    finally:
        for r in rs:
            r.close()


if __name__ == "__main__":
    sys.exit(main())
