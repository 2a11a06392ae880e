"""Does overlapping consecutive frames fill the SIMDs that a launch's tail leaves idle?
Renders K frames (rank 0's shard of a world-W row tiling) back to back on one context and
stream, then rotating over n contexts on n streams, and prints ms per frame of each.
Usage: [SCENE=cornellbox1] [CTX="1 2"] [LANES=0] [FIF=1] python tools/overlap_probe.py W [K]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

import bench  # noqa: E402

SCENE = os.environ.get("SCENE", "cornellbox1")
loader, W, H, SPP, DEPTH, _ = bench.SCENES[SCENE]
world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
NCTX = [int(c) for c in os.environ.get("CTX", "1 2").split()]
rs = [rtmi.Renderer(0) for _ in range(max(NCTX))]
for r in rs:
    getattr(rtmi, loader)(r, W, H)
outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in rs]
streams = [torch.cuda.Stream() for _ in rs]
LANES = int(os.environ.get("LANES", "0"))  # sub-streams per pixel (0 = auto)
FIF = os.environ.get("FIF", "1") == "1"  # RT_RENDER_FRAMES_IN_FLIGHT, as bench.py sets it with 3 contexts
p = rs[0].params(W, H, SPP, DEPTH, 1984, 0, 2, 0, world, LANES, bench.INTEGRATOR.get(SCENE, "rayColor"),
                 frames_in_flight=FIF)


def run(n_ctx):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        i = k % n_ctx
        rs[i].render_device(p, outs[i].data_ptr(), streams[i].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / K


for n in NCTX + NCTX:
    run(n)  # warm-up of this mode
    print(f"{SCENE} world {world} lanes {LANES}: {n} context(s) {run(n):.4f} ms/frame", flush=True)
