"""Kernel time of every rank's row shard on one GPU (default CornellBox1 512², 128 spp, d8;
SCENE=<bench.py scene name> for the others): the max over ranks is what a strong-scaling
frame waits for. Usage: [SCENE=spheres] python tools/shard_balance.py world:row_block[:lanes] ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

import bench  # noqa: E402  (scene table)

SCENE = os.environ.get("SCENE", "cornellbox1")
loader, W, H, SPP0, DEPTH, _ = bench.SCENES[SCENE]
SPP = int(os.environ.get("SPP", str(SPP0)))
r = rtmi.Renderer(0)
getattr(rtmi, loader)(r, W, H)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
for arg in sys.argv[1:] or ["8:8", "8:2", "8:1"]:
    parts = [int(v) for v in arg.split(":")]
    world, block = parts[0], parts[1]
    lanes = parts[2] if len(parts) > 2 else 0
    times = []
    for rank in range(world):
        p = r.params(W, H, SPP, DEPTH, 1984, 0, block, rank, world, lanes, bench.INTEGRATOR.get(SCENE, "rayColor"))
        best = 1e9
        for _ in range(3):
            r.render_device(p, out.data_ptr(), stream)
            best = min(best, r.stats()["kernel_ms"])
        times.append(best)
    print(f"{SCENE} world {world} row_block {block} refill {r.stats()['refill']} S {r.stats()['lanes_per_pixel']} max {max(times):.3f} "
          f"min {min(times):.3f} mean {sum(times) / len(times):.3f} ranks "
          + " ".join(f"{t:.3f}" for t in times), flush=True)
