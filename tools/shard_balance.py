"""Kernel time of every rank's row shard on one GPU (CornellBox1 512², 128 spp, d8):
the max over ranks is what a strong-scaling frame waits for.
Usage: python tools/shard_balance.py world:row_block[:lanes] ...   (e.g. 8:8 8:2 8:1)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

W = H = 512
SPP = int(os.environ.get("SPP", "128"))
r = rtmi.Renderer(0)
rtmi.cornell_box1(r, W, H)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
for arg in sys.argv[1:] or ["8:8", "8:2", "8:1"]:
    parts = [int(v) for v in arg.split(":")]
    world, block = parts[0], parts[1]
    lanes = parts[2] if len(parts) > 2 else 0
    times = []
    for rank in range(world):
        p = r.params(W, H, SPP, 8, 1984, 0, block, rank, world, lanes)
        best = 1e9
        for _ in range(3):
            r.render_device(p, out.data_ptr(), stream)
            best = min(best, r.stats()["kernel_ms"])
        times.append(best)
    print(f"world {world} row_block {block} S {r.stats()['lanes_per_pixel']} max {max(times):.3f} "
          f"min {min(times):.3f} mean {sum(times) / len(times):.3f} ranks "
          + " ".join(f"{t:.3f}" for t in times), flush=True)
