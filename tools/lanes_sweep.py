"""Kernel time of rank 0's row shard vs lanes_per_pixel (CornellBox1 512², 128 spp, d8).
Usage: python tools/lanes_sweep.py  (prints world, S, kernel ms; best of 3)"""
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
import sys as _s
combos = [tuple(int(v) for v in a.split(",")) for a in _s.argv[1:]] or [(1, 0), (2, 0), (4, 0), (8, 0)]
for world, lanes in combos:
    p = r.params(W, H, SPP, 8, 1984, 0, 8, 0, world, lanes)
    best = 1e9
    for _ in range(3):
        r.render_device(p, out.data_ptr(), stream)
        best = min(best, r.stats()["kernel_ms"])
    print(f"spp {SPP} world {world} S {lanes}->{r.stats()['lanes_per_pixel']} kernel_ms {best:.3f}", flush=True)
