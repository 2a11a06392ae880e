"""GPU BVH builder at larger sizes: random small triangles (seeded), GPU vs host
builder byte for byte through rt_commit's mesh BVH census and a render, plus the
build times. Usage: python tools/bvh_scale_check.py [n_tris ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import raytracingthenextweekcuda_amd as rtmi  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [100000, 400000]:
    rng = np.random.RandomState(n)
    c = rng.uniform(-0.4, 0.4, size=(n, 1, 3)).astype(np.float32)
    tris = (c + rng.uniform(-0.01, 0.01, size=(n, 3, 3)).astype(np.float32)).reshape(n, 9)
    tris[np.abs(tris) == 0] = 0.0  # no -0.0 (the GPU builder declines those)
    out = {}
    for builder in ("host", "gpu"):
        with rtmi.Renderer(0) as r:
            r.set_bvh_builder(builder)
            rtmi.cornell_box1(r, 64, 64, commit=False)
            r.lambertian(20, (0.6, 0.6, 0.6))
            r.mesh(20, tris, 20)
            r.commit()
            st = r.bvh_build_stats()
            img = r.render(64, 64, 2, 4)
            out[builder] = (st, r.object_counts()["bvh_node"], img)
    same = out["host"][1] == out["gpu"][1] and np.array_equal(out["host"][2], out["gpu"][2])
    print(f"{n} triangles: host {out['host'][0]['build_ms']:.1f} ms, gpu {out['gpu'][0]['build_ms']:.1f} ms "
          f"(gpu builds {out['gpu'][0]['gpu_builds']}), nodes {out['gpu'][1]}, identical render: {same}",
          flush=True)

# byte-level check through the `.bvh` image of a synthetic ASCII PLY (loadObject semantics)
import ctypes as C  # noqa: E402
import tempfile  # noqa: E402

from raytracingthenextweekcuda_amd import _lib  # noqa: E402

L = _lib.lib()
for n in [int(a) for a in sys.argv[1:]] or [100000, 400000]:
    rng = np.random.RandomState(n + 1)
    c = rng.uniform(-1.0, 1.0, size=(n, 1, 3))
    v = (c + rng.uniform(-0.02, 0.02, size=(n, 3, 3))).reshape(-1, 3)
    with tempfile.NamedTemporaryFile("w", suffix=".ply", delete=False) as fh:
        fh.write(f"ply\nformat ascii 1.0\nelement vertex {3 * n}\nproperty float x\nproperty float y\n"
                 f"property float z\nelement face {n}\nproperty list uchar int vertex_indices\nend_header\n")
        fh.write("\n".join(f"{a:.6f} {b:.6f} {d:.6f}" for a, b, d in v) + "\n")
        fh.write("\n".join(f"3 {3 * i} {3 * i + 1} {3 * i + 2}" for i in range(n)) + "\n")
        path = fh.name
    off = (C.c_float * 3)(0.0, 0.0, 0.0)
    size = C.c_int64()
    assert L.rt_ply_bvh_image(path.encode(), off, 1.0, None, 0, C.byref(size)) == 0
    host = (C.c_uint8 * size.value)()
    assert L.rt_ply_bvh_image(path.encode(), off, 1.0, host, size.value, C.byref(size)) == 0
    ms = C.c_double()
    assert L.rt_ply_bvh_image_gpu(0, path.encode(), off, 1.0, None, 0, C.byref(size), C.byref(ms)) == 0
    gpu = (C.c_uint8 * size.value)()
    assert L.rt_ply_bvh_image_gpu(0, path.encode(), off, 1.0, gpu, size.value, C.byref(size), None) == 0
    os.unlink(path)
    print(f"PLY {n} triangles: .bvh image {size.value} bytes, GPU == host byte for byte: "
          f"{bytes(host) == bytes(gpu)} (GPU build {ms.value:.1f} ms)", flush=True)
