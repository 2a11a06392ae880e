"""The GPU BVH builder (rt_bvh_gpu.hip) against the reference's own
`.bvh` cache files and against the host builder, byte for byte.

Golden fixtures shipped by the reference: resources/models/{bunny,dragon,materialball}
and suzanne/suzanne2.ply.bvh (tests/golden/bvh). bun_zipper (69,451 triangles) has no
reference cache; there the host builder, itself pinned by those files and by the
reference's own O(N x bins) split search (tests/test_bvh.py), is the oracle."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from raytracingthenextweekcuda_amd import _lib
from tests import scenes as S
from tests.test_bvh import bvh_image

pytestmark = pytest.mark.gpu


def gpu_bvh_image(path, offset=(0.0, 0.0, 0.0), max_coord=1.0):
    L = _lib.lib()
    size = C.c_int64()
    ms = C.c_double()
    off = (C.c_float * 3)(*offset)
    assert L.rt_ply_bvh_image_gpu(0, path.encode(), off, max_coord, None, 0, C.byref(size), C.byref(ms)) == 0
    buf = (C.c_uint8 * size.value)()
    assert L.rt_ply_bvh_image_gpu(0, path.encode(), off, max_coord, buf, size.value, C.byref(size), None) == 0
    return bytes(buf), ms.value


@pytest.mark.parametrize("model,offset,max_coord,golden", [
    ("bunny/bunny.ply", (0.0, 0.0, 0.0), 1.0, "bunny.ply.bvh"),
    ("dragon/dragon_vrip_res4.ply", (0.0, 0.0, 0.0), 1.2, "dragon_vrip_res4.ply.bvh"),
    ("materialball/materialball.ply", (0.1, 0.0, -1.0), 1.0, "materialball.ply.bvh"),
])
def test_gpu_builder_reproduces_reference_cache(model, offset, max_coord, golden):
    img, ms = gpu_bvh_image(os.path.join(S.MODELS, model), offset, max_coord)
    assert img == open(os.path.join(S.GOLDEN, "bvh", golden), "rb").read()
    assert ms > 0.0


def test_gpu_builder_equals_host_builder_bun_zipper():
    path = os.path.join(S.MODELS, "bunny", "bun_zipper.ply")
    for offset, max_coord in [((0.0, -0.15, -0.1), 0.35), ((0.0, 0.0, 0.0), 1.0)]:
        img, _ = gpu_bvh_image(path, offset, max_coord)
        assert img == bvh_image(path, offset, max_coord)
        assert struct.unpack("<II", img[:8])[1] == 69451


def test_gpu_builder_pathtrace_scene_three_files():
    # loadObject x3 + processTriangleData with the GPU builder: the reference's suzanne cache
    import raytracingthenextweekcuda_amd as rtmi

    with rtmi.Renderer(0) as r:
        r.set_bvh_builder("gpu")
        S.build_pathtrace_product(r, "suzanne")
        img = r.pathtrace_bvh_image()
        st = r.bvh_build_stats()
    assert img == open(os.path.join(S.GOLDEN, "bvh", "suzanne012.ply.bvh"), "rb").read()
    assert st["gpu_builds"] == 1


@pytest.mark.parametrize("scene", ["bunny", "spheres", "suzanne"])
def test_gpu_builder_scene_renders_identical(scene):
    # rt_commit's mesh / sphere-group BVHs from the GPU builder: same tables, same image
    import raytracingthenextweekcuda_amd as rtmi

    make = {"bunny": rtmi.bunny_cornell_box, "spheres": rtmi.random_spheres,
            "suzanne": rtmi.suzanne_cornell_box}[scene]
    w, h = 48, 32
    out = {}
    for builder in ("host", "gpu"):
        with rtmi.Renderer(0) as r:
            r.set_bvh_builder(builder)
            make(r, w, h)
            out[builder] = (r.render(w, h, 2, 6), r.object_counts(), r.stats()["node_visits"],
                            r.bvh_build_stats())
    assert np.array_equal(out["host"][0], out["gpu"][0])
    assert out["host"][1] == out["gpu"][1]
    # identical trees: the visit counts agree up to the cooperative traversal's
    # pruning order, which depends on which items share a wave (dynamic queue)
    assert abs(out["host"][2] - out["gpu"][2]) <= 1e-3 * out["gpu"][2]
    assert out["gpu"][3]["gpu_builds"] >= 1 and out["host"][3]["gpu_builds"] == 0


def test_gpu_builder_declines_negative_zero():
    # a -0.0 coordinate makes the reference's min3/max3 tie rule order-dependent: the
    # commit falls back to the host builder and says so in the stats
    import raytracingthenextweekcuda_amd as rtmi

    rng = np.random.RandomState(5)
    tris = rng.uniform(-0.4, 0.4, size=(80, 9)).astype(np.float32)
    tris[3, 1] = np.float32(-0.0)
    with rtmi.Renderer(0) as r:
        r.set_bvh_builder("gpu")
        rtmi.cornell_box1(r, 16, 16, commit=False)
        r.lambertian(20, (0.5, 0.5, 0.5))
        r.mesh(20, tris, 20)
        r.commit()
        assert r.bvh_build_stats()["gpu_builds"] == 0


def test_gpu_builder_random_ply_byte_identical(tmp_path):
    # 30k seeded random small triangles (deep, unbalanced splits): GPU == host builder
    n = 30000
    rng = np.random.RandomState(11)
    c = rng.uniform(-1.0, 1.0, size=(n, 1, 3)) * np.array([1.0, 0.2, 0.6])
    v = (c + rng.uniform(-0.02, 0.02, size=(n, 3, 3))).reshape(-1, 3)
    path = tmp_path / "random.ply"
    with open(path, "w") as fh:
        fh.write(f"ply\nformat ascii 1.0\nelement vertex {3 * n}\nproperty float x\nproperty float y\n"
                 f"property float z\nelement face {n}\nproperty list uchar int vertex_indices\nend_header\n")
        fh.write("\n".join(f"{a:.6f} {b:.6f} {d:.6f}" for a, b, d in v) + "\n")
        fh.write("\n".join(f"3 {3 * i} {3 * i + 1} {3 * i + 2}" for i in range(n)) + "\n")
    img, _ = gpu_bvh_image(str(path), (0.2, -0.1, 0.0), 0.8)
    assert img == bvh_image(str(path), (0.2, -0.1, 0.0), 0.8)
    assert struct.unpack("<II", img[:8])[1] == n
