"""Reading (and writing) the reference's `.bvh` cache files: UpdateBoundingVolumeHierarchy
(BVH.cpp:500-554) reads `<ply>.bvh` unless the PLY is newer, and writes it after a build.

The reference's own caches (tests/golden/bvh/) must load into exactly the tables a fresh
build produces: the pathTrace scene's `.bvh` image is byte-identical, and a rayColor
rt_mesh_ply scene commits to the same scene digest (objects, triangles, nodes, index maps
- so every render is the same). Cache files are untrusted input: malformed ones are
rejected and rebuilt, never read out of bounds."""
import ctypes as C
import os
import shutil
import struct

import numpy as np
import pytest

import raytracingthenextweekcuda_amd as rtmi
from tests import scenes as S

GOLD = os.path.join(S.GOLDEN, "bvh")

# golden cache -> (PLY files loaded in order, reflection types, processTriangleData offset, maxCoord)
CASES = {
    "bunny": (["bunny/bunny.ply"], ["COAT"], (0.0, 0.0, 0.0), 1.0, "bunny.ply.bvh"),
    "dragon": (["dragon/dragon_vrip_res4.ply"], ["COAT"], (0.0, 0.0, 0.0), 1.2, "dragon_vrip_res4.ply.bvh"),
    "materialball": (["materialball/materialball.ply"], ["COAT"], (0.1, 0.0, -1.0), 1.0, "materialball.ply.bvh"),
    # prepareCUDAscene's commented three-suzanne variant (main.cu:415-425): the cache is
    # named after the LAST file loaded
    "suzanne": (["suzanne/suzanne0.ply", "suzanne/suzanne1.ply", "suzanne/suzanne2.ply"],
                ["COAT", "REFRACTION", "METAL"], (0.0, 0.0, 0.0), 1.0, "suzanne012.ply.bvh"),
}


def _stage(tmp_path, case, cache_bytes=None, ply_newer=False):
    """Copies the case's PLYs into tmp_path with the golden cache next to the last one."""
    plys, _, _, _, gold = CASES[case]
    paths = []
    for rel in plys:
        dst = tmp_path / os.path.basename(rel)
        shutil.copyfile(os.path.join(S.MODELS, rel), dst)
        paths.append(str(dst))
    cache = paths[-1] + ".bvh"
    with open(cache, "wb") as fh:
        fh.write(cache_bytes if cache_bytes is not None else open(os.path.join(GOLD, gold), "rb").read())
    t = os.stat(paths[-1]).st_mtime
    os.utime(cache, (t + (-10 if ply_newer else 10), t + (-10 if ply_newer else 10)))
    return paths


def _pathtrace_image(paths, case, mode):
    _, kinds, off, mc, _ = CASES[case]
    r = rtmi.Renderer(-1)
    r.set_bvh_cache(mode)
    for p, k in zip(paths, kinds):
        r.load_object(p, k)
    r.process_triangle_data(off, mc)
    return r.pathtrace_bvh_image(), r.bvh_cache_stats()


@pytest.mark.parametrize("case", sorted(CASES))
def test_golden_cache_is_read_and_equals_a_fresh_build(tmp_path, case):
    paths = _stage(tmp_path, case)
    img, st = _pathtrace_image(paths, case, rtmi.BVH_CACHE_READ)
    assert st == {"reads": 1, "writes": 0, "rejected": 0}
    gold = open(os.path.join(GOLD, CASES[case][4]), "rb").read()
    assert img == gold
    fresh, st0 = _pathtrace_image(paths, case, rtmi.BVH_CACHE_OFF)
    assert st0["reads"] == 0 and fresh == gold


def test_stale_cache_is_rebuilt_and_rewritten(tmp_path):
    # bUpdateBVH = plyFileTime > bvhFileTime (BVH.cpp:508-514): a cache older than its PLY
    # is ignored; with WRITE the fresh build replaces it
    gold = open(os.path.join(GOLD, "bunny.ply.bvh"), "rb").read()
    corrupt = bytearray(gold)
    corrupt[8 + 12] ^= 0x40  # a node box coordinate: would render differently if read
    paths = _stage(tmp_path, "bunny", bytes(corrupt), ply_newer=True)
    img, st = _pathtrace_image(paths, "bunny", rtmi.BVH_CACHE_READ | rtmi.BVH_CACHE_WRITE)
    assert st == {"reads": 0, "writes": 1, "rejected": 0}
    assert img == gold
    assert open(paths[-1] + ".bvh", "rb").read() == gold


def _hostile(gold: bytes):
    nn, ni = struct.unpack_from("<II", gold)
    node = lambda i: 8 + 32 * i  # noqa: E731
    out = {"truncated": gold[:-4], "header_counts": struct.pack("<II", nn + 1, ni) + gold[8:],
           "index_count": struct.pack("<II", nn, ni - 1) + gold[8:-4]}
    b = bytearray(gold)
    struct.pack_into("<I", b, node(0) + 24, nn + 5)  # root's left child past the end
    out["child_out_of_range"] = bytes(b)
    b = bytearray(gold)
    struct.pack_into("<I", b, node(0) + 28, 0)  # root's right child = root (a cycle)
    out["cycle"] = bytes(b)
    b = bytearray(gold)
    idx = 8 + 32 * nn
    struct.pack_into("<i", b, idx, struct.unpack_from("<i", b, idx + 4)[0])  # a triangle listed twice
    out["not_a_permutation"] = bytes(b)
    b = bytearray(gold)
    struct.pack_into("<i", b, idx, 1 << 30)  # triangle index out of range
    out["index_out_of_range"] = bytes(b)
    b = bytearray(gold)
    for a in range(3):  # root box shrunk to a point: its triangles are outside it
        struct.pack_into("<f", b, node(0) + 4 * a, 0.0)
        struct.pack_into("<f", b, node(0) + 12 + 4 * a, 0.0)
    out["box_misses_triangles"] = bytes(b)
    b = bytearray(gold)
    leaf = next(i for i in range(nn) if struct.unpack_from("<I", gold, node(i) + 24)[0] & 0x80000000)
    struct.pack_into("<I", b, node(leaf) + 28, ni)  # leaf range starting past the list
    out["leaf_range"] = bytes(b)
    out["empty"] = b""
    return out


@pytest.mark.parametrize("kind", ["truncated", "header_counts", "index_count", "child_out_of_range", "cycle",
                                  "not_a_permutation", "index_out_of_range", "box_misses_triangles",
                                  "leaf_range", "empty"])
def test_hostile_cache_is_rejected_and_rebuilt(tmp_path, kind):
    gold = open(os.path.join(GOLD, "bunny.ply.bvh"), "rb").read()
    paths = _stage(tmp_path, "bunny", _hostile(gold)[kind])
    img, st = _pathtrace_image(paths, "bunny", rtmi.BVH_CACHE_READ)
    assert st == {"reads": 0, "writes": 0, "rejected": 1}, (kind, st)
    assert img == gold


def _ply_mesh_digest(path, off, mc, mode):
    r = rtmi.Renderer(-1)
    r.set_bvh_cache(mode)
    r.set_camera(rtmi.Camera((0, 0, 1), (0, 0, -1), (0, 1, 0), 1.0, 60.0, 0.0, 2.0))
    r.lambertian(0, (0.8, 0.8, 0.8))
    r.mesh_ply(0, path, off, mc, r.materials[0])
    r.commit()
    return r.scene_digest(), r.bvh_cache_stats(), r.object_counts()


@pytest.mark.parametrize("case", ["bunny", "dragon", "materialball"])
def test_mesh_ply_reads_the_cache_into_identical_tables(tmp_path, case):
    paths = _stage(tmp_path, case)
    _, _, off, mc, _ = CASES[case]
    d1, st1, counts = _ply_mesh_digest(paths[0], off, mc, rtmi.BVH_CACHE_READ)
    assert st1["reads"] == 1 and st1["rejected"] == 0, st1
    d0, st0, _ = _ply_mesh_digest(paths[0], off, mc, rtmi.BVH_CACHE_OFF)
    assert st0["reads"] == 0
    assert d1 == d0


def test_cache_of_another_placement_is_rejected(tmp_path):
    # the reference would read materialball's cache whatever the offset; the library
    # checks every box against the triangles it was loaded with and rebuilds instead
    paths = _stage(tmp_path, "materialball")
    d1, st1, _ = _ply_mesh_digest(paths[0], (0.0, 0.0, 0.0), 1.0, rtmi.BVH_CACHE_READ)
    assert st1 == {"reads": 0, "writes": 0, "rejected": 1}
    d0, _, _ = _ply_mesh_digest(paths[0], (0.0, 0.0, 0.0), 1.0, rtmi.BVH_CACHE_OFF)
    assert d1 == d0


@pytest.mark.gpu
def test_gpu_frames_equal_with_and_without_the_cache(tmp_path):
    paths = _stage(tmp_path, "materialball")
    frames = []
    for mode in (rtmi.BVH_CACHE_OFF, rtmi.BVH_CACHE_READ):
        with rtmi.Renderer(0) as r:
            r.set_bvh_cache(mode)
            rtmi.load_yaml_scene(r, os.path.join(S.SCENES, "cornellbox2.yaml"), 64, 64)
            r.load_object(paths[0], "COAT")
            r.process_triangle_data((0.1, 0.0, -1.0))
            frames.append(r.render(64, 64, 4, 5, integrator="pathTrace", lanes_per_pixel=0))
            assert r.bvh_cache_stats()["reads"] == (1 if mode else 0)
    assert np.array_equal(frames[0], frames[1])


def _chain_bvh(n_tris):
    """A structurally valid `.bvh` image whose tree is a chain: inner node k has a one-triangle
    leaf on the left and the rest of the chain on the right, so its depth is n_tris - 1."""
    big = 1e30
    box = struct.pack("<6f", -big, -big, -big, big, big, big)
    nodes = []
    for k in range(n_tris - 1):
        me = 2 * k
        nodes.append(box + struct.pack("<II", me + 1, me + 2))  # inner: left leaf, right chain
        nodes.append(box + struct.pack("<II", 0x80000001, k))    # leaf: triangle list entry k
    nodes.append(box + struct.pack("<II", 0x80000001, n_tris - 1))
    return struct.pack("<II", len(nodes), n_tris) + b"".join(nodes) + struct.pack(f"<{n_tris}i", *range(n_tris))


@pytest.mark.parametrize("n_tris,ok", [(32, True), (33, False), (40, False)])
def test_deep_cache_is_refused_not_launched(tmp_path, n_tris, ok):
    # the traversal keeps one pending subtree per tree level (LDS stacks sized by the depth):
    # like the reference's builder (BVH.cpp:469-496), a tree at least BVH_STACK_SIZE (32) deep is
    # refused with a clear error at process_triangle_data, here for a deep but valid cache file
    ply = tmp_path / "chain.ply"
    lines = ["ply", "format ascii 1.0", f"element vertex {3 * n_tris}", "property float x",
             "property float y", "property float z", f"element face {n_tris}",
             "property list uchar int vertex_indices", "end_header"]
    lines += [f"{k * 0.1} {y} 0" for k in range(n_tris) for y in (0.0, 1.0, 2.0)]
    lines += [f"3 {3 * k} {3 * k + 1} {3 * k + 2}" for k in range(n_tris)]
    ply.write_text("\n".join(lines) + "\n")
    cache = str(ply) + ".bvh"
    with open(cache, "wb") as fh:
        fh.write(_chain_bvh(n_tris))
    t = os.stat(ply).st_mtime
    os.utime(cache, (t + 10, t + 10))
    r = rtmi.Renderer(-1)
    r.set_bvh_cache(rtmi.BVH_CACHE_READ)
    r.load_object(str(ply), "DIFFUSE")
    if ok:
        info = r.process_triangle_data()
        assert info["depth"] == n_tris - 1 and r.bvh_cache_stats()["reads"] == 1
    else:
        with pytest.raises(rtmi.RTError, match="exceeds the traversal stack"):
            r.process_triangle_data()
