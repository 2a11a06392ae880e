"""pathTrace integrator (CUDAPathTracer.cu:358-622, the committed call of
renderKernel at main.cu:187) over the PLY scenes of prepareCUDAscene.

CPU tests pin the scene preparation against the reference's own `.bvh` cache
files (byte-identical: PLY loading, index offsets across several loadObject
calls, processTriangleData, the SAH builder) and check the oracle's math
helpers. GPU tests compare the HIP kernel with the oracle, which traverses the
reference's cache files as BVH_IntersectTriangles does (full DFS, strict `<`).
"""
import math
import os
import struct

import numpy as np
import pytest

from tests import scenes as S

# north_star: image within 1e-4 per-channel L-infinity of the reference.
TOL = 1e-4


def _product(device=-1):
    import raytracingthenextweekcuda_amd as rtmi

    return rtmi.Renderer(device)


@pytest.mark.parametrize("name", sorted(S.PT_SCENES))
def test_pathtrace_scene_bvh_matches_reference_cache(name):
    r = _product()
    info = S.build_pathtrace_product(r, name)
    img = r.pathtrace_bvh_image()
    golden = open(os.path.join(S.GOLDEN, "bvh", S.PT_SCENES[name][2]), "rb").read()
    assert img == golden
    nn, ni = struct.unpack("<II", golden[:8])
    assert (info["bvh_nodes"], info["tri_list"]) == (nn, ni)
    assert info["depth"] < 32  # fits BVH_STACK_SIZE (CUDAPathTracer.cu:43)
    r.close()


def test_load_object_offsets_indices_across_files():
    # three loadObject calls: counts add up (Loader.cpp:228, 282-284)
    r = _product()
    counts = []
    for path, kind in S.PT_SCENES["suzanne"][0]:
        r.load_object(os.path.join(S.MODELS, path), kind)
        counts.append(r.process_triangle_data()["triangles"])
    assert counts[0] < counts[1] < counts[2] == 6902
    r.close()


def test_load_object_errors():
    import raytracingthenextweekcuda_amd as rtmi

    r = _product()
    with pytest.raises(rtmi.RTError, match="RT_ERR_IO"):
        r.load_object("/nonexistent.ply", "COAT")
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.load_object(os.path.join(S.MODELS, "bunny", "bunny.ply"), 7)
    with pytest.raises(rtmi.RTError, match="RT_ERR_STATE"):
        r.pathtrace_bvh_image()
    r.close()


def test_oracle_sin_cos_pow_accuracy():
    from oracle import oracle as orc

    L = orc.lib()
    rng = np.random.RandomState(3)
    xs = np.concatenate([rng.uniform(0, 2 * math.pi, 4000), [0.0, 1e-8, math.pi / 4, math.pi / 2,
                                                             math.pi, 2 * math.pi]]).astype(np.float32)
    for x in xs:
        x = float(x)
        for f, ref in ((L.orc_pt_sinf, math.sin), (L.orc_pt_cosf, math.cos)):
            got, exact = f(x), ref(x)
            assert abs(got - exact) <= max(abs(exact), 1e-30) * 2 ** -23 + 1e-45, (f, x)
    for x in rng.uniform(0, 1, 4000).astype(np.float32):
        y = np.float32(1.0) / np.float32(21.0)
        got, exact = L.orc_pt_powf(float(x), float(y)), float(x) ** float(y)
        assert abs(got - exact) <= exact * 2 ** -23, x
    assert L.orc_pt_powf(0.0, float(np.float32(1 / 21))) == 0.0
    assert L.orc_pt_powf(1.0, 0.5) == 1.0


def test_oracle_rejects_malformed_bvh():
    pt, _ = S.build_pathtrace_oracle("bunny")
    with pytest.raises(ValueError):
        pt.set_bvh(b"\x01\x00\x00\x00\x00\x00\x00\x00")
    golden = open(os.path.join(S.GOLDEN, "bvh", "materialball.ply.bvh"), "rb").read()
    with pytest.raises(ValueError):  # indices beyond the bunny's triangles
        pt.set_bvh(golden)


def test_oracle_materialball_known_properties():
    pt, cam = S.build_pathtrace_oracle("materialball")
    img, st = pt.render(cam, 16, 16, 2, 5, threads=4)
    assert np.isfinite(img).all() and (img >= 0).all()
    assert st["overflow"] == 0
    # every path runs 5 segments unless it escapes (returns black) first
    assert st["segments"] <= 16 * 16 * 2 * 5
    # the ball (orange 0.9, 0.3, 0 albedo, COAT) fills the frame centre
    c = img[6:10, 6:10].mean(axis=(0, 1))
    assert c[0] > c[1] > c[2]


# ------------------------------ GPU parity ------------------------------
def _gpu_render(name, w, h, spp, bounces=5, **kw):
    r = _product(0)
    S.build_pathtrace_product(r, name)
    img = r.render(w, h, spp, bounces, integrator="pathTrace", **kw)
    st = r.stats()
    r.close()
    return img, st


def _assert_parity(a, b):
    assert a.shape == b.shape
    err = float(np.abs(a - b).max())
    assert err <= TOL, f"L-inf {err}, {(np.abs(a - b) > TOL).sum()} channels over"


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,spp", [("materialball", 40, 32, 4), ("suzanne", 32, 32, 4),
                                          ("bunny", 24, 24, 3)])
def test_gpu_pathtrace_parity(name, w, h, spp):
    pt, cam = S.build_pathtrace_oracle(name)
    want, ost = pt.render(cam, w, h, spp, 5, threads=8)
    got, st = _gpu_render(name, w, h, spp)
    _assert_parity(got, want)
    assert st["segments"] == ost["segments"]
    assert st["overflow"] == 0


@pytest.mark.gpu
def test_gpu_pathtrace_lanes_and_rows():
    pt, cam = S.build_pathtrace_oracle("materialball")
    want, _ = pt.render(cam, 32, 24, 8, 5, row_block=4, row_rank=1, row_world=3, threads=8,
                        lanes_per_pixel=4)
    got, _ = _gpu_render("materialball", 32, 24, 8, row_block=4, row_rank=1, row_world=3,
                         lanes_per_pixel=4)
    _assert_parity(got, want)


@pytest.mark.gpu
def test_gpu_pathtrace_bounce_count_and_seed():
    pt, cam = S.build_pathtrace_oracle("suzanne")
    for bounces, seed in ((1, 7), (8, 1984)):
        want, _ = pt.render(cam, 16, 16, 2, bounces, seed=seed, threads=8)
        got, _ = _gpu_render("suzanne", 16, 16, 2, bounces, seed=seed)
        _assert_parity(got, want)


@pytest.mark.gpu
def test_gpu_pathtrace_requires_processed_scene():
    import raytracingthenextweekcuda_amd as rtmi

    r = _product(0)
    r.set_camera(rtmi.Camera(*S.PT_CAMERA))
    with pytest.raises(rtmi.RTError, match="RT_ERR_STATE"):
        r.render(8, 8, 1, 5, integrator="pathTrace")
    r.process_triangle_data()  # spheres only: no triangles
    img = r.render(8, 8, 1, 5, integrator="pathTrace")
    assert np.isfinite(img).all()
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.render(8, 8, 1, 0, integrator="pathTrace")
    r.close()


@pytest.mark.gpu
def test_gpu_materialball_committed_configuration():
    # rtmi.materialball: cornellbox2.yaml camera + materialball COAT at (0.1, 0, -1)
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    w, h = 48, 40
    cam = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox2.yaml"), S.MODELS, w, h)
    pt, _ = S.build_pathtrace_oracle("materialball")
    want, _ = pt.render(cam, w, h, 4, 5, threads=8)
    r = _product(0)
    rtmi.materialball(r, w, h)
    got = r.render(w, h, 4, 5, integrator="pathTrace")
    r.close()
    _assert_parity(got, want)
    assert np.array_equal(got, want)  # bit-identical in practice (same IEEE op order)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_pathtrace_random_views(seed):
    # random camera, bounce count, seed and sub-stream layout per case
    rng = np.random.RandomState(100 + seed)
    name = sorted(S.PT_SCENES)[seed % 3]
    eye = (float(rng.uniform(-2.5, 2.5)), float(rng.uniform(-0.5, 2.0)), float(rng.uniform(1.5, 3.5)))
    cam = (eye, (0.1, 0.0, -0.5), (0.0, 1.0, 0.0), 1.25, float(rng.uniform(25, 70)),
           float(rng.uniform(0.0, 0.05)), 3.0, 0.0, 1.0)
    bounces, lanes = int(rng.randint(1, 9)), [1, 2, 8][seed % 3]
    pt, oc = S.build_pathtrace_oracle(name, cam)
    want, ost = pt.render(oc, 30, 24, 4, bounces, seed=seed, threads=8, lanes_per_pixel=lanes)
    r = _product(0)
    S.build_pathtrace_product(r, name, cam)
    got = r.render(30, 24, 4, bounces, seed=seed, lanes_per_pixel=lanes, integrator="pathTrace")
    st = r.stats()
    r.close()
    _assert_parity(got, want)
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]
