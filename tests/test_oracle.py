"""The CPU restatement against known answers: Random123 Philox4x32-10 KAT
vectors, curand's uniform mapping, the reference's cube_small.obj
triangulation, and hand-derived hit/scatter results."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from tests import scenes as S


# Random123 kat_vectors (philox4x32 10): counter, key -> output.
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_kat(ctr, key, out):
    assert orc.philox(ctr, key) == out


def _xoshiro128p(state, n):
    """xoshiro128+ 1.0 (Blackman & Vigna), restated in Python."""
    s = list(state)
    M = 0xFFFFFFFF
    rotl = lambda x, k: ((x << k) | (x >> (32 - k))) & M
    out = []
    for _ in range(n):
        out.append((s[0] + s[3]) & M)
        t = (s[1] << 9) & M
        s[2] ^= s[0]
        s[3] ^= s[1]
        s[1] ^= s[2]
        s[0] ^= s[3]
        s[2] ^= t
        s[3] = rotl(s[3], 11)
    return out


def test_uniform_stream_layout_and_range():
    """Stream of (seed, pixel, sample): Philox4x32-10(counter=(sample,0,0,0),
    key=(seed,pixel)) seeds xoshiro128+; uniforms use curand's (0,1] map."""
    u = orc.uniforms(1984, 12345, 7, 9)
    words = _xoshiro128p(orc.philox([7, 0, 0, 0], [1984, 12345]), 9)
    inv = np.float32(2.0 ** -32)
    expect = np.float32(words) * inv + inv / np.float32(2)
    assert np.array_equal(u, expect.astype(np.float32))
    assert (u > 0).all() and (u <= 1).all()
    # extremes of curand's mapping
    assert np.float32(0) * inv + inv / 2 > 0
    assert np.float32(0xFFFFFFFF) * inv + inv / 2 == np.float32(1.0)
    # distinct samples / pixels give distinct streams
    assert not np.array_equal(u, orc.uniforms(1984, 12345, 8, 9))
    assert not np.array_equal(u, orc.uniforms(1984, 12346, 7, 9))


def test_cube_small_triangulation():
    """tinyobjloader quad split (tiny_obj_loader.h:1475-1493): square faces have
    equal diagonals, so each quad (0,1,2,3) becomes (0,1,3),(1,2,3)."""
    tri = orc.load_obj(os.path.join(S.MODELS, "cube", "cube_small.obj"))
    assert tri.shape == (12, 9)
    # first face `f 1 2 4 3`: v1=(-.25,-.25,.25) v2=(-.25,.25,.25) v4=(-.25,.25,-.25) v3=(-.25,-.25,-.25)
    np.testing.assert_array_equal(tri[0], [-.25, -.25, .25, -.25, .25, .25, -.25, -.25, -.25])
    np.testing.assert_array_equal(tri[1], [-.25, .25, .25, -.25, .25, -.25, -.25, -.25, -.25])
    assert np.all(np.abs(tri) == 0.25)


def test_obj_transform_scale_rotate_offset():
    s, rot, off = (0.5, 1.0, 0.5), (0.0, 30.0, 0.0), (-0.25, -0.25, -0.25)
    tri = orc.load_obj(os.path.join(S.MODELS, "cube", "cube_small.obj"), s, rot, off)
    raw = orc.load_obj(os.path.join(S.MODELS, "cube", "cube_small.obj"))
    v = raw.reshape(-1, 3).astype(np.float32) * np.float32(s)
    r = np.float32(np.float32(3.1415926535897932) / np.float32(180.0)) * np.float32(30.0)
    c, sn = np.cos(np.float32(r), dtype=np.float32), np.sin(np.float32(r), dtype=np.float32)
    x = v[:, 0] * c + v[:, 2] * sn
    z = -v[:, 0] * sn + v[:, 2] * c
    exp = np.stack([x, v[:, 1], z], 1) + np.float32(off)
    np.testing.assert_allclose(tri.reshape(-1, 3), exp, rtol=0, atol=1e-7)


def test_product_obj_loader_matches_oracle():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    rtmi.cornell_box1(r, 8, 8)
    a = orc.load_obj(os.path.join(S.MODELS, "cube", "cube_small.obj"), (0.5, 1, 0.5), (0, 30, 0), (-.25, -.25, -.25))
    b = orc.load_obj(os.path.join(S.MODELS, "cube", "cube_small.obj"), (0.5, .5, 0.5), (0, -30, 0), (.25, -.375, -.25))
    assert np.array_equal(r.mesh_vertices(6), a)
    assert np.array_equal(r.mesh_vertices(7), b)
    r.close()


def _box_scene():
    sc = orc.OracleScene()
    orc.preseed_materials(sc)
    # cornellbox1 walls
    sc.plane(0, (0, 0.5, 0), (0, 1, 0), (.5, .5, .5), 3, 2, True)
    sc.plane(1, (0, -0.5, 0), (0, -1, 0), (.5, .5, .5), 3, 2, True)
    sc.plane(2, (-0.5, 0, 0), (-1, 0, 0), (.5, .5, .5), 4, 1, True)
    sc.plane(3, (0.5, 0, 0), (1, 0, 0), (.5, .5, .5), 5, 1, True)
    sc.plane(4, (0, 0, -0.5), (0, 0, -1), (.5, .5, .5), 3, 0, True)
    sc.plane(5, (0, 0.49, 0), (0, 1, 0), (.125, .125, .125), 8, 2, False)
    return sc


def test_plane_hits_known_answers():
    sc = _box_scene()
    # straight down -z from the eye: back wall (two-sided, n_out = (0,0,-1)) at t = 1.5.
    # setFaceNormal: front = dot(d, n_out) < FLT_EPSILON -> 1 < eps is false -> back face,
    # stored normal is -n_out = (-0, -0, 1).
    t, n, front, mat = sc.trace((0, 0, 1), (0, 0, -1))
    assert (t, mat) == (1.5, 3) and n == (0.0, 0.0, 1.0) and not front
    # the left wall seen from inside: t = 0.5, n_out = (-1,0,0), d = (-1,0,0) -> back face
    t, n, front, mat = sc.trace((0, 0, 0), (-1, 0, 0))
    assert (t, mat, front) == (0.5, 4, False) and n[0] == 1.0
    # grazing the open front: nothing is hit from outside looking +z
    assert sc.trace((0, 0, 1), (0, 0, 1)) is None


def test_one_sided_light_only_from_below():
    sc = _box_scene()
    up = sc.trace((0, 0, 0), (0, 1, 0))
    assert up[3] == 8 and abs(up[0] - 0.49) < 1e-7  # light (one-sided, normal +y, den > eps)
    sc2 = _box_scene()
    down = sc2.trace((0, 0.495, 0), (0, -1, 0))
    assert down[3] == 3 and abs(down[0] - 0.995) < 1e-6  # passes through the light's back side


def test_sphere_roots_and_inside():
    sc = orc.OracleScene()
    sc.material(0, 0, (0.5, 0.5, 0.5), 1.0)
    sc.sphere(0, (0, 0, -2), 0.5, 0)
    t, n, front, _ = sc.trace((0, 0, 0), (0, 0, -1))
    assert t == 1.5 and n == (0.0, 0.0, 1.0) and front
    t, n, front, _ = sc.trace((0, 0, -2), (0, 0, -1))  # from the centre: far root, back face
    assert t == 0.5 and n == (0.0, 0.0, 1.0) and not front
    assert sc.trace((0, 0, 0), (0, 1, 0)) is None


def test_cornellbox1_segments_per_sample():
    """CornellBox1 256x256 spp4 d4 (BASELINE config 1) traces 3.43 segments per
    sample, as measured from the reference's own code in the survey."""
    sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox1.yaml"), S.MODELS, 128, 128)
    img, st = sc.render(128, 128, 4, 4)
    assert 3.38 < st["segments"] / (128 * 128 * 4) < 3.48
    assert np.isfinite(img).all() and img.min() >= 0


def test_oracle_column_window_equals_the_full_rows():
    """rt_render_params' column window, restated: columns [c0, c0 + n) of a row are the full
    frame's pixels (camera and RNG keyed by the frame position), for both integrators."""
    from oracle import oracle as orc

    W, H = 40, 24
    sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox1.yaml"), S.MODELS, W, H)
    full, _ = sc.render(W, H, 4, 4, row_block=1, row_rank=5, row_world=6, lanes_per_pixel=2)
    win, st = sc.render(W, H, 4, 4, row_block=1, row_rank=5, row_world=6, lanes_per_pixel=2,
                        col_begin=7, col_count=13)
    assert win.shape == (full.shape[0], 13, 3)
    assert np.array_equal(win, full[:, 7:20])
    cam = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox2.yaml"), S.MODELS, W, H)
    pt, _ = S.build_pathtrace_oracle("materialball")
    fullp, _ = pt.render(cam, W, H, 2, 5, row_block=2, row_rank=1, row_world=3)
    winp, _ = pt.render(cam, W, H, 2, 5, row_block=2, row_rank=1, row_world=3, col_begin=30, col_count=10)
    assert np.array_equal(winp, fullp[:, 30:40])
