"""GPU parity for rays with special direction components through the axial-plane records.

rt_scene.cpp gives every plane with a +-1 normal the kObjPlaneAxial record kind, whose kernel test
(rt_kernel.hip plane_axial) forms den = n_K * d_K and num = (p_K - o_K) * n_K and takes the quotient as
v_rcp + Newton + Markstein, with an IEEE fallback for waves whose |num| or |den| reach 2^100. The CPU
test tests/test_plane_axial.py proves the axial form equal to Plane.cu's general one in numpy; these scenes
drive the GPU code itself through the cases it argues about, against the oracle's general Plane::hit:

  * zero direction components: a camera with fov 0 sends every ray along its forward vector, here
    (0, 0, -1) exactly, so planes of the other two orientations see den = +-0 for every camera ray, and
    fuzz-free metal mirrors keep the zeros on reflection (rays bounce between two XY mirrors);
  * tiny and subnormal components: the same camera looking along (1e-38, -1e-40, -1);
  * huge operands: a plane at z = -1e31 (|num| >= 2^100: the wave's IEEE fallback).
NaN directions cannot reach the kernel: rt_camera_apply refuses a non-finite view (a camera whose eye equals
its centre), which the last test pins, and no scatter produces one (refract takes sqrt(|1 - |perp|^2|),
Lambertian's near-zero guard replaces a vanishing direction by the normal).
"""
import numpy as np
import pytest

from tests.test_fuzz_parity import build_oracle, build_product

MATS = [("lambertian", 0, (0.7, 0.6, 0.5)), ("metal", 1, (0.9, 0.9, 0.9), 0.0), ("emission", 2, (1.0, 0.9, 0.8), 3.0),
        ("lambertian", 3, (0.2, 0.4, 0.8))]


def axial_box(extra=()):
    """Axial planes of all three orientations, one- and two-sided, both normal signs, two facing XY mirrors."""
    objs = [
        ("plane", 0, (0.0, 0.0, -1.0), (0.0, 0.0, 1.0), (1.0, 1.0, 1.0), 1, 0, True),     # XY mirror (back)
        ("plane", 1, (0.0, 0.0, 3.0), (0.0, 0.0, -1.0), (1.0, 1.0, 1.0), 1, 0, False),    # XY mirror behind the eye
        ("plane", 2, (0.0, -0.5, 0.0), (0.0, 1.0, 0.0), (1.0, 1.0, 4.0), 0, 2, True),     # XZ floor
        ("plane", 3, (0.0, 0.5, 0.0), (0.0, -1.0, 0.0), (0.3, 1.0, 0.3), 2, 2, False),    # XZ light, one-sided
        ("plane", 4, (-0.8, 0.0, 0.0), (1.0, 0.0, 0.0), (1.0, 1.0, 4.0), 3, 1, True),     # YZ wall
        ("plane", 5, (0.8, 0.0, 0.0), (-1.0, 0.0, 0.0), (1.0, 1.0, 4.0), 0, 1, False),    # YZ wall, one-sided
    ]
    for k, o in enumerate(extra):
        objs.append((o[0], 6 + k) + tuple(o[2:]))
    return objs


def spec(kind):
    up = (0.0, 1.0, 0.0)
    if kind == "zero":  # fov 0: every camera ray is (0, 0, -1)
        cam = ((0.0, 0.0, 2.0), (0.0, 0.0, 0.0), up, 1.0, 0.0, 0.0, 2.0, 0.0, 1.0)
        objs = axial_box()
    elif kind == "tiny":  # forward (1e-38, -1e-40, -1): tiny and subnormal components
        cam = ((0.0, 0.0, 2.0), (1e-38, -1e-40, 1.0), up, 1.0, 0.0, 0.0, 2.0, 0.0, 1.0)
        objs = axial_box()
    elif kind == "huge":  # a far XY plane: |num| >= 2^100 for the rays that reach it
        cam = ((0.0, 0.0, 2.0), (0.0, 0.0, 0.0), up, 1.0, 40.0, 0.0, 2.0, 0.0, 1.0)
        objs = axial_box(extra=[("plane", 0, (0.0, 0.0, -1e31), (0.0, 0.0, 1.0), (1e32, 1e32, 1.0), 3, 0, True)])
        objs = [o for o in objs if o[1] != 0]  # no back mirror: camera rays reach the far plane
    else:  # "nan": eye == centre
        cam = ((0.0, 0.0, 2.0), (0.0, 0.0, 2.0), up, 1.0, 60.0, 0.0, 2.0, 0.0, 1.0)
        objs = axial_box()
    return {"camera": cam, "materials": MATS, "objects": objs}


@pytest.mark.parametrize("kind", ["zero", "tiny", "huge"])
def test_degenerate_specs_render_on_the_oracle(kind):
    img, st = build_oracle(spec(kind)).render(8, 8, 2, 6, lanes_per_pixel=1)
    assert st["segments"] > 0 and np.isfinite(img).all()


def test_a_non_finite_view_is_refused():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    with pytest.raises(rtmi.RTError, match="non-finite view"):
        build_product(r, spec("nan"))
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zero", "tiny", "huge"])
def test_gpu_degenerate_rays_match_the_oracle(kind):
    import raytracingthenextweekcuda_amd as rtmi

    s = spec(kind)
    w, h, spp, depth = 32, 24, 8, 8
    r = rtmi.Renderer(0)
    build_product(r, s)
    got = r.render(w, h, spp, depth, lanes_per_pixel=4)
    st = r.stats()
    r.close()
    want, ost = build_oracle(s).render(w, h, spp, depth, lanes_per_pixel=4)
    assert st["segments"] == ost["segments"]
    assert np.array_equal(got, want)
