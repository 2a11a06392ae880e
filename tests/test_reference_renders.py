"""The integrator against images the REFERENCE rendered (tests/golden/ref_images/).

These are the parity pins of the full integrator composition: camera, closest hit,
materials, sky, bounce limit, sample mean, Canvas::gamma and the PNG row flip. The
reference's own renders are 8-bit and drawn from cuRAND XORWOW, so the comparison is
statistical (tests/refimg.py): the global mean and the 16x16 tile means, in 8-bit levels.

Thresholds ("reference renders"). The noise floor was measured with the
oracle itself: two renders of cornellbox0 at 256 spp with different seeds differ by a
tile p95 of 1.39 levels (median 0.40, max 2.66). Tile-mean noise scales with
sqrt(1/n_ours + 1/n_ref), so ours at 256 spp vs the reference's 1024 spp expects
p95 = 1.39 * sqrt(1/256 + 1/1024) / sqrt(2/256) = 1.10 -- measured 1.12. The thresholds
sit near 1.8x the noise floor. The global mean is biased low by gamma's concavity at
finite spp (-0.15 levels at 256 spp; -0.01 at 1024 spp), so its bound is 0.5 levels at
256 spp and 0.25 at the reference's own 1024 spp. Negative controls (GPU) show that the
statistic rejects a plausible mistake: the YAML's light intensity 10 instead of the
pre-seeded Emission x5 (main.cu:651), and glass of IOR 1.33 instead of 1.5.
"""
import os

import numpy as np
import pytest

from tests import refimg
from tests import scenes as S

THREADS = min(16, os.cpu_count() or 1)
W = H = 512

# (spp, global |delta| bound, tile p95 bound)
CB0_CPU = (256, 0.5, 2.0)
CB0_GPU = (1024, 0.25, 1.5)
MB = (32, 0.5, 4.0)  # the reference image's own 32 spp (R/main.cu:168)


def _check(stats, g_bound, p95_bound, what):
    assert stats["global_abs_max"] <= g_bound, (what, stats)
    assert stats["tile_p95"] <= p95_bound, (what, stats)


def _oracle_materialball(w, h):
    from oracle import oracle as orc

    cam = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox2.yaml"), S.MODELS, w, h)
    pt = orc.OraclePathTrace()
    pt.load_object(os.path.join(S.MODELS, "materialball", "materialball.ply"), "COAT")
    pt.process((0.1, 0.0, -1.0))
    with open(os.path.join(S.GOLDEN, "bvh", "materialball.ply.bvh"), "rb") as fh:
        pt.set_bvh(fh.read())
    return cam, pt


def test_ref_images_decode():
    for p in (refimg.CORNELLBOX0, refimg.MATERIALBALL):
        img = refimg.load_png(p)
        assert img.shape == (H, W, 3) and img.dtype == np.uint8


def test_oracle_cornellbox0_matches_reference_render():
    """rayColor (main.cu:63-94) over cornellbox0.yaml, 10 bounces (main.cu:23)."""
    from oracle import oracle as orc

    spp, g, p95 = CB0_CPU
    sc = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox0.yaml"), S.MODELS, W, H)
    img, _ = sc.render(W, H, spp, 10, threads=THREADS)
    st = refimg.compare(refimg.to_png_rows(orc.gamma_u8(img)), refimg.load_png(refimg.CORNELLBOX0))
    _check(st, g, p95, "oracle cornellbox0")


def test_oracle_materialball_matches_reference_render():
    """pathTrace (CUDAPathTracer.cu:358-622) as committed in main.cu:187: R/render.png."""
    from oracle import oracle as orc

    spp, g, p95 = MB
    cam, pt = _oracle_materialball(W, H)
    img, st = pt.render(cam, W, H, spp, 5, threads=THREADS)
    assert st["overflow"] == 0
    s = refimg.compare(refimg.to_png_rows(orc.gamma_u8(img)), refimg.load_png(refimg.MATERIALBALL))
    _check(s, g, p95, "oracle materialball")


@pytest.mark.gpu
def test_gpu_cornellbox0_matches_reference_render():
    """The HIP path at the reference image's own 1024 spp, through rt_render_u8 (the
    device-side Canvas::gamma), with the bench's automatic lane layout."""
    import raytracingthenextweekcuda_amd as rtmi

    spp, g, p95 = CB0_GPU
    ref = refimg.load_png(refimg.CORNELLBOX0)
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, os.path.join(S.SCENES, "cornellbox0.yaml"), W, H)
        u8 = r.render_u8(W, H, spp, 10, lanes_per_pixel=0)
        assert r.stats()["overflow"] == 0
    _check(refimg.compare(refimg.to_png_rows(u8), ref), g, p95, "gpu cornellbox0 @1024")

    # negative controls: the same statistic must reject plausible integration mistakes
    for tweak in ("light_x10", "ior_1.33"):
        with rtmi.Renderer(0) as r:
            rtmi.load_yaml_scene(r, os.path.join(S.SCENES, "cornellbox0.yaml"), W, H, commit=False)
            if tweak == "light_x10":
                r.emission(8, (1.0, 1.0, 1.0), 10.0)
            else:
                r.dielectric(7, 1.33)
            r.commit()
            u8 = r.render_u8(W, H, spp, 10, lanes_per_pixel=0)
        st = refimg.compare(refimg.to_png_rows(u8), ref)
        assert st["global_abs_max"] > g or st["tile_max"] > 3 * p95, (tweak, st)


@pytest.mark.gpu
def test_gpu_cornellbox0_matches_reference_render_at_256spp():
    """The CPU test's sample count on the GPU path (same thresholds as the oracle)."""
    import raytracingthenextweekcuda_amd as rtmi

    spp, g, p95 = CB0_CPU
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, os.path.join(S.SCENES, "cornellbox0.yaml"), W, H)
        u8 = r.render_u8(W, H, spp, 10, lanes_per_pixel=0)
    _check(refimg.compare(refimg.to_png_rows(u8), refimg.load_png(refimg.CORNELLBOX0)), g, p95,
           "gpu cornellbox0 @256")


@pytest.mark.gpu
def test_gpu_materialball_matches_reference_render():
    import raytracingthenextweekcuda_amd as rtmi

    spp, g, p95 = MB
    with rtmi.Renderer(0) as r:
        rtmi.materialball(r, W, H)
        u8 = r.render_u8(W, H, spp, 5, lanes_per_pixel=0, integrator="pathTrace")
        assert r.stats()["overflow"] == 0
    _check(refimg.compare(refimg.to_png_rows(u8), refimg.load_png(refimg.MATERIALBALL)), g, p95,
           "gpu materialball")
