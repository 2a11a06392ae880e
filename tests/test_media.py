"""Participating media (BASELINE config 5; a build extension: the reference has
no media). Semantics are those of "Ray Tracing: The Next Week" ConstantMedium +
isotropic with a cube boundary and the free-flight draw taken from the
sample's stream in slot order (include/rtmi.h rt_constant_medium). Parity is against the CPU restatement
only: unpinned against the reference, which has no such code."""
import math
import os

import numpy as np
import pytest

from tests import scenes as S

MEDIA_YAML = os.path.join(S.SCENES, "cornellbox_media.yaml")


def _medium_scene(density, albedo=(0.0, 0.0, 0.0)):
    from oracle import oracle as orc

    sc = orc.OracleScene()
    sc.camera((0, 0, 1), (0, 0, -1), (0, 1, 0), 1.0, 60.0, 0.0, 2.0, 0.0, 1.0)
    sc.material(0, 4, albedo, 0.0)
    sc.constant_medium(0, (0.0, 0.0, 0.0), (0.5, 0.5, 0.5), density, 0)
    return sc


def test_oracle_dense_medium_scatters_near_the_entry():
    hit = _medium_scene(1e6).trace((0, 0, 2), (0, 0, -1))
    assert hit is not None
    t, n, front, mat = hit
    assert 1.5 <= t < 1.5 + 1e-4 and n == (1.0, 0.0, 0.0) and front and mat == 0


def test_oracle_thin_medium_is_transparent():
    assert _medium_scene(1e-6).trace((0, 0, 2), (0, 0, -1)) is None


def test_oracle_medium_misses_outside_the_box():
    assert _medium_scene(1e6).trace((0.7, 0, 2), (0, 0, -1)) is None


def test_oracle_medium_transmittance_matches_beer_lambert():
    # fraction of camera rays through a 1-unit-thick slab that scatter ~ 1 - exp(-density)
    from oracle import oracle as orc

    density = 0.7
    sc = _medium_scene(density)
    img, st = sc.render(48, 48, 16, 2, threads=4)
    # rays that scatter (black isotropic albedo) contribute 0; escaping rays see the sky
    sky = orc.OracleScene()
    sky.camera((0, 0, 1), (0, 0, -1), (0, 1, 0), 1.0, 60.0, 0.0, 2.0, 0.0, 1.0)
    ref, _ = sky.render(48, 48, 16, 2, threads=4)
    centre = (slice(18, 30), slice(18, 30))  # rays crossing the full depth of the box (z 0.5 .. -0.5)
    frac = 1.0 - img[centre].mean() / ref[centre].mean()
    assert abs(frac - (1.0 - math.exp(-density))) < 0.05


def test_media_scene_loads_in_product_and_oracle():
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    r = rtmi.Renderer(-1)
    rtmi.cornell_box_media(r, 32, 32)
    assert r.object_counts()["sphere"] == 1
    r.close()
    orc.yaml_scene(MEDIA_YAML, S.MODELS, 32, 32)


def test_constant_medium_rejects_bad_density():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    r.isotropic(0, (1, 1, 1))
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.constant_medium(0, (0, 0, 0), (1, 1, 1), 0.0, r.materials[0])
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,spp,depth,lanes", [(48, 48, 8, 16, 1), (40, 24, 16, 16, 4), (16, 16, 4, 3, 1)])
def test_gpu_media_parity(w, h, spp, depth, lanes):
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    sc = orc.yaml_scene(MEDIA_YAML, S.MODELS, w, h)
    want, ost = sc.render(w, h, spp, depth, threads=8, lanes_per_pixel=lanes)
    r = rtmi.Renderer(0)
    rtmi.cornell_box_media(r, w, h)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    assert float(np.abs(got - want).max()) <= 1e-4
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]
