"""Radiance regression fixtures (tests/golden/radiance, made by
tests/golden/make_radiance_fixtures.py from the CPU restatement): the oracle must
reproduce them exactly on CPU, and the HIP path must match them bit for bit on
the GPU. They freeze the restatement; pinning against the reference is by the
component fixtures listed in DESIGN.md §2."""
import os

import numpy as np
import pytest

from tests import scenes as S
from tests.golden import make_radiance_fixtures as F


def _fixture(name, w, h):
    return np.fromfile(os.path.join(F.OUT, name + ".f32"), dtype="<f4").reshape(h, w, 3)


@pytest.mark.parametrize("name", sorted(F.FIXTURES))
def test_oracle_reproduces_fixture(name):
    kind, w, h, spp, depth = F.FIXTURES[name]
    assert np.array_equal(F.render(kind, w, h, spp, depth), _fixture(name, w, h))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(F.FIXTURES))
def test_gpu_matches_fixture(name):
    import raytracingthenextweekcuda_amd as rtmi

    kind, w, h, spp, depth = F.FIXTURES[name]
    r = rtmi.Renderer(0)
    if kind == "materialball":
        rtmi.materialball(r, w, h)
        got = r.render(w, h, spp, depth, integrator="pathTrace")
    elif kind == "media":
        rtmi.cornell_box_media(r, w, h)
        got = r.render(w, h, spp, depth)
    else:
        rtmi.cornell_box1(r, w, h)
        got = r.render(w, h, spp, depth)
    r.close()
    want = _fixture(name, w, h)
    assert float(np.abs(got - want).max()) <= 1e-4
    assert np.array_equal(got, want)
