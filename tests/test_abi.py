"""The C-ABI library loads and exports every symbol include/rtmi.h declares;
host-only (device = -1) scene building works without a GPU."""
import os
import re

import numpy as np
import pytest

from raytracingthenextweekcuda_amd import _lib
from tests import scenes as S

HEADER = os.path.join(S.REPO, "include", "rtmi.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:rt_status|int32_t|uint32_t|void|const char\*)\s+(rt_\w+)\s*\(", txt, re.M)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.rt_abi_version() == _lib.ABI_VERSION
    assert f"#define RTMI_ABI_VERSION {_lib.ABI_VERSION}" in open(HEADER).read()


def test_nodev_context_builds_scene_but_refuses_render():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    rtmi.cornell_box1(r, 16, 16)
    c = r.object_counts()
    assert c["plane"] == 6 and c["mesh"] == 2 and c["triangle"] == 24
    with pytest.raises(rtmi.RTError, match="RT_ERR_NODEV"):
        r.render(16, 16, 1, 1)
    r.close()


def test_preseeded_materials_win_over_yaml():
    """main.cu:643-651 vs the nullptr guards: light id 8 stays Emission x5."""
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    rtmi.cornell_box1(r, 16, 16, commit=False)
    assert r.materials[8] is not None and r.materials[9] is None
    r.close()


def test_invalid_arguments_are_reported_not_fatal():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.plane(0, (0, 0, 0), (0, 1, 0), (1, 1, 1), 0, orientation=5)
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.sphere(-1, (0, 0, 0), 1.0, 0)
    with pytest.raises(rtmi.RTError, match="RT_ERR_IO"):
        r.mesh_obj(0, "/nonexistent.obj", material=0)
    r.sphere(0, (0, 0, 0), 1.0, 3)  # material 3 never created
    with pytest.raises(rtmi.RTError, match="undefined material"):
        r.commit()
    with pytest.raises(rtmi.RTError, match="RT_ERR_INVALID"):
        r.sphere(1, (np.nan, 0, 0), 1.0, 0)
    r.close()


def test_gamma_u8_matches_canvas_gamma():
    from oracle import oracle as orc
    import raytracingthenextweekcuda_amd as rtmi

    x = np.linspace(-0.5, 3.0, 10007, dtype=np.float32)
    x[:5] = [0.0, 1.0, 0.998, 1e-30, 0.25]
    a = rtmi.gamma_u8(x)
    assert np.array_equal(a, orc.gamma_u8(x))
    assert a[1] == 255 and a[0] == 0 and a[4] == 127  # 255.99*0.5


def test_missing_library_fails_loudly():
    # the product path has no fallback: without librtmi.so the renderer refuses to start
    import subprocess
    import sys

    code = ("import raytracingthenextweekcuda_amd as r\n"
            "try:\n    r.Renderer(0)\nexcept ImportError as e:\n    print('IMPORT_ERROR', e)\n")
    env = dict(os.environ, RTMI_LIB="/nonexistent/librtmi.so")
    out = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         env=env, capture_output=True, text=True, timeout=300)
    assert "IMPORT_ERROR" in out.stdout and "no fallback" in out.stdout, out.stdout + out.stderr
