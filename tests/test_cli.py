"""Offline renderer CLI (python -m raytracingthenextweekcuda_amd): the reference's
main() for one scene file -> PNG/PPM."""
import os
import struct
import subprocess
import sys
import zlib

import numpy as np
import pytest

from tests import scenes as S


def _run(args, cwd):
    return subprocess.run([sys.executable, "-m", "raytracingthenextweekcuda_amd"] + args, cwd=cwd,
                          capture_output=True, text=True, env=dict(os.environ, PYTHONPATH=S.REPO))


def test_cli_help_and_argument_errors(tmp_path):
    out = _run(["--help"], tmp_path)
    assert out.returncode == 0 and "cornellbox1" in out.stdout
    assert _run(["cornellbox1", "--out", "x.jpg"], tmp_path).returncode != 0
    assert _run(["cornellbox1", "--spp", "0"], tmp_path).returncode != 0
    assert _run(["cornellbox1", "--devices", ""], tmp_path).returncode != 0


def _decode_png(path):
    png = open(path, "rb").read()
    off, chunks = 8, {}
    while off < len(png):
        n, tag = struct.unpack(">I4s", png[off:off + 8])
        chunks[tag] = chunks.get(tag, b"") + png[off + 8:off + 8 + n]
        off += 12 + n
    w, h = struct.unpack(">II", chunks[b"IHDR"][:8])
    raw = zlib.decompress(chunks[b"IDAT"])
    return np.frombuffer(raw, np.uint8).reshape(h, w * 3 + 1)[:, 1:].reshape(h, w, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["cornellbox1", os.path.join(S.SCENES, "cornellbox0.yaml")])
def test_cli_renders_scene_to_png(tmp_path, scene):
    import raytracingthenextweekcuda_amd as rtmi

    out = _run([scene, "--width", "40", "--height", "24", "--spp", "4", "--depth", "6", "--out", "r.png"],
               tmp_path)
    assert out.returncode == 0, out.stderr
    assert "Mrays/s" in out.stdout
    png = _decode_png(tmp_path / "r.png")
    with rtmi.Renderer(0) as r:
        if os.path.exists(scene):
            rtmi.load_yaml_scene(r, scene, 40, 24)
        else:
            rtmi.cornell_box1(r, 40, 24)
        img = r.render(40, 24, 4, 6, lanes_per_pixel=0)
    assert np.array_equal(png, rtmi.gamma_u8(img)[::-1])  # top row first, like Canvas::writeToPNG
