"""The C++ facade (include/rtmi.hpp) compiles against librtmi.so with g++ and
builds the reference-style CornellBox1 scene through the kernels.h-shaped
factories (examples/cornellbox.cpp). The GPU render is in test_gpu_examples."""
import os
import subprocess

import pytest

from tests import scenes as S

EX = os.path.join(S.REPO, "examples")


@pytest.fixture(scope="module")
def binary():
    subprocess.run(["make", "-s", "-C", EX, "cornellbox"], check=True)
    return os.path.join(EX, "cornellbox")


def test_facade_builds_scene_without_gpu(binary):
    out = subprocess.run([binary, "-1"], check=True, capture_output=True, text=True).stdout
    assert "6 planes, 2 meshes, 24 triangles" in out


@pytest.mark.gpu
def test_facade_renders_on_gpu(binary, tmp_path):
    out = subprocess.run([binary, "0", "64", "64", "4", "4"], check=True, capture_output=True,
                         text=True, cwd=tmp_path).stdout
    assert "Mrays/s" in out
    data = (tmp_path / "cornellbox.ppm").read_bytes()
    assert data.startswith(b"P6\n64 64\n255\n") and len(data) == len(b"P6\n64 64\n255\n") + 64 * 64 * 3


@pytest.fixture(scope="module")
def pt_binary():
    subprocess.run(["make", "-s", "-C", EX, "materialball"], check=True)
    return os.path.join(EX, "materialball")


def test_facade_pathtrace_scene_without_gpu(pt_binary):
    out = subprocess.run([pt_binary, "-1"], check=True, capture_output=True, text=True).stdout
    assert "46816 triangles, 42503 BVH nodes" in out


@pytest.mark.gpu
def test_facade_pathtrace_renders_on_gpu(pt_binary, tmp_path):
    out = subprocess.run([pt_binary, "0", "48", "32", "2"], check=True, capture_output=True,
                         text=True, cwd=tmp_path).stdout
    assert "Mrays/s" in out
    data = (tmp_path / "materialball.ppm").read_bytes()
    assert data.startswith(b"P6\n48 32\n255\n") and len(data) == len(b"P6\n48 32\n255\n") + 48 * 32 * 3


def test_facade_png_writer_matches_ppm(tmp_path):
    # Canvas::writeToPNG (stored-deflate PNG, no codec dependency) carries the same
    # gamma'd top-down rows as writeToPPM; decoded here with zlib
    import struct
    import zlib

    src = tmp_path / "png_check.cpp"
    src.write_text(r'''
#include "rtmi.hpp"
int main() {
    rtmi::Canvas c(37, 300);  // > 65535 raw bytes: several stored blocks
    for (int i = 0; i < 37 * 300 * 3; ++i) c.data()[i] = (float)((i * 7919) % 1000) / 999.0f;
    c.writeToPPM("out.ppm");
    c.writeToPNG("out.png");
    return 0;
}
''')
    exe = tmp_path / "png_check"
    lib = os.path.join(S.REPO, "raytracingthenextweekcuda_amd")
    subprocess.run(["g++", "-O1", "-std=c++17", f"-I{os.path.join(S.REPO, 'include')}", str(src), "-o", str(exe),
                    f"-L{lib}", "-lrtmi", f"-Wl,-rpath,{lib}"], check=True)
    subprocess.run([str(exe)], check=True, cwd=tmp_path)
    png = (tmp_path / "out.png").read_bytes()
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    chunks, off = {}, 8
    while off < len(png):
        n, tag = struct.unpack(">I4s", png[off:off + 8])
        data = png[off + 8:off + 8 + n]
        assert struct.unpack(">I", png[off + 8 + n:off + 12 + n])[0] == zlib.crc32(tag + data)
        chunks[tag] = data
        off += 12 + n
    w, h, depth, ctype = struct.unpack(">IIBB", chunks[b"IHDR"][:10])
    assert (w, h, depth, ctype) == (37, 300, 8, 2)
    raw = zlib.decompress(chunks[b"IDAT"])
    rows = [raw[y * (w * 3 + 1):(y + 1) * (w * 3 + 1)] for y in range(h)]
    assert all(r[0] == 0 for r in rows)
    ppm = (tmp_path / "out.ppm").read_bytes()
    header = b"P6\n37 300\n255\n"
    assert ppm.startswith(header) and b"".join(r[1:] for r in rows) == ppm[len(header):]


@pytest.fixture(scope="module")
def cli_binary():
    subprocess.run(["make", "-s", "-C", EX, "rtmi_render"], check=True)
    return os.path.join(EX, "rtmi_render")


def test_native_cli_scene_digest_matches_python_loader(cli_binary):
    # examples/rtmi_render reads the YAML with the library's own reader
    import raytracingthenextweekcuda_amd as rtmi

    path = os.path.join(S.SCENES, "suzanne_cornellbox.yaml")
    out = subprocess.run([cli_binary, path, "--device", "-1", "--width", "96", "--height", "64"], check=True,
                         capture_output=True, text=True).stdout
    r = rtmi.Renderer(-1)
    rtmi.load_yaml_scene(r, path, 96, 64)
    want = r.scene_digest()
    r.close()
    assert f"digest {want:016x}" in out, out
    bad = subprocess.run([cli_binary, os.path.join(S.SCENES, "scene.yaml"), "--device", "-1"],
                         capture_output=True, text=True)
    assert bad.returncode == 1 and "line 167" in bad.stderr


@pytest.mark.gpu
def test_native_cli_renders_the_python_frame(cli_binary, tmp_path):
    # main()-style native program vs the Python host layer: same scene, same frame, same bytes
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.canvas import Canvas

    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    w, h, spp, depth = 64, 48, 4, 6
    subprocess.run([cli_binary, path, "--width", str(w), "--height", str(h), "--spp", str(spp), "--depth",
                    str(depth), "--out", str(tmp_path / "native.ppm")], check=True, capture_output=True)
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        img = r.render(w, h, spp, depth, lanes_per_pixel=0)
    want = Canvas(w, h).pixels(img)[::-1].reshape(-1)  # writeToPPM's rows: top first
    data = (tmp_path / "native.ppm").read_bytes()
    head = f"P6\n{w} {h}\n255\n".encode()
    assert data.startswith(head)
    assert data[len(head):] == want.astype("uint8").tobytes()
