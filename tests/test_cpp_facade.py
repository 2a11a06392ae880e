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


@pytest.fixture(scope="module")
def driver_binary():
    subprocess.run(["make", "-s", "-C", EX, "main_driver"], check=True)
    return os.path.join(EX, "main_driver")


def _ppm_rows(path, w, h):
    data = path.read_bytes()
    head = f"P6\n{w} {h}\n255\n".encode()
    assert data.startswith(head)
    return data[len(head):]


def test_main_h_driver_initializes_without_gpu(driver_binary):
    # include/rtmi_main.hpp: initialize()/cleanup() of main.h over a scene YAML, device -1
    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    for extra in ([], ["--realtime", "--camera"]):
        out = subprocess.run([driver_binary, path, "--device", "-1", "--width", "40", "--height", "30", *extra],
                             check=True, capture_output=True, text=True).stdout
        assert "initialized 40x30, 3 channels" in out


@pytest.mark.gpu
def test_main_h_driver_offline_frame_equals_python(driver_binary, tmp_path):
    # offline pathTracing() (main.cu:889-897): one frame, imageData = gamma'd canvas
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.canvas import Canvas

    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    w, h, spp, depth = 64, 48, 4, 6
    subprocess.run([driver_binary, path, "--width", str(w), "--height", str(h), "--spp", str(spp), "--depth",
                    str(depth), "--out", str(tmp_path / "o.ppm")], check=True, capture_output=True)
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        img = r.render(w, h, spp, depth, lanes_per_pixel=0)
    want = Canvas(w, h).pixels(img)[::-1].reshape(-1)
    assert _ppm_rows(tmp_path / "o.ppm", w, h) == want.astype("uint8").tobytes()


@pytest.mark.gpu
def test_main_h_driver_realtime_frames_equal_accumulate(driver_binary, tmp_path):
    # GPU_REALTIME pathTracing() (main.cu:868-888): F frames of S fresh samples each into
    # the device accumulation == the same rt_accumulate sequence driven from Python
    import torch

    import raytracingthenextweekcuda_amd as rtmi

    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    w, h, spp, depth, frames = 48, 40, 2, 6, 3
    out = subprocess.run([driver_binary, path, "--width", str(w), "--height", str(h), "--spp", str(spp), "--depth",
                          str(depth), "--frames", str(frames), "--realtime", "--out", str(tmp_path / "rt.ppm")],
                         check=True, capture_output=True, text=True).stdout
    assert f"samples {frames * spp}" in out
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        acc = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
        px = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
        for f in range(frames):
            p = r.params(w, h, spp, depth, 1984, f * spp, 1, 0, 1, 0, "rayColor")
            r.accumulate_device(p, acc.data_ptr(), (f + 1) * spp, px.data_ptr())
        torch.cuda.synchronize()
        want = px.cpu().numpy()[::-1].reshape(-1)
    assert _ppm_rows(tmp_path / "rt.ppm", w, h) == want.tobytes()


@pytest.mark.gpu
def test_main_h_driver_camera_change_clears_accumulation(driver_binary, tmp_path):
    # camera->isDirty() -> clearBackBuffers() (main.cu:869-873): moving the camera before
    # frame 2 of 4 leaves exactly the image of 2 frames rendered from the moved camera
    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    w, h = 40, 32
    base = [driver_binary, path, "--width", str(w), "--height", str(h), "--spp", "2", "--depth", "5", "--realtime",
            "--camera"]

    def run(name, *extra):
        out = subprocess.run([*base, *extra, "--out", str(tmp_path / name)], check=True, capture_output=True,
                             text=True).stdout
        return out, _ppm_rows(tmp_path / name, w, h)

    out_a, a = run("a.ppm", "--frames", "4", "--move-at", "2")
    out_b, b = run("b.ppm", "--frames", "2", "--move-at", "0")
    _, c = run("c.ppm", "--frames", "4")
    assert "samples 4" in out_a and "samples 4" in out_b
    assert a == b and a != c
