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
