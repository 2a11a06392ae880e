"""Checkpoint / resume of a progressive render (SURVEY §5's accumulation dump; the reference
keeps its accumulation only in device memory and loses it on exit): the accumulation sums as a
little-endian PFM (bottom row first, the buffer's own order) plus `<file>.json` with the
counters, from the Python Canvas and from the C++ facade's Canvas (rt_canvas_read/write_accumulation).
A render resumed from a dump continues the sample sequence: it ends on the bytes of an
uninterrupted run."""
import json
import os
import subprocess

import numpy as np
import pytest

from tests import scenes as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples")


def test_python_canvas_round_trip(tmp_path):
    from raytracingthenextweekcuda_amd.canvas import Canvas, read_pfm

    cv = Canvas(5, 3)
    cv.accumulation[...] = np.random.RandomState(1).uniform(0, 40, (3, 5, 3)).astype(np.float32)
    cv.sampleCount, cv.renderingTime = 37, 123.5
    path = str(tmp_path / "acc.pfm")
    cv.save(path, rows=[0, 2, 4])
    raw = open(path, "rb").read()
    assert raw.startswith(b"PF\n5 3\n-1.0\n")
    # PFM rows run bottom to top: the first stored row is the buffer's row 0 (the bottom row)
    first = np.frombuffer(raw[len(b"PF\n5 3\n-1.0\n"):], "<f4", count=15)
    assert np.array_equal(first, cv.accumulation[0].reshape(-1))
    back = Canvas.load(path)
    assert np.array_equal(back.accumulation, cv.accumulation) and np.array_equal(read_pfm(path), cv.accumulation)
    assert (back.sampleCount, back.renderingTime, back.rows) == (37, 123.5, [0, 2, 4])
    assert json.load(open(path + ".json"))["sampleCount"] == 37


@pytest.fixture(scope="module")
def driver_binary():
    subprocess.run(["make", "-s", "-C", EX, "main_driver"], check=True)
    return os.path.join(EX, "main_driver")


@pytest.mark.gpu
def test_resumed_realtime_render_equals_an_uninterrupted_one(driver_binary, tmp_path):
    """main.h driver, GPU_REALTIME: 2 frames + dump, then a new process resumes for 3 frames ==
    5 frames in one run, byte for byte; the dump holds the 2 frames' sums of rt_accumulate."""
    import torch

    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd.canvas import Canvas

    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    w, h, spp, depth = 40, 32, 2, 5
    base = [driver_binary, path, "--width", str(w), "--height", str(h), "--spp", str(spp), "--depth", str(depth),
            "--realtime"]
    ck = str(tmp_path / "ck.pfm")
    subprocess.run([*base, "--frames", "5", "--out", str(tmp_path / "a.ppm")], check=True, capture_output=True)
    subprocess.run([*base, "--frames", "2", "--save", ck, "--out", str(tmp_path / "b1.ppm")], check=True,
                   capture_output=True)
    out = subprocess.run([*base, "--frames", "3", "--resume", ck, "--out", str(tmp_path / "b.ppm")], check=True,
                         capture_output=True, text=True).stdout
    assert "samples 10" in out
    assert (tmp_path / "a.ppm").read_bytes() == (tmp_path / "b.ppm").read_bytes()
    dump = Canvas.load(ck)
    assert dump.sampleCount == 2
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        acc = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda")
        for f in range(2):
            r.accumulate_device(r.params(w, h, spp, depth, 1984, f * spp, 1, 0, 1, 0, "rayColor"), acc.data_ptr(),
                                (f + 1) * spp)
        torch.cuda.synchronize()
        assert np.array_equal(dump.accumulation, acc.cpu().numpy())
