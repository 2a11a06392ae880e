"""The reference's Camera object (Camera.h:12-196) and Canvas counters through the C ABI
(rt_camera_*, rtmi.h) and the C++ facade (include/rtmi.hpp, include/rtmi_main.hpp), against
the restatement's Camera (oracle/rt_oracle.c OrcCam) and hand-derived known answers.

The realtime frontend (OpenGLFrontend.cpp) moves the camera with walk / strafe / raise / yaw /
pitch (:393-407, :586-611), edits aperture / FOV / speed through the getters' references
(:189-197) and calls updateViewMatrix every frame (:611); pathTracing() then clears the
accumulation while the camera is dirty (main.cu:877-881). Every field must land on the same
floats as the reference's arithmetic."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from tests import scenes as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples")
F32 = np.float32


def _fields(state):
    return bytes(memoryview(state).cast("B"))


def _pair(*args):
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    return rtmi.Camera(*args), orc.OracleCamera(*args)


def test_camera_known_answers():
    import raytracingthenextweekcuda_amd as rtmi

    cam = rtmi.Camera((0.0, 0.0, 1.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 1.0, 90.0, 0.5, 2.0, 0.0, 1.0)
    s = cam.state
    # initialize: movingSpeed 1.5, dirty, lensRadius = aperture / 2, scale = tan(45 deg)
    assert s.moving_speed == 1.5 and cam.isDirty() and s.lens_radius == 0.25
    assert tuple(s.forward) == (0.0, 0.0, -1.0) and tuple(s.right) == (1.0, 0.0, 0.0)
    assert s.scale == pytest.approx(1.0, abs=1e-6) and s.viewport_width == s.viewport_height
    # walk(1): eye += forward * 1.5 * 1 -> z = 1 - 1.5; the view is not updated until
    # updateViewMatrix (origin still at the old eye)
    cam.walk(1.0)
    assert tuple(s.eye) == (0.0, 0.0, -0.5) and tuple(s.center) == (0.0, 0.0, -2.5)
    assert tuple(s.origin) == (0.0, 0.0, 1.0)
    cam.updateViewMatrix()
    assert tuple(s.origin) == (0.0, 0.0, -0.5)
    # updateViewMatrix leaves the flag set (updateLensRadius); resetDiryFlag clears it and a
    # clean camera's updateViewMatrix changes nothing
    assert cam.isDirty()
    cam.resetDiryFlag()
    before = _fields(s)
    cam.updateViewMatrix()
    assert _fields(s) == before
    # yaw(pi/2) turns forward (0,0,-1) to about (-1,0,0) and center = eye + forward
    cam.yaw(float(F32(np.pi / 2)))
    assert s.forward[0] == pytest.approx(-1.0) and abs(s.forward[2]) < 1e-6 and cam.isDirty()
    assert tuple(s.center) == tuple(F32(s.eye[k]) + F32(s.forward[k]) for k in range(3))
    # setAperture -> lensRadius = aperture / 2 (Camera.h:105-113)
    cam.setAperture(0.3)
    assert s.lens_radius == F32(F32(0.3) / F32(2.0))


@pytest.mark.parametrize("seed", range(6))
def test_camera_moves_equal_the_restatement(seed):
    """Random sequences of the frontend's calls: every field bit-identical to the oracle's."""
    rng = np.random.RandomState(seed)
    eye = rng.uniform(-3, 3, 3)
    center = eye + rng.uniform(-2, 2, 3)
    prod, ref = _pair(tuple(eye), tuple(center), (0.0, 1.0, 0.0), float(rng.uniform(0.5, 2.0)),
                      float(rng.uniform(20, 90)), float(rng.uniform(0, 0.2)), float(rng.uniform(0.5, 5.0)), 0.0, 1.0)
    assert _fields(prod.state) == _fields(ref.state)
    for _ in range(60):
        op = rng.randint(10)
        d = float(rng.uniform(-0.3, 0.3))
        if op < 6:
            name = ["walk", "strafe", "raise_", "yaw", "pitch", "updateViewMatrix"][op]
            for cam in (prod, ref):
                (getattr(cam, name)(d) if op < 5 else cam.updateViewMatrix())
        elif op == 6:
            t = tuple(rng.uniform(-1, 1, 3))
            prod.orbit(t)
            ref.orbit(t)
        elif op == 7:
            prod.setAperture(abs(d))
            ref.setAperture(abs(d))
        elif op == 8:  # the FOV slider writes through getFOV() then setDirty()
            prod.state.fov = ref.state.fov = float(rng.uniform(20, 90))
            prod.setDirty()
            ref.setDirty()
        else:
            prod.resetDiryFlag()
            ref.resetDiryFlag()
        assert _fields(prod.state) == _fields(ref.state), op


def test_scene_camera_is_the_yaml_camera():
    """rt_get_camera after a scene file: the Camera object initialize() made (main.cu:632-638)."""
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    path = os.path.join(S.SCENES, "cornellbox0.yaml")
    r = rtmi.Renderer(-1)
    r.load_yaml_native(path, 96, 64, S.MODELS)
    assert _fields(r.get_camera().state) == _fields(orc.yaml_camera(path, 96, 64).state)


# ---- OpenGLFrontend.cpp's loop without a window (examples/frontend_loop.cpp) ----

def _replay(cam, frames):
    """frontend_loop.cpp's scripted input + processInput for `frames` frames, on `cam`
    (the restatement's Camera), with the C++ program's float / double conversions."""
    ft = F32(1.0) / F32(60.0)  # frameTime
    rad = lambda deg: float(F32(F32(3.1415926535897932) / F32(180.0)) * F32(deg))  # noqa: E731
    for f in range(frames):
        keys = set()
        if f == 0:  # onScrollCallback(yOffset = 1): walk(float(1.0 / 8.0f))
            cam.walk(float(F32(1.0 / 8.0)))
        elif f == 1:  # right drag 100,100 -> 94,103
            dx, dy = (100.0 - 94.0) * float(ft), (100.0 - 103.0) * float(ft)
            cam.yaw(rad(F32(dx * 5.0)))
            cam.pitch(rad(F32(dy * 5.0)))
        elif f == 2:  # middle drag 50,50 -> 53,48
            dx, dy = (50.0 - 53.0) * float(ft), (50.0 - 48.0) * float(ft)
            cam.strafe(float(F32(-dx / 4.0)))
            cam.raise_(float(F32(dy / 4.0)))
        elif f == 3:  # sliders: aperture, FOV (each then setDirty), camera speed
            cam.state.aperture = float(F32(0.05))
            cam.setDirty()
            cam.state.fov = 55.0
            cam.setDirty()
            cam.state.moving_speed = 2.0
        elif f == 4:
            keys = {"W", "D"}
        elif f == 5:
            keys = {"S", "Q"}
        elif f == 6:
            keys = {"A", "E"}
        # processInput (OpenGLFrontend.cpp:576-612): A, D, W, S, Q, E, then updateViewMatrix
        for k, fn, sign in (("A", "strafe", -1), ("D", "strafe", 1), ("W", "walk", 1), ("S", "walk", -1),
                            ("Q", "raise_", 1), ("E", "raise_", -1)):
            if k in keys:
                getattr(cam, fn)(float(ft) * sign)
        cam.updateViewMatrix()
        yield f


@pytest.fixture(scope="module")
def loop_binary():
    subprocess.run(["make", "-s", "-C", EX, "frontend_loop"], check=True)
    return os.path.join(EX, "frontend_loop")


def _printed_state(out):
    vals = {}
    for line in out.splitlines():
        parts = line.split()
        if parts and parts[0] in ("eye", "center", "forward", "right", "origin", "lower_left", "horizontal",
                                  "vertical"):
            vals[parts[0]] = tuple(float.fromhex(p) for p in parts[1:4])
        m = re.match(r"lens_radius (\S+) fov (\S+) moving_speed (\S+)", line)
        if m:
            vals["lens_radius"], vals["fov"], vals["moving_speed"] = (float.fromhex(x) for x in m.groups())
    return vals


def test_frontend_loop_camera_equals_the_restatement(loop_binary):
    """The GL-free OpenGLFrontend loop (compiled against rtmi_main.hpp, librtmi.so only) ends
    on the camera the restatement reaches with the same calls."""
    from oracle import oracle as orc

    path = os.path.join(S.SCENES, "cornellbox1.yaml")
    out = subprocess.run([loop_binary, path, "--device", "-1", "--width", "64", "--height", "48", "--frames", "7",
                          "--still", "0"], check=True, capture_output=True, text=True).stdout
    got = _printed_state(out)
    cam = orc.yaml_camera(path, 64, 48)
    for _ in _replay(cam, 7):
        pass
    st = cam.state
    for k in ("eye", "center", "forward", "right", "origin", "lower_left", "horizontal", "vertical"):
        assert got[k] == tuple(getattr(st, k)), k
    assert (got["lens_radius"], got["fov"], got["moving_speed"]) == (st.lens_radius, st.fov, st.moving_speed)


@pytest.mark.gpu
def test_frontend_loop_frame_equals_the_restatement(loop_binary, tmp_path):
    """The loop on the GPU: the moves of frames 0-6 each clear the accumulation, so the final
    image is frames 6-9 (4 samples per pixel) seen by the final camera - gamma(acc * 1/4) of
    the restatement's frames with the replayed camera, byte for byte."""
    from oracle import oracle as orc

    path = os.path.join(S.SCENES, "cornellbox1.yaml")
    w, h, depth = 48, 40, 6
    out = subprocess.run([loop_binary, path, "--width", str(w), "--height", str(h), "--frames", "7", "--still", "3",
                          "--depth", str(depth), "--out", str(tmp_path / "loop.ppm")], check=True,
                         capture_output=True, text=True).stdout
    assert "sample count 4 " in out
    cam = orc.yaml_camera(path, w, h)
    for _ in _replay(cam, 10):
        pass
    sc = orc.yaml_scene(path, S.MODELS, w, h)
    cam.apply(sc)
    acc = np.zeros((h, w, 3), np.float32)
    for n in range(4):
        frame, _ = sc.render(w, h, 1, depth, sample_offset=n, threads=8)
        acc = acc + frame
    want = orc.gamma_u8(acc * (F32(1.0) / F32(4.0)))[::-1].reshape(-1)
    data = (tmp_path / "loop.ppm").read_bytes()
    head = f"P6\n{w} {h}\n255\n".encode()
    assert data.startswith(head) and data[len(head):] == want.tobytes()


@pytest.mark.gpu
def test_yaw_and_walk_render_the_restatements_frame():
    """A yaw + walk sequence, then updateViewMatrix: the product renders the oracle camera's
    frame bit for bit (and before updateViewMatrix, the old view's frame)."""
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc

    path = os.path.join(S.SCENES, "cornellbox1.yaml")
    w, h, spp, depth = 48, 40, 4, 6
    ocam = orc.yaml_camera(path, w, h)
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        cam = r.get_camera()
        for c in (cam, ocam):
            c.yaw(0.12)
            c.walk(-0.2)
            c.strafe(0.05)
        r.set_camera(cam)
        stale = r.render(w, h, spp, depth)  # not updated yet: the initial view
        for c in (cam, ocam):
            c.updateViewMatrix()
        r.set_camera(cam)
        moved = r.render(w, h, spp, depth)
        st = r.stats()
    sc = orc.yaml_scene(path, S.MODELS, w, h)
    ref0, _ = sc.render(w, h, spp, depth)
    ocam.apply(sc)
    ref, ref_st = sc.render(w, h, spp, depth)
    assert np.array_equal(stale, ref0)
    assert np.array_equal(moved, ref) and st["segments"] == ref_st["segments"]
    assert not np.array_equal(moved, stale)


@pytest.mark.gpu
def test_device_canvas_accumulates_like_canvas_h():
    """rt_canvas_* (the facade Canvas's device buffers): F realtime frames of 1 sample, the
    pixel buffer = gamma(acc * (1.0f / F)) (Canvas.h:82-98, 166-169); clear zeroes the sums."""
    import raytracingthenextweekcuda_amd as rtmi
    from oracle import oracle as orc
    from raytracingthenextweekcuda_amd._lib import lib

    L = lib()
    path = os.path.join(S.SCENES, "cornellbox1.yaml")
    w, h, depth, frames = 32, 24, 5, 3
    with rtmi.Renderer(0) as r:
        rtmi.load_yaml_scene(r, path, w, h)
        cv = C.c_void_p()
        assert L.rt_canvas_create(r.ctx, w, h, C.byref(cv)) == 0
        try:
            for n in range(frames):
                p = r.params(w, h, 1, depth, 1984, n)
                assert L.rt_canvas_accumulate(cv, C.byref(p), n + 1) == 0
            px = np.zeros((h, w, 3), np.uint8)
            acc = np.zeros((h, w, 3), np.float32)
            assert L.rt_canvas_read_pixels(cv, px.ctypes.data_as(C.POINTER(C.c_uint8))) == 0
            assert L.rt_canvas_read_accumulation(cv, acc.ctypes.data_as(C.POINTER(C.c_float))) == 0
            assert L.rt_canvas_clear_accumulation(cv) == 0
            zero = np.ones((h, w, 3), np.float32)
            assert L.rt_canvas_read_accumulation(cv, zero.ctypes.data_as(C.POINTER(C.c_float))) == 0
        finally:
            L.rt_canvas_destroy(cv)
    sc = orc.yaml_scene(path, S.MODELS, w, h)
    want = np.zeros((h, w, 3), np.float32)
    for n in range(frames):
        want = want + sc.render(w, h, 1, depth, sample_offset=n, threads=8)[0]
    assert np.array_equal(acc, want)
    assert np.array_equal(px, orc.gamma_u8(want * (F32(1.0) / F32(frames))))
    assert not zero.any()
