"""ctypes front-end of the CPU restatement (rt_oracle.c).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker. The product package never imports
this module.

Scene construction follows the reference's host code independently of the
product package: YAML scenes with main.cu:629-786 semantics (pre-seeded
materials 0-8, first-key primitive type, meshes always on materials[3]).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_rt.so")

_f3 = C.c_float * 3
_lib = None


def build() -> str:
    """Compile liboracle_rt.so (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class OracleCameraState(C.Structure):
    """The restatement's Camera object (rt_oracle.c OrcCam: Camera.h:169-195's fields)."""
    _fields_ = [(n, C.c_float * 3) for n in ("eye", "center", "up", "forward", "right", "true_up", "origin",
                                             "horizontal", "vertical", "lower_left")] + \
        [(n, C.c_float) for n in ("aspect_ratio", "fov", "scale", "viewport_height", "viewport_width",
                                  "moving_speed", "aperture", "focus_distance", "lens_radius", "time0", "time1")] + \
        [("dirty", C.c_int32)]


class OracleCamera:
    """Camera (Camera.h:12-196) in the restatement: the same method names as the product's."""

    def __init__(self, eye, center, up, aspectRatio, fov=90.0, aperture=2.0, focusDistance=1.0,
                 time0=0.0, time1=0.0):
        self.L = lib()
        self.state = OracleCameraState()
        self.L.orc_cam_initialize(C.byref(self.state), f3(eye), f3(center), f3(up), aspectRatio, fov, aperture,
                                  focusDistance, time0, time1)

    def walk(self, d):
        self.L.orc_cam_walk(C.byref(self.state), d)

    def strafe(self, d):
        self.L.orc_cam_strafe(C.byref(self.state), d)

    def raise_(self, d):
        self.L.orc_cam_raise(C.byref(self.state), d)

    def yaw(self, d):
        self.L.orc_cam_yaw(C.byref(self.state), d)

    def pitch(self, d):
        self.L.orc_cam_pitch(C.byref(self.state), d)

    def orbit(self, target):
        self.L.orc_cam_orbit(C.byref(self.state), f3(target))

    def updateViewMatrix(self):
        self.L.orc_cam_update_view_matrix(C.byref(self.state))

    def setAperture(self, a):
        self.L.orc_cam_set_aperture(C.byref(self.state), a)

    def setDirty(self):
        self.state.dirty = 1

    def isDirty(self):
        return bool(self.state.dirty)

    def resetDiryFlag(self):
        self.state.dirty = 0

    def apply(self, scene: "OracleScene"):
        """The scene renders with this camera's current view (the fields getRay reads)."""
        self.L.orc_scene_camera_from(scene.h, C.byref(self.state))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        fp = C.POINTER(C.c_float)
        L.orc_scene_new.restype = vp
        L.orc_scene_free.argtypes = [vp]
        L.orc_material.argtypes = [vp, C.c_int, C.c_int, fp, C.c_float]
        L.orc_material_defined.argtypes = [vp, C.c_int]
        L.orc_sphere.argtypes = [vp, C.c_int, fp, C.c_float, C.c_int]
        L.orc_moving_sphere.argtypes = [vp, C.c_int, fp, fp, C.c_float, C.c_float, C.c_float, C.c_int]
        L.orc_plane.argtypes = [vp, C.c_int, fp, fp, fp, C.c_int, C.c_int, C.c_int]
        L.orc_cube.argtypes = [vp, C.c_int, fp, fp, C.c_int]
        L.orc_constant_medium.argtypes = [vp, C.c_int, fp, fp, C.c_float, C.c_int]
        L.orc_mesh.argtypes = [vp, C.c_int, fp, C.c_int, C.c_int]
        L.orc_mesh_obj.argtypes = [vp, C.c_int, C.c_char_p, fp, fp, fp, C.c_int]
        L.orc_load_obj.argtypes = [C.c_char_p, fp, fp, fp, C.POINTER(fp)]
        L.orc_free.argtypes = [vp]
        L.orc_load_ply.argtypes = [C.c_char_p, fp, C.c_float, C.POINTER(fp)]
        L.orc_bvh_image.restype = C.c_int64
        L.orc_bvh_image.argtypes = [fp, C.c_int, C.POINTER(C.POINTER(C.c_uint8))]
        L.orc_camera.argtypes = [vp, fp, fp, fp] + [C.c_float] * 6
        L.orc_length.argtypes = [fp]
        L.orc_length.restype = C.c_float
        L.orc_render.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                 C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, fp, C.POINTER(C.c_uint64),
                                 C.c_int, C.c_int]
        L.orc_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.orc_uniforms.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, fp]
        L.orc_trace.argtypes = [vp, fp, fp, C.c_float, fp, fp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_pt_new.restype = vp
        L.orc_pt_free.argtypes = [vp]
        L.orc_pt_load_object.argtypes = [vp, C.c_char_p, C.c_int]
        L.orc_pt_process.argtypes = [vp, fp, C.c_float]
        L.orc_pt_set_bvh.argtypes = [vp, C.POINTER(C.c_uint8), C.c_int64]
        L.orc_pt_render.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                    C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, fp,
                                    C.POINTER(C.c_uint64), C.c_int, C.c_int]
        L.orc_pt_sinf.argtypes = [C.c_float]
        L.orc_pt_sinf.restype = C.c_float
        L.orc_pt_cosf.argtypes = [C.c_float]
        L.orc_pt_cosf.restype = C.c_float
        L.orc_pt_powf.argtypes = [C.c_float, C.c_float]
        L.orc_pt_powf.restype = C.c_float
        L.orc_gamma_u8.argtypes = [fp, C.c_int64, C.POINTER(C.c_uint8)]
        cs = C.POINTER(OracleCameraState)
        L.orc_cam_initialize.argtypes = [cs, fp, fp, fp] + [C.c_float] * 6
        L.orc_cam_update_view_matrix.argtypes = [cs]
        for name in ("walk", "strafe", "raise", "yaw", "pitch", "set_aperture"):
            getattr(L, "orc_cam_" + name).argtypes = [cs, C.c_float]
        L.orc_cam_orbit.argtypes = [cs, fp]
        L.orc_scene_camera_from.argtypes = [vp, cs]
        _lib = L
    return _lib


def f3(v):
    return _f3(*[float(x) for x in v])


def philox(ctr, key):
    out = (C.c_uint32 * 4)()
    lib().orc_philox((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
    return list(out)


def uniforms(seed, pixel, sample, n):
    out = np.zeros(n, np.float32)
    lib().orc_uniforms(seed, pixel, sample, n, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def load_obj(path, scale=(1, 1, 1), rotate=(0, 0, 0), offset=(0, 0, 0)) -> np.ndarray:
    p = C.POINTER(C.c_float)()
    n = lib().orc_load_obj(path.encode(), f3(scale), f3(rotate), f3(offset), C.byref(p))
    if n < 0:
        raise IOError(f"oracle OBJ load failed: {path}")
    arr = np.ctypeslib.as_array(p, shape=(max(n, 1) * 9,)).copy()[: n * 9]
    lib().orc_free(p)
    return arr.reshape(n, 9)


def load_ply(path, offset=(0, 0, 0), max_coord=1.0) -> np.ndarray:
    p = C.POINTER(C.c_float)()
    n = lib().orc_load_ply(path.encode(), f3(offset), max_coord, C.byref(p))
    if n < 0:
        raise IOError(f"oracle PLY load failed: {path}")
    arr = np.ctypeslib.as_array(p, shape=(max(n, 1) * 9,)).copy()[: n * 9]
    lib().orc_free(p)
    return arr.reshape(n, 9)


def bvh_image(soup: np.ndarray) -> bytes:
    """CreateBVH + Recurse + CreateCFBVH (BVH.cpp:94-497) with the reference's own
    O(N x bins) split search over a triangle soup (n x 9 floats, e.g. load_ply's):
    the `.bvh` cache image."""
    soup = np.ascontiguousarray(soup, np.float32).reshape(-1, 9)
    p = C.POINTER(C.c_uint8)()
    n = lib().orc_bvh_image(soup.ctypes.data_as(C.POINTER(C.c_float)), len(soup), C.byref(p))
    if n < 0:
        raise ValueError("oracle BVH build failed")
    img = C.string_at(p, n)
    lib().orc_free(p)
    return img


def gamma_u8(rgb: np.ndarray) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(rgb.shape, np.uint8)
    lib().orc_gamma_u8(rgb.ctypes.data_as(C.POINTER(C.c_float)), rgb.size,
                       out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


class OracleScene:
    """Scene in the CPU restatement; method names follow kernels.h factories."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.orc_scene_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_scene_free(self.h)
            self.h = None

    def material(self, idx, mtype, albedo=(1, 1, 1), param=1.0):
        assert self.L.orc_material(self.h, idx, mtype, f3(albedo), param) == 0

    def defined(self, idx):
        return bool(self.L.orc_material_defined(self.h, idx))

    def sphere(self, idx, c, r, mat):
        assert self.L.orc_sphere(self.h, idx, f3(c), r, mat) == 0

    def moving_sphere(self, idx, c0, c1, t0, t1, r, mat):
        assert self.L.orc_moving_sphere(self.h, idx, f3(c0), f3(c1), t0, t1, r, mat) == 0

    def plane(self, idx, pos, n, ext, mat, orient, two):
        assert self.L.orc_plane(self.h, idx, f3(pos), f3(n), f3(ext), mat, orient, int(two)) == 0

    def cube(self, idx, c, ext, mat):
        assert self.L.orc_cube(self.h, idx, f3(c), f3(ext), mat) == 0

    def constant_medium(self, idx, c, ext, density, mat):
        assert self.L.orc_constant_medium(self.h, idx, f3(c), f3(ext), density, mat) == 0

    def mesh(self, idx, verts, mat):
        v = np.ascontiguousarray(verts, np.float32).reshape(-1)
        assert self.L.orc_mesh(self.h, idx, v.ctypes.data_as(C.POINTER(C.c_float)), v.size // 9, mat) == 0

    def mesh_obj(self, idx, path, scale, rotate, offset, mat):
        assert self.L.orc_mesh_obj(self.h, idx, path.encode(), f3(scale), f3(rotate), f3(offset), mat) == 0

    def camera(self, eye, center, up, aspect, fov, aperture, focus, t0=0.0, t1=0.0):
        self.L.orc_camera(self.h, f3(eye), f3(center), f3(up), aspect, fov, aperture, focus, t0, t1)

    def trace(self, o, d, time=0.0):
        t = C.c_float()
        n = _f3()
        front = C.c_int()
        mat = C.c_int()
        hit = self.L.orc_trace(self.h, f3(o), f3(d), time, C.byref(t), n, C.byref(front), C.byref(mat))
        if not hit:
            return None
        return float(t.value), tuple(n), bool(front.value), int(mat.value)

    def render(self, width, height, spp, depth, seed=1984, sample_offset=0, row_block=1,
               row_rank=0, row_world=1, threads=0, lanes_per_pixel=1, col_begin=0, col_count=0):
        rows = owned_rows(height, row_block, row_rank, row_world)
        out = np.zeros((rows, col_count or width, 3), np.float32)
        stats = (C.c_uint64 * 2)()
        rc = self.L.orc_render(self.h, width, height, spp, depth, seed, sample_offset, row_block,
                               row_rank, row_world, lanes_per_pixel, threads,
                               out.ctypes.data_as(C.POINTER(C.c_float)), stats, col_begin, col_count)
        if rc != 0:
            raise RuntimeError(f"orc_render failed with {rc}")
        return out, {"segments": int(stats[0]), "tri_tests": int(stats[1])}


REFLECTION_TYPES = {"DIFFUSE": 0, "METAL": 1, "SPECULAR": 2, "REFRACTION": 3, "COAT": 4}


class OraclePathTrace:
    """pathTrace scene of the CPU restatement (prepareCUDAscene, main.cu:404-553):
    PLY meshes via load_object, processTriangleData via process, and the BVH
    from a `.bvh` cache image (the reference's own files in the tests). The
    camera comes from an OracleScene (its `camera`)."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.orc_pt_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_pt_free(self.h)
            self.h = None

    def load_object(self, path, reflection_type="COAT"):
        t = REFLECTION_TYPES[reflection_type] if isinstance(reflection_type, str) else int(reflection_type)
        assert self.L.orc_pt_load_object(self.h, str(path).encode(), t) == 0, path

    def process(self, offset=(0.0, 0.0, 0.0), max_coord=1.0):
        assert self.L.orc_pt_process(self.h, f3(offset), max_coord) == 0

    def set_bvh(self, image: bytes):
        buf = (C.c_uint8 * len(image)).from_buffer_copy(image)
        rc = self.L.orc_pt_set_bvh(self.h, buf, len(image))
        if rc:
            raise ValueError(f"bad .bvh image ({rc})")

    def render(self, cam: OracleScene, width, height, spp, bounces=5, seed=1984, sample_offset=0,
               row_block=1, row_rank=0, row_world=1, threads=0, lanes_per_pixel=1, col_begin=0,
               col_count=0):
        rows = owned_rows(height, row_block, row_rank, row_world)
        out = np.zeros((rows, col_count or width, 3), np.float32)
        stats = (C.c_uint64 * 3)()
        rc = self.L.orc_pt_render(self.h, cam.h, width, height, spp, bounces, seed, sample_offset,
                                  row_block, row_rank, row_world, lanes_per_pixel, threads,
                                  out.ctypes.data_as(C.POINTER(C.c_float)), stats, col_begin, col_count)
        if rc != 0:
            raise RuntimeError(f"orc_pt_render failed with {rc}")
        return out, {"segments": int(stats[0]), "tri_tests": int(stats[1]), "overflow": int(stats[2])}


def owned_rows(height, block, rank, world):
    n = 0
    b = rank
    while b * block < height:
        r0 = b * block
        n += min(r0 + block, height) - r0
        b += world
    return n


# --------------------------------------------------------------------------
# YAML scenes, restating main.cu:629-786 (SCENE == 1) independently of the
# product package.
# --------------------------------------------------------------------------
def preseed_materials(sc: OracleScene):
    # main.cu:643-651
    sc.material(0, 0, (1.0, 0.0, 0.0), 1.0)
    sc.material(1, 0, (0.0, 1.0, 0.0), 1.0)
    sc.material(2, 0, (0.0, 0.0, 1.0), 1.0)
    sc.material(3, 0, (1.0, 1.0, 1.0), 1.0)
    sc.material(4, 0, (0.75, 0.25, 0.25), 1.0)
    sc.material(5, 0, (0.25, 0.25, 0.75), 1.0)
    sc.material(6, 1, (1.0, 1.0, 1.0), 0.0)
    sc.material(7, 2, (1.0, 1.0, 1.0), 1.5)
    sc.material(8, 3, (1.0, 1.0, 1.0), 5.0)


def yaml_camera(cfg, width: int, height: int) -> OracleCamera:
    """initialize()'s camera of a scene YAML (main.cu:632-638); `cfg` = the parsed file or its path."""
    if isinstance(cfg, str):
        import yaml

        with open(cfg) as fh:
            cfg = yaml.safe_load(fh)
    cam = cfg["camera"]
    eye, center, up = cam["eye"], cam["center"], cam["up"]
    focus = lib().orc_length(f3(np.float32(center) - np.float32(eye)))  # (center - eye).length()
    aspect = float(np.float32(width) / np.float32(height))              # Float(width) / height
    return OracleCamera(eye, center, up, aspect, float(cam["fov"]), float(cam["aperture"]), focus, 0.0, 1.0)


def yaml_scene(path: str, models_dir: str, width: int, height: int) -> OracleScene:
    import yaml

    with open(path) as fh:
        cfg = yaml.safe_load(fh)
    sc = OracleScene()
    yaml_camera(cfg, width, height).apply(sc)
    preseed_materials(sc)
    for i, entry in enumerate(cfg["objects"]):
        key = next(iter(entry))
        obj = entry[key]
        mat = obj["material"]
        mid = int(obj["materialId"])
        mtype = int(mat["type"])
        if not sc.defined(mid):
            if mtype == 0:
                sc.material(mid, 0, mat["albedo"], 1.0)
            elif mtype == 2:
                sc.material(mid, 2, (1, 1, 1), float(mat["indexOfRefraction"]))
            elif mtype == 1:
                sc.material(mid, 1, mat["albedo"], float(mat["fuzz"]))
            elif mtype == 3:
                sc.material(mid, 3, mat["albedo"], float(mat["intensity"]))
            elif mtype == 4:
                sc.material(mid, 4, mat["albedo"], 0.0)
        ptype = int(next(iter(obj.values())))  # first key of the object map (main.cu:706, 749)
        if ptype == 0:
            sc.sphere(i, obj["center"], float(obj["radius"]), mid)
        elif ptype == 1:
            sc.plane(i, obj["position"], obj["normal"], obj["extend"], mid, int(obj["orientation"]),
                     bool(obj["twoSide"]))
        elif ptype == 2:  # meshes always use materials[3] (main.cu:781)
            model = os.path.join(models_dir, obj["model"])
            if model.lower().endswith(".ply"):  # build extension (PLY placement)
                sc.mesh(i, load_ply(model, obj.get("offset", (0, 0, 0)), float(obj.get("maxCoord", 1.0))), 3)
            else:
                sc.mesh_obj(i, model, obj["scale"], obj["rotate"], obj["offset"], 3)
        elif ptype == 3:  # build extension: cube
            sc.cube(i, obj["center"], obj["extend"], mid)
        elif ptype == 4:  # build extension: constant medium
            sc.constant_medium(i, obj["center"], obj["extend"], float(obj["density"]), mid)
        else:
            raise ValueError(f"unknown primitive type {ptype}")
    return sc


def json_scene(path: str, width: int, height: int) -> OracleScene:
    """Object-list scenes (assets/scenes/random_spheres.json): one material per
    object slot, as the reference's SCENE 2 code (main.cu:792-848)."""
    import json

    with open(path) as fh:
        d = json.load(fh)
    sc = OracleScene()
    c = d["camera"]
    aspect = float(np.float32(width) / np.float32(height))
    sc.camera(c["eye"], c["center"], c["up"], aspect, float(c["fov"]), float(c["aperture"]),
              float(c["focus"]), float(c.get("time0", 0.0)), float(c.get("time1", 0.0)))
    kinds = {"lambertian": 0, "metal": 1, "dielectric": 2, "emission": 3}
    for i, o in enumerate(d["objects"]):
        m = o["material"]
        k = kinds[m["type"]]
        param = {0: 1.0, 1: m.get("fuzz", 0.0), 2: m.get("ior", 1.5), 3: m.get("intensity", 1.0)}[k]
        sc.material(i, k, m.get("albedo", (1, 1, 1)), float(param))
        if o["kind"] == "sphere":
            sc.sphere(i, o["center"], float(o["radius"]), i)
        else:
            sc.moving_sphere(i, o["center0"], o["center1"], float(o["time0"]), float(o["time1"]),
                             float(o["radius"]), i)
    return sc
