"""Host-side mirror of the reference's scene API over the C ABI.

The reference builds scenes with device-side factories that take a pointer
table and a slot index (kernels.h:50-154), a Camera (Camera.h) and a Canvas
(Canvas.h). This module keeps those names and argument meanings so scene code
written like main.cu:592-848 ports line by line:

    r = Renderer(device=0)
    materials, spheres = r.materials, r.objects          # createObjectPtrArray
    createLambertianMaterial(materials, 0, (1, 0, 0))    # kernels.h:54
    createSphere(spheres, 0, (-1, 0, -1), 0.5, materials[0])
    r.set_camera(Camera(eye, center, up, aspect, fov, aperture, focus, 0, 1))
    img = r.render(width, height, spp, depth)            # pathTracing()

`materials[i]` is None until slot i is created, so the reference's
`if (materials[id] == nullptr)` guards (main.cu:714-744) read the same.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import RT_OK, SCHEDULES, CameraState, RenderParams, RenderStats, RTError, lib, variant_name

_f3 = C.c_float * 3


def _v(x):
    return _f3(*[float(c) for c in x])


@dataclass(frozen=True)
class MaterialHandle:
    """Opaque non-null stand-in for a device `Material*`."""
    index: int


class _Table:
    def __init__(self, renderer: "Renderer"):
        self._r = renderer


class MaterialTable(_Table):
    """createObjectPtrArray<Material*>(n) (kernels.h:26-31)."""

    def __getitem__(self, i: int):
        return MaterialHandle(i) if lib().rt_material_defined(self._r.ctx, i) else None


class ObjectTable(_Table):
    """createObjectPtrArray<Hitable*>(n): slot order = closest-hit scan order."""


def _mat_index(m) -> int:
    if m is None:
        raise ValueError("material is nullptr (slot not created)")
    return m.index if isinstance(m, MaterialHandle) else int(m)


class Camera:
    """The reference's Camera (Camera.h:12-196) over the library's restatement of its
    methods (rt_camera_*, rtmi.h), so camera moves land on the reference's floats:
    Camera(eye, center, up, aspectRatio, fov=90, aperture=2, focusDistance=1, time0=0,
    time1=0) - the Camera.h:14-17 defaults. Renderer.set_camera hands the current view
    (the fields getRay reads) to a context."""

    def __init__(self, eye, center, up, aspectRatio, fov=90.0, aperture=2.0,
                 focusDistance=1.0, time0=0.0, time1=0.0):
        self.state = CameraState()
        self.initialize(eye, center, up, aspectRatio, fov, aperture, focusDistance, time0, time1)

    @classmethod
    def from_state(cls, state: CameraState) -> "Camera":
        cam = cls.__new__(cls)
        cam.state = CameraState()
        C.pointer(cam.state)[0] = state
        return cam

    def _call(self, name, *args):
        st = getattr(lib(), "rt_camera_" + name)(C.byref(self.state), *args)
        if st != RT_OK:
            raise RTError(st, f"rt_camera_{name}")

    def initialize(self, eye, center, up, aspectRatio, fov=90.0, aperture=2.0,
                   focusDistance=1.0, time0=0.0, time1=0.0):
        self._call("initialize", _v(eye), _v(center), _v(up), float(aspectRatio), float(fov), float(aperture),
                   float(focusDistance), float(time0), float(time1))

    # Camera.h:40-84
    def walk(self, delta):
        self._call("walk", float(delta))

    def strafe(self, delta):
        self._call("strafe", float(delta))

    def raise_(self, delta):  # `raise` is a Python keyword
        self._call("raise", float(delta))

    def yaw(self, delta):
        self._call("yaw", float(delta))

    def pitch(self, delta):
        self._call("pitch", float(delta))

    def orbit(self, target):
        self._call("orbit", _v(target))

    def updateViewMatrix(self):
        self._call("update_view_matrix")

    def setAperture(self, a):
        self._call("set_aperture", float(a))

    def getAperture(self):
        return self.state.aperture

    def getFOV(self):
        return self.state.fov

    def getMovingSpeed(self):
        return self.state.moving_speed

    def setDirty(self):
        self.state.dirty = 1

    def isDirty(self):
        return bool(self.state.dirty)

    def resetDiryFlag(self):  # reference spelling (Camera.h:147)
        self.state.dirty = 0

    # the constructor's parameters
    eye = property(lambda self: tuple(self.state.eye))
    center = property(lambda self: tuple(self.state.center))
    up = property(lambda self: tuple(self.state.up))
    aspectRatio = property(lambda self: self.state.aspect_ratio)
    fov = property(lambda self: self.state.fov)
    aperture = property(lambda self: self.state.aperture)
    focusDistance = property(lambda self: self.state.focus_distance)
    time0 = property(lambda self: self.state.time0)
    time1 = property(lambda self: self.state.time1)


class Renderer:
    """One rt_ctx on one HIP device (replaces initialize()/cleanup(), main.cu:555-936)."""

    def __init__(self, device: int = 0):
        self.L = lib()
        h = C.c_void_p()
        st = self.L.rt_create(device, C.byref(h))
        if st != RT_OK:
            raise RTError(st, f"rt_create(device={device}) failed")
        self.ctx = h
        self.device = device
        self.materials = MaterialTable(self)
        self.objects = ObjectTable(self)
        self._camera = None

    def close(self):
        if getattr(self, "ctx", None):
            self.L.rt_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st):
        if st != RT_OK:
            raise RTError(st, self.L.rt_last_error(self.ctx).decode(errors="replace"))

    # ---- scene ----
    def clear(self):
        self._check(self.L.rt_clear_scene(self.ctx))

    def lambertian(self, index, albedo, absorb=1.0):
        self._check(self.L.rt_material_lambertian(self.ctx, index, _v(albedo), absorb))

    def metal(self, index, albedo, fuzz=1.0):
        self._check(self.L.rt_material_metal(self.ctx, index, _v(albedo), fuzz))

    def dielectric(self, index, ior=1.5):
        self._check(self.L.rt_material_dielectric(self.ctx, index, ior))

    def emission(self, index, albedo, intensity=1.0):
        self._check(self.L.rt_material_emission(self.ctx, index, _v(albedo), intensity))

    def isotropic(self, index, albedo):
        """Phase function of participating media (build extension, rtmi.h)."""
        self._check(self.L.rt_material_isotropic(self.ctx, index, _v(albedo)))

    def sphere(self, index, center, radius, material, shading=True):
        self._check(self.L.rt_sphere(self.ctx, index, _v(center), radius, _mat_index(material), int(shading)))

    def moving_sphere(self, index, c0, c1, t0, t1, radius, material):
        self._check(self.L.rt_moving_sphere(self.ctx, index, _v(c0), _v(c1), t0, t1, radius,
                                            _mat_index(material)))

    def plane(self, index, position, normal, extend, material, orientation=2, two_side=True):
        self._check(self.L.rt_plane(self.ctx, index, _v(position), _v(normal), _v(extend),
                                    _mat_index(material), int(orientation), int(bool(two_side))))

    def cube(self, index, center, extend, material):
        self._check(self.L.rt_cube(self.ctx, index, _v(center), _v(extend), _mat_index(material)))

    def constant_medium(self, index, center, extend, density, material):
        """Constant-density medium in an axis-aligned cube (build extension, rtmi.h)."""
        self._check(self.L.rt_constant_medium(self.ctx, index, _v(center), _v(extend), density,
                                              _mat_index(material)))

    def mesh(self, index, tri_vertices, material):
        v = np.ascontiguousarray(tri_vertices, np.float32).reshape(-1)
        if v.size % 9:
            raise ValueError("mesh vertices must be 9 floats per triangle")
        self._check(self.L.rt_mesh(self.ctx, index, v.ctypes.data_as(C.POINTER(C.c_float)),
                                   v.size // 9, _mat_index(material)))

    def mesh_obj(self, index, path, scale=(1, 1, 1), rotate=(0, 0, 0), offset=(0, 0, 0), material=3):
        self._check(self.L.rt_mesh_obj(self.ctx, index, str(path).encode(), _v(scale), _v(rotate),
                                       _v(offset), _mat_index(material)))

    def mesh_ply(self, index, path, offset=(0, 0, 0), max_coord=1.0, material=3):
        """PLY mesh with loadObject + processTriangleData semantics (Loader.cpp)."""
        self._check(self.L.rt_mesh_ply(self.ctx, index, str(path).encode(), _v(offset), max_coord,
                                       _mat_index(material)))

    # ---- pathTrace scene (prepareCUDAscene, main.cu:404-553) ----
    def load_object(self, path, reflection_type="COAT"):
        """loadObject(file, ReflectionType, meshIndex) (Loader.cpp:207-319): append a PLY mesh."""
        self._check(self.L.rt_load_object(self.ctx, str(path).encode(), _reflection_type(reflection_type)))

    def process_triangle_data(self, offset=(0.0, 0.0, 0.0), max_coord=1.0) -> dict:
        """processTriangleData (Loader.cpp:98-205) + BVH build + upload. Returns the census."""
        out = (C.c_int32 * 4)()
        self._check(self.L.rt_process_triangle_data(self.ctx, _v(offset), max_coord, out))
        return {"triangles": out[0], "bvh_nodes": out[1], "tri_list": out[2], "depth": out[3]}

    def set_bvh_builder(self, builder: str = "host"):
        """BVH builder for rt_commit / process_triangle_data: "host" (Recurse on the
        host) or "gpu" (the byte-identical level-synchronous GPU restatement)."""
        code = {"host": 0, "gpu": 1}[builder]
        self._check(self.L.rt_set_bvh_builder(self.ctx, code))

    def set_bvh_cache(self, mode: int = 3):
        """rt_set_bvh_cache: 1 = read `<ply>.bvh` when fresh (UpdateBoundingVolumeHierarchy,
        BVH.cpp:500-554), 2 = write it after a build, 3 = both (the reference), 0 = off."""
        self._check(self.L.rt_set_bvh_cache(self.ctx, int(mode)))

    def bvh_cache_stats(self) -> dict:
        r, w, x = C.c_int32(), C.c_int32(), C.c_int32()
        self._check(self.L.rt_bvh_cache_stats(self.ctx, C.byref(r), C.byref(w), C.byref(x)))
        return {"reads": r.value, "writes": w.value, "rejected": x.value}

    def bvh_build_stats(self) -> dict:
        """Wall time of the last commit's + process_triangle_data's BVH builds, and
        how many the GPU builder ran."""
        ms, n = C.c_double(), C.c_int32()
        self._check(self.L.rt_bvh_build_stats(self.ctx, C.byref(ms), C.byref(n)))
        return {"build_ms": ms.value, "gpu_builds": n.value}

    def pathtrace_bvh_image(self) -> bytes:
        """The `.bvh` cache image of the processed pathTrace scene (BVH.cpp:537-540)."""
        size = C.c_int64()
        self._check(self.L.rt_pathtrace_bvh_image(self.ctx, None, 0, C.byref(size)))
        buf = (C.c_uint8 * size.value)()
        self._check(self.L.rt_pathtrace_bvh_image(self.ctx, buf, size.value, C.byref(size)))
        return bytes(buf)

    def mesh_vertices(self, index) -> np.ndarray:
        n = self.L.rt_mesh_triangle_count(self.ctx, index)
        out = np.zeros((n, 9), np.float32)
        if n:
            self._check(self.L.rt_mesh_vertices(self.ctx, index, out.ctypes.data_as(C.POINTER(C.c_float)), n))
        return out

    def set_camera(self, cam: Camera):
        """The context renders with the camera's current view (rt_camera_apply)."""
        self._camera = cam
        self._check(self.L.rt_camera_apply(self.ctx, C.byref(cam.state)))

    def get_camera(self) -> Camera:
        """The context's current Camera object (rt_get_camera): a scene file's camera too."""
        st = CameraState()
        self._check(self.L.rt_get_camera(self.ctx, C.byref(st)))
        return Camera.from_state(st)

    def commit(self):
        self._check(self.L.rt_commit(self.ctx))

    def object_counts(self) -> dict:
        """Census of the committed device tables (rt_scene_info)."""
        out = (C.c_int32 * 8)()
        self._check(self.L.rt_scene_info(self.ctx, out))
        keys = ["plane", "sphere", "moving_sphere", "mesh", "triangle", "material", "bvh_node",
                "grouped_spheres"]
        return {k: int(out[i]) for i, k in enumerate(keys)}

    def bvh_depth(self) -> int:
        """rt_scene_bvh_depth: the traversal stack entries per lane the committed scene needs."""
        out = C.c_int32()
        self._check(self.L.rt_scene_bvh_depth(self.ctx, C.byref(out)))
        return int(out.value)

    def scene_digest(self) -> int:
        """FNV-1a 64 digest of the committed host tables (rt_scene_digest)."""
        out = C.c_uint64()
        self._check(self.L.rt_scene_digest(self.ctx, C.byref(out)))
        return int(out.value)

    def load_yaml_native(self, path, width, height, models_dir):
        """The scene file through the library's own reader (rt_load_yaml_scene,
        initialize() of main.cu:623-786); does not commit."""
        self._check(self.L.rt_load_yaml_scene(self.ctx, str(path).encode(), str(models_dir).encode(),
                                              int(width), int(height)))

    # ---- render ----
    @staticmethod
    def params(width, height, spp, max_depth, seed=1984, sample_offset=0, row_block=1,
               row_rank=0, row_world=1, lanes_per_pixel=1, integrator="rayColor",
               keep_counters=False, col_begin=0, col_count=0, schedule="auto",
               frames_in_flight=False) -> RenderParams:
        """rt_render_params; schedule "auto" = the persistent work queue (the static grid when
        the frame's partial sums do not fit), "static" = the static grid (same image).
        frames_in_flight: the caller overlaps three or more launches (RT_RENDER_FRAMES_IN_FLIGHT;
        the auto layout of linear-scan launches then takes at most 16 sub-streams)."""
        flags = (KEEP_COUNTERS if keep_counters else 0) | (FRAMES_IN_FLIGHT if frames_in_flight else 0)
        return RenderParams(width, height, spp, max_depth, seed, sample_offset, row_block,
                            row_rank, row_world, lanes_per_pixel, _integrator(integrator),
                            flags, col_begin, col_count, SCHEDULES[schedule])

    def render(self, width, height, spp, max_depth, seed=1984, sample_offset=0, row_block=1,
               row_rank=0, row_world=1, lanes_per_pixel=1, integrator="rayColor",
               col_begin=0, col_count=0, schedule="auto", frames_in_flight=False) -> np.ndarray:
        """Mean radiance of the owned rows, shape (rows, width, 3), y = 0 bottom.
        lanes_per_pixel=1 keeps the reference's sequential per-pixel sample sum;
        0 lets the library pick a lane layout that fills the GPU. integrator
        "pathTrace" runs CUDAPathTracer.cu's integrator over the
        load_object/process_triangle_data scene (max_depth = its 5 bounces).
        col_count > 0 renders only columns [col_begin, col_begin + col_count) of the
        frame's rows (shape (rows, col_count, 3)); the pixels are the full frame's."""
        p = self.params(width, height, spp, max_depth, seed, sample_offset, row_block, row_rank,
                        row_world, lanes_per_pixel, integrator, False, col_begin, col_count, schedule,
                        frames_in_flight)
        rows = owned_rows(height, row_block, row_rank, row_world)
        out = np.zeros((rows, col_count or width, 3), np.float32)
        self._check(self.L.rt_render(self.ctx, C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def render_u8(self, width, height, spp, max_depth, seed=1984, sample_offset=0, row_block=1,
                  row_rank=0, row_world=1, lanes_per_pixel=1, integrator="rayColor") -> np.ndarray:
        """renderKernel's offline uint8 output: gamma(color / spp) per channel
        (Canvas::writePixel), computed on the device. Shape (rows, width, 3), y = 0 bottom."""
        p = self.params(width, height, spp, max_depth, seed, sample_offset, row_block, row_rank,
                        row_world, lanes_per_pixel, integrator)
        rows = owned_rows(height, row_block, row_rank, row_world)
        out = np.zeros((rows, width, 3), np.uint8)
        self._check(self.L.rt_render_u8(self.ctx, C.byref(p), out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def accumulate_device(self, params: RenderParams, accum_ptr: int, sample_count: int,
                          pixels_ptr: int = 0, stream_ptr: int = 0):
        """GPU_REALTIME progressive frame (Canvas::accumulatePixel): add this call's
        per-pixel sample sums to a caller-owned device float buffer and, if
        pixels_ptr is set, write gamma(acc * (1 / sample_count)) as uint8."""
        self._check(self.L.rt_accumulate(self.ctx, C.byref(params), C.c_void_p(accum_ptr),
                                         int(sample_count), C.c_void_p(pixels_ptr or None),
                                         C.c_void_p(stream_ptr)))

    def render_device(self, params: RenderParams, out_ptr: int, stream_ptr: int = 0):
        """Enqueue a render into a caller-owned device buffer (e.g. a torch tensor's
        data_ptr()) on a HIP stream (torch.cuda.Stream.cuda_stream)."""
        self._check(self.L.rt_render_device(self.ctx, C.byref(params), C.c_void_p(out_ptr),
                                            C.c_void_p(stream_ptr)))

    def assemble_rows_device(self, params: RenderParams, world: int, staging_ptr: int, frame_ptr: int,
                             stream_ptr: int = 0):
        """rt_assemble_rows: the gather root's row de-interleave (world tiles of
        rt_max_tile_rows rows, rank-major) into a (height, width, 3) device frame."""
        self._check(self.L.rt_assemble_rows(self.ctx, C.byref(params), int(world), C.c_void_p(staging_ptr),
                                            C.c_void_p(frame_ptr), C.c_void_p(stream_ptr)))

    def stats(self) -> dict:
        s = RenderStats()
        self._check(self.L.rt_sync_stats(self.ctx, C.byref(s)))
        d = {k: getattr(s, k) for k, _ in RenderStats._fields_}
        d["debug"] = list(s.debug)
        d["variant_name"] = variant_name(s.variant)  # the kernel symbol, as rocprofv3 prints it
        return d


REFLECTION_TYPES = {"DIFFUSE": 0, "METAL": 1, "SPECULAR": 2, "REFRACTION": 3, "COAT": 4}
INTEGRATORS = {"rayColor": 0, "pathTrace": 1}
KEEP_COUNTERS = 1  # rtmi.h RT_RENDER_KEEP_COUNTERS
FRAMES_IN_FLIGHT = 2  # rtmi.h RT_RENDER_FRAMES_IN_FLIGHT


def _reflection_type(t) -> int:
    if isinstance(t, str):
        return REFLECTION_TYPES[t.upper()]
    return int(t)


def _integrator(i) -> int:
    if isinstance(i, str):
        return INTEGRATORS[i]
    return int(i)


def render_multi(renderers, width, height, spp, max_depth, seed=1984, sample_offset=0, row_block=8,
                 lanes_per_pixel=0, integrator="rayColor") -> np.ndarray:
    """rt_render_multi: one host process renders a frame over several contexts
    (devices), renderer k taking the row tiles of rank k; returns (H, W, 3)."""
    L = lib()
    p = Renderer.params(width, height, spp, max_depth, seed, sample_offset, row_block, 0, 1,
                        lanes_per_pixel, integrator)
    arr = (C.c_void_p * len(renderers))(*[r.ctx for r in renderers])
    out = np.zeros((height, width, 3), np.float32)
    st = L.rt_render_multi(arr, len(renderers), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)))
    if st != 0:
        raise RTError(st, L.rt_last_error(renderers[0].ctx).decode())
    return out


def owned_rows(height, block, rank, world) -> int:
    n, b = 0, rank
    while b * block < height:
        r0 = b * block
        n += min(r0 + block, height) - r0
        b += world
    return n


def owned_row_ids(height, block, rank, world) -> np.ndarray:
    ids, b = [], rank
    while b * block < height:
        ids.extend(range(b * block, min(b * block + block, height)))
        b += world
    return np.asarray(ids, np.int64)


def gamma_u8(rgb: np.ndarray) -> np.ndarray:
    """Canvas::gamma (Canvas.h:198-200) through the native library."""
    rgb = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(rgb.shape, np.uint8)
    st = lib().rt_gamma_u8(rgb.ctypes.data_as(C.POINTER(C.c_float)), rgb.size,
                           out.ctypes.data_as(C.POINTER(C.c_uint8)))
    if st != RT_OK:
        raise RTError(st, "rt_gamma_u8")
    return out


# ---- kernels.h factory names (reference signatures) ----
def createLambertianMaterial(materials: MaterialTable, index, albedo, absorb=1.0):
    materials._r.lambertian(index, albedo, absorb)


def createMetalMaterial(materials: MaterialTable, index, albedo, fuzz=1.0):
    materials._r.metal(index, albedo, fuzz)


def createDieletricMaterial(materials: MaterialTable, index, indexOfRefraction=1.5):
    materials._r.dielectric(index, indexOfRefraction)


def createEmissionMaterial(materials: MaterialTable, index, albedo, intensity=1.0):
    materials._r.emission(index, albedo, intensity)


def createSphere(spheres: ObjectTable, index, center, radius, material, bShading=True):
    spheres._r.sphere(index, center, radius, material, bShading)


def createMovingSphere(spheres: ObjectTable, index, center0, center1, time0, time1, radius, material):
    spheres._r.moving_sphere(index, center0, center1, time0, time1, radius, material)


def createPlane(planes: ObjectTable, index, position, normal, extend, material, orientation, bTwoSide=True):
    planes._r.plane(index, position, normal, extend, material, orientation, bTwoSide)


def createCube(cubes: ObjectTable, index, center, extend, material):
    cubes._r.cube(index, center, extend, material)


def createMesh(meshes: ObjectTable, index, tri_vertices, material):
    meshes._r.mesh(index, tri_vertices, material)
