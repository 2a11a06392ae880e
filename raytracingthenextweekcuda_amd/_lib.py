"""ctypes binding of librtmi.so (include/rtmi.h).

The product path always goes through this native library: if librtmi.so is
missing, importing the renderer raises instead of falling back to anything.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "librtmi.so")
# Experiments only (A/B builds of the same sources, tools/variants.sh).
if os.environ.get("RTMI_LIB"):
    LIB_PATH = os.path.abspath(os.environ["RTMI_LIB"])

RT_OK = 0
STATUS_NAMES = {
    0: "RT_OK", 1: "RT_ERR_INVALID", 2: "RT_ERR_HIP", 3: "RT_ERR_IO", 4: "RT_ERR_STATE",
    5: "RT_ERR_OOM", 6: "RT_ERR_NODEV", 7: "RT_ERR_OVERFLOW", 8: "RT_ERR_COMM",
}
# rtmi.h rt_build_flags() bits; bench.py and smoke() refuse ABLATION / STAMPS builds
BUILD_ABLATION, BUILD_STAMPS, BUILD_AB = 1, 2, 4
BVH_CACHE_OFF, BVH_CACHE_READ, BVH_CACHE_WRITE = 0, 1, 2
GATHER_RCCL, GATHER_COPY = 1, 2

# Every symbol include/rtmi.h declares (checked by tests/test_abi.py).
ABI_VERSION = 10  # include/rtmi.h RTMI_ABI_VERSION

EXPORTS = [
    "rt_abi_version", "rt_create", "rt_destroy", "rt_last_error", "rt_clear_scene",
    "rt_material_lambertian", "rt_material_metal", "rt_material_dielectric",
    "rt_material_emission", "rt_material_isotropic", "rt_material_defined", "rt_constant_medium",
    "rt_sphere", "rt_moving_sphere", "rt_plane",
    "rt_cube", "rt_mesh", "rt_mesh_obj", "rt_mesh_triangle_count", "rt_mesh_vertices",
    "rt_mesh_ply", "rt_ply_bvh_image", "rt_load_object", "rt_process_triangle_data",
    "rt_pathtrace_bvh_image", "rt_set_bvh_builder", "rt_bvh_build_stats", "rt_ply_bvh_image_gpu",
    "rt_camera", "rt_commit", "rt_scene_info", "rt_scene_bvh_depth", "rt_scene_digest", "rt_load_yaml_scene",
    "rt_render", "rt_render_device", "rt_sync_stats",
    "rt_render_u8", "rt_accumulate", "rt_render_multi", "rt_gamma_u8",
    "rt_build_flags", "rt_set_bvh_cache", "rt_bvh_cache_stats",
    "rt_owned_rows", "rt_max_tile_rows", "rt_render_multi_device", "rt_comm_unique_id", "rt_comm_init",
    "rt_comm_destroy", "rt_gather_rows", "rt_assemble_rows", "rt_kernel_variant_name", "rt_kernel_source_sha",
    "rt_camera_initialize", "rt_camera_update_view_matrix", "rt_camera_walk", "rt_camera_strafe", "rt_camera_raise",
    "rt_camera_yaw", "rt_camera_pitch", "rt_camera_orbit", "rt_camera_set_aperture", "rt_camera_apply",
    "rt_get_camera", "rt_canvas_create", "rt_canvas_destroy", "rt_canvas_clear_accumulation",
    "rt_canvas_accumulate", "rt_canvas_read_pixels", "rt_canvas_read_accumulation", "rt_canvas_write_accumulation",
]

# rtmi.h RT_SCHEDULE_* and RT_VARIANT_* (rt_render_stats.variant)
SCHEDULES = {"auto": 0, "static": 1}
VARIANTS = {
    1: "SCAN_QUEUE", 2: "SCAN_MEDIA_QUEUE", 3: "SCAN_SIMPLE_QUEUE", 4: "BVH_QUEUE", 5: "BVH_MESH_QUEUE",
    6: "BVH_MESH_SIMPLE_QUEUE", 7: "BVH_GROUP_QUEUE", 8: "SCAN_STATIC", 9: "SCAN_MEDIA_STATIC",
    10: "SCAN_SIMPLE_STATIC", 11: "BVH_STATIC", 12: "PATHTRACE_QUEUE", 13: "PATHTRACE_STATIC",
}


class RTError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class RenderParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
        ("max_depth", C.c_int32), ("seed", C.c_uint32), ("sample_offset", C.c_uint32),
        ("row_block", C.c_int32), ("row_rank", C.c_int32), ("row_world", C.c_int32),
        ("lanes_per_pixel", C.c_int32), ("integrator", C.c_int32), ("flags", C.c_uint32),
        ("col_begin", C.c_int32), ("col_count", C.c_int32), ("schedule", C.c_int32),
    ]


class CameraState(C.Structure):
    """rt_camera_state (rtmi.h): the fields of the reference's Camera (Camera.h:169-195)."""
    _fields_ = [(n, C.c_float * 3) for n in ("eye", "center", "up", "forward", "right", "true_up", "origin",
                                             "horizontal", "vertical", "lower_left")] + \
        [(n, C.c_float) for n in ("aspect_ratio", "fov", "scale", "viewport_height", "viewport_width",
                                  "moving_speed", "aperture", "focus_distance", "lens_radius", "time0", "time1")] + \
        [("dirty", C.c_int32)]


class RenderStats(C.Structure):
    _fields_ = [
        ("segments", C.c_uint64), ("samples", C.c_uint64), ("node_visits", C.c_uint64),
        ("tri_tests", C.c_uint64), ("box_tests", C.c_uint64), ("kernel_ms", C.c_double),
        ("overflow", C.c_uint32), ("lanes_per_pixel", C.c_uint32),
        ("group_sphere_tests", C.c_uint64), ("group_moving_sphere_tests", C.c_uint64),
        ("debug", C.c_uint64 * 8),
        ("refill", C.c_uint32), ("queue_blocks", C.c_uint32), ("gather", C.c_uint32), ("launches", C.c_uint32),
        ("kernel_ms_sum", C.c_double), ("variant", C.c_uint32), ("substreams_per_item", C.c_uint32),
        ("stack_depth", C.c_uint32),
    ]


def build(arch: str = "gfx950") -> str:
    """Compile librtmi.so in-tree with hipcc (cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", CSRC, f"ARCH={arch}", "-j4"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: if torch (which bundles its own
    # libamdhip64) is importable, load it first so librtmi.so binds to the
    # already-loaded runtime instead of a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"librtmi.so not found at {LIB_PATH}: build it with __graft_entry__.build() "
            "(the renderer has no fallback path)")
    L = C.CDLL(LIB_PATH)
    check_source_digest(L)
    vp, fp, i32 = C.c_void_p, C.POINTER(C.c_float), C.c_int32
    L.rt_abi_version.restype = i32
    L.rt_create.argtypes = [i32, C.POINTER(vp)]
    L.rt_destroy.argtypes = [vp]
    L.rt_destroy.restype = None
    L.rt_last_error.argtypes = [vp]
    L.rt_last_error.restype = C.c_char_p
    L.rt_clear_scene.argtypes = [vp]
    L.rt_material_lambertian.argtypes = [vp, i32, fp, C.c_float]
    L.rt_material_metal.argtypes = [vp, i32, fp, C.c_float]
    L.rt_material_dielectric.argtypes = [vp, i32, C.c_float]
    L.rt_material_emission.argtypes = [vp, i32, fp, C.c_float]
    L.rt_material_defined.argtypes = [vp, i32]
    L.rt_material_isotropic.argtypes = [vp, i32, fp]
    L.rt_constant_medium.argtypes = [vp, i32, fp, fp, C.c_float, i32]
    L.rt_sphere.argtypes = [vp, i32, fp, C.c_float, i32, i32]
    L.rt_moving_sphere.argtypes = [vp, i32, fp, fp, C.c_float, C.c_float, C.c_float, i32]
    L.rt_plane.argtypes = [vp, i32, fp, fp, fp, i32, i32, i32]
    L.rt_cube.argtypes = [vp, i32, fp, fp, i32]
    L.rt_mesh.argtypes = [vp, i32, fp, i32, i32]
    L.rt_mesh_obj.argtypes = [vp, i32, C.c_char_p, fp, fp, fp, i32]
    L.rt_mesh_triangle_count.argtypes = [vp, i32]
    L.rt_mesh_vertices.argtypes = [vp, i32, fp, i32]
    L.rt_mesh_ply.argtypes = [vp, i32, C.c_char_p, fp, C.c_float, i32]
    L.rt_ply_bvh_image.argtypes = [C.c_char_p, fp, C.c_float, C.POINTER(C.c_uint8), C.c_int64,
                                   C.POINTER(C.c_int64)]
    L.rt_ply_bvh_image_gpu.argtypes = [i32, C.c_char_p, fp, C.c_float, C.POINTER(C.c_uint8), C.c_int64,
                                       C.POINTER(C.c_int64), C.POINTER(C.c_double)]
    L.rt_set_bvh_builder.argtypes = [vp, i32]
    L.rt_bvh_build_stats.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    L.rt_load_object.argtypes = [vp, C.c_char_p, i32]
    L.rt_process_triangle_data.argtypes = [vp, fp, C.c_float, C.POINTER(C.c_int32)]
    L.rt_pathtrace_bvh_image.argtypes = [vp, C.POINTER(C.c_uint8), C.c_int64, C.POINTER(C.c_int64)]
    L.rt_camera.argtypes = [vp, fp, fp, fp] + [C.c_float] * 6
    L.rt_commit.argtypes = [vp]
    L.rt_scene_info.argtypes = [vp, C.POINTER(C.c_int32)]
    L.rt_scene_bvh_depth.argtypes = [vp, C.POINTER(C.c_int32)]
    L.rt_scene_digest.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.rt_load_yaml_scene.argtypes = [vp, C.c_char_p, C.c_char_p, i32, i32]
    L.rt_render.argtypes = [vp, C.POINTER(RenderParams), fp]
    L.rt_render_device.argtypes = [vp, C.POINTER(RenderParams), vp, vp]
    L.rt_sync_stats.argtypes = [vp, C.POINTER(RenderStats)]
    L.rt_render_multi.argtypes = [C.POINTER(vp), i32, C.POINTER(RenderParams), fp]
    L.rt_render_u8.argtypes = [vp, C.POINTER(RenderParams), C.POINTER(C.c_uint8)]
    L.rt_accumulate.argtypes = [vp, C.POINTER(RenderParams), vp, C.c_uint32, vp, vp]
    L.rt_gamma_u8.argtypes = [fp, C.c_int64, C.POINTER(C.c_uint8)]
    L.rt_build_flags.restype = C.c_uint32
    L.rt_build_flags.argtypes = []
    cs = C.POINTER(CameraState)
    L.rt_camera_initialize.argtypes = [cs, fp, fp, fp] + [C.c_float] * 6
    L.rt_camera_update_view_matrix.argtypes = [cs]
    for name in ("walk", "strafe", "raise", "yaw", "pitch", "set_aperture"):
        getattr(L, "rt_camera_" + name).argtypes = [cs, C.c_float]
    L.rt_camera_orbit.argtypes = [cs, fp]
    L.rt_camera_apply.argtypes = [vp, cs]
    L.rt_get_camera.argtypes = [vp, cs]
    L.rt_canvas_create.argtypes = [vp, i32, i32, C.POINTER(vp)]
    L.rt_canvas_destroy.argtypes = [vp]
    L.rt_canvas_destroy.restype = None
    L.rt_canvas_clear_accumulation.argtypes = [vp]
    L.rt_canvas_accumulate.argtypes = [vp, C.POINTER(RenderParams), C.c_uint32]
    L.rt_canvas_read_pixels.argtypes = [vp, C.POINTER(C.c_uint8)]
    L.rt_canvas_read_accumulation.argtypes = [vp, fp]
    L.rt_canvas_write_accumulation.argtypes = [vp, fp]
    L.rt_kernel_variant_name.argtypes = [C.c_uint32]
    L.rt_kernel_variant_name.restype = C.c_char_p
    L.rt_kernel_source_sha.argtypes = []
    L.rt_kernel_source_sha.restype = C.c_char_p
    L.rt_set_bvh_cache.argtypes = [vp, i32]
    L.rt_bvh_cache_stats.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.rt_owned_rows.argtypes = [i32, i32, i32, i32]
    L.rt_owned_rows.restype = i32
    L.rt_max_tile_rows.argtypes = [i32, i32, i32]
    L.rt_max_tile_rows.restype = i32
    L.rt_render_multi_device.argtypes = [C.POINTER(vp), i32, C.POINTER(RenderParams), vp, vp]
    L.rt_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
    L.rt_comm_init.argtypes = [vp, C.POINTER(C.c_uint8), i32, i32, C.POINTER(vp)]
    L.rt_comm_destroy.argtypes = [vp]
    L.rt_gather_rows.argtypes = [vp, vp, C.POINTER(RenderParams), i32, i32, vp, vp, vp]
    L.rt_assemble_rows.argtypes = [vp, C.POINTER(RenderParams), i32, vp, vp, vp]
    _lib = L
    return L


class StaleLibraryError(ImportError):
    pass


def library_digest(L) -> str:
    """rt_kernel_source_sha() of a loaded library ('' for a library that predates it)."""
    f = getattr(L, "rt_kernel_source_sha", None)
    if f is None:
        return ""
    f.argtypes = []
    f.restype = C.c_char_p
    return (f() or b"").decode()


def tree_digest(csrc: str = CSRC) -> str | None:
    """The digest of the library's sources in this tree (None if they are not here)."""
    from .source_digest import source_digest

    if not os.path.exists(os.path.join(csrc, "Makefile")):
        return None
    return source_digest(csrc)


def check_source_digest(L, csrc: str = CSRC, lib_path: str | None = None) -> str:
    """Refuses a library that was not built from the sources next to it: its embedded digest
    (rt_kernel_source_sha, baked in by the Makefile) must equal the tree's. A library named by
    RTMI_LIB (an A/B build of other sources or flags, tools/) is exempt, and bench.py then reports
    the library's own digest. Returns the library's digest."""
    lib_path = lib_path or LIB_PATH
    have = library_digest(L)
    if os.environ.get("RTMI_LIB"):
        return have
    want = tree_digest(csrc)
    if want is not None and have != want:
        raise StaleLibraryError(
            f"stale {lib_path}: built from sources with digest {have or '(none)'}, but the tree's sources "
            f"hash to {want}; rebuild it (__graft_entry__.build() or make -C {csrc})")
    return have


def source_sha() -> str:
    """The loaded library's source digest (what bench.py stamps on its line)."""
    return library_digest(lib())


def build_flags() -> int:
    """rt_build_flags() of the loaded library (0 = the shipped parity build)."""
    return int(lib().rt_build_flags())


def variant_name(variant: int) -> str | None:
    """rt_kernel_variant_name: the kernel symbol of an RT_VARIANT_* id as rocprofv3 prints it."""
    n = lib().rt_kernel_variant_name(int(variant))
    return n.decode() if n else None


def require_parity_build(what: str) -> None:
    """Refuses a library compiled with an ablation (results differ from the
    restatement) or the instrumented timer build: `what` would not measure or
    check the shipped kernel."""
    f = build_flags()
    if f & (BUILD_ABLATION | BUILD_STAMPS):
        raise RuntimeError(f"{what}: {LIB_PATH} is a non-parity build (rt_build_flags = {f:#x}); "
                           "rebuild it without EXTRA=-DRT_ABL_* / -DRT_STAMPS")
