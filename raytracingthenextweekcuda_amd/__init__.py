"""rtmi — MI355X-native path tracer with the scene model of
erosnick/RayTracingTheNextWeekCUDA.

The renderer is librtmi.so (hand-written HIP megakernel for gfx950 + C ABI,
include/rtmi.h). This package is the host-side mirror of the reference's scene
API (Camera / create* factories) over that ABI, plus scene ingestion.
"""
from ._lib import (  # noqa: F401
    BVH_CACHE_OFF, BVH_CACHE_READ, BVH_CACHE_WRITE, GATHER_COPY, GATHER_RCCL, RTError, build, build_flags,
)
from .renderer import (  # noqa: F401
    Camera, MaterialHandle, Renderer, createCube, createDieletricMaterial,
    createEmissionMaterial, createLambertianMaterial, createMesh, createMetalMaterial,
    createMovingSphere, createPlane, createSphere, gamma_u8, owned_row_ids, owned_rows,
    render_multi,
)
from .scene import (  # noqa: F401
    bunny_cornell_box, cornell_box1, cornell_box_media, load_json_scene, load_yaml_scene, materialball, random_spheres,
    suzanne_cornell_box,
)
