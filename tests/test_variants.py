"""Every kernel instantiation the library can launch, against the CPU restatement.

renderKernel (main.cu:160-206) is one kernel with virtual hit/scatter calls; librtmi compiles
one instantiation per scene content and schedule (rtmi.h RT_VARIANT_*), and the host picks
one per launch (rt_kernel.hip select_variant). Each case below builds a scene that reaches
its variant, renders it through the C ABI, checks the variant the library reports (by id and
by the kernel symbol rocprofv3 prints), and compares the image with the restatement bit for
bit, segment count included. The static-grid cases are the product's fallback when a frame's
partial sums do not fit the work queue (rt_capi.cpp launch()); here they are forced with
rt_render_params.schedule = RT_SCHEDULE_STATIC."""
import os

import numpy as np
import pytest

from tests import scenes as S

W, H, SPP, LANES = 32, 24, 8, 4


def _yaml(name):
    def product(r, rtmi):
        rtmi.load_yaml_scene(r, os.path.join(S.SCENES, name), W, H)

    def oracle():
        from oracle import oracle as orc

        return orc.yaml_scene(os.path.join(S.SCENES, name), S.MODELS, W, H)
    return product, oracle


def _spec(maker):
    def product(r, rtmi):
        S.build_product(r, maker())

    def oracle():
        return S.build_oracle(maker())
    return product, oracle


def mesh_bvh_and_sphere_group_scene():
    """A BVH mesh (suzanne_small.obj, 968 triangles) next to >= 16 spheres (an object BVH):
    both traversal parts in one scene."""
    spec = S.duplicate_spheres_scene(20)
    spec["objects"].append(("mesh_obj", 26, os.path.join(S.MODELS, "suzanne", "suzanne_small.obj"),
                            (0.3, 0.3, 0.3), (0.0, 30.0, 0.0), (-0.6, 0.1, -1.4), 0))
    return spec


SCENES = {
    "spheres": _spec(S.spheres_scene),                # spheres, metal, glass: the general scan
    "media": _yaml("cornellbox_media.yaml"),          # participating media
    "cornellbox1": _yaml("cornellbox1.yaml"),         # planes + small meshes, Lambertian + emission
    "mesh_and_groups": _spec(mesh_bvh_and_sphere_group_scene),
    "suzanne": _yaml("suzanne_cornellbox.yaml"),      # BVH mesh + metal / glass spheres
    "bunny_small": _yaml("bunny_small_cornellbox.yaml"),  # BVH mesh, Lambertian + emission
    "sphere_groups": _spec(lambda: S.duplicate_spheres_scene(20)),
}

# (RT_VARIANT_* name, scene, schedule, depth)
CASES = [
    ("SCAN_QUEUE", "spheres", "auto", 10),
    ("SCAN_MEDIA_QUEUE", "media", "auto", 16),
    ("SCAN_SIMPLE_QUEUE", "cornellbox1", "auto", 8),
    ("BVH_QUEUE", "mesh_and_groups", "auto", 8),
    ("BVH_MESH_QUEUE", "suzanne", "auto", 10),
    ("BVH_MESH_SIMPLE_QUEUE", "bunny_small", "auto", 8),
    ("BVH_GROUP_QUEUE", "sphere_groups", "auto", 8),
    ("SCAN_STATIC", "spheres", "static", 10),
    ("SCAN_MEDIA_STATIC", "media", "static", 16),
    ("SCAN_SIMPLE_STATIC", "cornellbox1", "static", 8),
    ("BVH_STATIC", "suzanne", "static", 10),
    ("PATHTRACE_QUEUE", "materialball", "auto", 5),
    ("PATHTRACE_STATIC", "materialball", "static", 5),
]


def test_every_variant_has_a_case():
    from raytracingthenextweekcuda_amd._lib import VARIANTS

    assert sorted(c[0] for c in CASES) == sorted(VARIANTS.values())


def test_variant_names_are_the_profiled_symbols():
    """rt_kernel_variant_name spells each instantiation as rocprofv3 prints it (the
    template defaults included), so profiles can be matched to a launch's variant."""
    from raytracingthenextweekcuda_amd import _lib

    names = {k: _lib.variant_name(k) for k in _lib.VARIANTS}
    assert len(set(names.values())) == len(names)
    for k, n in names.items():
        kind = _lib.VARIANTS[k]
        if kind.startswith("PATHTRACE"):
            assert n == "pathtrace_kernel<%s>" % ("true" if kind.endswith("QUEUE") else "false")
        else:
            args = n[len("render_kernel<"):-1].split(", ")
            assert n.startswith("render_kernel<") and len(args) == 5, n
            assert args[1] == ("true" if kind.endswith("QUEUE") else "false"), n
            assert args[0] == ("true" if kind.startswith("BVH") else "false"), n
    assert _lib.variant_name(0) is None and _lib.variant_name(99) is None


@pytest.mark.gpu
@pytest.mark.parametrize("variant,scene,schedule,depth", CASES, ids=[c[0] for c in CASES])
def test_variant_parity(variant, scene, schedule, depth):
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd import _lib

    with rtmi.Renderer(0) as r:
        if scene == "materialball":
            rtmi.materialball(r, W, H)
            img = r.render(W, H, SPP, depth, lanes_per_pixel=LANES, integrator="pathTrace", schedule=schedule)
        else:
            SCENES[scene][0](r, rtmi)
            img = r.render(W, H, SPP, depth, lanes_per_pixel=LANES, schedule=schedule)
        st = r.stats()
    assert _lib.VARIANTS[st["variant"]] == variant, (st["variant"], st["variant_name"])
    assert st["variant_name"] == _lib.variant_name(st["variant"])
    assert (st["queue_blocks"] > 0) == (schedule == "auto")
    assert st["overflow"] == 0
    if scene == "materialball":
        from oracle import oracle as orc

        cam = orc.yaml_scene(os.path.join(S.SCENES, "cornellbox2.yaml"), S.MODELS, W, H)
        pt = orc.OraclePathTrace()
        pt.load_object(os.path.join(S.MODELS, "materialball", "materialball.ply"), "COAT")
        pt.process((0.1, 0.0, -1.0))
        with open(os.path.join(S.GOLDEN, "bvh", "materialball.ply.bvh"), "rb") as fh:
            pt.set_bvh(fh.read())
        ref, ref_st = pt.render(cam, W, H, SPP, depth, lanes_per_pixel=LANES)
    else:
        ref, ref_st = SCENES[scene][1]().render(W, H, SPP, depth, lanes_per_pixel=LANES)
    assert st["segments"] == ref_st["segments"], (variant, st["segments"], ref_st["segments"])
    assert np.array_equal(img, ref), (variant, float(np.max(np.abs(img - ref))))


@pytest.mark.gpu
@pytest.mark.parametrize("scene,variant", [("bunny_small", "BVH_MESH_SIMPLE_QUEUE"), ("suzanne", "BVH_MESH_QUEUE")])
def test_mesh_bvh_kernels_path_depth(scene, variant):
    """The mesh-BVH-only kernels keep a path's depth in bits 2-31 of the lane's LDS word W.grp_s, beside the
    deferral bits (rt_kernel.hip): paths of 0, 1 and 2 bounces match the restatement bit for bit, segment
    counts included, and max_depth >= 2^30 is refused (rt_capi.cpp validate)."""
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd import _lib

    oracle_scene = SCENES[scene][1]()
    with rtmi.Renderer(0) as r:
        SCENES[scene][0](r, rtmi)
        for depth in (0, 1, 2):
            img = r.render(W, H, SPP, depth, lanes_per_pixel=LANES)
            st = r.stats()
            assert _lib.VARIANTS[st["variant"]] == variant
            ref, ref_st = oracle_scene.render(W, H, SPP, depth, lanes_per_pixel=LANES)
            assert st["segments"] == ref_st["segments"], (depth, st["segments"], ref_st["segments"])
            assert np.array_equal(img, ref), (depth, float(np.max(np.abs(img - ref))))
        with pytest.raises(_lib.RTError, match=r"2\^30"):
            r.render(W, H, 1, 1 << 30)


@pytest.mark.gpu
def test_scan_kernel_depth_limit():
    """The linear-scan kernels keep the depth in 20 bits of the camera slot's spare word."""
    import raytracingthenextweekcuda_amd as rtmi
    from raytracingthenextweekcuda_amd import _lib

    with rtmi.Renderer(0) as r:
        SCENES["cornellbox1"][0](r, rtmi)
        with pytest.raises(_lib.RTError, match=r"2\^20"):
            r.render(W, H, 1, 1 << 20)
