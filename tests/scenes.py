"""Scene fixtures for parity tests: one neutral spec, built twice — through the
product's C ABI (librtmi.so) and through the CPU restatement (oracle/)."""
from __future__ import annotations

import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(REPO, "assets", "scenes")
MODELS = os.path.join(REPO, "assets", "models")
GOLDEN = os.path.join(REPO, "tests", "golden")


def _mtype(name):
    return {"lambertian": 0, "metal": 1, "dielectric": 2, "emission": 3}[name]


def build_product(r, spec):
    cam = spec["camera"]
    import raytracingthenextweekcuda_amd as rtmi

    r.set_camera(rtmi.Camera(*cam))
    for m in spec["materials"]:
        kind, idx = m[0], m[1]
        if kind == "lambertian":
            r.lambertian(idx, m[2], m[3] if len(m) > 3 else 1.0)
        elif kind == "metal":
            r.metal(idx, m[2], m[3])
        elif kind == "dielectric":
            r.dielectric(idx, m[2])
        else:
            r.emission(idx, m[2], m[3])
    for o in spec["objects"]:
        kind, idx = o[0], o[1]
        getattr(r, kind)(idx, *o[2:])
    r.commit()


def build_oracle(spec):
    from oracle import oracle as orc

    sc = orc.OracleScene()
    sc.camera(*spec["camera"])
    for m in spec["materials"]:
        kind, idx = m[0], m[1]
        if kind == "dielectric":
            sc.material(idx, 2, (1, 1, 1), m[2])
        elif kind == "lambertian":
            sc.material(idx, 0, m[2], m[3] if len(m) > 3 else 1.0)
        else:
            sc.material(idx, _mtype(kind), m[2], m[3])
    for o in spec["objects"]:
        kind, idx = o[0], o[1]
        if kind == "mesh":
            sc.mesh(idx, o[2], o[3])
        elif kind == "mesh_obj":
            sc.mesh_obj(idx, *o[2:])
        else:
            getattr(sc, kind)(idx, *o[2:])
    return sc


def spheres_scene():
    """RTNW-style SCENE 0 (main.cu:592-622) with a defocus aperture, a moving
    sphere, a hollow glass sphere (negative radius) and a metal sphere."""
    eye = (3.0, 3.0, 2.0)
    center = (0.0, 0.0, -1.0)
    d = np.float32(center) - np.float32(eye)
    focus = float(np.sqrt(np.float32(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])))
    return {
        "camera": (eye, center, (0.0, 1.0, 0.0), 1.0, 20.0, 0.1, focus, 0.0, 1.0),
        "materials": [
            ("dielectric", 0, 1.5), ("dielectric", 1, 1.5), ("lambertian", 2, (0.1, 0.2, 0.5)),
            ("metal", 3, (0.8, 0.6, 0.2), 0.3), ("lambertian", 4, (0.8, 0.8, 0.0)),
            ("emission", 5, (1.0, 0.9, 0.8), 4.0),
        ],
        "objects": [
            ("sphere", 0, (-1.0, 0.0, -1.0), 0.5, 0),
            ("sphere", 1, (-1.0, 0.0, -1.0), -0.4, 1),
            ("moving_sphere", 2, (0.0, 0.0, -1.0), (0.0, 0.5, -1.0), 0.0, 1.0, 0.5, 2),
            ("sphere", 3, (1.0, 0.0, -1.0), 0.5, 3),
            ("sphere", 4, (0.0, -100.5, -1.0), 100.0, 4),
            ("cube", 5, (0.0, 1.2, -1.5), (0.3, 0.05, 0.3), 5),
        ],
    }


def mixed_scene():
    """Planes (one- and two-sided, all orientations), a cube, a mesh and spheres."""
    tri = np.array([[-0.3, -0.3, -0.6, 0.3, -0.3, -0.6, 0.0, 0.3, -0.6],
                    [-0.2, 0.2, -0.4, 0.2, 0.2, -0.4, 0.0, -0.1, -0.3]], np.float32)
    return {
        "camera": ((0.0, 0.0, 1.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 1.5, 60.0, 0.0, 2.0, 0.0, 1.0),
        "materials": [
            ("lambertian", 0, (0.7, 0.7, 0.7)), ("metal", 1, (0.9, 0.9, 0.9), 0.0),
            ("dielectric", 2, 1.33), ("emission", 3, (1.0, 1.0, 1.0), 6.0),
            ("lambertian", 4, (0.2, 0.8, 0.3)),
        ],
        "objects": [
            ("plane", 0, (0.0, -0.5, 0.0), (0.0, -1.0, 0.0), (0.6, 0.6, 0.6), 0, 2, True),
            ("plane", 1, (0.0, 0.0, -0.8), (0.0, 0.0, -1.0), (0.6, 0.6, 0.6), 4, 0, True),
            ("plane", 2, (0.6, 0.0, -0.3), (1.0, 0.0, 0.0), (0.6, 0.6, 0.6), 1, 1, True),
            ("plane", 3, (0.0, 0.45, -0.3), (0.0, 1.0, 0.0), (0.2, 0.2, 0.2), 3, 2, False),
            ("cube", 4, (-0.3, -0.35, -0.4), (0.1, 0.15, 0.1), 0),
            ("mesh", 5, tri, 4),
            ("sphere", 6, (0.25, -0.3, -0.2), 0.15, 2),
            ("sphere", 7, (0.0, 0.1, -0.5), 0.1, 1),
        ],
    }


def duplicate_spheres_scene(n_extra=20):
    """Exact ties: identical spheres in several slots (the reference's inclusive
    sphere test makes the LAST one win) next to a plane, plus enough spheres to
    put them behind the object BVH. Materials differ per slot so a wrong tie
    rule changes the image."""
    objs = [
        ("plane", 0, (0.0, -0.5, 0.0), (0.0, 1.0, 0.0), (5.0, 5.0, 5.0), 0, 2, True),
        ("sphere", 1, (0.0, 0.0, -1.0), 0.5, 1),
        ("sphere", 2, (0.0, 0.0, -1.0), 0.5, 2),
        ("moving_sphere", 3, (0.6, 0.0, -1.2), (0.6, 0.0, -1.2), 0.0, 1.0, 0.3, 3),
        ("sphere", 4, (0.6, 0.0, -1.2), 0.3, 4),
        ("sphere", 5, (0.0, 0.0, -1.0), 0.5, 3),
    ]
    rng = np.random.RandomState(5)
    for k in range(n_extra):
        c = (float(rng.uniform(-3, 3)), float(rng.uniform(-0.4, 0.6)), float(rng.uniform(-6, -2)))
        objs.append(("sphere", 6 + k, c, 0.1 + 0.1 * (k % 3), k % 5))
    return {
        "camera": ((0.0, 0.3, 1.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 1.0, 50.0, 0.0, 2.0, 0.0, 1.0),
        "materials": [
            ("lambertian", 0, (0.5, 0.5, 0.5)), ("lambertian", 1, (0.9, 0.1, 0.1)),
            ("metal", 2, (0.8, 0.8, 0.8), 0.1), ("dielectric", 3, 1.5), ("lambertian", 4, (0.1, 0.1, 0.9)),
        ],
        "objects": objs,
    }


# ---- pathTrace integrator scenes (prepareCUDAscene, main.cu:404-553) ----
# Each names the PLY files (with their ReflectionType), the processTriangleData
# offset and the reference's own `.bvh` cache file for that combination.
PT_CAMERA = ((0.0, 0.5, 3.0), (0.1, 0.0, -1.0), (0.0, 1.0, 0.0), 1.0, 45.0, 0.0, 4.0, 0.0, 1.0)
PT_SCENES = {
    # the committed configuration (main.cu:430-432)
    "materialball": ([("materialball/materialball.ply", "COAT")], (0.1, 0.0, -1.0), "materialball.ply.bvh"),
    # the commented three-suzanne configuration (main.cu:418-428); its cache is
    # the reference's suzanne/suzanne2.ply.bvh
    "suzanne": ([("suzanne/suzanne0.ply", "COAT"), ("suzanne/suzanne1.ply", "REFRACTION"),
                 ("suzanne/suzanne2.ply", "METAL")], (0.0, 0.0, 0.0), "suzanne012.ply.bvh"),
    "bunny": ([("bunny/bunny.ply", "DIFFUSE")], (0.0, 0.0, 0.0), "bunny.ply.bvh"),
}


def build_pathtrace_product(r, name, camera=PT_CAMERA):
    import raytracingthenextweekcuda_amd as rtmi

    plys, offset, _ = PT_SCENES[name]
    r.set_camera(rtmi.Camera(*camera))
    for path, kind in plys:
        r.load_object(os.path.join(MODELS, path), kind)
    return r.process_triangle_data(offset)


def build_pathtrace_oracle(name, camera=PT_CAMERA):
    """(OraclePathTrace, camera OracleScene), the BVH from the reference's cache file."""
    from oracle import oracle as orc

    plys, offset, bvh = PT_SCENES[name]
    pt = orc.OraclePathTrace()
    for path, kind in plys:
        pt.load_object(os.path.join(MODELS, path), kind)
    pt.process(offset)
    with open(os.path.join(GOLDEN, "bvh", bvh), "rb") as fh:
        pt.set_bvh(fh.read())
    cam = orc.OracleScene()
    cam.camera(*camera)
    return pt, cam
