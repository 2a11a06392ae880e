"""Randomised parity: seeded random scenes built through the product's C ABI and
the CPU restatement alike (every primitive and material kind, moving spheres,
one- and two-sided planes of each orientation, cubes, small and BVH meshes,
media), rendered on the GPU and compared bit for bit with the oracle."""
import numpy as np
import pytest


MATS = ("lambertian", "metal", "dielectric", "emission")


def random_spec(seed):
    rng = np.random.RandomState(seed)
    u = lambda lo, hi: float(rng.uniform(lo, hi))  # noqa: E731
    v3 = lambda lo, hi: (u(lo, hi), u(lo, hi), u(lo, hi))  # noqa: E731
    mats = []
    for m in range(6):
        kind = MATS[rng.randint(len(MATS))]
        if kind == "lambertian":
            mats.append(("lambertian", m, v3(0.1, 0.9)))
        elif kind == "metal":
            mats.append(("metal", m, v3(0.3, 1.0), u(0.0, 1.2)))
        elif kind == "dielectric":
            mats.append(("dielectric", m, u(1.1, 2.0)))
        else:
            mats.append(("emission", m, v3(0.5, 1.0), u(1.0, 6.0)))
    objs = []
    slot = 0
    for _ in range(rng.randint(2, 7)):
        kind = rng.randint(6)
        m = int(rng.randint(6))
        if kind == 0:
            objs.append(("sphere", slot, v3(-1.0, 1.0), u(-0.3, 0.5), m))
        elif kind == 1:
            c0 = v3(-1.0, 1.0)
            objs.append(("moving_sphere", slot, c0, (c0[0], c0[1] + u(0, 0.4), c0[2]), 0.0, 1.0, u(0.05, 0.4), m))
        elif kind == 2:
            o = int(rng.randint(3))
            n = [(0.0, 0.0, 1.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0)][o]
            if rng.rand() < 0.5:
                n = tuple(-x for x in n)
            objs.append(("plane", slot, v3(-1.0, 1.0), n, v3(0.2, 1.5), m, o, bool(rng.rand() < 0.7)))
        elif kind == 3:
            objs.append(("cube", slot, v3(-0.8, 0.8), v3(0.05, 0.4), m))
        elif kind == 4:
            nt = int(rng.choice([3, 12, 80]))  # 80 > 64: BVH path
            base = np.float32(v3(-0.6, 0.6))
            tris = (base + rng.uniform(-0.4, 0.4, size=(nt, 3, 3)).astype(np.float32)).reshape(nt, 9)
            objs.append(("mesh", slot, tris, m))
        else:
            objs.append(("medium", slot, v3(-0.5, 0.5), v3(0.1, 0.5), u(0.5, 8.0), 6))
        slot += 1
    mats.append(("isotropic", 6, v3(0.2, 1.0)))
    eye = v3(-0.3, 0.3)
    eye = (eye[0], eye[1], eye[2] + 2.5)
    cam = (eye, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.33, u(30.0, 70.0), u(0.0, 0.1), 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def build_product(r, spec):
    import raytracingthenextweekcuda_amd as rtmi

    r.set_camera(rtmi.Camera(*spec["camera"]))
    for m in spec["materials"]:
        kind, idx = m[0], m[1]
        if kind == "isotropic":
            r.isotropic(idx, m[2])
        elif kind == "lambertian":
            r.lambertian(idx, m[2])
        elif kind == "metal":
            r.metal(idx, m[2], m[3])
        elif kind == "dielectric":
            r.dielectric(idx, m[2])
        else:
            r.emission(idx, m[2], m[3])
    for o in spec["objects"]:
        if o[0] == "medium":
            r.constant_medium(o[1], o[2], o[3], o[4], o[5])
        else:
            getattr(r, o[0])(o[1], *o[2:])
    r.commit()


def build_oracle(spec):
    from oracle import oracle as orc

    sc = orc.OracleScene()
    sc.camera(*spec["camera"])
    kinds = {"lambertian": 0, "metal": 1, "dielectric": 2, "emission": 3, "isotropic": 4}
    for m in spec["materials"]:
        kind, idx = m[0], m[1]
        if kind == "dielectric":
            sc.material(idx, 2, (1, 1, 1), m[2])
        elif kind in ("lambertian", "isotropic"):
            sc.material(idx, kinds[kind], m[2], 1.0 if kind == "lambertian" else 0.0)
        else:
            sc.material(idx, kinds[kind], m[2], m[3])
    for o in spec["objects"]:
        if o[0] == "mesh":
            sc.mesh(o[1], o[2], o[3])
        elif o[0] == "medium":
            sc.constant_medium(o[1], o[2], o[3], o[4], o[5])
        else:
            getattr(sc, o[0])(o[1], *o[2:])
    return sc


def test_random_specs_build_on_host():
    import raytracingthenextweekcuda_amd as rtmi

    for seed in range(20):
        spec = random_spec(seed)
        r = rtmi.Renderer(-1)
        build_product(r, spec)
        r.close()
        build_oracle(spec)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_gpu_random_scene_parity(seed):
    import raytracingthenextweekcuda_amd as rtmi

    spec = random_spec(seed)
    w, h, spp, depth = 32, 24, 4, 6
    lanes = [1, 2, 4][seed % 3]
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert float(np.abs(got - want).max()) <= 1e-4
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def mesh_run_spec(seed):
    """Runs of equal brute-force meshes for the kernel's mesh_run (rt_scene.cpp
    mark_mesh_runs): five 12-triangle meshes in a row (a run of 4, then 1), a 3-triangle
    mesh, a plane, a pair, a BVH mesh and a single one. Meshes 1 and 2 are the SAME
    triangles with different materials: at equal t the earlier mesh must win
    (the sequential hit()'s strict <), which the shading makes visible."""
    rng = np.random.RandomState(seed)
    mats = [("lambertian", 0, (0.8, 0.3, 0.3)), ("metal", 1, (0.9, 0.9, 0.5), 0.3),
            ("lambertian", 2, (0.2, 0.7, 0.3)), ("emission", 3, (1.0, 0.9, 0.8), 4.0),
            ("dielectric", 4, 1.5)]

    def soup(nt, centre):
        base = np.float32(centre)
        return (base + rng.uniform(-0.35, 0.35, size=(nt, 3, 3)).astype(np.float32)).reshape(nt, 9)

    objs, slot = [], 0

    def add(o):
        nonlocal slot
        objs.append(o)
        slot += 1

    twin = soup(12, (0.0, 0.0, 0.0))
    add(("mesh", slot, soup(12, (-0.5, 0.2, 0.1)), 0))
    add(("mesh", slot, twin, 1))
    add(("mesh", slot, twin.copy(), 2))
    add(("mesh", slot, soup(12, (0.4, -0.3, 0.0)), 0))
    add(("mesh", slot, soup(12, (0.1, 0.5, -0.2)), 4))
    add(("mesh", slot, soup(3, (-0.3, -0.4, 0.3)), 2))
    add(("plane", slot, (0.0, -0.8, 0.0), (0.0, 1.0, 0.0), (2.0, 2.0, 2.0), 0, 2, True))
    add(("mesh", slot, soup(12, (0.6, 0.4, 0.2)), 1))
    add(("mesh", slot, soup(12, (-0.6, -0.2, -0.3)), 2))
    add(("mesh", slot, soup(80, (0.2, 0.0, -0.6)), 0))
    add(("mesh", slot, soup(12, (0.0, -0.5, 0.5)), 3))
    add(("sphere", slot, (0.0, 1.5, 0.0), 0.6, 3))
    cam = ((0.2, 0.3, 2.6), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.33, 50.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def test_mesh_run_specs_build_on_host():
    import raytracingthenextweekcuda_amd as rtmi

    for seed in range(3):
        r = rtmi.Renderer(-1)
        build_product(r, mesh_run_spec(seed))
        r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,lanes", [(0, 1), (1, 4), (2, 32)])
def test_gpu_mesh_runs_parity(seed, lanes):
    import raytracingthenextweekcuda_amd as rtmi

    spec = mesh_run_spec(seed)
    w, h, spp, depth = 48, 36, 8, 6
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def large_leaf_spec(seed):
    """BVH leaves larger than a child-pair leaf reference holds (16 primitives: rt_scene.cpp
    build_mesh_pairs splits them into halves under the leaf's box): a 160-triangle mesh whose
    first 100 triangles are one triangle repeated (equal centroids: the SAH builder cannot split
    them, and at equal t the lowest mesh-local index must win), and 40 spheres of which 24 are
    one sphere repeated with different materials (a sphere-group leaf of 24; at equal t the
    highest scan order wins)."""
    rng = np.random.RandomState(seed)
    mats = [("lambertian", 0, (0.8, 0.3, 0.3)), ("metal", 1, (0.9, 0.9, 0.5), 0.3),
            ("lambertian", 2, (0.2, 0.7, 0.3)), ("emission", 3, (1.0, 0.9, 0.8), 4.0),
            ("dielectric", 4, 1.5)]
    one = rng.uniform(-0.4, 0.4, size=(1, 9)).astype(np.float32)
    rest = rng.uniform(-0.6, 0.6, size=(60, 9)).astype(np.float32)
    tris = np.concatenate([np.repeat(one, 100, axis=0), rest]).reshape(-1)
    objs = [("mesh", 0, tris, 0), ("plane", 1, (0.0, -0.8, 0.0), (0.0, 1.0, 0.0), (2.0, 2.0, 2.0), 0, 2, True)]
    slot = 2
    for k in range(40):
        c = (0.3, 0.9, -0.2) if k < 24 else tuple(rng.uniform(-1.2, 1.2, 3))
        objs.append(("sphere", slot, c, 0.25 if k < 24 else float(rng.uniform(0.05, 0.2)), k % 5))
        slot += 1
    cam = ((0.3, 0.4, 2.6), (0.0, 0.1, 0.0), (0.0, 1.0, 0.0), 1.33, 50.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def test_large_leaf_specs_build_on_host():
    import raytracingthenextweekcuda_amd as rtmi

    for seed in range(2):
        r = rtmi.Renderer(-1)
        build_product(r, large_leaf_spec(seed))
        c = r.object_counts()
        r.close()
        assert c["bvh_node"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,lanes", [(0, 1), (1, 8)])
def test_gpu_large_leaf_parity(seed, lanes):
    import raytracingthenextweekcuda_amd as rtmi

    spec = large_leaf_spec(seed)
    w, h, spp, depth = 48, 36, 8, 6
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert st["overflow"] == 0
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def division_edge_spec():
    """Planes whose quotient leaves the domain of the kernel's v_rcp + Newton / Markstein
    division (rt_kernel.hip rcp_nr / div_y): a floor 1e31 below the scene (|num| >= 2^100) and a
    wall with a huge, non-unit normal (|den| >= 2^100), next to ordinary objects. Waves that meet
    them take the IEEE division; the image must stay bit-identical to the restatement's."""
    mats = [("lambertian", 0, (0.7, 0.6, 0.5)), ("metal", 1, (0.9, 0.9, 0.9), 0.05),
            ("emission", 2, (1.0, 0.9, 0.8), 3.0), ("lambertian", 3, (0.3, 0.5, 0.8))]
    objs = [
        ("plane", 0, (0.0, -1.0e31, 0.0), (0.0, 1.0, 0.0), (1.0e38, 1.0e38, 1.0e38), 0, 2, True),
        ("plane", 1, (-1.5, 0.0, 0.0), (-3.0e31, 0.0, 0.0), (2.0, 2.0, 2.0), 2, 1, False),  # emissive: no scatter off a huge normal
        ("sphere", 2, (0.0, 0.0, 0.0), 0.5, 1),
        ("sphere", 3, (0.6, 0.9, -0.4), 0.3, 2),
        ("plane", 4, (0.0, 0.0, -1.2), (0.0, 0.0, 1.0), (2.0, 2.0, 2.0), 0, 0, True),
    ]
    cam = ((0.3, 0.8, 2.4), (0.0, -0.2, 0.0), (0.0, 1.0, 0.0), 1.33, 60.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def test_division_edge_spec_builds_on_host():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    build_product(r, division_edge_spec())
    r.close()
    build_oracle(division_edge_spec())


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 8])
def test_gpu_division_edge_parity(lanes):
    import raytracingthenextweekcuda_amd as rtmi

    spec = division_edge_spec()
    w, h, spp, depth = 40, 30, 8, 6
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert np.isfinite(got).all()
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def groups_with_medium_spec(seed):
    """24 spheres (a sphere group: >= 16 spheres go behind a BVH) beside a participating medium that sits
    in the scan BEFORE the group, and one more after it. The sphere-group-only kernel resumes an unfinished
    group traversal in the next loop trip by re-scanning the objects before the group, which would draw the
    medium's free-flight distance again from the ray's stream: such scenes must run a kernel
    that traverses each group in one pass, and match the restatement bit for bit."""
    rng = np.random.RandomState(seed)
    mats = [("lambertian", 0, (0.8, 0.3, 0.3)), ("metal", 1, (0.9, 0.9, 0.5), 0.3),
            ("dielectric", 2, 1.5), ("emission", 3, (1.0, 0.9, 0.8), 4.0), ("lambertian", 4, (0.3, 0.6, 0.8)),
            ("isotropic", 5, (0.7, 0.7, 0.9))]
    objs = [("plane", 0, (0.0, -0.8, 0.0), (0.0, 1.0, 0.0), (3.0, 3.0, 3.0), 4, 2, True),
            ("medium", 1, (0.0, 0.0, 0.0), (0.9, 0.6, 0.9), float(rng.uniform(0.8, 3.0)), 5)]
    slot = 2
    for k in range(24):
        objs.append(("sphere", slot, tuple(rng.uniform(-1.0, 1.0, 3)), float(rng.uniform(0.06, 0.22)), k % 5))
        slot += 1
    objs.append(("medium", slot, (0.5, 0.4, -0.3), (0.2, 0.2, 0.2), 4.0, 5))
    cam = ((0.2, 0.4, 2.7), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 1.33, 50.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def test_groups_with_medium_spec_builds_on_host():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    build_product(r, groups_with_medium_spec(0))
    c = r.object_counts()
    r.close()
    assert c["bvh_node"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,lanes", [(0, 1), (1, 8)])
def test_gpu_sphere_groups_with_medium_parity(seed, lanes):
    import raytracingthenextweekcuda_amd as rtmi

    spec = groups_with_medium_spec(seed)
    w, h, spp, depth = 48, 36, 16, 8
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    assert st["variant_name"] == "render_kernel<true, true, false, true, 3>"  # not the resuming group kernel
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert st["overflow"] == 0
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def deep_leaf_spec():
    """One triangle repeated 260 times: the SAH builder keeps them in one leaf, which build_mesh_pairs
    splits into halves under the same box (260 -> 130 -> 65 -> 33 -> 17 -> 9): five levels of pair
    records, every child of every node hit by any ray that hits the box.
    A lane descending it pushes at every level, so its stack reaches exactly the scene's bound
    (rt_scene_bvh_depth) while its non-pushing steps write the spare slot past it (rt_kernel.hip
    kStackSpare)."""
    one = np.array([[-0.6, -0.5, -0.2, 0.7, -0.4, -0.3, -0.1, 0.6, -0.25]], np.float32)
    mats = [("lambertian", 0, (0.8, 0.3, 0.3)), ("emission", 1, (1.0, 0.9, 0.8), 4.0)]
    objs = [("mesh", 0, np.repeat(one, 260, axis=0).reshape(-1), 0),
            ("plane", 1, (0.0, 0.9, 0.0), (0.0, -1.0, 0.0), (2.0, 2.0, 2.0), 1, 2, True),
            ("plane", 2, (0.0, -0.8, 0.0), (0.0, 1.0, 0.0), (2.0, 2.0, 2.0), 0, 2, True)]
    cam = ((0.1, 0.2, 2.2), (0.0, 0.0, -0.2), (0.0, 1.0, 0.0), 1.33, 40.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


def test_deep_leaf_spec_depth():
    import raytracingthenextweekcuda_amd as rtmi

    r = rtmi.Renderer(-1)
    build_product(r, deep_leaf_spec())
    assert r.bvh_depth() == 5  # child-pair records: 260 -> 130 -> 65 -> 33 -> 17 -> 9 (leaf references of <= 16)
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 16])
def test_gpu_stack_reaches_its_bound(lanes):
    import raytracingthenextweekcuda_amd as rtmi

    spec = deep_leaf_spec()
    w, h, spp, depth = 40, 30, 8, 4
    r = rtmi.Renderer(0)
    build_product(r, spec)
    bound = r.bvh_depth()
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    assert bound == 5 and st["stack_depth"] == bound and st["overflow"] == 0
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]


def resume_spec(seed):
    """A scene whose mesh traversal the kernel may defer to the next loop trip when few rays of a wave
    want it (rt_kernel.hip RT_MESH_DEFER; rt_scene.cpp build_mesh_pairs sets the mesh's flag): one BVH
    mesh (a 400-triangle soup, so traversals are deep and uneven) as the scan's only mesh, planes and
    spheres around it, no medium. Metal, glass and emission make the deferred rays' shading and draw
    order visible."""
    rng = np.random.RandomState(seed)
    mats = [("lambertian", 0, (0.8, 0.3, 0.3)), ("metal", 1, (0.9, 0.9, 0.5), 0.2),
            ("dielectric", 2, 1.5), ("emission", 3, (1.0, 0.9, 0.8), 4.0), ("lambertian", 4, (0.3, 0.6, 0.8))]
    soup = (np.float32((0.0, 0.0, -0.2)) + rng.uniform(-0.5, 0.5, size=(400, 3, 3)).astype(np.float32))
    objs = [("plane", 0, (0.0, -0.8, 0.0), (0.0, 1.0, 0.0), (2.0, 2.0, 2.0), 4, 2, True),
            ("sphere", 1, (-0.6, 0.1, 0.2), 0.25, 2),
            ("mesh", 2, soup.reshape(-1), int(rng.randint(2))),
            ("plane", 3, (0.0, 0.9, 0.0), (0.0, -1.0, 0.0), (2.0, 2.0, 2.0), 3, 2, True),
            ("sphere", 4, (0.6, -0.2, 0.3), 0.2, 1)]
    cam = ((0.1, 0.2, 2.2), (0.0, 0.0, -0.2), (0.0, 1.0, 0.0), 1.33, 45.0, 0.0, 2.5, 0.0, 1.0)
    return {"camera": cam, "materials": mats, "objects": objs}


@pytest.mark.gpu
@pytest.mark.parametrize("seed,lanes", [(0, 1), (1, 4), (2, 32)])
def test_gpu_resumed_mesh_traversal_parity(seed, lanes):
    """Bit-exact against the oracle where waves defer a mesh traversal few of their rays want to the next
    loop trip (the deferred rays scan again and shade a trip later; segment counts unchanged)."""
    import raytracingthenextweekcuda_amd as rtmi

    spec = resume_spec(seed)
    w, h, spp, depth = 48, 32, 8, 6
    r = rtmi.Renderer(0)
    build_product(r, spec)
    got = r.render(w, h, spp, depth, lanes_per_pixel=lanes)
    st = r.stats()
    r.close()
    want, ost = build_oracle(spec).render(w, h, spp, depth, lanes_per_pixel=lanes)
    assert st["overflow"] == 0
    assert np.array_equal(got, want)
    assert st["segments"] == ost["segments"]
