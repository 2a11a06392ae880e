// rt_scene.h — device scene layout (what lives in HBM) and the host-side scene
// builder behind the C ABI.
//
// Layout rationale: the closest-hit scan walks the object table
// in the same order for every lane of a wave, so object and triangle records
// are wave-uniform reads. They are packed AoS records sized for one scalar
// s_load_dwordx16 / x12 each (64 B / 48 B), which the SMEM path broadcasts to
// all 64 lanes. Materials are read per lane (divergent) and are 32 B records.
// BVH nodes (per-lane divergent traversal) are SoA-friendly 32 B records.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_math.h"

namespace rt {

enum ObjType : uint32_t {
    kObjSphere = 0,
    kObjMovingSphere = 1,
    kObjPlane = 2,
    kObjMesh = 3,
    kObjSphereGroup = 4,  // BVH over (moving) spheres: u0 = first member, u1 = count, u2 = root, f[8] = root pair ref
    kObjMedium = 5,       // constant medium in a cube: f = (center - extend) xyz, (center + extend) xyz, -1/density; u0 = slot
    // A plane whose normal is (0, 0, +-1) for XY, (+-1, 0, 0) for YZ, (0, +-1, 0) for XZ (every plane of the
    // reference's scenes): kObjPlaneAxial + orientation, the record otherwise a kObjPlane one. The kernel's
    // Plane::hit then forms the two dot products from their one non-zero term (rt_kernel.hip plane_axial),
    // and the scan dispatches on the type alone.
    kObjPlaneAxial = 6    // 6: XY, 7: YZ, 8: XZ
};
RT_HD bool is_plane(uint32_t type) { return type == kObjPlane || (type - kObjPlaneAxial) < 3u; }

// One hitable (Sphere.h, Plane.h, TriangleMesh.h). Cube is flattened into its
// six planes at build time: Cube::hit (Cube.cu:10-23) is a closest scan over its
// faces with the caller's closestSoFar, identical to scanning them inline.
struct alignas(16) ObjRec {
    uint32_t type;
    uint32_t material;
    uint32_t u0;  // plane: orientation | mesh: first triangle
    uint32_t u1;  // plane: twoSide (axial kinds: the bits of 1.0f or 0) | mesh: triangle count
    uint32_t u2;     // mesh / sphere group: BVH root node index, or kNoBvh (brute-force scan)
    uint32_t order;  // position in the reference's sequential hit() scan (tie rule)
    // sphere: center xyz, radius
    // moving sphere: center0 xyz, center1 xyz, time0, time1, radius
    // plane: position xyz, normal xyz, rectangle bounds (lo_a, hi_a, lo_b, hi_b) on the
    //        orientation's axes a, b (XY: x, y; YZ: y, z; XZ: x, z)
    // mesh: boundsMin xyz, boundsMax xyz (computeMeshAABB, main.cu:261-281), f[6] = the bits of
    //       ceil(2^32 / triangle count) (the brute-force compaction's division; BVH meshes: the node slot
    //       of their QFrame), f[7] = mesh-run length (brute force), f[8] = root child-pair reference
    //       (BVH meshes), f[9] = 1 (as u32 bits)
    //       for a brute-force mesh that is a convex shell (rt_scene.cpp convex_shell), 2 for a BVH
//       mesh whose traversal the kernel may defer to the next loop trip (build_mesh_pairs, rt_kernel.hip kMeshDefer)
    float f[10];
};
constexpr uint32_t kNoBvh = 0xFFFFFFFFu;
// Meshes with more triangles than this are traversed through a BVH.
constexpr uint32_t kBvhMinTris = 64;
constexpr uint32_t kMeshRunMax = 4;  // brute-force meshes compacted together (rt_kernel.hip mesh_run)
// Scenes with at least this many (moving) spheres get an object-level BVH.
constexpr uint32_t kSphereBvhMin = 16;
// Per-lane LDS traversal stack depth; the builder rejects deeper trees, like
// the reference's BVH_STACK_SIZE check (BVH.cpp:490-496, CUDAPathTracer.h:43).
constexpr int kBvhStackDepth = 32;
static_assert(sizeof(ObjRec) == 64, "ObjRec must be 64 B");

// Triangle as prepared by prepareTriangleData (main.cu:334-349): v0, E1, E2.
// The per-triangle normal normalize(cross(E1,E2)) that TriangleMesh::hit
// recomputes for every ray (TriangleMesh.cu:42) is ray-independent and is
// precomputed here with the same float operations.
struct alignas(16) TriRec {
    float v0x, v0y, v0z, nx;
    float e1x, e1y, e1z, ny;
    float e2x, e2y, e2z, nz;
};
static_assert(sizeof(TriRec) == 48, "TriRec must be 48 B");

// BVH node for traversal: the reference's CacheFriendlyBVHNode (BVH.h:46-67)
// with absolute child / triangle indices and conservatively inflated bounds.
// Inner: a = left child, b = right child. Leaf: a = first triangle (leaf order),
// b = 0x80000000 | count.
struct alignas(16) BvhNode {
    float lo[3];
    uint32_t a;
    float hi[3];
    uint32_t b;
};
static_assert(sizeof(BvhNode) == 32, "BvhNode must be 32 B");

// Child-pair record of a MESH BVH (rt_kernel.hip mesh_bvh_pairs; rt_scene.cpp QPairBuilder): one 32 B node
// slot holding both children's boxes as 16-bit grid coordinates of the mesh's frame (origin c, step s = 2^e):
// box = [c + qlo s, c + qhi s], rounded outward from the inflated float box, so the grid box contains it.
// q[0..2] = left (lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16), q[3..5] = right, then the two
// references (a pair slot index, or kLeafRef | (count - 1) << 27 | first triangle). Half the 64 B of a
// float pair, so twice the records per L2 line: the bunny's 2.0 MB of pair records become 1.0 MB.
struct alignas(32) QPair {
    uint32_t q[6];
    uint32_t ref[2];
};
static_assert(sizeof(QPair) == 32, "QPair must be 32 B");
// The frame of a mesh's QPairs, one node slot before its root pair (index in the mesh record's f[6]):
// c.xyz, s, then zeros.
struct alignas(32) QFrame {
    float c[3];
    float s;
    uint32_t pad[4];
};
static_assert(sizeof(QFrame) == 32, "QFrame must be 32 B");
constexpr int kQMax = 65535;  // largest grid coordinate



struct alignas(16) MatRec {
    uint32_t type;  // RT_LAMBERTIAN..RT_ISOTROPIC
    float a0, a1, a2;  // albedo (emission: albedo * intensity, Material.h:121)
    float p0;          // metal: fuzz (clamped to 1, Material.h:40) | dielectric: ior
    float pad0, pad1, pad2;
};
static_assert(sizeof(MatRec) == 32, "MatRec must be 32 B");

// Camera after updateViewMatrix (Camera.h:86-103), as read by getRay (151-168).
struct CamRec {
    v3 origin, lower_left, horizontal, vertical, right, true_up;
    float lens_radius, time0, time1;
};

struct SceneArgs {
    const ObjRec* objs;
    const TriRec* tris;
    const MatRec* mats;
    const BvhNode* nodes;
    const uint32_t* tri_orig;  // per TriRec j: [2j] mesh-local index, [2j+1] position of mesh-local index j - base
    int32_t n_objs;            // records scanned by hit(); sphere-group members follow them
    int32_t n_mats;
    bool has_bvh;  // any mesh carries a BVH (selects the kernel variant)
    int32_t stack_cap = kBvhStackDepth;  // traversal stack entries per lane (the scene's BVH depth)
    bool has_media = false;  // any participating medium in the scan list (selects the kernel variant)
    int32_t bvh_parts = 3;   // BVH scenes: 1 = mesh BVHs only, 2 = sphere groups only, 3 = both
    bool full_scan = true;  // spheres or non-Lambertian/emissive materials in the scan list (false: the simple-scene variant)
};

// ----------------------------------------------------------------------------
// Host-side scene (built by the C ABI, uploaded by commit()).
// ----------------------------------------------------------------------------
struct HostMaterial {
    bool defined = false;
    MatRec rec{};
};

struct HostObject {
    bool defined = false;
    uint32_t type = 0;        // kObj* or kHostCube
    uint32_t material = 0;
    uint32_t orientation = 0;
    uint32_t two_side = 1;
    float f[12] = {0};
    std::vector<float> tri_vertices;  // mesh: 9 floats / triangle
    std::string bvh_cache;            // rt_mesh_ply: the PLY path (its `<ply>.bvh` cache)
};
constexpr uint32_t kHostCube = 100;

struct HostScene {
    std::vector<HostMaterial> materials;
    std::vector<HostObject> objects;
    bool has_camera = false;
    CamRec camera{};

    // Flattened tables (valid after flatten()).
    std::vector<ObjRec> objs;  // scan list, then sphere-group members
    int n_scan = 0;
    std::vector<TriRec> tris;
    std::vector<MatRec> mats;
    std::vector<BvhNode> nodes;
    std::vector<uint32_t> tri_orig;  // 2 per triangle: (mesh-local index, inverse map), see flatten()
    int bvh_max_depth = 0;

    // BVH builder (rt_set_bvh_builder): host Recurse, or its GPU restatement on
    // `bvh_device` (byte-identical; falls back to the host when it declines).
    bool bvh_gpu = false;
    int bvh_device = -1;
    double bvh_build_ms = 0.0;  // summed wall time of the last flatten()'s builds
    int bvh_gpu_builds = 0;     // builds the GPU ran in the last flatten()
    // `.bvh` caches (rt_set_bvh_cache: bit 1 read, bit 2 write) and what the last
    // flatten() did with them
    int bvh_cache_mode = 0;
    int cache_reads = 0, cache_writes = 0, cache_rejected = 0;
    std::string cache_last_reject;

    // Returns "" on success or an error message.
    std::string flatten();
    std::string group_spheres();
    void mark_mesh_runs();
    std::string build_mesh_pairs();
    // A mesh BVH: read from `<cache_ply>.bvh` when the cache mode allows and the file is
    // fresh and valid, else built (and written when the mode says so).
    void build_bvh(const std::vector<v3>& vs, const std::vector<uint32_t>& ix, CFBvh& b,
                   const std::string& cache_ply = std::string());
    void build_bvh_boxes(const std::vector<v3>& lo, const std::vector<v3>& hi, CFBvh& b);
};

// TriRec from three world-space vertices (prepareTriangleData, main.cu:334-343).
TriRec make_triangle(v3 p0, v3 p1, v3 p2);

// OBJ loading with loadModel(file, scale, rotate, offset) semantics
// (ModelLoader.cpp:418-448). Returns "" on success.
std::string load_obj_transformed(const std::string& path, v3 scale, v3 rotate, v3 offset,
                                 std::vector<float>& out_tri_vertices);

}  // namespace rt
