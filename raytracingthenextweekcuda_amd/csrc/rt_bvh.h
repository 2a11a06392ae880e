// rt_bvh.h — PLY ingestion and the binned-SAH BVH builder.
//
// Restates, for byte-exact agreement with the reference's `.bvh` cache files
// (paths relative to RayTracingTheNextWeekCUDA/):
//   loadObject (ASCII PLY) ............. Loader.cpp:207-319
//   processTriangleData (centre/scale, Kuchkuda planes) Loader.cpp:98-205
//   CreateBVH / Recurse (binned SAH) .... BVH.cpp:94-392
//   CreateCFBVH / PopulateCacheFriendlyBVH (DFS, 32 B nodes) BVH.cpp:432-497
//   .bvh cache image .................... BVH.cpp:537-540
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "rt_math.h"

namespace rt {

struct PlyMesh {
    std::vector<v3> vertices;
    std::vector<uint32_t> indices;  // 3 per triangle, as read (idx1, idx2, idx3)
};

// Loader.cpp:207-319 (ASCII "element vertex / element face / end_header").
std::string load_ply(const std::string& path, PlyMesh& out);

// processTriangleData (Loader.cpp:98-205) vertex transform: centre the
// triangles' bounding box, scale so max |coord| = max_coord, add offset.
void process_ply_vertices(PlyMesh& m, v3 offset, float max_coord);

// CacheFriendlyBVHNode (BVH.h:46-67): bottom, top, {idxLeft, idxRight} or
// {0x80000000 | count, startIndexInTriIndexList}.
struct CFNode {
    float bottom[3];
    float top[3];
    uint32_t u0;
    uint32_t u1;
};
static_assert(sizeof(CFNode) == 32, "CFNode must be 32 B");

struct CFBvh {
    std::vector<CFNode> nodes;
    std::vector<int32_t> tri_index;  // leaf triangle lists (indices into the mesh)
    int max_depth = 0;
};

// Child-pair references of the batched traversals (rt_scene.cpp build_mesh_pairs,
// cf_child_pairs): a pair index q (the children's records at nodes[2q], nodes[2q + 1]), or
// kLeafRef | (count - 1) << 27 | first triangle / member for a leaf of 1..kLeafRefMax.
constexpr uint32_t kLeafRef = 0x80000000u;
constexpr uint32_t kLeafRefMax = 16;

// Child-pair records of a pathTrace BVH, appended to `nodes` from an even index (each pair
// one aligned 64 B line): per inner node (and per half of a leaf larger than kLeafRefMax)
// its two children's records with bottom/top as built, u0 = the child's reference and
// u1 = 1 when the child's box is a leaf's box (BVH_IntersectTriangles never box-tests a
// leaf: only the distance pruning applies to it), else 0. Returns the root's reference;
// *max_pairs = pair records on the longest root-to-leaf path (the stack entries a lane may
// need), *empty_leaf = a leaf without triangles was found.
uint32_t cf_child_pairs(std::vector<CFNode>& nodes, int* max_pairs, bool* empty_leaf);

// CreateBVH + CreateCFBVH over triangles given by vertex index triples.
// leaf_min_split = 4 is the reference's tree (byte-identical `.bvh` caches);
// rayColor meshes, which the reference brute-forces, may use larger leaves.
void build_cf_bvh(const std::vector<v3>& vertices, const std::vector<uint32_t>& indices,
                  CFBvh& out, int leaf_min_split = 4);

// Same builder over arbitrary primitive boxes (object-level BVH).
void build_cf_bvh_boxes(const std::vector<v3>& bottoms, const std::vector<v3>& tops, CFBvh& out,
                        int leaf_min_split = 4);

// The same builder on the GPU (rt_bvh_gpu.hip): level-synchronous, one
// workgroup per node, byte-identical output. Returns "" on success, else why it
// declined (-0.0 coordinates, allocation failure, ...): callers then use the
// host builder. *ms = wall time of the build (upload, levels, download).
std::string gpu_build_cf_bvh(int device, const std::vector<v3>& vertices, const std::vector<uint32_t>& indices,
                             CFBvh& out, int leaf_min_split, double* ms);
std::string gpu_build_cf_bvh_boxes(int device, const std::vector<v3>& lo, const std::vector<v3>& hi, CFBvh& out,
                                   int leaf_min_split, double* ms);

// Kuchkuda triangle record of the pathTrace integrator, as uploaded by
// prepareCUDAscene (main.cu:457-494) minus the unused centre: plane normal + d,
// three edge planes + d1..d3 (processTriangleData, Loader.cpp:166-202) and the
// triangle's ReflectionType.
struct alignas(16) KTri {
    float n[3], d;
    float e1[3], d1;
    float e2[3], d2;
    float e3[3], d3;
    float material, pad[3];
};
static_assert(sizeof(KTri) == 80, "KTri must be 80 B");

// processTriangleData's Kuchkuda precompute over (already transformed) vertices.
void kuchkuda_triangles(const PlyMesh& m, const std::vector<uint32_t>& materials,
                        std::vector<KTri>& out);

// loadObject appending to an existing mesh (Loader.cpp:228, 282-284: indices
// are offset by the vertices already loaded).
std::string append_ply(const std::string& path, PlyMesh& accum);

// The `.bvh` cache image: u32 nodes, u32 indices, nodes, int32 indices.
std::vector<uint8_t> bvh_image(const CFBvh& b);

// A `.bvh` cache image read back (UpdateBoundingVolumeHierarchy's reader,
// BVH.cpp:544-551) as UNTRUSTED input for the triangles (vertices, indices):
// the header counts must match the size and the triangle count, children must
// follow their parent (DFS order) and be referenced once, every node reachable,
// the leaves must partition the triangle list, the list must be a permutation,
// and every box must contain its triangles / children. Returns "" or why not.
std::string parse_bvh_image(const uint8_t* data, size_t size, const std::vector<v3>& vertices,
                            const std::vector<uint32_t>& indices, CFBvh& out);

// UpdateBoundingVolumeHierarchy's cache rule for `<ply>.bvh`: 1 = read and valid,
// 0 = no usable file (absent, or the PLY is newer: plyFileTime > bvhFileTime),
// -1 = present and fresh but rejected (*why says why).
int read_bvh_cache(const std::string& ply_path, const std::vector<v3>& vertices,
                   const std::vector<uint32_t>& indices, CFBvh& out, std::string* why);
// The writer (BVH.cpp:535-541): true if `<ply>.bvh` was written.
bool write_bvh_cache(const std::string& ply_path, const CFBvh& b);

}  // namespace rt
