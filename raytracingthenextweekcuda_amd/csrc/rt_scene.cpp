// rt_scene.cpp — host-side scene preparation: camera, triangle records, OBJ
// ingestion and flattening of the reference's Hitable list into the device
// tables of rt_scene.h. Compiled with -ffp-contract=off (see Makefile).
#include "rt_scene.h"

#include <chrono>

#include "rt_bvh.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace rt {

namespace {
// Math::radians (Constants.h:29-31): pi / 180.0f * degree.
inline float radians(float deg) { return 3.1415926535897932f / 180.0f * deg; }

// rotateY (LinearAlgebra.h:74-77) with the float cos/sin of CUDATypes.h:23-24.
inline v3 rotate_y(v3 v, float r) {
    return v3{v.x * cosf(r) + v.z * sinf(r), v.y, -v.x * sinf(r) + v.z * cosf(r)};
}
}  // namespace

// A brute-force mesh the kernels may skip for rays that start on its own surface (rt_kernel.hip
// mesh_run, the convex-shell skip): a convex polyhedral shell whose face planes meet at angles of at least
// 30 degrees and whose parallel faces are apart. A ray that leaves such a mesh outward from a point
// well inside a face (closest_hit's caller checks both, with margins) stays outside every face
// plane it could cross from the front, so TriangleMesh::hit (TriangleMesh.cu:34-117, which culls
// back faces) accepts none of its triangles at t >= tMin: the geometric argument is in DESIGN §4.
// Computed in double from the triangles the kernel tests (their precomputed normals and v0).
bool convex_shell(const TriRec* t, size_t nt) {
    if (nt < 4) return false;
    struct P { double n[3], d; };
    std::vector<P> pl(nt);
    std::vector<double> vs;  // every vertex
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (size_t i = 0; i < nt; ++i) {
        const TriRec& r = t[i];
        const double v0[3] = {r.v0x, r.v0y, r.v0z}, e1[3] = {r.e1x, r.e1y, r.e1z}, e2[3] = {r.e2x, r.e2y, r.e2z};
        const double n[3] = {r.nx, r.ny, r.nz};
        if (!std::isfinite(n[0]) || !std::isfinite(n[1]) || !std::isfinite(n[2])) return false;
        const double len = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (!(std::fabs(len - 1.0) < 1e-5)) return false;
        for (int a = 0; a < 3; ++a) pl[i].n[a] = n[a] / len;
        pl[i].d = pl[i].n[0] * v0[0] + pl[i].n[1] * v0[1] + pl[i].n[2] * v0[2];
        for (int k = 0; k < 3; ++k)
            for (int a = 0; a < 3; ++a) {
                const double x = v0[a] + (k == 1 ? e1[a] : k == 2 ? e2[a] : 0.0);
                vs.push_back(x);
                lo[a] = std::min(lo[a], x);
                hi[a] = std::max(hi[a], x);
            }
    }
    const double scale = std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                   (hi[2] - lo[2]) * (hi[2] - lo[2]));
    if (!(scale > 0.0) || !std::isfinite(scale)) return false;
    // the kernel's margins (1e-3 of a triangle's height from its edges) must dwarf the rounding of a hit
    // point: every triangle at least 1e-2 high relative to the mesh's largest coordinate (and to 1)
    double maxabs = 1.0, hmin = 1e300;
    for (double x : vs) maxabs = std::max(maxabs, std::fabs(x));
    for (size_t i = 0; i < nt; ++i) {
        const TriRec& r = t[i];
        const double e1[3] = {r.e1x, r.e1y, r.e1z}, e2[3] = {r.e2x, r.e2y, r.e2z};
        const double e3[3] = {e2[0] - e1[0], e2[1] - e1[1], e2[2] - e1[2]};
        const double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2],
                     cz = e1[0] * e2[1] - e1[1] * e2[0];
        const double area2 = std::sqrt(cx * cx + cy * cy + cz * cz);
        auto len = [](const double* e) { return std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]); };
        const double longest = std::max(len(e1), std::max(len(e2), len(e3)));
        hmin = std::min(hmin, area2 / longest);
    }
    if (!(hmin >= 1e-2 * maxabs)) return false;
    for (size_t i = 0; i < nt; ++i)  // every vertex on or behind every triangle's plane (outward normals)
        for (size_t k = 0; k < vs.size(); k += 3)
            if (pl[i].n[0] * vs[k] + pl[i].n[1] * vs[k + 1] + pl[i].n[2] * vs[k + 2] - pl[i].d > 1e-6 * scale)
                return false;
    for (size_t i = 0; i < nt; ++i)
        for (size_t j = i + 1; j < nt; ++j) {
            const double c = pl[i].n[0] * pl[j].n[0] + pl[i].n[1] * pl[j].n[1] + pl[i].n[2] * pl[j].n[2];
            if (c > 1.0 - 1e-9) {  // the same face: coplanar
                if (std::fabs(pl[i].d - pl[j].d) > 1e-6 * scale) return false;
            } else if (c < -1.0 + 1e-9) {  // opposite faces: apart
                if (std::fabs(pl[i].d + pl[j].d) < 1e-3 * scale) return false;
            } else if (c * c > 0.75) {  // planes within 30 degrees of each other
                return false;
            }
        }
    return true;
}

TriRec make_triangle(v3 p0, v3 p1, v3 p2) {
    v3 e1 = sub(p1, p0);
    v3 e2 = sub(p2, p0);
    v3 n = normalize(cross(e1, e2));
    TriRec t;
    t.v0x = p0.x; t.v0y = p0.y; t.v0z = p0.z; t.nx = n.x;
    t.e1x = e1.x; t.e1y = e1.y; t.e1z = e1.z; t.ny = n.y;
    t.e2x = e2.x; t.e2y = e2.y; t.e2z = e2.z; t.nz = n.z;
    return t;
}

// ---------------------------------------------------------------------------
// OBJ ingestion. Restates the parts of tinyobjloader v2.0 (vendored by the
// reference as tinyobjloader/tiny_obj_loader.h) that decide triangle output:
// its decimal parser (tryParseDouble, :837-965, cast to float in parseReal
// :967-975), 1-based / negative index fix-up, and the quad split on the
// shorter diagonal (:1397-1495). n-gons (> 4 vertices) use tinyobjloader's
// ear clipping, which this loader does not restate: they are rejected.
//
// tinyobjloader is distributed under the MIT licence:
//   The MIT License (MIT)
//   Copyright (c) 2012-Present, Syoyo Fujita and many contributors.
//   Permission is hereby granted, free of charge, to any person obtaining a copy
//   of this software and associated documentation files (the "Software"), to deal
//   in the Software without restriction, including without limitation the rights
//   to use, copy, modify, merge, publish, distribute, sublicense, and/or sell
//   copies of the Software, and to permit persons to whom the Software is
//   furnished to do so, subject to the following conditions: The above copyright
//   notice and this permission notice shall be included in all copies or
//   substantial portions of the Software. THE SOFTWARE IS PROVIDED "AS IS",
//   WITHOUT WARRANTY OF ANY KIND, EXPRESS OR IMPLIED.
// ---------------------------------------------------------------------------
namespace {

bool parse_obj_double(const char* s, const char* e, double* out) {
    if (s >= e) return false;
    double mant = 0.0;
    int expo = 0;
    char sign = '+', esign = '+';
    const char* c = s;
    int read = 0;
    bool lead_dot = false;
    if (*c == '+' || *c == '-') {
        sign = *c++;
        if (c != e && *c == '.') lead_dot = true;
    } else if (*c >= '0' && *c <= '9') {
    } else if (*c == '.') {
        lead_dot = true;
    } else {
        return false;
    }
    if (!lead_dot) {
        while (c != e && *c >= '0' && *c <= '9') {
            mant *= 10;
            mant += (int)(*c - '0');
            ++c;
            ++read;
        }
        if (read == 0) return false;
    }
    if (c != e) {
        if (*c == '.') {
            ++c;
            read = 1;
            static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (c != e && *c >= '0' && *c <= '9') {
                mant += (int)(*c - '0') * (read < 8 ? lut[read] : pow(10.0, -read));
                ++read;
                ++c;
            }
        }
        if (c != e && (*c == 'e' || *c == 'E')) {
            ++c;
            if (c != e && (*c == '+' || *c == '-')) {
                esign = *c++;
            } else if (!(c != e && *c >= '0' && *c <= '9')) {
                return false;
            }
            read = 0;
            while (c != e && *c >= '0' && *c <= '9') {
                expo = expo * 10 + (int)(*c - '0');
                ++c;
                ++read;
            }
            expo *= (esign == '+' ? 1 : -1);
            if (read == 0) return false;
        }
    }
    *out = (sign == '+' ? 1 : -1) * (expo ? ldexp(mant * pow(5.0, expo), expo) : mant);
    return true;
}

float parse_obj_real(const char*& p) {
    p += strspn(p, " \t");
    const char* end = p + strcspn(p, " \t\r");
    double v = 0.0;
    parse_obj_double(p, end, &v);
    p = end;
    return (float)v;
}

}  // namespace

std::string load_obj_transformed(const std::string& path, v3 scl, v3 rot, v3 off,
                                 std::vector<float>& out) {
    std::ifstream in(path);
    if (!in) return "cannot open OBJ file: " + path;
    std::vector<float> pos;  // raw positions
    std::vector<int> idx;    // triangulated position indices
    std::string line;
    int lineno = 0;
    bool first_shape_done = false;
    bool in_shape = false;
    while (std::getline(in, line)) {
        ++lineno;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* p = line.c_str();
        p += strspn(p, " \t");
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            p += 2;
            float x = parse_obj_real(p);
            float y = parse_obj_real(p);
            float z = parse_obj_real(p);
            pos.push_back(x);
            pos.push_back(y);
            pos.push_back(z);
        } else if ((p[0] == 'o' || p[0] == 'g') && (p[1] == ' ' || p[1] == '\t')) {
            // loadModel(file, scale, rotate, offset) keeps only the first mesh
            // (getMeshes()[0], ModelLoader.cpp:421).
            if (in_shape && !idx.empty()) first_shape_done = true;
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            if (first_shape_done) continue;
            in_shape = true;
            p += 2;
            std::vector<int> face;
            const int nv = (int)(pos.size() / 3);
            while (*p) {
                p += strspn(p, " \t");
                if (!*p) break;
                int v = atoi(p);
                if (v > 0) v -= 1;
                else if (v < 0) v = nv + v;
                else return "OBJ face index 0 at line " + std::to_string(lineno);
                face.push_back(v);
                p += strcspn(p, " \t");
            }
            if (face.size() < 3) continue;  // degenerate face: skipped (tiny_obj_loader.h:1389-1395)
            for (int v : face)
                if (v < 0 || v >= nv) return "OBJ vertex index out of range at line " + std::to_string(lineno);
            if (face.size() == 3) {
                idx.insert(idx.end(), face.begin(), face.end());
            } else if (face.size() == 4) {
                const float* a = &pos[3 * face[0]];
                const float* b = &pos[3 * face[1]];
                const float* c = &pos[3 * face[2]];
                const float* d = &pos[3 * face[3]];
                float e02x = c[0] - a[0], e02y = c[1] - a[1], e02z = c[2] - a[2];
                float e13x = d[0] - b[0], e13y = d[1] - b[1], e13z = d[2] - b[2];
                float s02 = e02x * e02x + e02y * e02y + e02z * e02z;
                float s13 = e13x * e13x + e13y * e13y + e13z * e13z;
                if (s02 < s13) {
                    int t[6] = {face[0], face[1], face[2], face[0], face[2], face[3]};
                    idx.insert(idx.end(), t, t + 6);
                } else {
                    int t[6] = {face[0], face[1], face[3], face[1], face[2], face[3]};
                    idx.insert(idx.end(), t, t + 6);
                }
            } else {
                return "OBJ n-gon with " + std::to_string(face.size()) +
                       " vertices is not supported (line " + std::to_string(lineno) + ")";
            }
        }
    }
    // ModelLoader.cpp:438-445: vertex *= scale; rotateY(radians(rotate.y)); += offset.
    out.clear();
    out.reserve(idx.size() * 3);
    const float ry = radians(rot.y);
    for (int i : idx) {
        v3 v{pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]};
        v = mul(v, scl);
        v = rotate_y(v, ry);
        v = add(v, off);
        out.push_back(v.x);
        out.push_back(v.y);
        out.push_back(v.z);
    }
    return "";
}

// Leaf threshold of the BVHs over rayColor meshes and sphere groups (the reference's Recurse
// makes a leaf below 4 entries, BVH.cpp:106). Any tree gives the same hits (the closest-hit merge
// restates the sequential scan); the pathTrace tree is always the reference's.
#ifndef RT_MESH_LEAF_MIN
#define RT_MESH_LEAF_MIN 4
#endif
#ifndef RT_GROUP_LEAF_MIN
#define RT_GROUP_LEAF_MIN 4
#endif

void HostScene::build_bvh(const std::vector<v3>& vs, const std::vector<uint32_t>& ix, CFBvh& b,
                          const std::string& cache_ply) {
    const auto t0 = std::chrono::steady_clock::now();
    int got = 0;
    if (!cache_ply.empty() && (bvh_cache_mode & 1)) {
        got = read_bvh_cache(cache_ply, vs, ix, b, &cache_last_reject);
        if (got > 0) ++cache_reads;
        else if (got < 0) ++cache_rejected;
    }
    if (got <= 0) {
        if (bvh_gpu && gpu_build_cf_bvh(bvh_device, vs, ix, b, RT_MESH_LEAF_MIN, nullptr).empty()) ++bvh_gpu_builds;
        else build_cf_bvh(vs, ix, b, RT_MESH_LEAF_MIN);
        // rt_mesh_ply meshes read caches but never write them: a mesh placed with another
        // offset / maxCoord than the pathTrace scene's would overwrite that scene's cache (and
        // the two would keep rebuilding and replacing each other's file). The reference writes
        // `<ply>.bvh` from UpdateBoundingVolumeHierarchy only, i.e. the pathTrace scene
        // (rt_process_triangle_data).
    }
    bvh_build_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void HostScene::build_bvh_boxes(const std::vector<v3>& lo, const std::vector<v3>& hi, CFBvh& b) {
    const auto t0 = std::chrono::steady_clock::now();
    if (bvh_gpu && gpu_build_cf_bvh_boxes(bvh_device, lo, hi, b, RT_GROUP_LEAF_MIN, nullptr).empty()) ++bvh_gpu_builds;
    else build_cf_bvh_boxes(lo, hi, b, RT_GROUP_LEAF_MIN);
    bvh_build_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

std::string HostScene::flatten() {
    bvh_build_ms = 0.0;
    bvh_gpu_builds = 0;
    cache_reads = cache_writes = cache_rejected = 0;
    objs.clear();
    n_scan = 0;
    tris.clear();
    mats.clear();
    nodes.clear();
    tri_orig.clear();
    bvh_max_depth = 0;
    for (size_t i = 0; i < materials.size(); ++i) {
        MatRec m = materials[i].rec;
        if (!materials[i].defined) m.type = 0xFFFFFFFFu;  // never referenced by a defined object
        mats.push_back(m);
    }
    auto check_mat = [&](uint32_t m) -> bool {
        return m < materials.size() && materials[m].defined;
    };
    for (size_t i = 0; i < objects.size(); ++i) {
        const HostObject& o = objects[i];
        if (!o.defined) continue;  // null slots are skipped (main.cu:49)
        if (!check_mat(o.material))
            return "object " + std::to_string(i) + " references undefined material " +
                   std::to_string(o.material);
        if (o.type == kHostCube) {
            // createCube (kernels.h:139-154): six two-sided planes.
            v3 c{o.f[0], o.f[1], o.f[2]};
            v3 e{o.f[3], o.f[4], o.f[5]};
            struct Face { v3 p, n; uint32_t orient; };
            const Face faces[6] = {
                {{c.x - e.x, c.y, c.z}, {-1.0f, 0.0f, 0.0f}, 1},
                {{c.x + e.x, c.y, c.z}, {1.0f, 0.0f, 0.0f}, 1},
                {{c.x, c.y + e.y, c.z}, {0.0f, 1.0f, 0.0f}, 2},
                {{c.x, c.y - e.y, c.z}, {0.0f, -1.0f, 0.0f}, 2},
                {{c.x, c.y, c.z + e.z}, {0.0f, 0.0f, 1.0f}, 0},
                {{c.x, c.y, c.z - e.z}, {0.0f, 0.0f, -1.0f}, 0},
            };
            for (const Face& f : faces) {
                ObjRec r{};
                r.u2 = kNoBvh;
                r.type = kObjPlane;
                r.material = o.material;
                r.u0 = f.orient;
                r.u1 = 1;
                r.f[0] = f.p.x; r.f[1] = f.p.y; r.f[2] = f.p.z;
                r.f[3] = f.n.x; r.f[4] = f.n.y; r.f[5] = f.n.z;
                r.f[6] = e.x; r.f[7] = e.y; r.f[8] = e.z;
                objs.push_back(r);
            }
            continue;
        }
        ObjRec r{};
        r.type = o.type;
        r.material = o.material;
        r.u2 = kNoBvh;
        memcpy(r.f, o.f, sizeof(r.f));
        if (o.type == kObjMedium) {
            r.u0 = (uint32_t)i;             // slot: keys the free-flight draw
            r.f[6] = -1.0f / o.f[6];        // neg_inv_density
            // the boundary's face coordinates and rectangle bounds, center -/+ extend per axis: the
            // same floats the restatement computes per face (p.a -/+ e.a), evaluated once here
            for (int a = 0; a < 3; ++a) {
                r.f[a] = o.f[a] - o.f[3 + a];
                r.f[3 + a] = o.f[a] + o.f[3 + a];
            }
        } else if (o.type == kObjPlane) {
            r.u0 = o.orientation;
            r.u1 = o.two_side;
        } else if (o.type == kObjMesh) {
            const size_t nt = o.tri_vertices.size() / 9;
            if (nt == 0) continue;  // empty meshes are not created (main.cu:777)
            r.u0 = (uint32_t)tris.size();
            r.u1 = (uint32_t)nt;
            r.u2 = kNoBvh;
            // computeMeshAABB (main.cu:261-281): per-axis min / max of all vertices.
            v3 lo{o.tri_vertices[0], o.tri_vertices[1], o.tri_vertices[2]}, hi = lo;
            for (size_t k = 0; k < nt * 3; ++k) {
                const float* p = &o.tri_vertices[3 * k];
                lo.x = std::min(lo.x, p[0]); lo.y = std::min(lo.y, p[1]); lo.z = std::min(lo.z, p[2]);
                hi.x = std::max(hi.x, p[0]); hi.y = std::max(hi.y, p[1]); hi.z = std::max(hi.z, p[2]);
            }
            r.f[0] = lo.x; r.f[1] = lo.y; r.f[2] = lo.z;
            r.f[3] = hi.x; r.f[4] = hi.y; r.f[5] = hi.z;
            // the compaction's pair -> ray division p / nt as a multiply-high:
            // magic = ceil(2^32 / nt), exact for p < 2^26 (rt_kernel.hip mesh_compact)
            const uint32_t magic = nt > 1 ? 0xFFFFFFFFu / (uint32_t)nt + 1u : 0u;
            memcpy(&r.f[6], &magic, 4);
            std::vector<int32_t> order(nt);
            for (size_t t = 0; t < nt; ++t) order[t] = (int32_t)t;
            if (nt > kBvhMinTris) {
                // The reference's binned-SAH builder over this mesh's triangles.
                std::vector<v3> vs(nt * 3);
                std::vector<uint32_t> ix(nt * 3);
                for (size_t k = 0; k < nt * 3; ++k) {
                    vs[k] = v3{o.tri_vertices[3 * k], o.tri_vertices[3 * k + 1], o.tri_vertices[3 * k + 2]};
                    ix[k] = (uint32_t)k;
                }
                CFBvh b;
                build_bvh(vs, ix, b, o.bvh_cache);  // reference leaves (larger: measured slower)
                if (b.max_depth >= kBvhStackDepth)
                    return "mesh " + std::to_string(i) + ": BVH depth " + std::to_string(b.max_depth) +
                           " exceeds the traversal stack (" + std::to_string(kBvhStackDepth) + ")";
                bvh_max_depth = std::max(bvh_max_depth, b.max_depth);
                order.assign(b.tri_index.begin(), b.tri_index.end());
                const uint32_t nb = (uint32_t)nodes.size();
                r.u2 = nb;
                for (const CFNode& c : b.nodes) {
                    BvhNode n;
                    for (int a = 0; a < 3; ++a) {
                        // Conservative inflation: node tests may never cull a
                        // triangle the exact test accepts.
                        const float m = std::max(fabsf(c.bottom[a]), fabsf(c.top[a]));
                        const float pad = m * 1e-5f + 1e-30f;
                        n.lo[a] = c.bottom[a] - pad;
                        n.hi[a] = c.top[a] + pad;
                    }
                    if (c.u0 & 0x80000000u) {
                        n.a = r.u0 + c.u1;
                        n.b = c.u0;
                    } else {
                        n.a = nb + c.u0;
                        n.b = nb + c.u1;
                    }
                    nodes.push_back(n);
                }
            }
            // tri_orig pairs per leaf-order position j = base + t: (mesh-local index of the
            // triangle at j, position of the triangle whose mesh-local index is t)
            const size_t pair0 = tri_orig.size();
            tri_orig.resize(pair0 + 2 * nt);
            for (size_t t = 0; t < nt; ++t) {
                const float* p = &o.tri_vertices[9 * (size_t)order[t]];
                tris.push_back(make_triangle(v3{p[0], p[1], p[2]}, v3{p[3], p[4], p[5]},
                                             v3{p[6], p[7], p[8]}));
                tri_orig[pair0 + 2 * t] = (uint32_t)order[t];
                tri_orig[pair0 + 2 * (size_t)order[t] + 1] = r.u0 + (uint32_t)t;
            }
            // f[9] (brute-force meshes): 1 = a convex shell the kernels skip for rays leaving its surface
            const uint32_t convex = nt <= kBvhMinTris && convex_shell(&tris[r.u0], nt) ? 1u : 0u;
            memcpy(&r.f[9], &convex, 4);
        }
        objs.push_back(r);
    }
    for (size_t k = 0; k < objs.size(); ++k) objs[k].order = (uint32_t)k;  // sequential scan position
    // Plane::hit's rectangle bounds (Plane.cu:25-45: position -/+ extend on the two axes
    // of the orientation), evaluated once here with the same float ops; the kernel
    // compares the hit point against f[6..9] = (lo_a, hi_a, lo_b, hi_b).
    for (ObjRec& r : objs) {
        if (r.type != kObjPlane) continue;
        const int a = r.u0 == 1u ? 1 : 0, b = r.u0 == 0u ? 1 : 2;
        const float pa = r.f[a], ea = r.f[6 + a], pb = r.f[b], eb = r.f[6 + b];
        r.f[6] = pa - ea;
        r.f[7] = pa + ea;
        r.f[8] = pb - eb;
        r.f[9] = pb + eb;
        const int k = r.u0 == 0u ? 2 : r.u0 == 1u ? 0 : 1;  // the orientation's normal axis
        const float nk = r.f[3 + k];
        if ((nk == 1.0f || nk == -1.0f) && r.f[3 + (k + 1) % 3] == 0.0f && r.f[3 + (k + 2) % 3] == 0.0f &&
            r.u0 < 3u) {
            r.type = kObjPlaneAxial + r.u0;
            r.u1 = r.u1 ? 0x3F800000u : 0u;  // twoSide as the float 1 or 0 (still non-zero iff two-sided)
        }
    }
    n_scan = (int)objs.size();
    const std::string err = group_spheres();
    if (!err.empty()) return err;
    mark_mesh_runs();
    return build_mesh_pairs();
}

namespace {
// Child-pair records of one mesh BVH (see HostScene::build_mesh_pairs).
struct PairBuilder {
    std::vector<BvhNode>& nodes;
    int max_pairs = 0;  // pair records on the longest root-to-leaf path = stack entries a lane may need
    bool empty_leaf = false;

    uint32_t alloc() {
        const size_t at = nodes.size();
        nodes.resize(at + 2, BvhNode{});
        return (uint32_t)(at / 2);
    }
    void set(uint32_t q, BvhNode l, uint32_t ref_l, BvhNode r, uint32_t ref_r) {
        l.a = ref_l;
        l.b = 0;
        r.a = ref_r;
        r.b = 0;
        nodes[2 * (size_t)q] = l;
        nodes[2 * (size_t)q + 1] = r;
    }
    // reference to triangles [first, first + count) of a leaf whose box is `box`; `above` = pairs above it
    uint32_t leaf(BvhNode box, uint32_t first, uint32_t count, int above) {
        if (count <= kLeafRefMax) {
            empty_leaf |= count == 0u;
            max_pairs = std::max(max_pairs, above);
            return kLeafRef | ((count - 1u) << 27) | first;
        }
        const uint32_t q = alloc();  // a larger leaf: two halves under the same box
        const uint32_t half = count / 2u;
        const uint32_t l = leaf(box, first, half, above + 1), r = leaf(box, first + half, count - half, above + 1);
        set(q, box, l, box, r);
        return q;
    }
    uint32_t node(uint32_t i, int above) {
        const BvhNode n = nodes[i];
        if (n.b & 0x80000000u) return leaf(n, n.a, n.b & 0x7FFFFFFFu, above);
        const uint32_t q = alloc();
        const uint32_t l = node(n.a, above + 1), r = node(n.b, above + 1);
        set(q, nodes[n.a], l, nodes[n.b], r);
        return q;
    }
};


// Quantized child-pair records of one MESH BVH (rt_scene.h QPair; see HostScene::build_mesh_pairs): the
// PairBuilder tree, one 32 B slot per pair, boxes on the 16-bit grid of the mesh's frame.
struct QPairBuilder {
    std::vector<BvhNode>& nodes;
    float c[3] = {0.0f, 0.0f, 0.0f};
    double s = 0.0;  // grid step, a power of two
    int max_pairs = 0;
    bool empty_leaf = false;
    bool bad = false;  // a box off the grid (never, by the frame's construction)

    void extent(uint32_t i, float lo[3], float hi[3]) const {
        const BvhNode n = nodes[i];
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], n.lo[a]);
            hi[a] = std::max(hi[a], n.hi[a]);
        }
        if (!(n.b & 0x80000000u)) {
            extent(n.a, lo, hi);
            extent(n.b, lo, hi);
        }
    }
    // The frame: s = the smallest power of two that puts every box of the tree on a grid of kQMax steps
    // with two spare steps at each end (and at least 2^-40 of the coordinates' magnitude), c = the boxes'
    // minimum less two steps, rounded down to a float.
    void frame(uint32_t root) {
        float lo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
        float hi[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
        extent(root, lo, hi);
        double ext = 0.0, mag = 0.0;
        for (int a = 0; a < 3; ++a) {
            ext = std::max(ext, (double)hi[a] - (double)lo[a]);
            mag = std::max(mag, std::max(std::fabs((double)lo[a]), std::fabs((double)hi[a])));
        }
        s = std::ldexp(1.0, -126);
        while (s * (kQMax - 8) < ext || s < mag * 0x1p-40) s *= 2.0;
        for (int a = 0; a < 3; ++a) {
            const double want = (double)lo[a] - 2.0 * s;
            float cf = (float)want;
            if ((double)cf > want) cf = std::nextafter(cf, -__builtin_huge_valf());
            c[a] = cf;
        }
    }
    // grid coordinates of a box, one more step outward than its floor / ceil
    void quantize(const BvhNode& b, uint32_t* q) {
        uint32_t v[6];
        for (int a = 0; a < 3; ++a) {
            const double l = std::floor(((double)b.lo[a] - (double)c[a]) / s) - 1.0;
            const double h = std::ceil(((double)b.hi[a] - (double)c[a]) / s) + 1.0;
            if (!(l >= 0.0) || !(h <= (double)kQMax)) bad = true;
            v[a] = (uint32_t)std::max(0.0, std::min(l, (double)kQMax));
            v[3 + a] = (uint32_t)std::max(0.0, std::min(h, (double)kQMax));
        }
        q[0] = v[0] | v[1] << 16;
        q[1] = v[2] | v[3] << 16;
        q[2] = v[4] | v[5] << 16;
    }
    uint32_t alloc() {
        nodes.emplace_back();
        return (uint32_t)(nodes.size() - 1);
    }
    void set(uint32_t q, const BvhNode& l, uint32_t ref_l, const BvhNode& r, uint32_t ref_r) {
        QPair p{};
        quantize(l, &p.q[0]);
        quantize(r, &p.q[3]);
        p.ref[0] = ref_l;
        p.ref[1] = ref_r;
        memcpy(&nodes[q], &p, sizeof p);
    }
    uint32_t leaf(const BvhNode& box, uint32_t first, uint32_t count, int above) {
        if (count <= kLeafRefMax) {
            empty_leaf |= count == 0u;
            max_pairs = std::max(max_pairs, above);
            return kLeafRef | ((count - 1u) << 27) | first;
        }
        const uint32_t q = alloc();  // a larger leaf: two halves under the same box
        const uint32_t half = count / 2u;
        const uint32_t l = leaf(box, first, half, above + 1), r = leaf(box, first + half, count - half, above + 1);
        set(q, box, l, box, r);
        return q;
    }
    uint32_t node(uint32_t i, int above) {
        const BvhNode n = nodes[i];
        if (n.b & 0x80000000u) return leaf(n, n.a, n.b & 0x7FFFFFFFu, above);
        const uint32_t q = alloc();
        const uint32_t l = node(n.a, above + 1), r = node(n.b, above + 1);
        const BvhNode nl = nodes[n.a], nr = nodes[n.b];
        set(q, nl, l, nr, r);
        return q;
    }
};
}  // namespace

// The batched traversals (rt_kernel.hip mesh_bvh_pairs, sphere_group_batched) read each inner
// node of a mesh or sphere-group BVH as one 64 B child-pair record - both children's boxes, each with a reference word: a
// pair index (the child's own pair at nodes[2q], nodes[2q + 1]) or a leaf reference
// (kLeafRef | (count - 1) << 27 | first triangle or member, count <= 16; larger leaves become pairs of
// halves under the leaf's box). A lane therefore never loads a node to learn what its stack
// entry is: one dependent load per inner step, none for leaves. The records follow the
// node table (from an even index, so each pair is one aligned 64 B line); the mesh or group
// record keeps its node root in u2 and carries its root reference in f[8] (as u32 bits). Any
// tree over the same primitives gives the same hit (conservative boxes, the (t, index) minimum).
std::string HostScene::build_mesh_pairs() {
    auto tree = [&](const ObjRec& r) {
        return (r.type == kObjMesh || r.type == kObjSphereGroup) && r.u2 != kNoBvh;
    };
    bool any = false;
    for (int k = 0; k < n_scan; ++k) any |= tree(objs[k]);
    if (!any) return "";
    if (tris.size() >= (size_t(1) << 26) || objs.size() >= (size_t(1) << 26))
        return "too many triangles or objects for the BVH references (2^26)";
    if (nodes.size() & 1u) nodes.push_back(BvhNode{});
    // the LDS stacks are sized by what the traversals below may push (not the binary depth)
    bvh_max_depth = 0;
    for (int k = 0; k < n_scan; ++k) {
        ObjRec& r = objs[k];
        if (!tree(r)) continue;
        if (r.type == kObjMesh) {  // quantized 32 B pairs after the mesh's QFrame (rt_scene.h)
            QPairBuilder qb{nodes};
            qb.frame(r.u2);
            const uint32_t fs = qb.alloc();
            const uint32_t root = qb.node(r.u2, 0);
            if (qb.empty_leaf) return "BVH with an empty leaf";
            if (qb.bad) return "mesh BVH box off its quantization grid";
            if (qb.max_pairs > kBvhStackDepth)
                return "BVH pair depth " + std::to_string(qb.max_pairs) + " exceeds the traversal stack (" +
                       std::to_string(kBvhStackDepth) + ")";
            if (nodes.size() >= ((size_t)1 << 31)) return "too many BVH nodes (2^31)";
            QFrame fr{};
            for (int a = 0; a < 3; ++a) fr.c[a] = qb.c[a];
            fr.s = (float)qb.s;
            memcpy(&nodes[fs], &fr, sizeof fr);
            bvh_max_depth = std::max(bvh_max_depth, qb.max_pairs);
            memcpy(&r.f[8], &root, 4);
            memcpy(&r.f[6], &fs, 4);
            continue;
        }
        if (nodes.size() & 1u) nodes.push_back(BvhNode{});
        PairBuilder pb{nodes};
        const uint32_t root = pb.node(r.u2, 0);
        if (pb.empty_leaf) return "BVH with an empty leaf";
        if (pb.max_pairs > kBvhStackDepth)
            return "BVH pair depth " + std::to_string(pb.max_pairs) + " exceeds the traversal stack (" +
                   std::to_string(kBvhStackDepth) + ")";
        bvh_max_depth = std::max(bvh_max_depth, pb.max_pairs);
        memcpy(&r.f[8], &root, 4);
    }
    // f[9] = 2 (as u32 bits): the kernel may defer this mesh's traversal for its few wanting rays to the next
    // loop trip (rt_kernel.hip kMeshDefer). A deferred ray scans the list again, so only when no object of
    // the scan draws from the ray's stream (a participating medium) or counts its tests per scan (a
    // brute-force mesh), and this is the scan's only mesh (no sphere group either).
    int meshes = 0, others = 0;
    for (int k = 0; k < n_scan; ++k) {
        const ObjRec& r = objs[k];
        meshes += r.type == kObjMesh;
        others += r.type == kObjMedium || r.type == kObjSphereGroup || (r.type == kObjMesh && !tree(r));
    }
    if (meshes == 1 && others == 0)
        for (int k = 0; k < n_scan; ++k)
            if (objs[k].type == kObjMesh) {
                const uint32_t defer = 2u;
                memcpy(&objs[k].f[9], &defer, 4);
            }
    return "";
}

// Runs for the kernel's mesh_run: consecutive brute-force meshes of the final scan list
// with the same triangle count, consecutive triangle ranges and consecutive scan orders
// (up to kMeshRunMax). The first record of a run carries its length in f[7] (as u32
// bits), the others 0; a brute-force mesh outside any run is a run of 1.
void HostScene::mark_mesh_runs() {
    auto brute = [&](size_t k) { return objs[k].type == kObjMesh && objs[k].u2 == kNoBvh; };
    const size_t n = (size_t)n_scan;
    for (size_t k = 0; k < n;) {
        if (!brute(k)) {
            ++k;
            continue;
        }
        const ObjRec& a = objs[k];
        size_t e = k + 1;
        while (e < n && e - k < kMeshRunMax && brute(e) && objs[e].u1 == a.u1 &&
               objs[e].u0 == a.u0 + (uint32_t)(e - k) * a.u1 && objs[e].order == a.order + (uint32_t)(e - k))
            ++e;
        for (size_t j = k; j < e; ++j) {
            const uint32_t g = j == k ? (uint32_t)(e - k) : 0u;
            memcpy(&objs[j].f[7], &g, 4);
        }
        k = e;
    }
}

// Moves the (moving) spheres of a large scene behind one kObjSphereGroup record
// with the reference's binned-SAH builder over their boxes. The kernel merges
// hits with the sequential scan's tie rule (ObjRec::order), so the result is
// the same as scanning them in slot order.
std::string HostScene::group_spheres() {
    std::vector<ObjRec> scan, members;
    for (const ObjRec& r : objs) {
        if (r.type == kObjSphere || r.type == kObjMovingSphere) members.push_back(r);
        else scan.push_back(r);
    }
    if (members.size() < kSphereBvhMin) return "";
    const float t0 = has_camera ? camera.time0 : 0.0f, t1 = has_camera ? camera.time1 : 0.0f;
    std::vector<v3> lo(members.size()), hi(members.size());
    for (size_t k = 0; k < members.size(); ++k) {
        const float* f = members[k].f;
        v3 a, b;
        float r;
        if (members[k].type == kObjSphere) {
            a = b = v3{f[0], f[1], f[2]};
            r = fabsf(f[3]);
        } else {
            // The centre is affine in the ray time, and ray times lie in the
            // camera's shutter interval: its endpoints bound the motion.
            auto centre = [&](float t) {
                const float w = (t - f[6]) / (f[7] - f[6]);
                return v3{f[0] + w * (f[3] - f[0]), f[1] + w * (f[4] - f[1]), f[2] + w * (f[5] - f[2])};
            };
            a = centre(t0);
            b = centre(t1);
            r = fabsf(f[8]);
        }
        v3 l{std::min(a.x, b.x) - r, std::min(a.y, b.y) - r, std::min(a.z, b.z) - r};
        v3 h{std::max(a.x, b.x) + r, std::max(a.y, b.y) + r, std::max(a.z, b.z) + r};
        if (!(std::isfinite(l.x) && std::isfinite(l.y) && std::isfinite(l.z) && std::isfinite(h.x) &&
              std::isfinite(h.y) && std::isfinite(h.z)))
            return "sphere with non-finite bounds (degenerate moving-sphere time range?)";
        lo[k] = l;
        hi[k] = h;
    }
    // Spheres far larger than the rest (RTNW's r = 1000 ground) stay in the linear scan:
    // inside the tree their box would enlarge every node on their root path, and every
    // ray would descend it. Any split of the objects between the scan and the group
    // gives the same hit (Hit::merge restates the sequential tie rule).
    {
        std::vector<float> ext(members.size());
        for (size_t k = 0; k < members.size(); ++k)
            ext[k] = std::max(hi[k].x - lo[k].x, std::max(hi[k].y - lo[k].y, hi[k].z - lo[k].z));
        std::vector<float> sorted = ext;
        std::nth_element(sorted.begin(), sorted.begin() + sorted.size() / 2, sorted.end());
        const float core_cap = 8.0f * sorted[sorted.size() / 2];
        v3 cl{FLT_MAX, FLT_MAX, FLT_MAX}, ch{-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (size_t k = 0; k < members.size(); ++k) {
            if (ext[k] > core_cap) continue;
            cl = v3{std::min(cl.x, lo[k].x), std::min(cl.y, lo[k].y), std::min(cl.z, lo[k].z)};
            ch = v3{std::max(ch.x, hi[k].x), std::max(ch.y, hi[k].y), std::max(ch.z, hi[k].z)};
        }
        const float core_ext = std::max(ch.x - cl.x, std::max(ch.y - cl.y, ch.z - cl.z));
        std::vector<ObjRec> keep;
        std::vector<v3> klo, khi;
        for (size_t k = 0; k < members.size(); ++k) {
            if (ext[k] > 0.5f * core_ext) {
                scan.push_back(members[k]);
                continue;
            }
            keep.push_back(members[k]);
            klo.push_back(lo[k]);
            khi.push_back(hi[k]);
        }
        if (keep.size() < kSphereBvhMin) return "";  // not worth a tree: scan everything
        members.swap(keep);
        lo.swap(klo);
        hi.swap(khi);
    }
    CFBvh b;
    build_bvh_boxes(lo, hi, b);
    if (b.max_depth >= kBvhStackDepth)
        return "sphere BVH depth " + std::to_string(b.max_depth) + " exceeds the traversal stack";
    bvh_max_depth = std::max(bvh_max_depth, b.max_depth);
    ObjRec g{};
    g.type = kObjSphereGroup;
    g.order = 0xFFFFFFFFu;
    g.u0 = (uint32_t)(scan.size() + 1);  // members follow the scan list
    g.u1 = (uint32_t)members.size();
    g.u2 = (uint32_t)nodes.size();
    const uint32_t nb = (uint32_t)nodes.size();
    for (const CFNode& c : b.nodes) {
        BvhNode n;
        for (int a = 0; a < 3; ++a) {
            const float m = std::max(fabsf(c.bottom[a]), fabsf(c.top[a]));
            const float pad = m * 1e-5f + 1e-30f;
            n.lo[a] = c.bottom[a] - pad;
            n.hi[a] = c.top[a] + pad;
        }
        if (c.u0 & 0x80000000u) {
            n.a = g.u0 + c.u1;
            n.b = c.u0;
        } else {
            n.a = nb + c.u0;
            n.b = nb + c.u1;
        }
        nodes.push_back(n);
    }
    scan.push_back(g);
    n_scan = (int)scan.size();
    for (int32_t k : b.tri_index) scan.push_back(members[(size_t)k]);
    objs.swap(scan);
    return "";
}

}  // namespace rt
