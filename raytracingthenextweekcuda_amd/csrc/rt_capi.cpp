// rt_capi.cpp — the C ABI of include/rtmi.h.
//
// Replaces the reference's host driver (main.cu initialize/pathTracing/cleanup,
// main.cu:555-936) and the device-side `new` factories of kernels.h with a
// context that owns a host scene description and its device tables.
#include "../../include/rtmi.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <stdexcept>
#include <chrono>
#include <string>
#include <vector>

#include "rt_bvh.h"
#include "rt_ctx.h"
#include "rt_kernel.h"
#include "rt_scene.h"
#include "rt_yaml.h"

namespace rtc {

rt_status fail(rt_ctx* c, rt_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

rt_status hip_fail(rt_ctx* c, hipError_t e, const char* what) {
    return fail(c, RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

rt_status ensure_device(rt_ctx* c, void** buf, size_t* have, size_t bytes) {
    if (bytes <= *have) return RT_OK;
    (void)hipFree(*buf);
    *buf = nullptr;
    *have = 0;
    RT_HIP(c, hipMalloc(buf, bytes));
    *have = bytes;
    return RT_OK;
}

}  // namespace rtc

using rtc::fail;
using rtc::hip_fail;
using rtc::launch;
using rtc::validate;

namespace {

bool finite3(const float* v) { return v && isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]); }

rt::HostMaterial* mat_slot(rt_ctx* c, int32_t index) {
    if (index < 0 || index > (1 << 24)) return nullptr;
    if ((size_t)index >= c->scene.materials.size()) c->scene.materials.resize(index + 1);
    c->committed = false;
    return &c->scene.materials[index];
}

rt::HostObject* obj_slot(rt_ctx* c, int32_t index) {
    if (index < 0 || index > (1 << 24)) return nullptr;
    if ((size_t)index >= c->scene.objects.size()) c->scene.objects.resize(index + 1);
    c->committed = false;
    return &c->scene.objects[index];
}

void free_device(rt_ctx* c) {
    if (c->device < 0) return;
    (void)hipFree(c->d_objs);
    (void)hipFree(c->d_tris);
    (void)hipFree(c->d_mats);
    (void)hipFree(c->d_nodes);
    (void)hipFree(c->d_tri_orig);
    c->d_objs = nullptr;
    c->d_tris = nullptr;
    c->d_mats = nullptr;
    c->d_nodes = nullptr;
    c->d_tri_orig = nullptr;
}

void free_pathtrace(rt_ctx* c) {
    if (c->device >= 0) {
        (void)hipFree(c->d_pt_tris);
        (void)hipFree(c->d_pt_nodes);
        (void)hipFree(c->d_pt_list);
    }
    c->d_pt_tris = nullptr;
    c->d_pt_nodes = nullptr;
    c->d_pt_list = nullptr;
    c->pt_ready = false;
    c->pt_tris = 0;
    c->pt_root_ref = 0;
    c->pt_pair_depth = 0;
}

}  // namespace

extern "C" {

int32_t rt_abi_version(void) { return RTMI_ABI_VERSION; }

rt_status rt_create(int32_t device, rt_ctx** out) {
    if (!out) return RT_ERR_INVALID;
    *out = nullptr;
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return RT_ERR_OOM;
    c->device = device;
    if (device >= 0) {
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess || n == 0) {
            delete c;
            return RT_ERR_NODEV;
        }
        if (device >= n) {
            delete c;
            return RT_ERR_INVALID;
        }
        if (hipSetDevice(device) != hipSuccess ||
            hipMalloc(&c->d_counters, rt::kNumCounters * sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc(&c->d_cam, sizeof(rt::CamRec)) != hipSuccess ||
            hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
            delete c;
            return RT_ERR_HIP;
        }
        c->have_events = true;
        if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            hipMalloc(&c->d_queue, rt::kQueueHeadWords * sizeof(uint32_t)) != hipSuccess) {
            rt_destroy(c);
            return RT_ERR_HIP;
        }
    }
    *out = c;
    return RT_OK;
}

void rt_destroy(rt_ctx* c) {
    if (!c) return;
    if (c->device >= 0) {
        (void)hipSetDevice(c->device);
        free_device(c);
        free_pathtrace(c);
        (void)hipFree(c->d_counters);
        (void)hipFree(c->d_cam);
        (void)hipFree(c->d_out);
        (void)hipFree(c->d_u8);
        (void)hipFree(c->d_queue);
        (void)hipFree(c->d_partial);
        (void)hipFree(c->d_stage);
        (void)hipFree(c->d_frame);
        rtc::destroy_multi(c);
        for (hipEvent_t e : c->kev0) (void)hipEventDestroy(e);
        for (hipEvent_t e : c->kev1) (void)hipEventDestroy(e);
        if (c->have_events) {
            (void)hipEventDestroy(c->ev0);
            (void)hipEventDestroy(c->ev1);
        }
    }
    delete c;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

rt_status rt_clear_scene(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    c->scene = rt::HostScene();
    c->committed = false;
    if (c->device >= 0) (void)hipSetDevice(c->device);
    free_pathtrace(c);
    c->pt_raw = rt::PlyMesh();
    c->pt_last_file.clear();
    c->pt_materials.clear();
    return RT_OK;
}

// ---- materials (kernels.h:50-84) ----
rt_status rt_material_lambertian(rt_ctx* c, int32_t index, const float albedo[3], float absorb) {
    (void)absorb;  // stored but unused by the reference's Lambertian::scatter (Material.h:35)
    if (!c) return RT_ERR_INVALID;
    if (!finite3(albedo)) return fail(c, RT_ERR_INVALID, "lambertian: albedo must be 3 finite floats");
    rt::HostMaterial* m = mat_slot(c, index);
    if (!m) return fail(c, RT_ERR_INVALID, "material index out of range");
    m->defined = true;
    m->rec = rt::MatRec{RT_LAMBERTIAN, albedo[0], albedo[1], albedo[2], 0.0f, 0, 0, 0};
    return RT_OK;
}

rt_status rt_material_metal(rt_ctx* c, int32_t index, const float albedo[3], float fuzz) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(albedo) || !isfinite(fuzz))
        return fail(c, RT_ERR_INVALID, "metal: albedo/fuzz must be finite");
    rt::HostMaterial* m = mat_slot(c, index);
    if (!m) return fail(c, RT_ERR_INVALID, "material index out of range");
    m->defined = true;
    // Metal ctor: fuzz(inFuzz < 1.0f ? inFuzz : 1.0f) (Material.h:40).
    m->rec = rt::MatRec{RT_METAL, albedo[0], albedo[1], albedo[2], fuzz < 1.0f ? fuzz : 1.0f, 0, 0, 0};
    return RT_OK;
}

rt_status rt_material_dielectric(rt_ctx* c, int32_t index, float ior) {
    if (!c) return RT_ERR_INVALID;
    if (!isfinite(ior) || ior <= 0.0f) return fail(c, RT_ERR_INVALID, "dielectric: ior must be > 0");
    rt::HostMaterial* m = mat_slot(c, index);
    if (!m) return fail(c, RT_ERR_INVALID, "material index out of range");
    m->defined = true;
    m->rec = rt::MatRec{RT_DIELECTRIC, 1.0f, 1.0f, 1.0f, ior, 0, 0, 0};
    return RT_OK;
}

rt_status rt_material_emission(rt_ctx* c, int32_t index, const float albedo[3], float intensity) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(albedo) || !isfinite(intensity))
        return fail(c, RT_ERR_INVALID, "emission: albedo/intensity must be finite");
    rt::HostMaterial* m = mat_slot(c, index);
    if (!m) return fail(c, RT_ERR_INVALID, "material index out of range");
    m->defined = true;
    // attenuation = albedo * intensity (Material.h:121), precomputed.
    m->rec = rt::MatRec{RT_EMISSION, albedo[0] * intensity, albedo[1] * intensity,
                        albedo[2] * intensity, intensity, 0, 0, 0};
    return RT_OK;
}

rt_status rt_material_isotropic(rt_ctx* c, int32_t index, const float albedo[3]) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(albedo)) return fail(c, RT_ERR_INVALID, "isotropic: albedo must be 3 finite floats");
    rt::HostMaterial* m = mat_slot(c, index);
    if (!m) return fail(c, RT_ERR_INVALID, "material index out of range");
    m->defined = true;
    m->rec = rt::MatRec{RT_ISOTROPIC, albedo[0], albedo[1], albedo[2], 0.0f, 0, 0, 0};
    return RT_OK;
}

int32_t rt_material_defined(const rt_ctx* c, int32_t index) {
    if (!c || index < 0 || (size_t)index >= c->scene.materials.size()) return 0;
    return c->scene.materials[index].defined ? 1 : 0;
}

// ---- hitables (kernels.h:99-154) ----
rt_status rt_sphere(rt_ctx* c, int32_t index, const float center[3], float radius,
                    int32_t material, int32_t shading) {
    (void)shading;  // Sphere::bShading is stored but never read on the hot path
    if (!c) return RT_ERR_INVALID;
    if (!finite3(center) || !isfinite(radius)) return fail(c, RT_ERR_INVALID, "sphere: non-finite input");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kObjSphere;
    o->material = (uint32_t)material;
    memcpy(o->f, center, 3 * sizeof(float));
    o->f[3] = radius;
    return RT_OK;
}

rt_status rt_moving_sphere(rt_ctx* c, int32_t index, const float c0[3], const float c1[3],
                           float t0, float t1, float radius, int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(c0) || !finite3(c1) || !isfinite(t0) || !isfinite(t1) || !isfinite(radius))
        return fail(c, RT_ERR_INVALID, "moving sphere: non-finite input");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kObjMovingSphere;
    o->material = (uint32_t)material;
    memcpy(o->f, c0, 3 * sizeof(float));
    memcpy(o->f + 3, c1, 3 * sizeof(float));
    o->f[6] = t0;
    o->f[7] = t1;
    o->f[8] = radius;
    return RT_OK;
}

rt_status rt_plane(rt_ctx* c, int32_t index, const float pos[3], const float normal[3],
                   const float extend[3], int32_t material, int32_t orientation, int32_t two_side) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(pos) || !finite3(normal) || !finite3(extend))
        return fail(c, RT_ERR_INVALID, "plane: non-finite input");
    if (orientation < 0 || orientation > 2) return fail(c, RT_ERR_INVALID, "plane: orientation must be 0..2");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kObjPlane;
    o->material = (uint32_t)material;
    o->orientation = (uint32_t)orientation;
    o->two_side = two_side ? 1u : 0u;
    memcpy(o->f, pos, 3 * sizeof(float));
    memcpy(o->f + 3, normal, 3 * sizeof(float));
    memcpy(o->f + 6, extend, 3 * sizeof(float));
    return RT_OK;
}

rt_status rt_constant_medium(rt_ctx* c, int32_t index, const float center[3],
                             const float extend[3], float density, int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(center) || !finite3(extend) || !isfinite(density) || !(density > 0.0f))
        return fail(c, RT_ERR_INVALID, "constant medium: non-finite input or density <= 0");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kObjMedium;
    o->material = (uint32_t)material;
    memcpy(o->f, center, 3 * sizeof(float));
    memcpy(o->f + 3, extend, 3 * sizeof(float));
    o->f[6] = density;
    return RT_OK;
}

rt_status rt_cube(rt_ctx* c, int32_t index, const float center[3], const float extend[3],
                  int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(center) || !finite3(extend)) return fail(c, RT_ERR_INVALID, "cube: non-finite input");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kHostCube;
    o->material = (uint32_t)material;
    memcpy(o->f, center, 3 * sizeof(float));
    memcpy(o->f + 3, extend, 3 * sizeof(float));
    return RT_OK;
}

static rt_status rt_mesh_impl(rt_ctx* c, int32_t index, const float* v, int32_t n_tris, int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (n_tris < 0 || (n_tris > 0 && !v)) return fail(c, RT_ERR_INVALID, "mesh: bad vertex array");
    for (int64_t i = 0; i < (int64_t)n_tris * 9; ++i)
        if (!isfinite(v[i])) return fail(c, RT_ERR_INVALID, "mesh: non-finite vertex");
    rt::HostObject* o = obj_slot(c, index);
    if (!o) return fail(c, RT_ERR_INVALID, "object index out of range");
    *o = rt::HostObject();
    o->defined = true;
    o->type = rt::kObjMesh;
    o->material = (uint32_t)material;
    o->tri_vertices.assign(v, v + (size_t)n_tris * 9);
    return RT_OK;
}

static rt_status rt_mesh_obj_impl(rt_ctx* c, int32_t index, const char* path, const float scale[3],
                      const float rotate[3], const float offset[3], int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (!path || !finite3(scale) || !finite3(rotate) || !finite3(offset))
        return fail(c, RT_ERR_INVALID, "mesh_obj: bad arguments");
    std::vector<float> verts;
    std::string e = rt::load_obj_transformed(path, rt::v3{scale[0], scale[1], scale[2]},
                                             rt::v3{rotate[0], rotate[1], rotate[2]},
                                             rt::v3{offset[0], offset[1], offset[2]}, verts);
    if (!e.empty()) return fail(c, RT_ERR_IO, e);
    return rt_mesh(c, index, verts.data(), (int32_t)(verts.size() / 9), material);
}

static rt_status rt_mesh_ply_impl(rt_ctx* c, int32_t index, const char* path, const float offset[3],
                      float max_coord, int32_t material) {
    if (!c) return RT_ERR_INVALID;
    if (!path || !finite3(offset) || !isfinite(max_coord) || max_coord <= 0.0f)
        return fail(c, RT_ERR_INVALID, "mesh_ply: bad arguments");
    rt::PlyMesh m;
    std::string e = rt::load_ply(path, m);
    if (!e.empty()) return fail(c, RT_ERR_IO, e);
    rt::process_ply_vertices(m, rt::v3{offset[0], offset[1], offset[2]}, max_coord);
    std::vector<float> verts;
    verts.reserve(m.indices.size() * 3);
    for (uint32_t i : m.indices) {
        verts.push_back(m.vertices[i].x);
        verts.push_back(m.vertices[i].y);
        verts.push_back(m.vertices[i].z);
    }
    rt_status st = rt_mesh(c, index, verts.data(), (int32_t)(verts.size() / 9), material);
    if (st == RT_OK) c->scene.objects[(size_t)index].bvh_cache = path;  // its `<ply>.bvh` (BVH.cpp:503-504)
    return st;
}

static rt_status rt_ply_bvh_image_impl(const char* path, const float offset[3], float max_coord,
                           uint8_t* out, int64_t capacity, int64_t* size) {
    if (!path || !finite3(offset) || !size || !(max_coord > 0.0f)) return RT_ERR_INVALID;
    rt::PlyMesh m;
    if (!rt::load_ply(path, m).empty()) return RT_ERR_IO;
    rt::process_ply_vertices(m, rt::v3{offset[0], offset[1], offset[2]}, max_coord);
    rt::CFBvh b;
    rt::build_cf_bvh(m.vertices, m.indices, b);
    std::vector<uint8_t> img = rt::bvh_image(b);
    *size = (int64_t)img.size();
    if (out && capacity > 0) memcpy(out, img.data(), (size_t)std::min<int64_t>(capacity, *size));
    return RT_OK;
}

static rt_status rt_ply_bvh_image_gpu_impl(int32_t device, const char* path, const float offset[3], float max_coord,
                               uint8_t* out, int64_t capacity, int64_t* size, double* build_ms) {
    if (device < 0 || !path || !finite3(offset) || !size || !(max_coord > 0.0f)) return RT_ERR_INVALID;
    rt::PlyMesh m;
    if (!rt::load_ply(path, m).empty()) return RT_ERR_IO;
    rt::process_ply_vertices(m, rt::v3{offset[0], offset[1], offset[2]}, max_coord);
    rt::CFBvh b;
    double ms = 0.0;
    if (!rt::gpu_build_cf_bvh(device, m.vertices, m.indices, b, 4, &ms).empty()) return RT_ERR_HIP;
    if (build_ms) *build_ms = ms;
    std::vector<uint8_t> img = rt::bvh_image(b);
    *size = (int64_t)img.size();
    if (out && capacity > 0) memcpy(out, img.data(), (size_t)std::min<int64_t>(capacity, *size));
    return RT_OK;
}

rt_status rt_set_bvh_builder(rt_ctx* c, int32_t builder) {
    if (!c) return RT_ERR_INVALID;
    if (builder != RT_BVH_HOST && builder != RT_BVH_GPU) return fail(c, RT_ERR_INVALID, "unknown BVH builder");
    if (builder == RT_BVH_GPU && c->device < 0) return fail(c, RT_ERR_NODEV, "the GPU builder needs a device context");
    c->scene.bvh_gpu = builder == RT_BVH_GPU;
    c->scene.bvh_device = c->device;
    return RT_OK;
}

rt_status rt_set_bvh_cache(rt_ctx* c, int32_t mode) {
    if (!c) return RT_ERR_INVALID;
    if (mode & ~(RT_BVH_CACHE_READ | RT_BVH_CACHE_WRITE)) return fail(c, RT_ERR_INVALID, "unknown BVH cache mode");
    c->scene.bvh_cache_mode = mode;
    c->committed = false;
    c->pt_ready = false;
    return RT_OK;
}

rt_status rt_bvh_cache_stats(const rt_ctx* c, int32_t* reads, int32_t* writes, int32_t* rejected) {
    if (!c) return RT_ERR_INVALID;
    if (reads) *reads = c->scene.cache_reads + c->pt_cache_reads;
    if (writes) *writes = c->scene.cache_writes + c->pt_cache_writes;
    if (rejected) *rejected = c->scene.cache_rejected + c->pt_cache_rejected;
    return RT_OK;
}

rt_status rt_bvh_build_stats(const rt_ctx* c, double* build_ms, int32_t* gpu_builds) {
    if (!c) return RT_ERR_INVALID;
    if (build_ms) *build_ms = c->scene.bvh_build_ms + c->pt_build_ms;
    if (gpu_builds) *gpu_builds = c->scene.bvh_gpu_builds + c->pt_gpu_builds;
    return RT_OK;
}

int32_t rt_mesh_triangle_count(const rt_ctx* c, int32_t index) {
    if (!c || index < 0 || (size_t)index >= c->scene.objects.size()) return 0;
    const rt::HostObject& o = c->scene.objects[index];
    if (!o.defined || o.type != rt::kObjMesh) return 0;
    return (int32_t)(o.tri_vertices.size() / 9);
}

static rt_status rt_mesh_vertices_impl(const rt_ctx* c, int32_t index, float* out, int32_t max_tris) {
    int32_t n = rt_mesh_triangle_count(c, index);
    if (!c || !out || n == 0) return RT_ERR_INVALID;
    if (max_tris < n) return RT_ERR_INVALID;
    memcpy(out, c->scene.objects[index].tri_vertices.data(), (size_t)n * 9 * sizeof(float));
    return RT_OK;
}

// ---- pathTrace scene (main.cu:404-553) ----
static rt_status rt_load_object_impl(rt_ctx* c, const char* path, int32_t reflection_type) {
    if (!c) return RT_ERR_INVALID;
    if (!path || reflection_type < RT_PT_DIFFUSE || reflection_type > RT_PT_COAT)
        return fail(c, RT_ERR_INVALID, "load_object: bad arguments");
    std::string e = rt::append_ply(path, c->pt_raw);
    if (!e.empty()) return fail(c, RT_ERR_IO, e);
    c->pt_last_file = path;  // UpdateBoundingVolumeHierarchy(sceneFile) (main.cu:435)
    c->pt_materials.resize(c->pt_raw.indices.size() / 3, (uint32_t)reflection_type);
    c->pt_ready = false;
    return RT_OK;
}

static rt_status rt_process_triangle_data_impl(rt_ctx* c, const float offset[3], float max_coord,
                                   int32_t out_info[4]) {
    if (!c) return RT_ERR_INVALID;
    if (!finite3(offset) || !isfinite(max_coord) || max_coord <= 0.0f)
        return fail(c, RT_ERR_INVALID, "process_triangle_data: bad arguments");
    if (c->device >= 0) RT_HIP(c, hipSetDevice(c->device));
    free_pathtrace(c);
    c->pt_build_ms = 0.0;
    c->pt_gpu_builds = 0;
    c->pt_cache_reads = c->pt_cache_writes = c->pt_cache_rejected = 0;
    rt::PlyMesh m = c->pt_raw;
    float scale_max = 0.0f;
    std::vector<rt::KTri> kt;
    rt::CFBvh b;
    if (!m.indices.empty()) {
        rt::process_ply_vertices(m, rt::v3{offset[0], offset[1], offset[2]}, max_coord);
        rt::kuchkuda_triangles(m, c->pt_materials, kt);
        for (uint32_t i : m.indices) {
            const rt::v3 v = m.vertices[i];
            scale_max = std::max(scale_max, std::max(fabsf(v.x), std::max(fabsf(v.y), fabsf(v.z))));
        }
        const auto t0 = std::chrono::steady_clock::now();
        const int mode = c->scene.bvh_cache_mode;
        int got = 0;
        if ((mode & RT_BVH_CACHE_READ) && !c->pt_last_file.empty()) {
            std::string why;
            got = rt::read_bvh_cache(c->pt_last_file, m.vertices, m.indices, b, &why);
            if (got > 0) c->pt_cache_reads = 1;
            else if (got < 0) c->pt_cache_rejected = 1;
        }
        if (got <= 0) {
            if (c->scene.bvh_gpu && rt::gpu_build_cf_bvh(c->device, m.vertices, m.indices, b, 4, nullptr).empty())
                c->pt_gpu_builds = 1;
            else
                rt::build_cf_bvh(m.vertices, m.indices, b);
            if ((mode & RT_BVH_CACHE_WRITE) && !c->pt_last_file.empty() && rt::write_bvh_cache(c->pt_last_file, b))
                c->pt_cache_writes = 1;
        }
        c->pt_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        // the traversal keeps one pending subtree per level in LDS; the reference's builder
        // refuses trees as deep as its BVH_STACK_SIZE (BVH.cpp:469-496), and so does this one
        // (a `.bvh` cache file is untrusted input: its depth is checked here, not assumed)
        if (b.max_depth >= rt::kBvhStackDepth)
            return fail(c, RT_ERR_INVALID, "pathTrace BVH depth " + std::to_string(b.max_depth) +
                                               " exceeds the traversal stack (" + std::to_string(rt::kBvhStackDepth) + ")");
    }
    // the traversal's references pack a list position in 27 bits (kLeafRef | (count - 1) << 27 |
    // first) and its leaf queue entries pack (position << 6 | owner lane) in 32: positions and
    // triangles stay below 2^26, as build_mesh_pairs requires for the rayColor meshes
    if (kt.size() >= (size_t(1) << 26) || b.tri_index.size() >= (size_t(1) << 26) ||
        b.nodes.size() >= (size_t(1) << 30))
        return fail(c, RT_ERR_INVALID, "pathTrace scene too large for the BVH references (2^26 triangles)");
    std::vector<rt::CFNode> dev_nodes = b.nodes;  // + the traversal's child-pair records
    int pair_depth = 0;
    bool empty_leaf = false;
    const uint32_t root_ref = rt::cf_child_pairs(dev_nodes, &pair_depth, &empty_leaf);
    if (empty_leaf) return fail(c, RT_ERR_INVALID, "pathTrace BVH with an empty leaf");
    if (pair_depth > rt::kBvhStackDepth)
        return fail(c, RT_ERR_INVALID, "pathTrace BVH pair depth " + std::to_string(pair_depth) +
                                           " exceeds the traversal stack (" + std::to_string(rt::kBvhStackDepth) + ")");
    if (out_info) {
        out_info[0] = (int32_t)kt.size();
        out_info[1] = (int32_t)b.nodes.size();
        out_info[2] = (int32_t)b.tri_index.size();
        out_info[3] = b.max_depth;
    }
    if (c->device >= 0) {
        auto up = [&](auto** dst, const auto& vec) -> hipError_t {
            size_t bytes = vec.size() * sizeof(vec[0]);
            hipError_t err = hipMalloc((void**)dst, bytes ? bytes : 64);
            if (err != hipSuccess || !bytes) return err;
            return hipMemcpy(*dst, vec.data(), bytes, hipMemcpyHostToDevice);
        };
        // the kernel reads the triangles in the DFS list order of its leaf references (the reference's
        // cudaTriIdxList indirection resolved here): record i is triangle tri_index[i], whose index the
        // record keeps in pad[0] for avoidSelf; a leaf test is then one dependent load, not two
        std::vector<rt::KTri> lt(b.tri_index.size());
        for (size_t i = 0; i < lt.size(); ++i) {
            const uint32_t idx = (uint32_t)b.tri_index[i];
            if (idx >= kt.size()) return fail(c, RT_ERR_INVALID, "pathTrace triangle list index out of range");
            lt[i] = kt[idx];
            memcpy(&lt[i].pad[0], &idx, 4);
        }
        RT_HIP(c, up(&c->d_pt_tris, lt));
        RT_HIP(c, up(&c->d_pt_nodes, dev_nodes));
        RT_HIP(c, up(&c->d_pt_list, b.tri_index));
    }
    c->pt_tris = (int)kt.size();
    c->pt_scale = scale_max;
    c->pt_root_ref = root_ref;
    c->pt_pair_depth = pair_depth;
    c->pt_bvh = std::move(b);
    c->pt_ready = true;
    return RT_OK;
}

static rt_status rt_pathtrace_bvh_image_impl(const rt_ctx* c, uint8_t* out, int64_t capacity, int64_t* size) {
    if (!c || !size) return RT_ERR_INVALID;
    if (!c->pt_ready) return RT_ERR_STATE;
    std::vector<uint8_t> img = rt::bvh_image(c->pt_bvh);
    *size = (int64_t)img.size();
    if (out && capacity > 0) memcpy(out, img.data(), (size_t)std::min<int64_t>(capacity, *size));
    return RT_OK;
}

rt_status rt_camera(rt_ctx* c, const float eye[3], const float center[3], const float up[3],
                    float aspect, float fov, float aperture, float focus, float t0, float t1) {
    if (!c) return RT_ERR_INVALID;
    // Camera::initialize + updateViewMatrix (rt_camera.cpp), then the view getRay reads
    rt_camera_state st;
    if (rt_camera_initialize(&st, eye, center, up, aspect, fov, aperture, focus, t0, t1) != RT_OK)
        return fail(c, RT_ERR_INVALID, "camera: non-finite input");
    return rt_camera_apply(c, &st);
}

rt_status rt_get_camera(const rt_ctx* c, rt_camera_state* out) {
    if (!c || !out) return RT_ERR_INVALID;
    if (!c->scene.has_camera) return RT_ERR_STATE;
    *out = c->cam_state;
    return RT_OK;
}

static rt_status rt_commit_impl(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    std::string e = c->scene.flatten();
    if (!e.empty()) return fail(c, RT_ERR_INVALID, e);
    if (c->device < 0) {
        c->committed = true;
        return RT_OK;
    }
    RT_HIP(c, hipSetDevice(c->device));
    free_device(c);
    const auto& S = c->scene;
    // `pad` zeroed bytes after the table: the scan kernels prefetch the record after the last one
    auto up = [&](auto** dst, const auto& vec, size_t pad = 0) -> hipError_t {
        size_t bytes = vec.size() * sizeof(vec[0]) + pad;
        if (bytes == 0) bytes = 64;  // keep a valid pointer for empty tables
        hipError_t err = hipMalloc((void**)dst, bytes);
        if (err != hipSuccess) return err;
        if (pad) err = hipMemset((char*)*dst + vec.size() * sizeof(vec[0]), 0, pad);
        if (err == hipSuccess && !vec.empty())
            err = hipMemcpy(*dst, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice);
        return err;
    };
    RT_HIP(c, up(&c->d_objs, S.objs, sizeof(rt::ObjRec)));
    RT_HIP(c, up(&c->d_tris, S.tris));
    RT_HIP(c, up(&c->d_mats, S.mats));
    RT_HIP(c, up(&c->d_nodes, S.nodes));
    RT_HIP(c, up(&c->d_tri_orig, S.tri_orig));
    c->n_objs = S.n_scan;
    c->n_mats = (int)S.mats.size();
    c->has_media = false;
    c->full_scan = false;
    c->bvh_parts = 0;
    for (int32_t i = 0; i < S.n_scan && i < (int32_t)S.objs.size(); ++i) {
        const uint32_t t = S.objs[(size_t)i].type;
        if (t == rt::kObjMedium) c->has_media = true;
        if (t == rt::kObjSphere || t == rt::kObjMovingSphere) c->full_scan = true;
        if (t == rt::kObjMesh && S.objs[(size_t)i].u2 != rt::kNoBvh) c->bvh_parts |= 1;
        if (t == rt::kObjSphereGroup) c->bvh_parts |= 2;
        // the simple-scene kernel variant shades Lambertian (0) and emissive (3) materials only
        const uint32_t mi = S.objs[(size_t)i].material;
        const uint32_t mt = mi < S.mats.size() ? S.mats[mi].type : 0xFFFFFFFFu;
        if (mt != 0u && mt != 3u) c->full_scan = true;
    }
    c->committed = true;
    return RT_OK;
}

rt_status rt_scene_info(const rt_ctx* c, int32_t out[8]) {
    if (!c || !out) return RT_ERR_INVALID;
    if (!c->committed) return RT_ERR_STATE;
    for (int i = 0; i < 8; ++i) out[i] = 0;
    for (const rt::ObjRec& o : c->scene.objs) {
        if (rt::is_plane(o.type)) ++out[0];
        else if (o.type == rt::kObjSphere) ++out[1];
        else if (o.type == rt::kObjMovingSphere) ++out[2];
        else if (o.type == rt::kObjMesh) ++out[3];
    }
    out[4] = (int32_t)c->scene.tris.size();
    out[5] = (int32_t)c->scene.mats.size();
    out[6] = (int32_t)c->scene.nodes.size();
    out[7] = (int32_t)(c->scene.objs.size() - (size_t)c->scene.n_scan);
    return RT_OK;
}

rt_status rt_scene_bvh_depth(const rt_ctx* c, int32_t* out) {
    if (!c || !out) return RT_ERR_INVALID;
    if (!c->committed) return RT_ERR_STATE;
    *out = c->scene.nodes.empty() ? 0 : (int32_t)c->scene.bvh_max_depth;
    return RT_OK;
}

}  // extern "C"

rt_status rtc::validate(rt_ctx* c, const rt_render_params* p, rt::RenderLaunch& L) {
    if (!p) return fail(c, RT_ERR_INVALID, "null params");
    if (c->device < 0) return fail(c, RT_ERR_NODEV, "context has no device");
    if (p->flags & ~(uint32_t)(RT_RENDER_KEEP_COUNTERS | RT_RENDER_FRAMES_IN_FLIGHT))
        return fail(c, RT_ERR_INVALID, "unknown flags");
    if (p->integrator != RT_INTEGRATOR_RAYCOLOR && p->integrator != RT_INTEGRATOR_PATHTRACE)
        return fail(c, RT_ERR_INVALID, "unknown integrator");
    if (p->integrator == RT_INTEGRATOR_RAYCOLOR && !c->committed)
        return fail(c, RT_ERR_STATE, "scene not committed (call rt_commit)");
    if (p->integrator == RT_INTEGRATOR_PATHTRACE && !c->pt_ready)
        return fail(c, RT_ERR_STATE, "pathTrace scene not processed (call rt_process_triangle_data)");
    if (p->integrator == RT_INTEGRATOR_PATHTRACE && p->max_depth < 1)
        return fail(c, RT_ERR_INVALID, "pathTrace needs max_depth >= 1");
    if (!c->scene.has_camera) return fail(c, RT_ERR_STATE, "camera not set");
    if (p->width < 2 || p->height < 2) return fail(c, RT_ERR_INVALID, "width/height must be >= 2");
    if ((int64_t)p->width * p->height > (int64_t)1 << 31) return fail(c, RT_ERR_INVALID, "frame too large");
    if (p->spp < 1 || p->max_depth < 0) return fail(c, RT_ERR_INVALID, "spp must be >= 1, max_depth >= 0");
    // the linear-scan rayColor kernels (scenes without BVHs) keep a path's depth in 20 bits of an LDS
    // word (rt_kernel.hip, the camera slot's spare word), the mesh-BVH-only kernels in 30 bits of one
    // (W.grp_s); the other BVH kernels and pathTrace keep it in a register
    if (p->integrator == RT_INTEGRATOR_RAYCOLOR && c->scene.nodes.empty() && p->max_depth >= (1 << 20))
        return fail(c, RT_ERR_INVALID, "max_depth must be < 2^20 for a scene without BVHs");
    if (p->integrator == RT_INTEGRATOR_RAYCOLOR && p->max_depth >= (1 << 30))
        return fail(c, RT_ERR_INVALID, "max_depth must be < 2^30");
    if (p->row_block < 1 || p->row_world < 1 || p->row_rank < 0 || p->row_rank >= p->row_world)
        return fail(c, RT_ERR_INVALID, "bad row tiling");
    L.width = p->width;
    L.height = p->height;
    L.spp = p->spp;
    L.max_depth = p->max_depth;
    L.seed = p->seed;
    L.sample_offset = p->sample_offset;
    L.row_block = p->row_block;
    L.row_rank = p->row_rank;
    L.row_world = p->row_world;
    L.local_rows = rt::owned_rows(p->height, p->row_block, p->row_rank, p->row_world);
    if (p->col_begin < 0 || p->col_count < 0 || (int64_t)p->col_begin + p->col_count > p->width ||
        (p->col_count == 0 && p->col_begin != 0))
        return fail(c, RT_ERR_INVALID, "bad column window");
    L.col0 = p->col_begin;
    L.cols = p->col_count ? p->col_count : p->width;
    const int32_t s = p->lanes_per_pixel;
    if (p->schedule != RT_SCHEDULE_AUTO && p->schedule != RT_SCHEDULE_STATIC)
        return fail(c, RT_ERR_INVALID, "unknown schedule");
    const bool queue = p->schedule == RT_SCHEDULE_AUTO;
    // work-queue launches split a pixel into up to 128 sub-streams (items); the
    // static grid maps one pixel's sub-streams onto lanes of one wave (<= 64)
    if (s < 0 || s > (queue ? 128 : 64) || (s & (s - 1)) != 0)
        return fail(c, RT_ERR_INVALID, "lanes_per_pixel must be 0 (auto) or a power of two <= 128 (64 static)");
    const bool bvh = p->integrator == RT_INTEGRATOR_PATHTRACE || !c->scene.nodes.empty();
    rt::choose_layout(L, s, queue, bvh);
    // Work items of several sub-streams (the image is that of S regardless). Frames in flight: with
    // three launches overlapped, CornellBox1 ran faster with items of 8 samples (round 3, as S = 16:
    // N = 1 5.55 vs 5.68 ms/frame, N = 8 shard 0.816 vs 0.834) and slower alone (5.85 vs 5.83):
    // longer items cut the dequeues, and the next frames fill their longer tail (DESIGN §7,
    // profiles/r03/lanes/). Here the same item length comes from groups of S' = 16 sub-streams of
    // the auto S, so the flag no longer changes the image. BVH launches keep one sub-stream per item.
    L.grp_log2 = 0;
#ifndef RT_FIF_GROUPS
#define RT_FIF_GROUPS 1  // 0 (A/B only): frames in flight lower the auto S to 16 instead (round 3)
#endif
#ifndef RT_FIF_ITEMS
#define RT_FIF_ITEMS 16  // work items per pixel with frames in flight (A/B builds only)
#endif
    if (RT_FIF_GROUPS && queue && !bvh && (p->flags & RT_RENDER_FRAMES_IN_FLIGHT))
        while ((L.lanes_per_pixel >> L.grp_log2) > RT_FIF_ITEMS) ++L.grp_log2;
    if (!RT_FIF_GROUPS && s == 0 && queue && !bvh && (p->flags & RT_RENDER_FRAMES_IN_FLIGHT) && L.lanes_per_pixel > 16)
        rt::choose_layout(L, 16, queue, bvh);
    L.accumulate = 0;
    L.accum_scale = 0.0f;
    L.u8 = nullptr;
    L.queue = 0;
    L.tiles_x = (L.cols + 7) / 8;
    L.n_items = 0;
    L.n_qitems = 0;
    L.n_pix = 0;
    L.tiles_x_div = rt::make_udiv((uint32_t)L.tiles_x);
    L.row_block_div = rt::make_udiv((uint32_t)L.row_block);
    L.refill = 8;
    L.q_counter = c->d_queue;
    L.partial = nullptr;
    L.pt_has_mesh = c->pt_tris > 0 ? 1 : 0;
    // LDS traversal stacks hold one pending subtree per level below the root: the scene's
    // deepest BVH (rayColor meshes and sphere groups, or the pathTrace tree) sizes them
    const int depth = p->integrator == RT_INTEGRATOR_PATHTRACE ? std::max(c->pt_bvh.max_depth, c->pt_pair_depth)
                                                                : c->scene.bvh_max_depth;
    L.stack_depth = depth > 0 ? depth : 1;
    L.pt_scale = c->pt_scale;
    L.pt_root_ref = c->pt_root_ref;
    return RT_OK;
}

rt_status rtc::launch(rt_ctx* c, const rt_render_params* p, const rt::RenderLaunch& L0, float* out,
                        hipStream_t st) {
    RT_HIP(c, hipSetDevice(c->device));
    // The context's work queue, partial sums and counters are reused by every
    // launch: a launch on another stream waits for the previous one.
    if (c->launched) RT_HIP(c, hipStreamWaitEvent(st, c->ev1, 0));
    c->launched = true;
    rt::RenderLaunch L = L0;
    // Work-queue mode (rt_kernel.h): persistent grid + partial sums, bit-identical
    // to the static layout with the same lanes_per_pixel. RT_SCHEDULE_STATIC selects the
    // static grid.
    const bool pathtrace = p->integrator == RT_INTEGRATOR_PATHTRACE;
    const bool bvh = !c->scene.nodes.empty();
    if (p->schedule == RT_SCHEDULE_AUTO && L.local_rows > 0) {
        const uint64_t tiles = (uint64_t)L.tiles_x * (uint64_t)((L.local_rows + 7) / 8);
        const uint64_t items = tiles * 64u * (uint64_t)L.lanes_per_pixel;
        const size_t bytes = (size_t)items * 3 * sizeof(float);
        // partial sums: 12 B per item (up to a few GB of the 288 GB HBM); a frame whose
        // items do not fit the 31-bit item index (bit 31 is the kernels' camera-slot flag) or the
        // allocation runs on the static grid
        bool have = items < 0x80000000ull && bytes <= ((size_t)16 << 30);
        if (have && bytes > c->d_partial_bytes) {
            (void)hipFree(c->d_partial);
            c->d_partial = nullptr;
            c->d_partial_bytes = 0;
            if (hipMalloc(&c->d_partial, bytes) == hipSuccess) {
                c->d_partial_bytes = bytes;
            } else {
                (void)hipGetLastError();  // clear the sticky allocation error
                have = false;
            }
        }
        if (have) {
            const uint32_t qv = rt::select_variant(pathtrace, true, bvh, c->has_media, c->full_scan, c->bvh_parts);
            L.queue = rt::queue_blocks(c->n_cu, qv, L);
            L.n_items = (uint32_t)items;
            L.n_qitems = L.n_items >> L.grp_log2;
            L.n_pix = (uint32_t)(items >> L.sp_log2);
            // refill threshold (idle lanes a wave collects before one dequeue): 4 for long
            // items (>= 16 samples each: waiting for 8 idle lanes wastes lane time), else 8
            // (fewer dequeues). Same-box A/B, ms, 4 vs 8: bunny (16 samples/item) 544.9 / 548.2,
            // media (128) 1798 / 1846 (profiles/r01/ab_refill*.log); N = 8 shards (4 samples/item,
            // profiles/r02/refill_shards.log) CB1 1.205 / 1.207, spheres 10.86 / 10.81, Suzanne
            // 0.876 / 0.860 - round 1's extra "short shard -> 4" rule is not supported there.
            const int per_item = ((L.spp + L.lanes_per_pixel - 1) / L.lanes_per_pixel) << L.grp_log2;
            L.refill = per_item >= 16 ? 4 : 8;
            L.partial = c->d_partial;
            RT_HIP(c, hipMemsetAsync(c->d_queue, 0, rt::kQueueHeadWords * sizeof(uint32_t), st));
        }
    }
    const uint32_t variant = rt::select_variant(pathtrace, L.queue != 0, bvh, c->has_media, c->full_scan, c->bvh_parts);
    if (L.queue == 0 || pathtrace) {  // the static grid and pathTrace: one sub-stream per item
        L.grp_log2 = 0;
        L.n_qitems = L.n_items;
    }
    if (L.queue == 0 && L.lanes_per_pixel > 64)  // the static grid keeps a pixel's sub-streams in one wave
        return fail(c, RT_ERR_INVALID, "lanes_per_pixel > 64 needs the work queue, which this frame does not fit");
    const bool keep = (p->flags & RT_RENDER_KEEP_COUNTERS) != 0;
    if (!keep) {
        RT_HIP(c, hipMemsetAsync(c->d_counters, 0, rt::kNumCounters * sizeof(unsigned long long), st));
        c->n_kev = 0;
    }
    // this launch's (start, end of megakernel) event pair; kept for every launch of a
    // KEEP_COUNTERS chain (up to 65,536) so rt_sync_stats can sum them
    hipEvent_t k0 = nullptr, k1 = nullptr;
    if (c->n_kev < 65536u) {
        while (c->kev0.size() <= c->n_kev) {
            hipEvent_t a = nullptr, b = nullptr;
            RT_HIP(c, hipEventCreate(&a));
            if (hipEventCreate(&b) != hipSuccess) {
                (void)hipEventDestroy(a);
                return fail(c, RT_ERR_HIP, "hipEventCreate failed");
            }
            c->kev0.push_back(a);
            c->kev1.push_back(b);
        }
        k0 = c->kev0[c->n_kev];
        k1 = c->kev1[c->n_kev];
        ++c->n_kev;
    }
    // the kernels read the camera from device memory; refresh it when it changed (after
    // the previous launch, which may still be reading it, has finished)
    if (!c->cam_uploaded || memcmp(&c->cam_on_device, &c->scene.camera, sizeof(rt::CamRec)) != 0) {
        if (c->launched_before) RT_HIP(c, hipEventSynchronize(c->ev1));
        RT_HIP(c, hipMemcpy(c->d_cam, &c->scene.camera, sizeof(rt::CamRec), hipMemcpyHostToDevice));
        c->cam_on_device = c->scene.camera;
        c->cam_uploaded = true;
    }
    c->launched_before = true;
    RT_HIP(c, hipEventRecord(c->ev0, st));
    if (k0) RT_HIP(c, hipEventRecord(k0, st));
    if (p->integrator == RT_INTEGRATOR_PATHTRACE) {
        rt::PtSceneArgs pt{c->d_pt_tris, c->d_pt_nodes, c->d_pt_list};
        RT_HIP(c, rt::launch_pathtrace(pt, c->d_cam, L, out, c->d_counters, st, k1));
    } else {
        rt::SceneArgs sc{c->d_objs,   c->d_tris,  c->d_mats,  c->d_nodes,
                         c->d_tri_orig, c->n_objs, c->n_mats, !c->scene.nodes.empty()};
        sc.has_media = c->has_media;
        sc.full_scan = c->full_scan;
        sc.bvh_parts = c->bvh_parts;
        RT_HIP(c, rt::launch_render(variant, sc, c->d_cam, L, out, c->d_counters, st, k1));
    }
    RT_HIP(c, hipEventRecord(c->ev1, st));
    const uint64_t prev_samples = keep ? c->last.samples : 0;
    c->last = rt_render_stats{};
    c->last.samples = prev_samples + (uint64_t)L.local_rows * (uint64_t)L.cols * (uint64_t)L.spp;
    c->last.lanes_per_pixel = (uint32_t)L.lanes_per_pixel;
    c->last.refill = L.queue ? (uint32_t)L.refill : 0u;
    c->last.queue_blocks = (uint32_t)L.queue;
    c->last.variant = variant;
    c->last.substreams_per_item = L.queue ? 1u << L.grp_log2 : 1u;
    c->last.stack_depth = (pathtrace ? c->pt_tris > 0 : bvh) ? (uint32_t)L.stack_depth : 0u;
    c->stats_pending = true;
    return RT_OK;
}

extern "C" {

static rt_status rt_render_device_impl(rt_ctx* c, const rt_render_params* p, float* out, void* stream) {
    if (!c) return RT_ERR_INVALID;
    rt::RenderLaunch L;
    rt_status s = validate(c, p, L);
    if (s != RT_OK) return s;
    if (!out && L.local_rows > 0) return fail(c, RT_ERR_INVALID, "null output");
    return launch(c, p, L, out, (hipStream_t)stream);
}

static rt_status rt_accumulate_impl(rt_ctx* c, const rt_render_params* p, float* accum, uint32_t sample_count,
                        uint8_t* pixels, void* stream) {
    if (!c) return RT_ERR_INVALID;
    rt::RenderLaunch L;
    rt_status s = validate(c, p, L);
    if (s != RT_OK) return s;
    if (!accum && L.local_rows > 0) return fail(c, RT_ERR_INVALID, "null accumulation buffer");
    if (pixels && sample_count == 0) return fail(c, RT_ERR_INVALID, "sample_count must be >= 1");
    L.accumulate = 1;
    L.u8 = pixels;
    // Canvas::incrementSampleCount: scale = 1.0f / sampleCount (Canvas.h:166-169).
    L.accum_scale = sample_count ? 1.0f / (float)sample_count : 0.0f;
    return launch(c, p, L, accum, (hipStream_t)stream);
}

rt_status rt_sync_stats(rt_ctx* c, rt_render_stats* out) {
    if (!c) return RT_ERR_INVALID;
    if (c->stats_pending) {
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipEventSynchronize(c->ev1));
        unsigned long long h[rt::kNumCounters];
        RT_HIP(c, hipMemcpy(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost));
        float ms = 0.0f;
        double sum = 0.0;
        for (uint32_t k = 0; k < c->n_kev; ++k) {
            float e = 0.0f;
            RT_HIP(c, hipEventElapsedTime(&e, c->kev0[k], c->kev1[k]));
            sum += e;
            ms = e;
        }
        c->last.launches = c->n_kev;
        c->last.kernel_ms_sum = sum;
        c->last.segments = h[0];
        c->last.tri_tests = h[1];
        c->last.box_tests = h[2];
        c->last.node_visits = h[3];
        c->last.overflow = h[4] ? 1u : 0u;
        c->last.group_sphere_tests = h[5];
        c->last.group_moving_sphere_tests = h[6];
        c->last.kernel_ms = ms;
        for (int k = 0; k < 8; ++k) c->last.debug[k] = h[8 + k];
        c->stats_pending = false;
    }
    if (out) *out = c->last;
    return RT_OK;
}

static rt_status rt_render_impl(rt_ctx* c, const rt_render_params* p, float* out_host) {
    if (!c) return RT_ERR_INVALID;
    rt::RenderLaunch L;
    rt_status s = validate(c, p, L);
    if (s != RT_OK) return s;
    size_t bytes = (size_t)L.local_rows * L.cols * 3 * sizeof(float);
    if (!out_host && bytes) return fail(c, RT_ERR_INVALID, "null output");
    RT_HIP(c, hipSetDevice(c->device));
    if (bytes > c->d_out_bytes) {
        (void)hipFree(c->d_out);
        c->d_out = nullptr;
        c->d_out_bytes = 0;
        RT_HIP(c, hipMalloc(&c->d_out, bytes));
        c->d_out_bytes = bytes;
    }
    s = rt_render_device(c, p, c->d_out, nullptr);
    if (s != RT_OK) return s;
    RT_HIP(c, hipStreamSynchronize(nullptr));
    if (bytes) RT_HIP(c, hipMemcpy(out_host, c->d_out, bytes, hipMemcpyDeviceToHost));
    s = rt_sync_stats(c, nullptr);
    if (s != RT_OK) return s;
    if (c->last.overflow) return fail(c, RT_ERR_OVERFLOW, "BVH traversal stack overflow");
    return RT_OK;
}

static rt_status rt_render_u8_impl(rt_ctx* c, const rt_render_params* p, uint8_t* out_host) {
    if (!c) return RT_ERR_INVALID;
    rt::RenderLaunch L;
    rt_status s = validate(c, p, L);
    if (s != RT_OK) return s;
    const size_t n = (size_t)L.local_rows * L.cols * 3;
    if (!out_host && n) return fail(c, RT_ERR_INVALID, "null output");
    RT_HIP(c, hipSetDevice(c->device));
    if (n * sizeof(float) > c->d_out_bytes) {
        (void)hipFree(c->d_out);
        c->d_out = nullptr;
        c->d_out_bytes = 0;
        RT_HIP(c, hipMalloc(&c->d_out, n * sizeof(float)));
        c->d_out_bytes = n * sizeof(float);
    }
    if (n > c->d_u8_bytes) {
        (void)hipFree(c->d_u8);
        c->d_u8 = nullptr;
        c->d_u8_bytes = 0;
        RT_HIP(c, hipMalloc(&c->d_u8, n));
        c->d_u8_bytes = n;
    }
    L.u8 = c->d_u8;
    s = launch(c, p, L, c->d_out, nullptr);
    if (s != RT_OK) return s;
    RT_HIP(c, hipStreamSynchronize(nullptr));
    if (n) RT_HIP(c, hipMemcpy(out_host, c->d_u8, n, hipMemcpyDeviceToHost));
    s = rt_sync_stats(c, nullptr);
    if (s != RT_OK) return s;
    if (c->last.overflow) return fail(c, RT_ERR_OVERFLOW, "BVH traversal stack overflow");
    return RT_OK;
}

rt_status rt_gamma_u8(const float* rgb, int64_t n, uint8_t* out) {
    if (n < 0 || (n > 0 && (!rgb || !out))) return RT_ERR_INVALID;
    for (int64_t i = 0; i < n; ++i) {
        // Canvas::gamma (Canvas.h:198-200) with clamp = fmaxf(a, fminf(f, b)) (cutil_math.h:1100-1103).
        float v = fmaxf(0.0f, fminf(sqrtf(rgb[i]), 0.999f));
        out[i] = (uint8_t)(uint32_t)(255.99f * v);
    }
    return RT_OK;
}

}  // extern "C"

// ---- scene files (initialize(), main.cu:623-786, SCENE == 1) ----

namespace {

namespace Y = rt::yaml;

bool vec3(const Y::Node* n, float out[3]) {
    if (!n || n->kind != Y::Node::kSeq || n->seq.size() != 3) return false;
    for (int k = 0; k < 3; ++k) {
        double v;
        if (!Y::as_double(n->seq[k], v)) return false;
        out[k] = (float)v;
    }
    return true;
}

// Python-style int(x) of a YAML int or float scalar (the reference reads these
// fields with as<int>()).
bool int_of(const Y::Node* n, long& out) {
    if (!n) return false;
    if (Y::as_int(*n, out)) return true;
    double v;
    if (!Y::as_double(*n, v)) return false;
    out = (long)v;
    return true;
}

bool float_of(const Y::Node* n, float& out) {
    double v;
    if (!n || !Y::as_double(*n, v)) return false;
    out = (float)v;
    return true;
}

bool bool_of(const Y::Node* n, bool& out) {
    if (!n) return false;
    if (Y::as_bool(*n, out)) return true;
    double v;
    if (!Y::as_double(*n, v)) return false;
    out = v != 0.0;
    return true;
}

std::string where(const Y::Node* n, const std::string& what) {
    return "line " + std::to_string(n ? n->line : 0) + ": " + what;
}

}  // namespace

extern "C" {

static rt_status rt_load_yaml_scene_impl(rt_ctx* c, const char* path, const char* models_dir, int32_t width,
                             int32_t height) {
    if (!c) return RT_ERR_INVALID;
    if (!path || !models_dir) return fail(c, RT_ERR_INVALID, "null path");
    if (width < 1 || height < 1) return fail(c, RT_ERR_INVALID, "width and height must be >= 1");
    Y::Node root;
    std::string e = Y::parse_file(path, root);
    if (!e.empty()) return fail(c, e.rfind("cannot open", 0) == 0 ? RT_ERR_IO : RT_ERR_INVALID, e);
    const Y::Node* cam = root.get("camera");
    const Y::Node* objects = root.get("objects");
    if (!cam || cam->kind != Y::Node::kMap) return fail(c, RT_ERR_INVALID, "scene has no camera map");

    // camera (main.cu:632-638): focus = |center - eye| in float, aspect = float(w) / h
    float eye[3], center[3], up[3], fov, aperture;
    if (!vec3(cam->get("eye"), eye) || !vec3(cam->get("center"), center) || !vec3(cam->get("up"), up) ||
        !float_of(cam->get("fov"), fov) || !float_of(cam->get("aperture"), aperture))
        return fail(c, RT_ERR_INVALID, where(cam, "camera needs eye, center, up, fov and aperture"));
    const float dx = center[0] - eye[0], dy = center[1] - eye[1], dz = center[2] - eye[2];
    const float focus = sqrtf(dx * dx + dy * dy + dz * dz);
    const float aspect = (float)width / (float)height;
    if (!objects || objects->kind != Y::Node::kSeq) return fail(c, RT_ERR_INVALID, "scene has no objects list");
    rt_status s = rt_camera(c, eye, center, up, aspect, fov, aperture, focus, 0.0f, 1.0f);
    if (s != RT_OK) return s;

    // materials 0-8 exist before any object (main.cu:643-651)
    const float red[3] = {1, 0, 0}, green[3] = {0, 1, 0}, blue[3] = {0, 0, 1}, white[3] = {1, 1, 1};
    const float wl[3] = {0.75f, 0.25f, 0.25f}, wr[3] = {0.25f, 0.25f, 0.75f};
    if ((s = rt_material_lambertian(c, 0, red, 1.0f)) || (s = rt_material_lambertian(c, 1, green, 1.0f)) ||
        (s = rt_material_lambertian(c, 2, blue, 1.0f)) || (s = rt_material_lambertian(c, 3, white, 1.0f)) ||
        (s = rt_material_lambertian(c, 4, wl, 1.0f)) || (s = rt_material_lambertian(c, 5, wr, 1.0f)) ||
        (s = rt_material_metal(c, 6, white, 0.0f)) || (s = rt_material_dielectric(c, 7, 1.5f)) ||
        (s = rt_material_emission(c, 8, white, 5.0f)))
        return s;

    for (size_t i = 0; i < objects->seq.size(); ++i) {
        const Y::Node& entry = objects->seq[i];
        if (entry.kind != Y::Node::kMap || entry.map.empty() || entry.map[0].second.kind != Y::Node::kMap ||
            entry.map[0].second.map.empty())
            return fail(c, RT_ERR_INVALID, where(&entry, "object entry must be 'kind: {type: ...}'"));
        const Y::Node& obj = entry.map[0].second;  // the first key names the object (main.cu:706)
        const Y::Node* mat = obj.get("material");
        long mid, mtype, ptype;
        if (!mat || !int_of(obj.get("materialId"), mid) || !int_of(mat->get("type"), mtype))
            return fail(c, RT_ERR_INVALID, where(&obj, "object needs materialId and material.type"));
        if (mid < 0 || mid > INT32_MAX) return fail(c, RT_ERR_INVALID, where(&obj, "materialId out of range"));
        if (!rt_material_defined(c, (int32_t)mid)) {  // the nullptr guards (main.cu:714-744)
            float albedo[3], p;
            if (mtype == 0 || mtype == 1 || mtype == 3 || mtype == 4) {
                if (!vec3(mat->get("albedo"), albedo))
                    return fail(c, RT_ERR_INVALID, where(mat, "material needs albedo"));
            }
            if (mtype == 0) {
                s = rt_material_lambertian(c, (int32_t)mid, albedo, 1.0f);
            } else if (mtype == 2) {
                if (!float_of(mat->get("indexOfRefraction"), p))
                    return fail(c, RT_ERR_INVALID, where(mat, "dielectric needs indexOfRefraction"));
                s = rt_material_dielectric(c, (int32_t)mid, p);
            } else if (mtype == 1) {
                if (!float_of(mat->get("fuzz"), p)) return fail(c, RT_ERR_INVALID, where(mat, "metal needs fuzz"));
                s = rt_material_metal(c, (int32_t)mid, albedo, p);
            } else if (mtype == 3) {
                if (!float_of(mat->get("intensity"), p))
                    return fail(c, RT_ERR_INVALID, where(mat, "emission needs intensity"));
                s = rt_material_emission(c, (int32_t)mid, albedo, p);
            } else if (mtype == 4) {  // build extension: isotropic phase function
                s = rt_material_isotropic(c, (int32_t)mid, albedo);
            }
            if (s != RT_OK) return s;
        }
        // the primitive type is the object map's first value (main.cu:749)
        if (!int_of(&obj.map[0].second, ptype))
            return fail(c, RT_ERR_INVALID, where(&obj, "the first field must be the primitive type"));
        const int32_t idx = (int32_t)i, m = (int32_t)mid;
        float a[3], b[3], d[3], f;
        if (ptype == 0) {
            if (!vec3(obj.get("center"), a) || !float_of(obj.get("radius"), f))
                return fail(c, RT_ERR_INVALID, where(&obj, "sphere needs center and radius"));
            s = rt_sphere(c, idx, a, f, m, 1);
        } else if (ptype == 1) {
            long orient;
            bool two;
            if (!vec3(obj.get("position"), a) || !vec3(obj.get("normal"), b) || !vec3(obj.get("extend"), d) ||
                !int_of(obj.get("orientation"), orient) || !bool_of(obj.get("twoSide"), two))
                return fail(c, RT_ERR_INVALID,
                            where(&obj, "plane needs position, normal, extend, orientation and twoSide"));
            s = rt_plane(c, idx, a, b, d, m, (int32_t)orient, two ? 1 : 0);
        } else if (ptype == 2) {
            const Y::Node* model = obj.get("model");
            if (!model || model->kind != Y::Node::kScalar)
                return fail(c, RT_ERR_INVALID, where(&obj, "mesh needs a model path"));
            const std::string file = std::string(models_dir) + "/" + model->scalar;
            std::string lower = file;
            for (char& ch : lower) ch = (char)tolower((unsigned char)ch);
            // meshes always take materials[3] (main.cu:781)
            if (lower.size() >= 4 && lower.compare(lower.size() - 4, 4, ".ply") == 0) {
                // build extension: PLY meshes with loadObject/processTriangleData placement
                float off[3] = {0, 0, 0}, max_coord = 1.0f;
                if (obj.get("offset") && !vec3(obj.get("offset"), off))
                    return fail(c, RT_ERR_INVALID, where(&obj, "bad offset"));
                if (obj.get("maxCoord") && !float_of(obj.get("maxCoord"), max_coord))
                    return fail(c, RT_ERR_INVALID, where(&obj, "bad maxCoord"));
                s = rt_mesh_ply(c, idx, file.c_str(), off, max_coord, 3);
            } else {
                if (!vec3(obj.get("scale"), a) || !vec3(obj.get("rotate"), b) || !vec3(obj.get("offset"), d))
                    return fail(c, RT_ERR_INVALID, where(&obj, "OBJ mesh needs scale, rotate and offset"));
                s = rt_mesh_obj(c, idx, file.c_str(), a, b, d, 3);
            }
        } else if (ptype == 3) {  // build extension: cube (createCube, kernels.h:139-154)
            if (!vec3(obj.get("center"), a) || !vec3(obj.get("extend"), d))
                return fail(c, RT_ERR_INVALID, where(&obj, "cube needs center and extend"));
            s = rt_cube(c, idx, a, d, m);
        } else if (ptype == 4) {  // build extension: constant medium in a cube
            if (!vec3(obj.get("center"), a) || !vec3(obj.get("extend"), d) || !float_of(obj.get("density"), f))
                return fail(c, RT_ERR_INVALID, where(&obj, "medium needs center, extend and density"));
            s = rt_constant_medium(c, idx, a, d, f, m);
        } else {
            return fail(c, RT_ERR_INVALID, where(&obj, "unknown primitive type " + std::to_string(ptype)));
        }
        if (s != RT_OK) return s;
    }
    return RT_OK;
}

rt_status rt_scene_digest(const rt_ctx* c, uint64_t* out) {
    if (!c || !out) return RT_ERR_INVALID;
    if (!c->committed) return RT_ERR_STATE;
    uint64_t h = 1469598103934665603ull;  // FNV-1a 64
    auto mix = [&h](const void* p, size_t n) {
        const unsigned char* b = (const unsigned char*)p;
        for (size_t k = 0; k < n; ++k) {
            h ^= b[k];
            h *= 1099511628211ull;
        }
    };
    const auto& S = c->scene;
    const uint64_t sizes[5] = {S.objs.size(), S.tris.size(), S.mats.size(), S.nodes.size(), S.tri_orig.size()};
    mix(sizes, sizeof(sizes));
    mix(&S.n_scan, sizeof(S.n_scan));
    if (!S.objs.empty()) mix(S.objs.data(), S.objs.size() * sizeof(S.objs[0]));
    if (!S.tris.empty()) mix(S.tris.data(), S.tris.size() * sizeof(S.tris[0]));
    for (const rt::MatRec& m : S.mats) {  // padding words excluded
        mix(&m.type, 4);
        mix(&m.a0, 16);
    }
    if (!S.nodes.empty()) mix(S.nodes.data(), S.nodes.size() * sizeof(S.nodes[0]));
    if (!S.tri_orig.empty()) mix(S.tri_orig.data(), S.tri_orig.size() * sizeof(S.tri_orig[0]));
    const rt::CamRec& k = S.camera;
    const float cam[21] = {k.origin.x, k.origin.y, k.origin.z, k.lower_left.x, k.lower_left.y, k.lower_left.z,
                           k.horizontal.x, k.horizontal.y, k.horizontal.z, k.vertical.x, k.vertical.y, k.vertical.z,
                           k.right.x, k.right.y, k.right.z, k.true_up.x, k.true_up.y, k.true_up.z,
                           k.lens_radius, k.time0, k.time1};
    mix(cam, sizeof(cam));
    *out = h;
    return RT_OK;
}

}  // extern "C"

// Exceptions must not cross the C ABI: host-side allocations (scene tables, BVH
// builds, file loaders) report RT_ERR_OOM instead of terminating the caller.
extern "C" {

rt_status rt_mesh(rt_ctx* c, int32_t index, const float* v, int32_t n_tris, int32_t material) {
    try {
        return rt_mesh_impl(c, index, v, n_tris, material);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_mesh_obj(rt_ctx* c, int32_t index, const char* path, const float scale[3],
                      const float rotate[3], const float offset[3], int32_t material) {
    try {
        return rt_mesh_obj_impl(c, index, path, scale, rotate, offset, material);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_mesh_ply(rt_ctx* c, int32_t index, const char* path, const float offset[3],
                      float max_coord, int32_t material) {
    try {
        return rt_mesh_ply_impl(c, index, path, offset, max_coord, material);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_ply_bvh_image(const char* path, const float offset[3], float max_coord,
                           uint8_t* out, int64_t capacity, int64_t* size) {
    try {
        return rt_ply_bvh_image_impl(path, offset, max_coord, out, capacity, size);
    } catch (const std::bad_alloc&) {
        return RT_ERR_OOM;
    } catch (const std::exception&) {
        return RT_ERR_INVALID;
    }
}

rt_status rt_ply_bvh_image_gpu(int32_t device, const char* path, const float offset[3], float max_coord,
                               uint8_t* out, int64_t capacity, int64_t* size, double* build_ms) {
    try {
        return rt_ply_bvh_image_gpu_impl(device, path, offset, max_coord, out, capacity, size, build_ms);
    } catch (const std::bad_alloc&) {
        return RT_ERR_OOM;
    } catch (const std::exception&) {
        return RT_ERR_INVALID;
    }
}

rt_status rt_load_object(rt_ctx* c, const char* path, int32_t reflection_type) {
    try {
        return rt_load_object_impl(c, path, reflection_type);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_process_triangle_data(rt_ctx* c, const float offset[3], float max_coord,
                                   int32_t out_info[4]) {
    try {
        return rt_process_triangle_data_impl(c, offset, max_coord, out_info);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_pathtrace_bvh_image(const rt_ctx* c, uint8_t* out, int64_t capacity, int64_t* size) {
    try {
        return rt_pathtrace_bvh_image_impl(c, out, capacity, size);
    } catch (const std::bad_alloc&) {
        return RT_ERR_OOM;
    } catch (const std::exception&) {
        return RT_ERR_INVALID;
    }
}

rt_status rt_commit(rt_ctx* c) {
    try {
        return rt_commit_impl(c);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_load_yaml_scene(rt_ctx* c, const char* path, const char* models_dir, int32_t width,
                             int32_t height) {
    try {
        return rt_load_yaml_scene_impl(c, path, models_dir, width, height);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_render(rt_ctx* c, const rt_render_params* p, float* out_host) {
    try {
        return rt_render_impl(c, p, out_host);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_render_device(rt_ctx* c, const rt_render_params* p, float* out, void* stream) {
    try {
        return rt_render_device_impl(c, p, out, stream);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_render_u8(rt_ctx* c, const rt_render_params* p, uint8_t* out_host) {
    try {
        return rt_render_u8_impl(c, p, out_host);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_accumulate(rt_ctx* c, const rt_render_params* p, float* accum, uint32_t sample_count,
                        uint8_t* pixels, void* stream) {
    try {
        return rt_accumulate_impl(c, p, accum, sample_count, pixels, stream);
    } catch (const std::bad_alloc&) {
        return fail(c, RT_ERR_OOM, "out of host memory");
    } catch (const std::exception& ex) {
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());
    }
}

rt_status rt_mesh_vertices(const rt_ctx* c, int32_t index, float* out, int32_t max_tris) {
    try {
        return rt_mesh_vertices_impl(c, index, out, max_tris);
    } catch (const std::bad_alloc&) {
        return RT_ERR_OOM;
    } catch (const std::exception&) {
        return RT_ERR_INVALID;
    }
}
}  // extern "C"

// ---- the reference's Canvas buffers on the device (Canvas.h:20-200) ----
struct rt_canvas {
    rt_ctx* ctx;
    int32_t device;  // rt_canvas_destroy needs only this (safe after the context is gone)
    int32_t width, height;
    float* accum;     // accumulationBuffer (float RGB)
    uint8_t* pixels;  // pixelBuffer (Canvas::gamma RGB8)
};

// The canvas entry points keep C++ exceptions (std::bad_alloc from an error message, say)
// inside the ABI, as the *_impl wrappers of the other entry points do.
template <typename F>
static rt_status canvas_guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return RT_ERR_OOM;
    } catch (...) {
        return RT_ERR_INVALID;
    }
}

extern "C" {

rt_status rt_canvas_create(rt_ctx* c, int32_t width, int32_t height, rt_canvas** out) {
    return canvas_guarded([&]() -> rt_status {
        if (!c || !out) return RT_ERR_INVALID;
        *out = nullptr;
        if (c->device < 0) return fail(c, RT_ERR_NODEV, "canvas: context has no device");
        if (width < 2 || height < 2 || (int64_t)width * height > ((int64_t)1 << 31))
            return fail(c, RT_ERR_INVALID, "canvas: bad size");
        RT_HIP(c, hipSetDevice(c->device));
        const size_t n = (size_t)width * (size_t)height * 3;
        rt_canvas* k = new (std::nothrow) rt_canvas{c, c->device, width, height, nullptr, nullptr};
        if (!k) return fail(c, RT_ERR_OOM, "out of host memory");
        if (hipMalloc((void**)&k->accum, n * sizeof(float)) != hipSuccess ||
            hipMalloc((void**)&k->pixels, n) != hipSuccess || hipMemset(k->accum, 0, n * sizeof(float)) != hipSuccess ||
            hipMemset(k->pixels, 0, n) != hipSuccess) {
            (void)hipGetLastError();
            rt_canvas_destroy(k);
            return fail(c, RT_ERR_OOM, "canvas: device allocation failed");
        }
        *out = k;
        return RT_OK;
    });
}

void rt_canvas_destroy(rt_canvas* k) {
    if (!k) return;
    (void)hipSetDevice(k->device);
    (void)hipFree(k->accum);
    (void)hipFree(k->pixels);
    delete k;
}

rt_status rt_canvas_clear_accumulation(rt_canvas* k) {
    return canvas_guarded([&]() -> rt_status {
        if (!k) return RT_ERR_INVALID;
        rt_ctx* c = k->ctx;
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipMemset(k->accum, 0, (size_t)k->width * k->height * 3 * sizeof(float)));
        return RT_OK;
    });
}

rt_status rt_canvas_accumulate(rt_canvas* k, const rt_render_params* p, uint32_t sample_count) {
    return canvas_guarded([&]() -> rt_status {
        if (!k || !p) return RT_ERR_INVALID;
        rt_ctx* c = k->ctx;
        if (p->width != k->width || p->height != k->height || p->row_world != 1 || p->col_count != 0)
            return fail(c, RT_ERR_INVALID, "canvas_accumulate: params must cover the canvas's full frame");
        if (sample_count == 0) return fail(c, RT_ERR_INVALID, "canvas_accumulate: sample_count must be >= 1");
        rt_status s = rt_accumulate(c, p, k->accum, sample_count, k->pixels, nullptr);
        if (s != RT_OK) return s;
        RT_HIP(c, hipStreamSynchronize(nullptr));
        s = rt_sync_stats(c, nullptr);
        if (s != RT_OK) return s;
        if (c->last.overflow) return fail(c, RT_ERR_OVERFLOW, "BVH traversal stack overflow");
        return RT_OK;
    });
}

rt_status rt_canvas_read_pixels(const rt_canvas* k, uint8_t* out) {
    return canvas_guarded([&]() -> rt_status {
        if (!k || !out) return RT_ERR_INVALID;
        rt_ctx* c = k->ctx;
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipMemcpy(out, k->pixels, (size_t)k->width * k->height * 3, hipMemcpyDeviceToHost));
        return RT_OK;
    });
}

rt_status rt_canvas_write_accumulation(rt_canvas* k, const float* in) {
    return canvas_guarded([&]() -> rt_status {
        if (!k || !in) return RT_ERR_INVALID;
        rt_ctx* c = k->ctx;
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipMemcpy(k->accum, in, (size_t)k->width * k->height * 3 * sizeof(float), hipMemcpyHostToDevice));
        return RT_OK;
    });
}

rt_status rt_canvas_read_accumulation(const rt_canvas* k, float* out) {
    return canvas_guarded([&]() -> rt_status {
        if (!k || !out) return RT_ERR_INVALID;
        rt_ctx* c = k->ctx;
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipMemcpy(out, k->accum, (size_t)k->width * k->height * 3 * sizeof(float), hipMemcpyDeviceToHost));
        return RT_OK;
    });
}

}  // extern "C"
