// rt_ctx.h — the context object behind include/rtmi.h's opaque rt_ctx, shared by
// the C ABI's translation units (rt_capi.cpp: scene, render; rt_multi.cpp: RCCL
// multi-GPU frames). Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_bvh.h"
#include "rt_kernel.h"
#include "rt_scene.h"

namespace rtc {
struct MultiGroup;
}

struct rt_ctx {
    int device = -1;
    std::string err;
    rt::HostScene scene;
    bool committed = false;

    // device tables
    rt::ObjRec* d_objs = nullptr;
    rt::TriRec* d_tris = nullptr;
    rt::MatRec* d_mats = nullptr;
    rt::BvhNode* d_nodes = nullptr;
    uint32_t* d_tri_orig = nullptr;
    int n_objs = 0;
    bool has_media = false;   // the committed scan list holds a participating medium (kernel variant)
    int bvh_parts = 3;        // 1: mesh BVHs, 2: sphere groups in the committed scan list (kernel variant)
    bool full_scan = true;  // the committed scan list needs the general kernel (spheres, metal, glass, isotropic)
    int n_mats = 0;
    unsigned long long* d_counters = nullptr;
    rt::CamRec* d_cam = nullptr;  // device copy of scene.camera read by the kernels
    rt_camera_state cam_state{};  // the Camera object scene.camera was taken from (rt_get_camera)
    rt::CamRec cam_on_device{};   // what d_cam holds (valid when cam_uploaded)
    bool cam_uploaded = false;
    bool launched_before = false;  // ev1 has been recorded by a launch
    float* d_out = nullptr;   // staging buffer for rt_render (host output)
    size_t d_out_bytes = 0;
    uint8_t* d_u8 = nullptr;  // staging buffer for rt_render_u8
    size_t d_u8_bytes = 0;
    int n_cu = 0;                 // compute units (persistent work-queue grid)
    uint32_t* d_queue = nullptr;  // work-queue head
    float* d_partial = nullptr;   // work-queue partial sums
    size_t d_partial_bytes = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool have_events = false;
    // one (start, end-of-megakernel) event pair per launch since the counters were last
    // reset: rt_sync_stats sums them (kernel_ms_sum) without a host sync per launch
    std::vector<hipEvent_t> kev0, kev1;
    uint32_t n_kev = 0;
    rt_render_stats last{};
    bool stats_pending = false;
    bool launched = false;

    // pathTrace scene (prepareCUDAscene): raw loaded PLY data + device tables
    rt::PlyMesh pt_raw;
    std::vector<uint32_t> pt_materials;  // ReflectionType per triangle
    bool pt_ready = false;
    int pt_tris = 0;
    float pt_scale = 0.0f;  // max |coordinate| of the processed triangles
    rt::CFBvh pt_bvh;  // host copy (the `.bvh` cache image source)
    rt::KTri* d_pt_tris = nullptr;
    rt::CFNode* d_pt_nodes = nullptr;  // the tree's nodes, then its child-pair records (cf_child_pairs)
    uint32_t pt_root_ref = 0;          // the root's child-pair reference
    int pt_pair_depth = 0;             // pair records on the longest root-to-leaf path
    int32_t* d_pt_list = nullptr;
    double pt_build_ms = 0.0;
    int pt_gpu_builds = 0;
    int pt_cache_reads = 0, pt_cache_writes = 0, pt_cache_rejected = 0;
    std::string pt_last_file;  // the last loadObject path: its `.bvh` is the scene's cache (main.cu:435)

    // multi-GPU (rt_multi.cpp): RCCL communicators of an rt_render_multi device set
    // (owned by the first context of the set), and the root's gather staging buffer
    rtc::MultiGroup* group = nullptr;
    float* d_stage = nullptr;
    size_t d_stage_bytes = 0;
    float* d_frame = nullptr;  // rt_render_multi's device frame (host output path)
    size_t d_frame_bytes = 0;
};

namespace rtc {

// Records `msg` as the context's last error and returns `s`.
rt_status fail(rt_ctx* c, rt_status s, const std::string& msg);
rt_status hip_fail(rt_ctx* c, hipError_t e, const char* what);

// rt_render_params -> launch description (checks the scene state and arguments).
rt_status validate(rt_ctx* c, const rt_render_params* p, rt::RenderLaunch& L);
// Enqueues one render of the validated launch on `st` into the device buffer `out`.
rt_status launch(rt_ctx* c, const rt_render_params* p, const rt::RenderLaunch& L, float* out, hipStream_t st);
// (Re)allocates a device buffer to at least `bytes` (contents not kept).
rt_status ensure_device(rt_ctx* c, void** buf, size_t* have, size_t bytes);
// Releases the multi-GPU state a context owns (rt_destroy).
void destroy_multi(rt_ctx* c);

}  // namespace rtc

#define RT_HIP(c, call)                                             \
    do {                                                            \
        hipError_t _e = (call);                                     \
        if (_e != hipSuccess) return rtc::hip_fail(c, _e, #call);   \
    } while (0)
