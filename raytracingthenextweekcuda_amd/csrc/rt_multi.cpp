// rt_multi.cpp — multi-GPU frames behind the C ABI (SURVEY §8(b) "Threading" and
// §8(e)): pixel-row tiles, one RCCL ncclGather over xGMI, and a device-side row
// de-interleave on the root. Replaces pathTracing's single renderKernel launch
// (main.cu:875-898); the reference has no multi-GPU path.
//
// Two host shapes share the exchange:
//  * rt_render_multi[_device]: one host process drives every device; communicators
//    come from ncclCommInitAll and stay cached on the first context;
//  * rt_comm_* + rt_gather_rows: one process per GPU (the scaling path), each rank
//    rendering its tile with rt_render_device and joining one ncclGather.
#include <rccl/rccl.h>
#include <string.h>

#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_ctx.h"

namespace rtc {

struct MultiGroup {
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
};

void destroy_multi(rt_ctx* c) {
    if (!c || !c->group) return;
    for (ncclComm_t m : c->group->comms) (void)ncclCommDestroy(m);
    delete c->group;
    c->group = nullptr;
}

namespace {

rt_status nccl_fail(rt_ctx* c, ncclResult_t r, const char* what) {
    return fail(c, RT_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

#define RT_NCCL(c, call)                                          \
    do {                                                          \
        ncclResult_t _r = (call);                                 \
        if (_r != ncclSuccess) return nccl_fail(c, _r, #call);    \
    } while (0)

rt_status check_frame(rt_ctx* c, const rt_render_params* p, int32_t world) {
    if (!p) return fail(c, RT_ERR_INVALID, "null params");
    if (p->width < 2 || p->height < 2 || p->row_block < 1 || world < 1)
        return fail(c, RT_ERR_INVALID, "bad frame or row tiling");
    if (p->col_begin != 0 || (p->col_count != 0 && p->col_count != p->width))
        return fail(c, RT_ERR_INVALID, "multi-GPU frames cover the whole width (no column window)");
    if ((int64_t)p->width * p->height > (int64_t)1 << 31) return fail(c, RT_ERR_INVALID, "frame too large");
    return RT_OK;
}

// Communicators over `devs` (one rank per device), cached on the set's first context.
rt_status group_for(rt_ctx* c0, const std::vector<int>& devs, MultiGroup** out) {
    if (c0->group && c0->group->devices == devs) {
        *out = c0->group;
        return RT_OK;
    }
    destroy_multi(c0);
    MultiGroup* g = new MultiGroup();
    g->devices = devs;
    g->comms.resize(devs.size());
    const ncclResult_t r = ncclCommInitAll(g->comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) {
        delete g;
        return nccl_fail(c0, r, "ncclCommInitAll");
    }
    c0->group = g;
    *out = g;
    return RT_OK;
}

rt_status render_multi_device(rt_ctx* const* ctxs, int32_t n, const rt_render_params* p, float* frame,
                              hipStream_t st0) {
    if (!ctxs || n < 1 || !p) return RT_ERR_INVALID;
    for (int32_t k = 0; k < n; ++k)
        if (!ctxs[k]) return RT_ERR_INVALID;
    rt_ctx* c0 = ctxs[0];
    rt_status s = check_frame(c0, p, n);
    if (s != RT_OK) return s;
    if (!frame) return fail(c0, RT_ERR_INVALID, "null frame");
    const int32_t W = p->width, H = p->height, rb = p->row_block;
    const int32_t max_rows = rt::max_tile_rows(H, rb, n);
    const size_t tile_floats = (size_t)max_rows * (size_t)W * 3;

    // 1. every context renders its rank's tiles into a max_rows tile (the gather's
    //    equal count); all launches are issued before anything is awaited
    std::vector<int> devs((size_t)n);
    bool distinct = true;
    for (int32_t k = 0; k < n; ++k) {
        rt_ctx* c = ctxs[k];
        devs[k] = c->device;
        for (int32_t j = 0; j < k; ++j) distinct = distinct && devs[j] != devs[k];
        rt_render_params pk = *p;
        pk.row_rank = k;
        pk.row_world = n;
        rt::RenderLaunch L;
        s = validate(c, &pk, L);
        if (s != RT_OK) return s;
        RT_HIP(c, hipSetDevice(c->device));
        s = ensure_device(c, (void**)&c->d_out, &c->d_out_bytes, tile_floats * sizeof(float));
        if (s != RT_OK) return s;
        s = launch(c, &pk, L, c->d_out, k == 0 ? st0 : nullptr);
        if (s != RT_OK) return s;
    }

    // 2. the tiles meet on the root: one ncclGather (distinct devices) or device copies
    RT_HIP(c0, hipSetDevice(c0->device));
    s = ensure_device(c0, (void**)&c0->d_stage, &c0->d_stage_bytes, (size_t)n * tile_floats * sizeof(float));
    if (s != RT_OK) return s;
    uint32_t mode;
    if (distinct) {
        MultiGroup* g = nullptr;
        s = group_for(c0, devs, &g);
        if (s != RT_OK) return s;
        RT_NCCL(c0, ncclGroupStart());
        for (int32_t k = 0; k < n; ++k) {
            const ncclResult_t r = ncclGather(ctxs[k]->d_out, k == 0 ? c0->d_stage : nullptr, tile_floats,
                                              ncclFloat32, 0, g->comms[k], k == 0 ? st0 : nullptr);
            if (r != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_fail(c0, r, "ncclGather");
            }
        }
        RT_NCCL(c0, ncclGroupEnd());
        mode = RT_GATHER_RCCL;
    } else {
        for (int32_t k = 0; k < n; ++k) {
            rt_ctx* c = ctxs[k];
            if (k > 0) RT_HIP(c0, hipStreamWaitEvent(st0, c->ev1, 0));  // rank k's render is done
            RT_HIP(c0, hipMemcpyPeerAsync(c0->d_stage + (size_t)k * tile_floats, c0->device, c->d_out, c->device,
                                          tile_floats * sizeof(float), st0));
        }
        mode = RT_GATHER_COPY;
    }
    // 3. de-interleave on the root device
    RT_HIP(c0, hipSetDevice(c0->device));
    RT_HIP(c0, rt::launch_assemble_rows(c0->d_stage, frame, W, H, rb, n, max_rows, st0));
    c0->last.gather = mode;
    return RT_OK;
}

}  // namespace
}  // namespace rtc

using rtc::fail;

extern "C" {

int32_t rt_owned_rows(int32_t height, int32_t row_block, int32_t rank, int32_t world) {
    if (height < 0 || row_block < 1 || world < 1 || rank < 0 || rank >= world) return -1;
    return rt::owned_rows(height, row_block, rank, world);
}

int32_t rt_max_tile_rows(int32_t height, int32_t row_block, int32_t world) {
    if (height < 0 || row_block < 1 || world < 1) return -1;
    return rt::max_tile_rows(height, row_block, world);
}

static rt_status rt_render_multi_device_impl(rt_ctx* const* ctxs, int32_t n, const rt_render_params* p,
                                             float* frame, void* stream) {
    return rtc::render_multi_device(ctxs, n, p, frame, (hipStream_t)stream);
}

static rt_status rt_render_multi_impl(rt_ctx* const* ctxs, int32_t n, const rt_render_params* p, float* out_host) {
    if (!ctxs || n < 1 || !p || !out_host || !ctxs[0]) return RT_ERR_INVALID;
    rt_ctx* c0 = ctxs[0];
    const size_t bytes = (size_t)p->width * (size_t)(p->height > 0 ? p->height : 0) * 3 * sizeof(float);
    if (p->width >= 2 && p->height >= 2) {
        RT_HIP(c0, hipSetDevice(c0->device));
        rt_status s = rtc::ensure_device(c0, (void**)&c0->d_frame, &c0->d_frame_bytes, bytes);
        if (s != RT_OK) return s;
    }
    rt_status s = rtc::render_multi_device(ctxs, n, p, c0->d_frame, nullptr);
    if (s != RT_OK) return s;
    const uint32_t mode = c0->last.gather;
    RT_HIP(c0, hipSetDevice(c0->device));
    RT_HIP(c0, hipMemcpyAsync(out_host, c0->d_frame, bytes, hipMemcpyDeviceToHost, nullptr));
    RT_HIP(c0, hipStreamSynchronize(nullptr));
    for (int32_t k = 0; k < n; ++k) {
        rt_ctx* c = ctxs[k];
        RT_HIP(c, hipSetDevice(c->device));
        RT_HIP(c, hipStreamSynchronize(nullptr));
        s = rt_sync_stats(c, nullptr);
        if (s != RT_OK) return s;
        if (c->last.overflow) return fail(c, RT_ERR_OVERFLOW, "BVH traversal stack overflow");
    }
    c0->last.gather = mode;
    return RT_OK;
}

static rt_status rt_comm_unique_id_impl(uint8_t id[128]) {
    if (!id) return RT_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RT_ERR_COMM;
    memcpy(id, &u, sizeof(u));
    return RT_OK;
}

static rt_status rt_comm_init_impl(rt_ctx* c, const uint8_t id[128], int32_t world, int32_t rank, void** comm) {
    if (!c || !id || !comm) return RT_ERR_INVALID;
    if (c->device < 0) return fail(c, RT_ERR_NODEV, "context has no device");
    if (world < 1 || rank < 0 || rank >= world) return fail(c, RT_ERR_INVALID, "bad rank / world");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    RT_HIP(c, hipSetDevice(c->device));
    ncclComm_t m = nullptr;
    const ncclResult_t r = ncclCommInitRank(&m, world, u, rank);
    if (r != ncclSuccess) return fail(c, RT_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    *comm = m;
    return RT_OK;
}

static rt_status rt_gather_rows_impl(rt_ctx* c, void* comm, const rt_render_params* p, int32_t rank, int32_t world,
                                     const float* tile, float* frame, void* stream) {
    if (!c || !comm) return RT_ERR_INVALID;
    rt_status s = rtc::check_frame(c, p, world);
    if (s != RT_OK) return s;
    if (rank < 0 || rank >= world) return fail(c, RT_ERR_INVALID, "bad rank");
    if (c->device < 0) return fail(c, RT_ERR_NODEV, "context has no device");
    const int32_t max_rows = rt::max_tile_rows(p->height, p->row_block, world);
    const size_t tile_floats = (size_t)max_rows * (size_t)p->width * 3;
    if (!tile && tile_floats) return fail(c, RT_ERR_INVALID, "null tile");
    if (rank == 0 && !frame) return fail(c, RT_ERR_INVALID, "null frame on the root");
    RT_HIP(c, hipSetDevice(c->device));
    if (rank == 0) {
        s = rtc::ensure_device(c, (void**)&c->d_stage, &c->d_stage_bytes, (size_t)world * tile_floats * sizeof(float));
        if (s != RT_OK) return s;
    }
    const ncclResult_t r = ncclGather(tile, rank == 0 ? c->d_stage : nullptr, tile_floats, ncclFloat32, 0,
                                      (ncclComm_t)comm, (hipStream_t)stream);
    if (r != ncclSuccess) return fail(c, RT_ERR_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
    if (rank == 0)
        RT_HIP(c, rt::launch_assemble_rows(c->d_stage, frame, p->width, p->height, p->row_block, world, max_rows,
                                           (hipStream_t)stream));
    return RT_OK;
}

static rt_status rt_assemble_rows_impl(rt_ctx* c, const rt_render_params* p, int32_t world, const float* staging,
                                       float* frame, void* stream) {
    if (!c) return RT_ERR_INVALID;
    rt_status s = rtc::check_frame(c, p, world);
    if (s != RT_OK) return s;
    if (c->device < 0) return fail(c, RT_ERR_NODEV, "context has no device");
    if (!staging || !frame) return fail(c, RT_ERR_INVALID, "null buffer");
    RT_HIP(c, hipSetDevice(c->device));
    RT_HIP(c, rt::launch_assemble_rows(staging, frame, p->width, p->height, p->row_block, world,
                                       rt::max_tile_rows(p->height, p->row_block, world), (hipStream_t)stream));
    return RT_OK;
}

// Exceptions must not cross the C ABI.
#define RT_GUARD(c, expr)                                                              \
    try {                                                                              \
        return expr;                                                                   \
    } catch (const std::bad_alloc&) {                                                  \
        return fail(c, RT_ERR_OOM, "out of host memory");                             \
    } catch (const std::exception& ex) {                                               \
        return fail(c, RT_ERR_INVALID, std::string("internal error: ") + ex.what());  \
    }

rt_status rt_render_multi(rt_ctx* const* ctxs, int32_t n, const rt_render_params* p, float* out_host) {
    rt_ctx* c0 = (ctxs && n > 0) ? ctxs[0] : nullptr;
    RT_GUARD(c0, rt_render_multi_impl(ctxs, n, p, out_host))
}

rt_status rt_render_multi_device(rt_ctx* const* ctxs, int32_t n, const rt_render_params* p, float* frame,
                                 void* stream) {
    rt_ctx* c0 = (ctxs && n > 0) ? ctxs[0] : nullptr;
    RT_GUARD(c0, rt_render_multi_device_impl(ctxs, n, p, frame, stream))
}

rt_status rt_comm_unique_id(uint8_t id[128]) { RT_GUARD(nullptr, rt_comm_unique_id_impl(id)) }

rt_status rt_comm_init(rt_ctx* c, const uint8_t id[128], int32_t world, int32_t rank, void** comm) {
    RT_GUARD(c, rt_comm_init_impl(c, id, world, rank, comm))
}

rt_status rt_comm_destroy(void* comm) {
    if (!comm) return RT_ERR_INVALID;
    return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? RT_OK : RT_ERR_COMM;
}

rt_status rt_gather_rows(rt_ctx* c, void* comm, const rt_render_params* p, int32_t rank, int32_t world,
                         const float* tile, float* frame, void* stream) {
    RT_GUARD(c, rt_gather_rows_impl(c, comm, p, rank, world, tile, frame, stream))
}

rt_status rt_assemble_rows(rt_ctx* c, const rt_render_params* p, int32_t world, const float* staging, float* frame,
                           void* stream) {
    RT_GUARD(c, rt_assemble_rows_impl(c, p, world, staging, frame, stream))
}

uint32_t rt_build_flags(void) { return rt::kernel_build_flags(); }
const char* rt_kernel_variant_name(uint32_t variant) { return rt::variant_name(variant); }

}  // extern "C"
