// rt_kernel.h — launch interface between the C ABI (rt_capi.cpp) and the HIP
// megakernel (rt_kernel.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/rtmi.h"
#include "rt_scene.h"

namespace rt {

// Unsigned division by a launch-invariant divisor without a divide: the multiply-high
// with add-back of Granlund & Montgomery (the sequence compilers emit for constant
// divisors), exact for every 32-bit dividend. The kernel's generic divisions by
// launch parameters otherwise keep per-lane reciprocal constants alive in VGPRs for
// the whole persistent loop (and the traversal kernel spilled them to scratch).
struct UDiv {
    uint32_t d, m, s1, s2;
};
inline UDiv make_udiv(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && ((uint64_t)1 << l) < d) ++l;  // ceil(log2 d)
    UDiv r;
    r.d = d;
    r.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    r.s1 = l < 1 ? l : 1;
    r.s2 = l > 1 ? l - 1 : 0;
    return r;
}
__host__ __device__ __forceinline__ uint32_t udiv(uint32_t x, const UDiv& D) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t t = __umulhi(x, D.m);
#else
    const uint32_t t = (uint32_t)(((uint64_t)x * D.m) >> 32);
#endif
    return (t + ((x - t) >> D.s1)) >> D.s2;
}

// Per-launch parameters (rt_render_params after validation).
struct RenderLaunch {
    int32_t width, height, spp, max_depth;
    uint32_t seed, sample_offset;
    int32_t row_block, row_rank, row_world;
    int32_t local_rows;  // rows owned by this shard (output has local_rows * cols pixels)
    int32_t col0, cols;  // column window [col0, col0 + cols) of each owned row (full: 0, width)
    int32_t lanes_per_pixel;  // S: power of two in [1, 128]
    int32_t sp_log2;          // log2 S
    int32_t tile_w, tile_h;   // per-wave pixel tile, tile_w * tile_h = 64 / S
    int32_t pt_has_mesh;      // pathTrace: a triangle BVH is present
    int32_t stack_depth;      // BVH traversal stack entries per lane = the scene's BVH depth (>= 1): an
                              // ordered traversal holds at most one pending subtree per level below the
                              // root, so the LDS stacks are sized per scene (dynamic LDS)
    float pt_scale;           // pathTrace: max |coordinate| of the triangles
    uint32_t pt_root_ref;     // pathTrace: the root's child-pair reference (rt_bvh.h cf_child_pairs)
    // Pixel output (Canvas.h:58-98): accumulate = 0 writes the mean color/spp to
    // `out` (and gamma(mean) to u8 when set: writePixel); accumulate = 1 adds the
    // sample sum to `out` (accumulatePixel) and, when u8 is set, writes
    // gamma(acc * accum_scale) with accum_scale = 1.0f / sampleCount.
    int32_t accumulate;
    float accum_scale;
    uint8_t* u8;
    // Work-queue mode (queue = 1): a persistent grid whose lanes take items
    // (pixel, sub-stream c) from a global counter; each item's sample sum goes
    // to partial[item] and a combine pass sums the S partials of a pixel in
    // the fixed order of the static layout. Items are numbered in 8x8 pixel
    // tiles (tiles_x per tile row), S per pixel.
    int32_t queue;
    int32_t tiles_x;
    uint32_t n_items;
    // A work item is a group of 1 << grp_log2 sub-streams of one pixel, c, c + S', c + 2S', ...
    // with S' = S >> grp_log2: the lane runs them one after the other and stores each one's
    // partial sum. The image depends on S only; the group size is the schedule's item length.
    int32_t grp_log2;
    uint32_t n_qitems;        // n_items >> grp_log2: what the queue hands out
    uint32_t n_pix;           // n_items / S: the pixels of the launch (one partial-sum plane)
    UDiv tiles_x_div;         // tile -> (tile row, tile column)
    UDiv row_block_div;       // local row -> local row block
    int32_t refill;  // idle lanes that trigger a wave's refill (set per launch, see rt_capi.cpp)
    uint32_t* q_counter;
    float* partial;
};

// Lane-layout choice: S = lanes_per_pixel (0 = auto). Adjacent lanes that
// share a pixel trace nearly identical camera rays, so larger S means more
// coherent waves (less divergence in BVH traversal and mesh compaction).
// Work-queue launches (the default) take the largest power of two
// S <= min(32, spp) with pixels * S <= 2^25 items (the partial-sum buffer stays
// <= 400 MB); launches that traverse BVHs (`bvh`: rayColor meshes / sphere groups,
// or pathTrace) the largest S <= min(128, spp) with pixels * S <= 2^27 (1.6 GB): a
// whole wave on one pixel keeps the traversal coherent (same box, frame overlap on:
// random spheres S = 32 / 64 / 128 -> 76.7 / 73.8 / 71.8 ms, bunny 517.0 / 518.6 / 516.5,
// while CornellBox1 without BVHs is best at 32: 7.39 vs 7.61 at 64;
// profiles/r02/lanes_sweep.txt). Static launches take the largest S <= min(32, spp)
// with pixels * S <= 2^24 lanes.
// `pixels` is the FULL frame (width * height), not this shard's rows: every rank
// of a row-sharded frame then folds a pixel's samples with the same S, so the
// assembled frame is bit-identical for any world size (and N > 1 shards do the
// same per-item work as N = 1).
// Measured on one MI355X, ms/frame (static S=1 -> static auto -> queue auto):
// CornellBox1 11.9 -> 10.7 -> 8.9, random spheres 245 -> 164 -> 113,
// materialball 34.5 -> 14.5 -> 11.7, bunny 999 -> 950 -> 765, media 1982 -> 2015 -> 1883.
inline void choose_layout(RenderLaunch& L, int32_t requested, bool queue, bool bvh) {
    int32_t s = requested;
    if (s <= 0) {
        s = 1;
        const int64_t px = (int64_t)L.height * L.width;
        const bool wide = queue && bvh;
        const int64_t cap = wide ? (int64_t(1) << 27) : queue ? (int64_t(1) << 25) : (int64_t(1) << 24);
        const int32_t smax = wide ? 128 : 32;
        while (2 * s <= smax && 2 * s <= L.spp && px * 2 * s <= cap) s *= 2;
    }
    L.lanes_per_pixel = s;
    L.sp_log2 = 0;
    while ((1 << L.sp_log2) < s) ++L.sp_log2;
    const int32_t p = s <= 64 ? 64 / s : 1;  // S > 64 (work queue only): no static tile
    L.tile_w = p >= 8 ? 8 : p;
    L.tile_h = p / L.tile_w;
}

// Work-queue heads: up to 64 shards, one 128 B line (32 words) each.
constexpr int kQueueHeadWords = 64 * 32;

// counters[0] = segments, [1] = triangle tests, [2] = mesh-box tests,
// [3] = BVH node visits, [4] = traversal overflow flag, [5] / [6] = spheres /
// moving spheres tested in object-BVH leaves.
// [8..15] = diagnostic section timers (RT_STAMPS builds only).
constexpr int kNumCounters = 16;

struct KTri;
struct CFNode;
// Device tables of the pathTrace integrator (prepareCUDAscene, main.cu:404-553).
struct PtSceneArgs {
    const KTri* ktris;        // in tri_list order (record i = triangle tri_list[i], its index in pad[0])
    const CFNode* nodes;      // the reference's CacheFriendlyBVHNode array, exact bounds
    const int32_t* tri_list;  // leaf triangle lists in DFS order
};

// `main_done` (may be null) is recorded on `stream` right after the megakernel,
// before the work queue's combine pass.
// `cam`: the camera record in device memory (rt_capi.cpp keeps it current).
hipError_t launch_pathtrace(const PtSceneArgs& sc, const CamRec* cam, const RenderLaunch& L,
                            float* out, unsigned long long* counters, hipStream_t stream,
                            hipEvent_t main_done);

// Workgroups of the persistent work-queue grid (n_cu x resident 4-wave blocks per CU: the
// variant's occupancy, capped by the LDS its tables and L's traversal stacks take).
int queue_blocks(int n_cu, uint32_t variant, const RenderLaunch& L);
// The kernel instantiation of a launch (rtmi.h RT_VARIANT_*) from the integrator, the
// schedule and the committed scene's content; the occupancy it is compiled for (waves per
// SIMD); its symbol as rocprofv3 prints it (nullptr for an unknown id).
uint32_t select_variant(bool pathtrace, bool queue, bool bvh, bool media, bool full, int bvh_parts);
int variant_waves(uint32_t variant);
const char* variant_name(uint32_t variant);

// `variant` = select_variant(false, L.queue != 0, ...) of the committed scene.
hipError_t launch_render(uint32_t variant, const SceneArgs& sc, const CamRec* cam, const RenderLaunch& L,
                         float* out, unsigned long long* counters, hipStream_t stream, hipEvent_t main_done);

// Frame assembly on the gather root (rt_rows.hip): staging = world tiles of
// max_rows x width x 3 floats, rank-major -> frame (height x width x 3).
hipError_t launch_assemble_rows(const float* staging, float* frame, int32_t width, int32_t height,
                                int32_t row_block, int32_t world, int32_t max_rows, hipStream_t stream);

// Build options compiled into the kernels (rtmi.h RT_BUILD_*).
uint32_t kernel_build_flags();

// Rows of [0, height) owned by (row_block, row_rank, row_world).
inline int32_t owned_rows(int32_t height, int32_t block, int32_t rank, int32_t world) {
    int32_t n = 0;
    for (int32_t b = rank; b * block < height; b += world) {
        int32_t r0 = b * block, r1 = r0 + block < height ? r0 + block : height;
        n += r1 - r0;
    }
    return n;
}

// The largest owned_rows over the ranks (rank 0 owns the most: blocks are dealt from it).
inline int32_t max_tile_rows(int32_t height, int32_t block, int32_t world) {
    int32_t m = 0;
    for (int32_t k = 0; k < world && k * block < height; ++k) {
        const int32_t r = owned_rows(height, block, k, world);
        m = r > m ? r : m;
    }
    return m;
}

}  // namespace rt
