/*
 * rtmi.h — C ABI of the MI355X-native path tracer (librtmi.so).
 *
 * This is the drop-in boundary for the reference's per-pixel path-tracing
 * hot path (erosnick/RayTracingTheNextWeekCUDA). Every entry point below names
 * the reference interface it replaces (paths relative to
 * RayTracingTheNextWeekCUDA/). Plain C types only: no HIP, no torch types.
 *
 * Ownership: the library owns every device buffer; the caller owns its host
 * input arrays (copied during the call) and its output buffers.
 * Errors: every export returns rt_status (0 = RT_OK). The message for the last
 * failure on a context is rt_last_error(ctx). The library never calls exit()
 * (replaces gpuErrorCheck -> cudaDeviceReset -> exit, Utils.h:125-133).
 * Threading: one rt_ctx per HIP device; calls on one ctx are not thread-safe.
 * Launches on one ctx run in issue order even across streams (each waits for
 * the previous one: they share the context's work queue and counters).
 */
#ifndef RTMI_H_
#define RTMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTMI_ABI_VERSION 10

typedef int32_t rt_status;
enum {
    RT_OK = 0,
    RT_ERR_INVALID = 1,  /* bad argument / index / shape */
    RT_ERR_HIP = 2,      /* HIP runtime failure */
    RT_ERR_IO = 3,       /* file could not be read / parsed */
    RT_ERR_STATE = 4,    /* call out of order (e.g. render before commit) */
    RT_ERR_OOM = 5,      /* allocation failure */
    RT_ERR_NODEV = 6,    /* no GPU / context created without a device */
    RT_ERR_OVERFLOW = 7, /* BVH traversal stack overflow flagged by the kernel */
    RT_ERR_COMM = 8      /* RCCL (communicator / collective) failure */
};

/* Material kinds (Material.h:8-13 MaterialType) + the isotropic phase function
 * of participating media (build extension, see rt_constant_medium). */
enum { RT_LAMBERTIAN = 0, RT_METAL = 1, RT_DIELECTRIC = 2, RT_EMISSION = 3, RT_ISOTROPIC = 4 };
/* Plane orientation (Plane.h:5-9 PlaneOrientation). */
enum { RT_PLANE_XY = 0, RT_PLANE_YZ = 1, RT_PLANE_XZ = 2 };
/* Integrator run by renderKernel: rayColor (main.cu:60-113, the Hitable scene)
 * or pathTrace (CUDAPathTracer.cu:358-622, the committed call at main.cu:187). */
enum { RT_INTEGRATOR_RAYCOLOR = 0, RT_INTEGRATOR_PATHTRACE = 1 };
/* pathTrace surface kinds (CUDAPathTracer.h ReflectionType). */
enum { RT_PT_DIFFUSE = 0, RT_PT_METAL = 1, RT_PT_SPECULAR = 2, RT_PT_REFRACTION = 3, RT_PT_COAT = 4 };

typedef struct rt_ctx rt_ctx;

/* Render parameters. Replaces the compile-time knobs of renderKernel
 * (main.cu:160-206: samplesPerPixel 165-169, BOUNCES 23, curand_init seed 1984
 * at 127) and adds row tiling for multi-GPU sharding.
 * Rows are numbered with y = 0 at the BOTTOM (reference convention,
 * main.cu:183). Row tiling: global row y belongs to this call iff
 * (y / row_block) % row_world == row_rank. Output holds only the owned rows,
 * in increasing y, each width*3 floats (col_count*3 with a column window).
 * row_world = 1 renders the full frame. */
typedef struct rt_render_params {
    int32_t width;
    int32_t height;
    int32_t spp;            /* samples per pixel (reference: 32 offline, 1 realtime) */
    int32_t max_depth;      /* reference BOUNCES (main.cu:23); rayColor: < 2^30, < 2^20 for a scene without BVHs */
    uint32_t seed;          /* reference 1984 (main.cu:127) */
    uint32_t sample_offset; /* first global sample index (progressive accumulation) */
    int32_t row_block;      /* rows per tile block (>= 1) */
    int32_t row_rank;       /* this shard's rank */
    int32_t row_world;      /* number of shards (>= 1) */
    int32_t lanes_per_pixel;/* sub-streams that split one pixel's samples: 0 = auto,
                               or a power of two <= 128 (<= 64 on the static grid).
                               Partial sums are combined in a fixed order, so
                               results are deterministic for a given value; 1 (and
                               spp) = the reference's sequential sum. */
    int32_t integrator;     /* RT_INTEGRATOR_RAYCOLOR (0) or RT_INTEGRATOR_PATHTRACE (1).
                               pathTrace bounces max_depth times (reference: 5). */
    uint32_t flags;         /* RT_RENDER_KEEP_COUNTERS: add this launch's counters to the
                               previous ones instead of resetting them (one rt_sync_stats
                               after many launches, no per-launch host sync).
                               RT_RENDER_FRAMES_IN_FLIGHT: the caller keeps three or more
                               launches in flight on other contexts/streams (frame overlap);
                               a linear-scan rayColor work-queue launch then hands out work
                               items of several sub-streams (at most 16 items per pixel:
                               longer items, whose longer tail the next frames fill). The
                               sub-streams, and so the image, are those of lanes_per_pixel:
                               the flag never changes a pixel. */
    /* Column window of every owned row: columns [col_begin, col_begin + col_count);
     * col_count = 0 = the whole width. Output rows are col_count wide. The pixels are
     * those of the full frame (camera and RNG keyed by the frame position). */
    int32_t col_begin;
    int32_t col_count;
    /* Launch schedule: RT_SCHEDULE_AUTO (0) = the persistent work queue, or the static grid
     * when the frame's partial sums do not fit (2^31 items or more - bit 31 of an item index
     * is the kernels' camera-slot flag - or more than 16 GB);
     * RT_SCHEDULE_STATIC (1) = the static grid (one lane per (pixel, sub-stream), the
     * reference's launch shape). Both compute the same partial sums: the image is
     * bit-identical. rt_render_stats.variant reports the kernel that ran. */
    int32_t schedule;
} rt_render_params;
enum { RT_RENDER_KEEP_COUNTERS = 1, RT_RENDER_FRAMES_IN_FLIGHT = 2 };
enum { RT_SCHEDULE_AUTO = 0, RT_SCHEDULE_STATIC = 1 };

/* The megakernel instantiation a launch ran (rt_render_stats.variant). renderKernel
 * (main.cu:160-206) is one kernel with virtual calls; this library compiles one
 * instantiation per scene content (BVH traversal parts, media, spheres / non-Lambertian
 * materials) and schedule, each with its own register budget. rt_kernel_variant_name
 * gives the template tuple as rocprofv3 prints the symbol. */
enum {
    RT_VARIANT_NONE = 0,
    RT_VARIANT_SCAN_QUEUE = 1,             /* render_kernel<false, true, false, true, 3>: linear scan */
    RT_VARIANT_SCAN_MEDIA_QUEUE = 2,       /* render_kernel<false, true, true, true, 3>: + media */
    RT_VARIANT_SCAN_SIMPLE_QUEUE = 3,      /* render_kernel<false, true, false, false, 3>: planes/meshes,
                                              Lambertian + emission only (CornellBox1) */
    RT_VARIANT_BVH_QUEUE = 4,              /* render_kernel<true, true, false, true, 3>: mesh BVHs + sphere groups */
    RT_VARIANT_BVH_MESH_QUEUE = 5,         /* render_kernel<true, true, false, true, 1>: mesh BVHs */
    RT_VARIANT_BVH_MESH_SIMPLE_QUEUE = 6,  /* render_kernel<true, true, false, false, 1>: mesh BVHs, simple scene */
    RT_VARIANT_BVH_GROUP_QUEUE = 7,        /* render_kernel<true, true, false, true, 2>: sphere groups */
    RT_VARIANT_SCAN_STATIC = 8,            /* render_kernel<false, false, false, true, 3> */
    RT_VARIANT_SCAN_MEDIA_STATIC = 9,      /* render_kernel<false, false, true, true, 3> */
    RT_VARIANT_SCAN_SIMPLE_STATIC = 10,    /* render_kernel<false, false, false, false, 3> */
    RT_VARIANT_BVH_STATIC = 11,            /* render_kernel<true, false, false, true, 3> */
    RT_VARIANT_PATHTRACE_QUEUE = 12,       /* pathtrace_kernel<true> */
    RT_VARIANT_PATHTRACE_STATIC = 13,      /* pathtrace_kernel<false> */
    RT_VARIANT_COUNT = 14
};

typedef struct rt_render_stats {
    uint64_t segments;      /* closest-hit queries traced (camera ray = 1, +1 per scatter) */
    uint64_t samples;       /* camera samples = owned pixels * spp (summed over kept launches) */
    uint64_t node_visits;   /* BVH node visits (0 for linear-scan scenes) */
    uint64_t tri_tests;     /* triangle records tested */
    uint64_t box_tests;     /* mesh bounding boxes tested */
    double kernel_ms;       /* duration of the last launch's render kernel alone (hipEvents around the
                               megakernel; the work queue's combine pass is not included) */
    uint32_t overflow;      /* 1 if any lane overflowed the traversal stack */
    uint32_t lanes_per_pixel; /* lane layout used by the last render */
    uint64_t group_sphere_tests;        /* spheres tested in object-BVH leaves */
    uint64_t group_moving_sphere_tests; /* moving spheres tested in object-BVH leaves */
    uint64_t debug[8];      /* diagnostic section timers (instrumented builds only; 0 otherwise) */
    uint32_t refill;        /* work-queue refill threshold of the last launch (idle lanes per dequeue); 0 = static grid */
    uint32_t queue_blocks;  /* persistent work-queue workgroups of the last launch; 0 = static grid */
    uint32_t gather;        /* rt_render_multi*: RT_GATHER_RCCL or RT_GATHER_COPY (first context only) */
    uint32_t launches;      /* launches summed in these counters (RT_RENDER_KEEP_COUNTERS chains; else 1) */
    double kernel_ms_sum;   /* render-kernel time summed over those launches (one event pair each) */
    uint32_t variant;       /* RT_VARIANT_* of the last launch */
    uint32_t substreams_per_item; /* sub-streams a work item runs in sequence (work queue; 1 on the static
                                     grid): the schedule's item length, which does not change the image */
    uint32_t stack_depth;         /* BVH traversal stack entries per lane of the launch (the scene's deepest
                                     path; 0 for a launch without BVH traversal) */
} rt_render_stats;

#define RT_GATHER_RCCL 1 /* one ncclGather over the contexts' devices */
#define RT_GATHER_COPY 2 /* device-to-device copies (contexts share a device; RCCL needs distinct ones) */

/* ---- context (replaces initialize()/cleanup(), main.cu:555-936) ---- */
int32_t rt_abi_version(void);
/* Build options of the loaded library. 0 = the shipped parity build. Non-zero bits:
 * RT_BUILD_ABLATION: an RT_ABL_* ablation is compiled in (results DIFFER from the
 * reference restatement: never for parity or bench numbers); RT_BUILD_STAMPS: the
 * instrumented timer build; RT_BUILD_AB: an A/B variant of the schedule (results
 * identical, performance not the shipped one). bench.py and smoke() refuse
 * ABLATION and STAMPS builds. */
#define RT_BUILD_ABLATION 1u
#define RT_BUILD_STAMPS 2u
#define RT_BUILD_AB 4u
uint32_t rt_build_flags(void);
/* The symbol of RT_VARIANT_* `variant` as rocprofv3 prints it, e.g.
 * "render_kernel<false, true, false, false, 3>"; NULL for an unknown id. */
const char* rt_kernel_variant_name(uint32_t variant);
/* 16 hex digits: sha256 of the library's native sources (the .hip, .cpp and .h files of csrc, its Makefile,
 * this header) and EXTRA build flags, computed at build time by source_digest.py. The Python
 * binding refuses an in-tree library whose digest differs from its source tree's (a stale
 * binary), and bench.py stamps it on every line and profile. */
const char* rt_kernel_source_sha(void);
/* device >= 0: HIP ordinal. device = -1: scene-building only (no GPU calls). */
rt_status rt_create(int32_t device, rt_ctx** out);
void rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
/* Drops every material, object and the camera (scene reset). */
rt_status rt_clear_scene(rt_ctx* ctx);

/* ---- materials (kernels.h:50-84 create*Material) ---- */
rt_status rt_material_lambertian(rt_ctx* ctx, int32_t index, const float albedo[3], float absorb);
rt_status rt_material_metal(rt_ctx* ctx, int32_t index, const float albedo[3], float fuzz);
rt_status rt_material_dielectric(rt_ctx* ctx, int32_t index, float index_of_refraction);
rt_status rt_material_emission(rt_ctx* ctx, int32_t index, const float albedo[3], float intensity);
/* Isotropic phase function (build extension for BASELINE config 5; the reference
 * has no media): scatter = Ray(p, randomInUnitSphere(), time), attenuation =
 * albedo (Ray Tracing: The Next Week's `isotropic`). */
rt_status rt_material_isotropic(rt_ctx* ctx, int32_t index, const float albedo[3]);
/* 1 if material slot `index` has been created (the `materials[id] == nullptr`
 * guards of main.cu:714,723,733,743), else 0. */
int32_t rt_material_defined(const rt_ctx* ctx, int32_t index);

/* ---- hitables (kernels.h:99-154 create*; object slot = closest-hit scan
 *      order of hit(), main.cu:43-57) ---- */
rt_status rt_sphere(rt_ctx* ctx, int32_t index, const float center[3], float radius,
                    int32_t material, int32_t shading);
rt_status rt_moving_sphere(rt_ctx* ctx, int32_t index, const float center0[3],
                           const float center1[3], float time0, float time1, float radius,
                           int32_t material);
rt_status rt_plane(rt_ctx* ctx, int32_t index, const float position[3], const float normal[3],
                   const float extend[3], int32_t material, int32_t orientation,
                   int32_t two_side);
rt_status rt_cube(rt_ctx* ctx, int32_t index, const float center[3], const float extend[3],
                  int32_t material);
/* Constant-density medium bounded by an axis-aligned cube (build extension for
 * BASELINE config 5; the reference has no media). Boundary = the six two-sided
 * faces of rt_cube. Per segment: entry t1 (any t) and exit t2 (> t1 + 1e-4) of
 * the boundary; t1 clamps to 0.001; free flight hd = -ln(u) / density with u the
 * sample's next uniform, drawn when the ray crosses the boundary (ConstantMedium's
 * random_double(); media are tested in slot order, hit()'s order); hit at
 * t1 + hd/|d| when hd <= (t2 - t1)|d|; closest rule strict like planes. */
rt_status rt_constant_medium(rt_ctx* ctx, int32_t index, const float center[3],
                             const float extend[3], float density, int32_t material);
/* Triangle mesh from world-space vertices, 9 floats per triangle
 * (createTriangleMeshData + createMesh, main.cu:384-401, kernels.h:126-133). */
rt_status rt_mesh(rt_ctx* ctx, int32_t index, const float* tri_vertices, int32_t n_tris,
                  int32_t material);
/* OBJ mesh with the loadModel(file, scale, rotate, offset) transform
 * (ModelLoader.cpp:418-448; tinyobjloader quad split, tiny_obj_loader.h:1397-1495). */
rt_status rt_mesh_obj(rt_ctx* ctx, int32_t index, const char* path, const float scale[3],
                      const float rotate[3], const float offset[3], int32_t material);
/* Number of triangles of the mesh in slot `index` (0 if not a mesh). */
int32_t rt_mesh_triangle_count(const rt_ctx* ctx, int32_t index);
/* Copies the world-space vertices (9 floats/tri) of mesh slot `index`. */
rt_status rt_mesh_vertices(const rt_ctx* ctx, int32_t index, float* out, int32_t max_tris);

/* PLY mesh with loadObject + processTriangleData semantics (Loader.cpp:207-319,
 * 98-205): centred, scaled so max |coord| = max_coord (reference 1.0,
 * MaxCoordAfterRescale Loader.cpp:58), then offset. The mesh is accelerated
 * by the reference's binned-SAH BVH (BVH.cpp:94-497). */
rt_status rt_mesh_ply(rt_ctx* ctx, int32_t index, const char* path, const float offset[3],
                      float max_coord, int32_t material);
/* The reference's `.bvh` cache image for a PLY file (BVH.cpp:500-554 with
 * UpdateBoundingVolumeHierarchy's writer, 537-540): u32 node count, u32 index
 * count, 32 B CacheFriendlyBVHNode[], int32 triangle indices. Writes up to
 * `capacity` bytes to `out` (may be NULL) and the full size to *size. */
rt_status rt_ply_bvh_image(const char* path, const float offset[3], float max_coord,
                           uint8_t* out, int64_t capacity, int64_t* size);

/* ---- BVH builder ----
 * RT_BVH_HOST (default): the reference's Recurse + PopulateCacheFriendlyBVH on the
 * host (BVH.cpp:94-497; rt_bvh.cpp, exact O(N log N) split search).
 * RT_BVH_GPU: the same builder restated level by level on the context's device
 * (rt_bvh_gpu.hip), byte-identical trees; used by rt_commit (mesh and sphere
 * BVHs) and rt_process_triangle_data. It declines inputs with -0.0 coordinates
 * (the reference's min3/max3 tie rule is order-dependent there); those are built
 * on the host. */
#define RT_BVH_HOST 0
#define RT_BVH_GPU 1
rt_status rt_set_bvh_builder(rt_ctx* ctx, int32_t builder);
/* Wall time (ms) of the BVH builds of the last rt_commit + rt_process_triangle_data,
 * and how many of them the GPU builder ran. */
rt_status rt_bvh_build_stats(const rt_ctx* ctx, double* build_ms, int32_t* gpu_builds);
/* rt_ply_bvh_image with the GPU builder on `device`; *build_ms (may be NULL) = the
 * build's wall time (upload, levels, numbering, download). */
rt_status rt_ply_bvh_image_gpu(int32_t device, const char* path, const float offset[3], float max_coord,
                               uint8_t* out, int64_t capacity, int64_t* size, double* build_ms);

/* ---- `.bvh` cache files (UpdateBoundingVolumeHierarchy, BVH.cpp:500-554) ----
 * RT_BVH_CACHE_OFF (default): every BVH is built. RT_BVH_CACHE_READ: a BVH over a PLY
 * file's triangles is read from `<ply>.bvh` when that file exists and the PLY is not
 * newer than it (the reference's `plyFileTime > bvhFileTime` rebuild rule), for the
 * pathTrace scene (the last rt_load_object path, as main.cu:435 passes sceneFile)
 * and for rt_mesh_ply meshes (read at rt_commit). RT_BVH_CACHE_WRITE: after a build,
 * write `<ply>.bvh` (BVH.cpp:535-541) - the pathTrace scene only, as in the reference
 * (rt_mesh_ply meshes may be placed differently, so they read caches but never write them).
 * READ | WRITE is the reference's behaviour.
 * Cache files are untrusted input: the header counts must match the file size and
 * the triangle count, every node index and leaf range must be in bounds, children
 * must follow their parent (DFS order), the leaves must partition the triangle list
 * and the list must be a permutation; a file that fails is ignored (rebuilt) and
 * counted in rt_bvh_cache_stats. */
#define RT_BVH_CACHE_OFF 0
#define RT_BVH_CACHE_READ 1
#define RT_BVH_CACHE_WRITE 2
rt_status rt_set_bvh_cache(rt_ctx* ctx, int32_t mode);
/* Since the last rt_commit + rt_process_triangle_data: caches read, written, and
 * rejected as invalid. */
rt_status rt_bvh_cache_stats(const rt_ctx* ctx, int32_t* reads, int32_t* writes, int32_t* rejected);

/* ---- pathTrace scene (prepareCUDAscene, main.cu:404-553) ----
 * loadObject (Loader.cpp:207-319): appends a PLY mesh whose triangles carry
 * `reflection_type` (RT_PT_*); indices are offset by the vertices already
 * loaded. */
rt_status rt_load_object(rt_ctx* ctx, const char* path, int32_t reflection_type);
/* processTriangleData(offset) (Loader.cpp:98-205, max |coord| = max_coord,
 * reference 1.0) + UpdateBoundingVolumeHierarchy (BVH.cpp:500-554) + the
 * device upload of prepareCUDAscene. The six built-in spheres
 * (CUDAPathTracer.cu:94-121) need no call. out_info (may be NULL):
 * [0] triangles, [1] BVH nodes, [2] triangle-list entries, [3] tree depth. */
rt_status rt_process_triangle_data(rt_ctx* ctx, const float offset[3], float max_coord,
                                   int32_t out_info[4]);
/* The `.bvh` cache image UpdateBoundingVolumeHierarchy writes for the processed
 * pathTrace scene (BVH.cpp:537-540; same layout as rt_ply_bvh_image). */
rt_status rt_pathtrace_bvh_image(const rt_ctx* ctx, uint8_t* out, int64_t capacity, int64_t* size);

/* ---- camera (Camera.h:19-34 initialize, 86-103 updateViewMatrix) ---- */
rt_status rt_camera(rt_ctx* ctx, const float eye[3], const float center[3], const float up[3],
                    float aspect_ratio, float fov, float aperture, float focus_distance,
                    float time0, float time1);

/* ---- the reference's Camera object (Camera.h:12-196) ----
 * rt_camera_state holds Camera's fields; the rt_camera_* functions below restate its methods
 * with the reference's float operations, so a realtime frontend's camera moves
 * (OpenGLFrontend.cpp:393-407 mouse, 586-611 keys, 189-197 sliders) land on the reference's
 * floats. The state is the caller's (plain memory, no context needed). Like the reference, a
 * move changes eye / center / forward / right but not the view that getRay reads
 * (origin, lower_left, horizontal, vertical, right, true_up, lens_radius) until
 * rt_camera_update_view_matrix runs while the state is dirty. */
typedef struct rt_camera_state {
    float eye[3], center[3], up[3];
    float forward[3], right[3], true_up[3];
    float origin[3], horizontal[3], vertical[3], lower_left[3];
    float aspect_ratio, fov, scale, viewport_height, viewport_width;
    float moving_speed; /* 1.5 after initialize (Camera.h:28); the frontend's "Camera Speed" slider */
    float aperture, focus_distance, lens_radius, time0, time1;
    int32_t dirty;      /* bIsDirty */
} rt_camera_state;
/* Camera::initialize (Camera.h:19-34): fields, movingSpeed 1.5, dirty, updateViewMatrix. */
rt_status rt_camera_initialize(rt_camera_state* cam, const float eye[3], const float center[3], const float up[3],
                               float aspect_ratio, float fov, float aperture, float focus_distance, float time0,
                               float time1);
/* Camera::updateViewMatrix (Camera.h:86-103): recomputes the view while dirty and leaves the
 * state dirty (updateLensRadius, Camera.h:110-113, sets the flag); the caller clears it
 * (resetDiryFlag: cam->dirty = 0), as pathTracing does (main.cu:877-881). */
rt_status rt_camera_update_view_matrix(rt_camera_state* cam);
/* walk / strafe / raise (Camera.h:40-56): eye and center += axis * movingSpeed * delta along
 * forward / right / up. yaw (58-67): forward and right rotateY by delta radians, center =
 * eye + forward. pitch (69-76): forward rotated about right. orbit (78-84): eye turned 0.01 rad
 * about the vertical through `target`. setAperture (105-108). All set the dirty flag. */
rt_status rt_camera_walk(rt_camera_state* cam, float delta);
rt_status rt_camera_strafe(rt_camera_state* cam, float delta);
rt_status rt_camera_raise(rt_camera_state* cam, float delta);
rt_status rt_camera_yaw(rt_camera_state* cam, float delta);
rt_status rt_camera_pitch(rt_camera_state* cam, float delta);
rt_status rt_camera_orbit(rt_camera_state* cam, const float target[3]);
rt_status rt_camera_set_aperture(rt_camera_state* cam, float aperture);
/* The context renders with the state's current view (what renderKernel's getRay reads from
 * the managed Camera); rt_camera() is rt_camera_initialize + rt_camera_apply. */
rt_status rt_camera_apply(rt_ctx* ctx, const rt_camera_state* cam);
/* The Camera object of the context's current camera (set by rt_camera, rt_camera_apply or a
 * scene file): the `camera` a frontend drives after initialize(). RT_ERR_STATE if none. */
rt_status rt_get_camera(const rt_ctx* ctx, rt_camera_state* out);

/* ---- the reference's Canvas buffers (Canvas.h:20-200) on the device ----
 * An accumulation buffer (float RGB) and a pixel buffer (uint8 RGB, Canvas::gamma) of
 * width x height in the context's device memory, row 0 = the bottom row. Destroy canvases
 * before their context. The sample / rendering-time counters are host state of the
 * caller's Canvas (the C++ facade keeps them). */
typedef struct rt_canvas rt_canvas;
rt_status rt_canvas_create(rt_ctx* ctx, int32_t width, int32_t height, rt_canvas** out);
void rt_canvas_destroy(rt_canvas* canvas);
/* clearAccumulationBuffer (Canvas.h:162-164) - to zero: the reference's cudaMemset(..., 1,
 * ...) leaves 2.4e-38 per float, a bug with no visible effect after gamma. */
rt_status rt_canvas_clear_accumulation(rt_canvas* canvas);
/* One GPU_REALTIME frame (renderKernel -> accumulatePixel, main.cu:195-196, Canvas.h:82-98)
 * into the canvas: rt_accumulate on the full frame with `sample_count` = the samples per
 * pixel accumulated after this frame (the reference: incrementSampleCount() before the
 * launch, 1 sample per frame); synchronous, like pathTracing's cudaDeviceSynchronize. */
rt_status rt_canvas_accumulate(rt_canvas* canvas, const rt_render_params* params, uint32_t sample_count);
/* getPixelBuffer (Canvas.h:105-107): width x height x 3 uint8; the accumulation buffer. */
rt_status rt_canvas_read_pixels(const rt_canvas* canvas, uint8_t* out_host);
rt_status rt_canvas_read_accumulation(const rt_canvas* canvas, float* out_host);
/* Restores an accumulation buffer read earlier (checkpoint / resume of a long progressive
 * render: SURVEY §5's accumulation dump; the reference loses it on exit). */
rt_status rt_canvas_write_accumulation(rt_canvas* canvas, const float* in_host);

/* Builds the device scene tables and uploads them (replaces the device-side
 * `new` factories + cudaMemcpyToSymbol, main.cu:850-851). */
rt_status rt_commit(rt_ctx* ctx);
/* Committed scene census: out[0] planes (cube faces included), [1] spheres,
 * [2] moving spheres, [3] meshes, [4] triangles, [5] material slots,
 * [6] BVH nodes, [7] spheres placed behind the object BVH (the counts
 * [1]/[2] include them). */
rt_status rt_scene_info(const rt_ctx* ctx, int32_t out[8]);
/* The rayColor BVHs' deepest root-to-leaf path in child-pair records (meshes of more than 64
 * triangles, sphere groups): the traversal stack entries per lane a render needs (rt_render_stats.
 * stack_depth; at most 32, the builder's limit like BVH_STACK_SIZE, CUDAPathTracer.h:43); 0 without BVHs. */
rt_status rt_scene_bvh_depth(const rt_ctx* ctx, int32_t* out);
/* FNV-1a 64 digest of the committed host tables (objects, triangles, materials,
 * BVH nodes, triangle maps, camera): two scene builds that agree on it upload
 * identical device data. Works on device -1 contexts. */
rt_status rt_scene_digest(const rt_ctx* ctx, uint64_t* out);

/* ---- scene files ----
 * initialize() for SCENE == 1 (main.cu:623-786): reads a scene YAML of the
 * reference's schema (the .yaml files under resources/scenes) with a built-in block-style
 * reader (the reference links yaml-cpp 0.7.0) and creates its camera,
 * materials and objects without committing:
 *   camera: eye, center, up, fov, aperture; focus = |center - eye|, aspect =
 *     float(width) / height, shutter [0, 1] (main.cu:632-638);
 *   materials 0-8 pre-created first (main.cu:643-651), so a YAML material whose
 *     id is taken is ignored (the nullptr guards, main.cu:714-744);
 *   object slot i = list position; the primitive type is the first field of
 *     the object's map (main.cu:706, 749): 0 sphere, 1 plane, 2 mesh (OBJ with
 *     scale/rotate/offset; meshes use materials[3], main.cu:781), and the build
 *     extensions 3 cube, 4 constant medium, `.ply` meshes (offset, maxCoord).
 * Model paths are relative to `models_dir`. Parse errors name the line. */
rt_status rt_load_yaml_scene(rt_ctx* ctx, const char* path, const char* models_dir, int32_t width,
                             int32_t height);

/* ---- render (renderKernel, main.cu:160-206, launched by pathTracing 875-898) ----
 * Output: float32 RGB mean radiance (color / spp, BEFORE Canvas::gamma). */
rt_status rt_render(rt_ctx* ctx, const rt_render_params* params, float* out_rgb_host);
/* Same, into a caller-owned device buffer, enqueued on `hip_stream`
 * (hipStream_t, NULL = default). Asynchronous: stats are valid after the
 * stream has completed and rt_sync_stats() has been called. */
rt_status rt_render_device(rt_ctx* ctx, const rt_render_params* params, float* out_rgb_device,
                           void* hip_stream);
rt_status rt_sync_stats(rt_ctx* ctx, rt_render_stats* out);
/* ---- multi-GPU frames: pixel-row tiles + one RCCL gather ----
 * Rank k of n owns the row blocks b = k, k + n, k + 2n, ... of params->row_block rows
 * (y = 0 at the bottom). The RNG is keyed by the global pixel, so the assembled frame
 * is bit-identical for every n. */
int32_t rt_owned_rows(int32_t height, int32_t row_block, int32_t rank, int32_t world);
/* The largest tile of a frame = the gather's equal per-rank count, in rows. */
int32_t rt_max_tile_rows(int32_t height, int32_t row_block, int32_t world);

/* Single-process multi-device frame (replaces pathTracing's single renderKernel
 * launch, main.cu:875-898, with SURVEY §8(b)'s `tiles + ncclGather`): ctxs[k] renders
 * rank k's tiles on its own device (params->row_rank / row_world are set per
 * context); all launches are issued before any is awaited. When the contexts sit on
 * distinct devices the tiles meet on ctxs[0]'s device through ONE ncclGather over
 * communicators from ncclCommInitAll (created on first use and kept by ctxs[0] for
 * later frames over the same devices); contexts that share a device are copied
 * device to device instead (RCCL needs one rank per device). A device kernel then
 * de-interleaves the rows. Each context needs the same committed scene and camera. */
rt_status rt_render_multi(rt_ctx* const* ctxs, int32_t n, const rt_render_params* params,
                          float* out_rgb_host);
/* Same, leaving the frame (height x width x 3 floats) in `frame_device` on ctxs[0]'s
 * device, ordered on `hip_stream` (of that device; NULL = default). */
rt_status rt_render_multi_device(rt_ctx* const* ctxs, int32_t n, const rt_render_params* params,
                                 float* frame_device, void* hip_stream);

/* One process per GPU (the scaling path): communicator plumbing for C/C++ hosts.
 * Rank 0 calls rt_comm_unique_id and ships the 128 bytes to every rank (MPI, a file,
 * a socket); every rank calls rt_comm_init for its context's device. `comm` is an
 * ncclComm_t. */
rt_status rt_comm_unique_id(uint8_t id[128]);
rt_status rt_comm_init(rt_ctx* ctx, const uint8_t id[128], int32_t world, int32_t rank, void** comm);
rt_status rt_comm_destroy(void* comm);
/* The frame exchange of one rank: `tile_device` holds this rank's rendered tile
 * (rt_render_device with row_rank = rank, row_world = world) with room for
 * rt_max_tile_rows rows; ONE ncclGather on `hip_stream` moves every tile to rank 0,
 * whose device de-interleaves them into `frame_device` (height x width x 3 floats;
 * ignored on other ranks). Asynchronous. */
rt_status rt_gather_rows(rt_ctx* ctx, void* comm, const rt_render_params* params, int32_t rank, int32_t world,
                         const float* tile_device, float* frame_device, void* hip_stream);
/* The de-interleave alone: `staging_device` = world x rt_max_tile_rows x width x 3
 * floats, rank-major (what the gather delivers) -> `frame_device`. */
rt_status rt_assemble_rows(rt_ctx* ctx, const rt_render_params* params, int32_t world,
                           const float* staging_device, float* frame_device, void* hip_stream);
/* renderKernel's offline output (Canvas::writePixel(index, color / spp), Canvas.h:58-71):
 * gamma-corrected uint8 RGB of the owned rows, computed on the device. */
rt_status rt_render_u8(rt_ctx* ctx, const rt_render_params* params, uint8_t* out_rgb8_host);
/* GPU_REALTIME progressive mode (renderKernel -> Canvas::accumulatePixel, Canvas.h:73-98,
 * main.cu:876-888): adds each owned pixel's sample SUM over params->spp samples
 * (reference: 1 per frame) to the caller's device buffer `accum_device` (float RGB,
 * same layout as the output) and, when `pixels_device` is not NULL, writes
 * gamma(acc * (1.0f / sample_count)) to it as uint8 RGB. `sample_count` is the
 * canvas's count after incrementSampleCount (total samples per pixel so far);
 * use params->sample_offset = samples already accumulated so each frame draws
 * fresh samples. Clearing the buffer (clearAccumulationBuffer on a camera
 * change) is the caller's: it owns the memory. Asynchronous on `hip_stream`. */
rt_status rt_accumulate(rt_ctx* ctx, const rt_render_params* params, float* accum_device,
                        uint32_t sample_count, uint8_t* pixels_device, void* hip_stream);

/* Canvas::gamma (Canvas.h:198-200): u8 = uint(255.99 * clamp(sqrt(c), 0, 0.999)). */
rt_status rt_gamma_u8(const float* rgb, int64_t n, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* RTMI_H_ */
