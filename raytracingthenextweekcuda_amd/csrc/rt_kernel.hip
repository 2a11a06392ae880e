// rt_kernel.hip — the per-pixel path-tracing megakernels for gfx950 (MI355X).
//
// Replaces renderKernel (main.cu:160-206) + rayColor (main.cu:63-94) + hit (main.cu:43-57) + the Hitable /
// Material virtual calls (Sphere.cu, Plane.cu, Cube.cu, TriangleMesh.cu, AABBox.h, Material.h/.cu) +
// Camera::getRay (Camera.h:151-168) + cuRAND (main.cu:120-129), and pathTrace (CUDAPathTracer.cu:358-622).
//
// Execution model:
//  * a persistent grid takes work items (pixel, sub-stream of S = lanes_per_pixel) from 8 sharded queue heads
//    (one per XCD band), one atomic per wave once L.refill lanes are idle; each lane folds its sub-stream's
//    samples in order and stores a partial sum, and combine_kernel sums a pixel's S partials in a fixed order
//    (the static grid, RT_SCHEDULE_STATIC, computes the same sums);
//  * path regeneration: a lane whose path ends starts its next sample in the same loop trip; once the queue is
//    dry, idle lanes trace other lanes' last samples (tail stealing);
//  * the main loop is wave-uniform (it exits on an empty __ballot), so the whole wave can cooperate in a trip;
//  * small meshes (the reference's brute-force TriangleMesh) are tested by two-phase ballot compaction over runs
//    of equal meshes; per-ray results merge with a 64-bit LDS atomic-min on (t, triangle index);
//  * large meshes, sphere groups and the pathTrace triangles use the reference's binned-SAH BVH (BVH.cpp) over
//    child-pair records (quantized for meshes), with per-lane LDS stacks, cooperative traversal (idle lanes
//    steal pending subtrees) and leaf tests deferred to wave-wide batches;
//  * scan records are read at wave-uniform addresses (scalar loads); counter-based RNG (rt_math.h).
//
// Numerics: compiled with -ffp-contract=off and IEEE div/sqrt (fast paths only where they give the same bits);
// every expression keeps the reference's evaluation order (rt_math.h): the output is bit-identical to the CPU
// restatement in oracle/.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rt_bvh.h"
#include "rt_kernel.h"

namespace rt {

namespace {

constexpr float kInf = __builtin_huge_valf();
constexpr int kWavesPerBlock = 4;  // static-grid blocks: 2 x 2 wave tiles
// Waves per block of the persistent work-queue grid. A block's LDS is released only when all its
// waves have retired, so at the end of a launch a block with one long wave holds the LDS of all;
// smaller blocks hand SIMD resources to the next launch in flight wave by wave.
#ifndef RT_QUEUE_BLOCK_WAVES
#define RT_QUEUE_BLOCK_WAVES 4
#endif
constexpr int kQueueBlockWaves = RT_QUEUE_BLOCK_WAVES;
static_assert(kQueueBlockWaves == 1 || kQueueBlockWaves == 2 || kQueueBlockWaves == 4, "queue block waves");
constexpr int block_waves(bool queue) { return queue ? kQueueBlockWaves : kWavesPerBlock; }

struct Ray {
    v3 o, d;
    float time;
};

// AABBox::intersect (AABBox.h:14-111). Uses the Ray ctor's inverse direction
// and signs (Ray.h:10-16); tMin/tMax are ignored like the reference.
__device__ __forceinline__ bool box_hit(const float* f, v3 o, v3 inv) {
    const bool sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
    float tminx = ((sx ? f[3] : f[0]) - o.x) * inv.x;
    float tmaxx = ((sx ? f[0] : f[3]) - o.x) * inv.x;
    float tminy = ((sy ? f[4] : f[1]) - o.y) * inv.y;
    float tmaxy = ((sy ? f[1] : f[4]) - o.y) * inv.y;
    if ((tminx > tmaxy) || (tminy > tmaxx)) return false;
    if (tminy > tminx) tminx = tminy;
    if (tmaxy < tmaxx) tmaxx = tmaxy;
    float tminz = ((sz ? f[5] : f[2]) - o.z) * inv.z;
    float tmaxz = ((sz ? f[2] : f[5]) - o.z) * inv.z;
    if ((tminx > tmaxz) || (tminz > tmaxx)) return false;
    if (tminz > tminx) tminx = tminz;
    if (tmaxz < tmaxx) tmaxx = tmaxz;
    float t = tminx;
    if (t < 0.0f) {
        t = tmaxx;
        if (t < 0.0f) return false;
    }
    return true;
}

// Conservative BVH node test (boxes are inflated at build time; NaN slabs from
// 0 * inf are ignored by fminf/fmaxf, i.e. never cull): entry <= min(exit, tmax).
__device__ __forceinline__ bool node_hit(const BvhNode& n, v3 o, v3 inv, float tmax, float& tnear) {
    const float tx0 = (n.lo[0] - o.x) * inv.x, tx1 = (n.hi[0] - o.x) * inv.x;
    const float ty0 = (n.lo[1] - o.y) * inv.y, ty1 = (n.hi[1] - o.y) * inv.y;
    const float tz0 = (n.lo[2] - o.z) * inv.z, tz1 = (n.hi[2] - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    tnear = tn;
    return tn <= fminf(tf, tmax * 1.00001f + 1e-30f);
}

// The mesh traversal's slab terms on a QPair grid (rt_scene.h): the plane c + q s of axis a is entered at
// t(q) = fma(q, A_a, B_a) with A = s * inv (exact: s is a power of two) and B = (c - o) * inv, once per ray.
// |t(q) - (c + q s - o) inv| <= 2^-22 (|B_a| + kQMax |A_a|) for every grid coordinate q <= kQMax (two roundings
// in B, one in the fma); E is 4x that bound over the axes and qpair_hit widens the interval by it, so it accepts
// every ray whose exact slab interval meets the grid box, which contains round 5's inflated float box.
struct QRay {
    v3 A, B;
    float E;
};
__device__ __forceinline__ QRay qray(const float4 fr, v3 o, v3 inv) {
    QRay r;
    r.A = v3{fr.w * inv.x, fr.w * inv.y, fr.w * inv.z};
    r.B = v3{(fr.x - o.x) * inv.x, (fr.y - o.y) * inv.y, (fr.z - o.z) * inv.z};
    const float q = (float)kQMax;
    const float m = fmaxf(fmaxf(fabsf(r.B.x) + q * fabsf(r.A.x), fabsf(r.B.y) + q * fabsf(r.A.y)),
                          fabsf(r.B.z) + q * fabsf(r.A.z));
    r.E = m * 0x1p-20f;  // 2 x (twice the bound): the interval is widened by E at both ends
    return r;
}
// One child box of a QPair (three words: lo.x | lo.y, lo.z | hi.x, hi.y | hi.z): node_hit's test on the
// grid box with the interval widened by E; `tmaxe` = the pruning bound (with node_hit's slack) + E.
__device__ __forceinline__ bool qpair_hit(uint32_t w0, uint32_t w1, uint32_t w2, const QRay& r, float tmaxe,
                                          float& tnear) {
    const float tx0 = __builtin_fmaf((float)(w0 & 0xFFFFu), r.A.x, r.B.x);
    const float ty0 = __builtin_fmaf((float)(w0 >> 16), r.A.y, r.B.y);
    const float tz0 = __builtin_fmaf((float)(w1 & 0xFFFFu), r.A.z, r.B.z);
    const float tx1 = __builtin_fmaf((float)(w1 >> 16), r.A.x, r.B.x);
    const float ty1 = __builtin_fmaf((float)(w2 & 0xFFFFu), r.A.y, r.B.y);
    const float tz1 = __builtin_fmaf((float)(w2 >> 16), r.A.z, r.B.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    tnear = tn;
    return tn <= fminf(tf + r.E, tmaxe);
}

// Sphere::hit / MovingSphere::hit root selection (Sphere.cu:3-37, 39-73). `inva` = 1.0f / dot(d, d), the
// same IEEE quotient for every sphere a ray tests: the caller forms it once per ray (sphere_inva).
__device__ __forceinline__ float sphere_inva(v3 d) { return fdiv(1.0f, dot(d, d)); }
__device__ __forceinline__ bool sphere_root(v3 o, v3 d, v3 c, float r, float tmin, float tmax,
                                            float& root, float inva) {
    v3 oc = sub(o, c);
    float a = dot(d, d);
    float hb = dot(oc, d);
    float cc = dot(oc, oc) - r * r;
    float disc = hb * hb - a * cc;
    if (!(disc > kFltEpsilon)) return false;
    float sq = fsqrt(disc);
    float t = (-hb - sq) * inva;
    if (t < tmin || tmax < t) {
        t = (-hb + sq) * inva;
        if (t < tmin || tmax < t) return false;
    }
    root = t;
    return true;
}

// MovingSphere::center (Sphere.cu:75-78).
__device__ __forceinline__ v3 moving_center(const float* f, float time) {
    v3 c0{f[0], f[1], f[2]}, c1{f[3], f[4], f[5]};
    return add(c0, scale(sub(c1, c0), (time - f[6]) / (f[7] - f[6])));
}

// Deferred leaf tests run when this many pairs are queued (64: full batches; fewer measured slower).
#ifndef RT_BATCH_MIN
#define RT_BATCH_MIN 64  // mesh_bvh_pairs
#endif
#ifndef RT_GROUP_BATCH_MIN
#define RT_GROUP_BATCH_MIN 64  // sphere_group_batched
#endif
#ifndef RT_PT_BATCH_MIN
#define RT_PT_BATCH_MIN 64  // pt_traverse_coop_batched
#endif
#ifndef RT_DEFER_MIN
#define RT_DEFER_MIN 32  // the mesh-BVH-only kernels defer a traversal when fewer than this many lanes want it
#endif
// The mesh-BVH-only kernels (no sphere groups, whose counters use W.grp_s / W.grp_m: here they hold the
// per-lane deferral bits) defer a traversal that only a few lanes want: those rays skip shading and scan
// again in the next loop trip, beside the rays that want the mesh then. A wave never defers twice in a row,
// so a deferred ray is traced in the next trip.
template <bool kBvh, int kParts>
constexpr bool kMeshDefer() { return kBvh && kParts == 1; }
// TriangleMesh.cu:74-105's acceptance of a Moller-Trumbore solution: t >= FLT_EPSILON, t >= tMin
// (implied by the first for every t: tMin > FLT_EPSILON), b1, b2 and 1 - b1 - b2 >= FLT_EPSILON.
// Returns t if all hold, else NaN.
__device__ __forceinline__ float tri_accept(float t, float b1, float b2) {
    const float u = 1.0f - b1 - b2;
    // x >= c iff x - (the float below c) > 0, for every float x with gradual underflow (the difference
    // of two distinct floats is never rounded to zero; +-inf and NaN compare the same way). The four
    // differences meet in gfx950's NaN-propagating minimum (v_minimum3_f32): it is > 0 iff every
    // condition holds, with no lane-mask ANDs (scalar instructions, a co-bound of these kernels).
    const float m = __builtin_elementwise_minimum(
        __builtin_elementwise_minimum(t - 0x1.0624dcp-10f /* the float below kTMin */, b1 - 0x1.fffffep-24f),
        __builtin_elementwise_minimum(b2 - 0x1.fffffep-24f /* the float below FLT_EPSILON */, u - 0x1.fffffep-24f));
    return m > 0.0f ? t : __builtin_nanf("");
}

// Correctly rounded reciprocal and quotient without the IEEE division expansion (11 VALU): v_rcp_f32 + one Newton
// step is RN(1/b) for every 2^-126 <= |b| < 2^126 (exhaustive GPU check, tools/div_check.hip), and Markstein's
// q0 + r y with that y is RN(a/b) for |a|, |b| in [2^-100, 2^101) and |a/b| in [2^-121, 2^125). Callers use them
// only where the operands provably lie there, or fall back to the IEEE division for the wave.
__device__ __forceinline__ float rcp_nr(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, y0, 1.0f), y0, y0);
}
__device__ __forceinline__ float div_y(float a, float b, float y) {
    const float q0 = a * y;
    return __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
}

// TriangleMesh.cu:84's 1.0f / det, correctly rounded, for the brute-force meshes' batched tests (all 64 lanes at once; the
// batched tests): v_rcp_f32 + one Newton step is RN(1 / b) for every |b| in [2^-126, 2^126) (exhaustive GPU
// check, tools/div_check.hip); a wave with any other det (zero, subnormal, huge, inf, NaN) takes the IEEE
// division.
__device__ __forceinline__ float tri_rcp(float det) {
    float y = rcp_nr(det);
    const float a = fabsf(det);
    if (__builtin_expect(__ballot(!(a >= 0x1p-126f && a < 0x1p126f)) != 0, 0)) y = fdiv(1.0f, det);
    return y;
}

// One triangle of TriangleMesh::hit (TriangleMesh.cu:40-108) without the closestSoFar comparison: returns t if
// every other acceptance test passes, else NaN (compares false with anything); the caller applies
// closestSoFar. The backface cull (TriangleMesh.cu:40-43) is the final select, not an early return, so the
// caller's record loads all issue at once instead of the normal first and the edges after the cull (the
// batched BVH leaf tests: one dependent load round trip per batch instead of two; round 6).
__device__ __forceinline__ float tri_t(const TriRec& tr, v3 o, v3 d) {
    v3 n{tr.nx, tr.ny, tr.nz};
    const bool cull = dot(d, n) > kFltEpsilon;
    v3 e1{tr.e1x, tr.e1y, tr.e1z}, e2{tr.e2x, tr.e2y, tr.e2z};
    v3 s = sub(o, v3{tr.v0x, tr.v0y, tr.v0z});
    v3 s1 = cross(d, e2);
    v3 s2 = cross(s, e1);
    const float coef = fdiv(1.0f, dot(s1, e1));
    float t = coef * dot(s2, e2);
    float b1 = coef * dot(s1, s);
    float b2 = coef * dot(s2, d);
    const float ta = tri_accept(t, b1, b2);
    return cull ? __builtin_nanf("") : ta;
}

// tri_t for a pair already known to pass the backface cull.
template <bool kRcp>
__device__ __forceinline__ float tri_t_culled(const TriRec& tr, v3 o, v3 d) {
    v3 e1{tr.e1x, tr.e1y, tr.e1z}, e2{tr.e2x, tr.e2y, tr.e2z};
    v3 s = sub(o, v3{tr.v0x, tr.v0y, tr.v0z});
    v3 s1 = cross(d, e2);
    v3 s2 = cross(s, e1);
    const float coef = kRcp ? tri_rcp(dot(s1, e1)) : fdiv(1.0f, dot(s1, e1));
    float t = coef * dot(s2, e2);
    float b1 = coef * dot(s1, s);
    float b2 = coef * dot(s2, d);
    return tri_accept(t, b1, b2);
}

// Closest-hit state with the reference's sequential tie rule (hit(), main.cu:43-57, each object called with
// tMax = closestSoFar): planes and triangles accept t < closestSoFar, spheres t <= closestSoFar (Sphere.cu:25).
// At the minimal t the lowest scan order wins, unless a higher-order sphere is also there (then the highest such
// sphere). Merging candidates in any order with this rule reproduces the sequential scan.
struct Hit {
    float t;
    int32_t obj;     // winner so far by lowest order (-1: none)
    int32_t tri;     // its triangle (meshes)
    uint32_t mi;     // lowest order at t
    int32_t ms_obj;  // highest-order sphere at t (-1: none)
    uint32_t ms;     // its order

    __device__ __forceinline__ void merge(float tc, uint32_t order, bool sphere, int32_t o, int32_t tr) {
        if (tc < t) {
            t = tc;
            mi = order;
            obj = o;
            tri = tr;
            ms_obj = sphere ? o : -1;
            ms = order;
        } else if (tc == t) {
            if (order < mi) {
                mi = order;
                obj = o;
                tri = tr;
            }
            if (sphere && (ms_obj < 0 || order > ms)) {
                ms_obj = o;
                ms = order;
            }
        }
    }
    // merge() for candidates that arrive in increasing scan order (the linear-scan kernel:
    // no sphere groups, so objects, mesh runs and media merge in slot order): an equal t of
    // a later object never lowers mi, so only the strict-less update and a later sphere at
    // the same t remain. Same result as merge() for such sequences.
    template <bool kOrdered>
    __device__ __forceinline__ void merge_seq(float tc, uint32_t order, bool sphere, int32_t o, int32_t tr) {
        if constexpr (!kOrdered) {
            merge(tc, order, sphere, o, tr);
        } else {
            // as selects on the compare's lane mask (VALU), without a divergent branch's exec-mask
            // saves and restores (scalar instructions: DESIGN §4)
            const bool lt = tc < t, eq = sphere && tc == t;
            ms_obj = lt ? (sphere ? o : -1) : eq ? o : ms_obj;
            ms = (lt || eq) ? order : ms;
            t = lt ? tc : t;
            mi = lt ? order : mi;
            obj = lt ? o : obj;
            tri = lt ? tr : tri;
        }
    }
    __device__ __forceinline__ void finish() {
        if (ms_obj >= 0 && ms > mi) {
            obj = ms_obj;
            tri = -1;
        }
    }
};

constexpr int kMaxRun = (int)kMeshRunMax;  // meshes per run (rt_scene.cpp marks the runs)
// The render kernels' traversal stacks hold L.stack_depth entries per lane (the scene's deepest path in pair
// records), PLUS one spare slot in kernels that traverse sphere groups: sphere_group_batched's non-pushing lanes
// write their would-be entry to slot L.stack_depth (lane selects). mesh_bvh_pairs writes it to the lane's W.src
// word instead, dead until the next trip's steal round, so the mesh-BVH-only kernels need no spare (round 6).
// The kernel's stack base and the launch's LDS size (stack_bytes) both count it; tests/test_fuzz_parity.py
// reaches the deepest pair of a chain BVH with both children hit.
template <int kParts>
constexpr int stack_spare() { return (kParts & 2) != 0 ? 1 : 0; }

// A wave's LDS tables. The mesh-BVH-only kernels (kParts = 1: the bunny, Suzanne) use the core alone: they
// keep no sphere-group counts, and their brute-force compaction's cull ring lives in the wave's traversal
// stacks (empty between two mesh traversals: nothing is carried across) - 512 B per wave less, which with the
// spare slot's 256 B lets six 4-wave blocks of the bunny's kernel (18-entry stacks) fit a CU's 160 KB.
struct WaveLdsCore {
    unsigned long long key[64];  // per-ray (t bits << 32 | triangle) minima
    int32_t src[64];             // rank -> lane of the rays wanting a mesh
    uint32_t slot[kMaxRun * 64];  // mesh_run ray slots / the BVH traversals' deferred leaf pairs
    uint32_t grp_s[64];          // sphere-group test counts / (kParts = 1) deferral bits 0-1, path depth bits 2-31
};
struct WaveLds : WaveLdsCore {
    uint32_t grp_m[64];  // per-lane moving-sphere test counts (Counters::grp drained per trip)
    uint16_t ring[128];  // pair ids that passed the backface cull, awaiting the full test
};

// The sphere-group traversal's per-lane state that outlives a loop trip (kResume): a lane whose
// traversal is still running when the wave leaves it keeps its reference, stack depth and (t, ~order)
// minimum here and resumes in the next trip (the member stack stays in the LDS stacks).
struct GroupLds {
    unsigned long long key[64];  // per-ray (t bits << 32 | ~order) minimum over accepted members
    int32_t src[64];             // the member that set it
    uint32_t cur[64];            // pair index or leaf reference to continue from
    uint32_t st[64];             // bit 31: pending; bit 8: `has`; bits 0-7: stack depth
};

// Event counters of one wave, laid out to keep VGPRs free: per-lane amounts stay per lane (node visits, BVH-leaf
// triangle tests); wave-uniform events (segments, mesh-box tests, brute-force triangle tests) are scalars from
// ballots; the two sphere-group counts share one VGPR (16 | 16 bits, drained to LDS every trip); a stack
// overflow is a flag stored straight into the device counters.
struct Counters {
    uint32_t tri_tests, node_visits;     // per lane
    uint32_t grp;                        // per lane, this trip: spheres | moving spheres << 16
    uint32_t segs, box_tests, tri_wave;  // wave-uniform
    unsigned long long* overflow_flag;   // counters[4]
    // low word only (the counters are zeroed per launch): a 32-bit constant the compiler
    // rematerialises instead of keeping a 64-bit one in two VGPRs for the whole kernel
    __device__ __forceinline__ void overflow() const { *reinterpret_cast<uint32_t*>(overflow_flag) = 1u; }
};

// Camera slots of one wave (linear-scan kernels): each lane's NEXT sample of its
// item, prepared ahead - the camera ray and the sample's stream state right after the camera's
// draws (o.xyz d.x | d.yz time s0 | s1 s2 s3 -). A lane that finishes a sample starts the
// prepared one from here; the camera pass itself then runs for many lanes at once (render_kernel).
struct CamSlots {
    float4 a[64], b[64];
    uint4 c[64];
};

// Diagnostic build only (RT_STAMPS): wave-uniform s_memtime section timers,
// summed per wave into counters[8..15]. Never enabled in shipped builds.
#ifdef RT_STAMPS
__device__ __forceinline__ uint64_t stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define RT_STAMP(var) const uint64_t var = stamp()
#define RT_ACC(slot, a, b) (tm[slot] += (b) - (a))
#else
#define RT_STAMP(var)
#define RT_ACC(slot, a, b)
#endif
// RT_STAMPS: the BVH traversals count their loop trips (slot 3) and the lanes with work in them (slot 6):
// their lane utilisation (tools/stamps_breakdown.py)
#ifdef RT_STAMPS
#define RT_TM_PARAM , uint64_t* tm
#define RT_TM_ARG , tm
#define RT_TRIP_COUNT(busy) (tm[3] += 1, tm[6] += (uint64_t)__popcll(__ballot(busy)))
#else
#define RT_TM_PARAM
#define RT_TM_ARG
#define RT_TRIP_COUNT(busy) ((void)0)
#endif

// A constant materialised at its use (the empty asm makes each call a fresh VGPR):
// the register allocator otherwise keeps shared constant tuples - a zero vector,
// a 64-bit all-ones - live across the whole persistent loop, and in the BVH kernel
// spilled them to scratch instead of rematerialising them.
__device__ __forceinline__ uint32_t fresh_u32(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ float fresh_f32(float v) {
    asm volatile("" : "+v"(v));
    return v;
}

// __shfl(v, src, 64) without HIP's lane-id arithmetic: ds_bpermute reads lane (address / 4) mod 64,
// the same lane __shfl picks. HIP's version derives its own lane id (mbcnt) for the width mask,
// a value the register allocator kept live across the persistent loop - and spilled to scratch.
__device__ __forceinline__ int lane_read(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ float lane_read(float v, int src) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}

// Sets an LDS 64-bit minimum slot to +inf (all ones).
__device__ __forceinline__ void key_reset(unsigned long long& k) {
    const uint32_t ones = fresh_u32(~0u);
    uint32_t* w = reinterpret_cast<uint32_t*>(&k);
    w[0] = ones;
    w[1] = ones;
}

// The lane's rank among the set bits of `mask` below it.
__device__ __forceinline__ int lane_rank(uint64_t mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// The megakernels' launch parameters (their FIRST argument: kernarg offset 0) behind an
// opaque pointer. Each loop trip re-reads the fields it uses with scalar loads at their
// use, instead of the compiler holding ~40 of them in SGPRs across the persistent loop
// (SGPRs are the scarce resource: their spills take VGPR lanes, whose spills go to scratch).
__device__ __forceinline__ const RenderLaunch& launch_args() {
    const __attribute__((address_space(4))) char* p =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *reinterpret_cast<const RenderLaunch*>((const char*)p);
}

// The batched mesh traversal over quantized child-pair records (rt_scene.h QPair). A lane holds one reference
// word: a pair index (one 32 B load, two box tests; the nearer hit child becomes the reference, the farther
// is pushed) or a leaf reference (first triangle, count), whose triangles are queued - up to three per trip -
// for the wave's batched tests: once 64 pairs are queued the wave tests them one per lane, merging accepted
// hits into each ray's LDS minimum of (t, mesh-local index), which is then the lanes' pruning bound. Idle
// lanes steal the oldest pending subtree of another ray. Pruning is conservative, so the candidate set holds
// the sequential scan's winner and the (t, index) minimum picks it.
__device__ __forceinline__ void mesh_bvh_pairs(const TriRec* __restrict__ tris,
                                               const uint32_t* __restrict__ tri_orig,
                                               const BvhNode* __restrict__ nodes, uint32_t root, uint32_t frame,
                                               uint32_t base, bool want, v3 o, v3 d, v3 inv, Hit& h, int32_t obj,
                                               uint32_t order, uint32_t* wstack, WaveLdsCore& W, int lane,
                                               Counters& cnt, int cap RT_TM_PARAM) {
    const uint64_t wm = __ballot(want);
    if (wm == 0) return;
    key_reset(W.key[lane]);
    int owner = lane;
    // the ray's slab terms on the mesh's QPair grid (the frame is one wave-uniform 16 B load)
    QRay qr = qray(*reinterpret_cast<const float4*>(nodes + frame), o, inv);
    float best = h.t;  // pruning bound for the current ray (its closestSoFar until a hit lands)
    uint32_t cur = root;  // pair index or leaf reference
    bool has = want;
    int sp = 0, bot = 0;            // pending references: wstack[k * 64 + lane], bot <= k < sp
    uint32_t qtail = 0, qdone = 0;  // wave-uniform positions in the pair queue W.slot (256 entries)
    constexpr uint32_t kQ = (uint32_t)kMaxRun * 64u;
    static_assert(kQ >= 256, "the pair queue holds 63 + 3 x 64 pairs");
    __builtin_amdgcn_wave_barrier();
    // test `count` (<= 64) queued pairs, one per lane (wave-uniform)
    auto batch = [&](uint32_t count) {
        const bool act = (uint32_t)lane < count;
        const uint32_t e = act ? W.slot[(qdone + (uint32_t)lane) & (kQ - 1)] : 0u;
        const uint32_t k = e >> 6;
        const int own = (int)(e & 63u);
        const v3 po{lane_read(o.x, own), lane_read(o.y, own), lane_read(o.z, own)};
        const v3 pd{lane_read(d.x, own), lane_read(d.y, own), lane_read(d.z, own)};
        const float pt0 = lane_read(h.t, own);
        // lanes past `count` test triangle 0 (valid) and drop the result: no branch around the loads. The
        // triangle's 48 B and its mesh-local index are loaded together, before the test needs either
        const TriRec tr = tris[k];
        const uint32_t orig = tri_orig[2 * k];
        const float t = tri_t(tr, po, pd);
        asm volatile("" ::"v"(orig));  // (keeps the index load beside the record's, not behind the test)
        if (act && t <= pt0) atomicMin(&W.key[own], ((unsigned long long)__float_as_uint(t) << 32) | orig);
        qdone += count;
        __builtin_amdgcn_wave_barrier();
    };
    for (;;) {
        if (__ballot(has || sp > bot) == 0) break;
        RT_TRIP_COUNT(has || sp > bot);
        // steal: pair the r-th idle lane with the r-th lane that has a spare reference
        const bool idle = !has && sp == bot;
        const bool spare = sp - bot >= (has ? 1 : 2);
        const uint64_t im = __ballot(idle), vm = __ballot(spare);
        if (im != 0 && vm != 0) {
            const int nv = __popcll(vm), ni = __popcll(im);
            if (spare) W.src[lane_rank(vm)] = lane;
            __builtin_amdgcn_wave_barrier();
            const bool thief = idle && lane_rank(im) < nv;
            const int vr = W.src[lane_rank(im)];  // (read by every lane: the rank is below 64)
            const int vic = thief ? vr : lane;
            const int vt = lane_read(bot, vic);  // the victim's oldest pending reference
            auto take = [&](float& x) {
                const float v = lane_read(x, vic);
                if (thief) x = v;
            };
            {
                const int v_owner = lane_read(owner, vic);
                if (thief) owner = v_owner;
            }
            take(qr.A.x); take(qr.A.y); take(qr.A.z);
            take(qr.B.x); take(qr.B.y); take(qr.B.z);
            take(qr.E);
            take(best);
            {
                const uint32_t vref = wstack[vt * 64 + vic];  // (a valid slot for every lane)
                const float kb = __uint_as_float((uint32_t)(W.key[owner] >> 32));
                cur = thief ? vref : cur;
                best = thief ? fminf(best, kb) : best;
                sp = thief ? 0 : sp;
                bot = thief ? 0 : bot + (spare && lane_rank(vm) < ni ? 1 : 0);  // robbed
                has = has || thief;
            }
            __builtin_amdgcn_wave_barrier();
        }
        {  // pop as lane selects (the read of slot 0 by lanes that do not pop is discarded)
            const bool pop = !has && sp > bot;
            const uint32_t v = wstack[(pop ? sp - 1 : 0) * 64 + lane];
            const float kb = __uint_as_float((uint32_t)(W.key[owner] >> 32));
            cur = pop ? v : cur;
            best = pop ? fminf(best, kb) : best;
            sp -= pop ? 1 : 0;
            has = has || pop;
            const bool empty = !has && sp == bot;
            sp = empty ? 0 : sp;
            bot = empty ? 0 : bot;
        }
        if (has && !(cur & kLeafRef)) {
            const QPair pr = *reinterpret_cast<const QPair*>(nodes + cur);  // one 32 B record
            cnt.node_visits += 2;
            float tl, tr;
            const float tmaxe = best * 1.00001f + 1e-30f + qr.E;
            const bool hl = qpair_hit(pr.q[0], pr.q[1], pr.q[2], qr, tmaxe, tl);
            const bool hr = qpair_hit(pr.q[3], pr.q[4], pr.q[5], qr, tmaxe, tr);
            // as lane selects; a lane that does not push writes the spare slot `cap` (never read)
            const bool both = hl && hr, lf = tl <= tr;
            const bool ovf = both && sp + 1 > cap;
            if (__builtin_expect(__ballot(ovf) != 0, 0))
                if (ovf) cnt.overflow();
            const bool push = both && !ovf;
            // (a lane that does not push writes its own W.src word, dead until the next trip's steal round)
            uint32_t* const dst = push ? wstack + sp * 64 + lane : reinterpret_cast<uint32_t*>(&W.src[lane]);
            *dst = lf ? pr.ref[1] : pr.ref[0];
            sp = ovf ? 0 : sp + (push ? 1 : 0);
            bot = ovf ? 0 : bot;
            cur = both ? (lf ? pr.ref[0] : pr.ref[1]) : (hl ? pr.ref[0] : pr.ref[1]);
            has = (hl || hr) && !ovf;
        }
        uint32_t lk = 0, ln = 0;  // this trip's leaf pairs: triangles lk .. lk + ln - 1
        {
            const bool leaf = has && (cur & kLeafRef);
            const uint32_t nt = ((cur >> 27) & 15u) + 1u;
            lk = cur & 0x07FFFFFFu;
            ln = leaf ? (nt < 3u ? nt : 3u) : 0u;
            // a larger leaf keeps this lane for more trips
            cur = leaf && nt > 3u ? (kLeafRef | ((nt - 4u) << 27) | (lk + 3u)) : cur;
            has = has && !(leaf && nt <= 3u);
            cnt.tri_tests += ln;
        }
        // enqueue the leaf pairs (converged): a lane's slots follow those of the lanes below it
        const uint64_t b1 = __ballot(ln >= 1u), b2 = __ballot(ln >= 2u), b3 = __ballot(ln >= 3u);
        if (b1) {
            const uint32_t at = qtail + (uint32_t)(lane_rank(b1) + lane_rank(b2) + lane_rank(b3));
            const uint32_t tag = (uint32_t)owner;
            for (uint32_t j = 0; j < ln; ++j) W.slot[(at + j) & (kQ - 1)] = ((lk + j) << 6) | tag;
            qtail += (uint32_t)(__popcll(b1) + __popcll(b2) + __popcll(b3));
            __builtin_amdgcn_wave_barrier();
            if (qtail - qdone >= (uint32_t)RT_BATCH_MIN) {
                while (qtail - qdone >= 64u) batch(64u);
                if ((uint32_t)RT_BATCH_MIN < 64u && qtail - qdone >= (uint32_t)RT_BATCH_MIN) batch(qtail - qdone);  // an early partial batch
                if (has || sp > bot) best = fminf(best, __uint_as_float((uint32_t)(W.key[owner] >> 32)));
            }
        }
    }
    if (qtail > qdone) batch(qtail - qdone);
    __builtin_amdgcn_wave_barrier();
    if (want) {
        const unsigned long long key = W.key[lane];
        if (key != ~0ull) {
            const uint32_t k = tri_orig[2 * (base + (uint32_t)(key & 0xFFFFFFFFu)) + 1];
            h.merge(__uint_as_float((uint32_t)(key >> 32)), order, false, obj, (int32_t)k);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// One object record (64 B) as a single wave-uniform scalar load; the same
// helper serves per-lane loads of sphere-group members.
__device__ __forceinline__ ObjRec load_obj(const ObjRec* __restrict__ objs, int i) {
    const uint4* q = reinterpret_cast<const uint4*>(objs + i);
    const uint4 a = q[0], b = q[1], c = q[2], e = q[3];
    ObjRec r;
    r.type = a.x;
    r.material = a.y;
    r.u0 = a.z;
    r.u1 = a.w;
    r.u2 = b.x;
    r.order = b.y;
    r.f[0] = __uint_as_float(b.z);
    r.f[1] = __uint_as_float(b.w);
    r.f[2] = __uint_as_float(c.x);
    r.f[3] = __uint_as_float(c.y);
    r.f[4] = __uint_as_float(c.z);
    r.f[5] = __uint_as_float(c.w);
    r.f[6] = __uint_as_float(e.x);
    r.f[7] = __uint_as_float(e.y);
    r.f[8] = __uint_as_float(e.z);
    r.f[9] = __uint_as_float(e.w);
    return r;
}

// A run of g consecutive brute-force meshes with the same triangle count m (g in the first record's f[7])
// compacted together: the rays wanting each mesh (box early-out, TriangleMesh.cu:34-38) become ray slots (lane,
// triangle base); the run's slot x triangle pairs are packed over 64 lanes, backface-culled, then tested in
// batches of 64. The triangles are consecutive in `tris`, so the per-lane minimum of (t, global triangle index)
// is what the sequential hit() keeps. `skip`: a convex mesh the ray starts on and leaves (rt_scene.cpp
// convex_shell) takes no slot; the counters still count the reference's AABB passes and tests. kLin (the scan
// kernels): branch-free cull loop and tri_rcp's 1 / det (the BVH kernels keep the exec-mask form: registers).
template <bool kOrdered, bool kLin>
__device__ __forceinline__ void mesh_run(const ObjRec* __restrict__ objs, const TriRec* __restrict__ tris,
                                         int i0, uint32_t g, uint32_t m, uint32_t magic, bool live, v3 o, v3 d,
                                         v3 inv, Hit& h, Counters& cnt, WaveLdsCore& W, uint16_t* ring, int lane,
                                         int skip) {
    uint32_t nslot = 0;  // wave-uniform
    bool any = false;
    const uint32_t lives = (uint32_t)__popcll(__ballot(live));
    for (uint32_t j = 0; j < g; ++j) {
        const ObjRec ob = load_obj(objs, i0 + (int)j);
        const bool want = live && box_hit(ob.f, o, inv);
        const uint64_t mask = __ballot(want);
        cnt.box_tests += lives;
        cnt.tri_wave += (uint32_t)__popcll(mask) * m;
        const bool take = want && skip != i0 + (int)j;
        const uint64_t tmask = __ballot(take);
        if (take) W.slot[nslot + (uint32_t)lane_rank(tmask)] = (uint32_t)lane | (ob.u0 << 6);
        nslot += (uint32_t)__popcll(tmask);
        any = any || take;
    }
    if (nslot == 0) return;
    if (any) key_reset(W.key[lane]);
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = nslot * m;
    const float t0 = h.t;
    uint32_t queued = 0, tested = 0;  // wave-uniform ring positions (phase 1: cull, phase 2: full test)
    constexpr bool kSel = kLin;
    // the pair's ray slot r = p / m as a multiply-high (kSel: magic = 0 for m = 1, where r = p; no branch)
    const uint32_t onem = m == 1u ? 0xFFFFFFFFu : 0u;  // wave-uniform
    auto slot_of = [&](uint32_t p) { return kSel ? (__umulhi(p, magic) | (p & onem)) : m > 1u ? __umulhi(p, magic) : p; };
    auto full_test = [&](uint32_t count) {
        const uint32_t i = tested + (uint32_t)lane;
        const bool act = (uint32_t)lane < count;
        const uint32_t p = act ? (uint32_t)ring[i & 127u] : 0u;
        const uint32_t r = slot_of(p);
        const uint32_t e = W.slot[r];
        const int src = (int)(e & 63u);
        const uint32_t tri = (e >> 6) + (p - r * m);
        const v3 ro{lane_read(o.x, src), lane_read(o.y, src), lane_read(o.z, src)};
        const v3 rd{lane_read(d.x, src), lane_read(d.y, src), lane_read(d.z, src)};
        const float rt0 = lane_read(t0, src);
        // inactive lanes test the pair of slot 0 (a valid triangle) and drop the result: no divergent
        // branch around the loads
        const float t = tri_t_culled<kLin>(tris[tri], ro, rd);
        if (act && t <= rt0) atomicMin(&W.key[src], ((unsigned long long)__float_as_uint(t) << 32) | tri);
        tested += count;
    };
    for (uint32_t p0 = 0; p0 < total; p0 += 64) {
        const uint32_t p = p0 + (uint32_t)lane;
        const bool act = p < total;
        const uint32_t pc = act ? p : 0u;  // inactive lanes read pair 0 (valid) and keep nothing
        const uint32_t r = slot_of(pc);
        const uint32_t e = W.slot[r];
        const int src = (int)(e & 63u);
        const v3 rd{lane_read(d.x, src), lane_read(d.y, src), lane_read(d.z, src)};
        const TriRec& tr = tris[(e >> 6) + (pc - r * m)];
        if constexpr (kSel) {
        // every lane loads its normal and writes a ring entry (no exec-mask branches: scalar instructions);
        // the lanes that keep nothing write position queued + 63, past the keepers' [queued, queued + K) for
        // K <= 63 and outside the pending [tested, queued), which holds fewer than 64 entries here
        const float dn = dot(rd, v3{tr.nx, tr.ny, tr.nz});
        // lanes past `total` compare +inf: one compare whose mask is the ballot (act & !(...) would be a
        // scalar AND, then a VALU round trip for the ballot); a NaN dn keeps, as !(dn > eps) does
        float lim = act ? -kInf : kInf;
        asm volatile("" : "+v"(lim));
        const bool keep = !(fmaxf(dn, lim) > kFltEpsilon);  // TriangleMesh.cu:72
        const uint64_t km = __ballot(keep);
        // (a non-keeper's rank is <= K <= 63, so rank | 63 = 63)
        ring[(queued + ((uint32_t)lane_rank(km) | (keep ? 0u : 63u))) & 127u] = (uint16_t)p;
        queued += (uint32_t)__popcll(km);
        } else {
        const bool keep = act && !(dot(rd, v3{tr.nx, tr.ny, tr.nz}) > kFltEpsilon);  // TriangleMesh.cu:72
        const uint64_t km = __ballot(keep);
        if (keep) ring[(queued + (uint32_t)lane_rank(km)) & 127u] = (uint16_t)p;
        queued += (uint32_t)__popcll(km);
        }
        __builtin_amdgcn_wave_barrier();
        if (queued - tested >= 64u) full_test(64u);
    }
    if (queued > tested) full_test(queued - tested);
    __builtin_amdgcn_wave_barrier();
    if (any) {
        const unsigned long long key = W.key[lane];
        if (key != ~0ull) {
            const uint32_t tri = (uint32_t)(key & 0xFFFFFFFFu);
            const uint32_t base0 = objs[i0].u0;  // wave-uniform
            const uint32_t j = m > 1u ? __umulhi(tri - base0, magic) : tri - base0;  // the mesh in the run
            h.merge_seq<kOrdered>(__uint_as_float((uint32_t)(key >> 32)), objs[i0].order + j, false, i0 + (int)j,
                                  (int32_t)tri);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Candidate root of a (moving) sphere independent of closestSoFar: the near
// root if >= tMin, else the far root (Sphere.cu:20-31 with tMax = +inf; the
// sequential tMax test is applied by Hit::merge). NaN = no candidate.
__device__ __forceinline__ float sphere_candidate(const ObjRec& ob, v3 o, v3 d, float time, float inva) {
    const float* f = ob.f;
    const bool moving = ob.type == kObjMovingSphere;
    const v3 c = moving ? moving_center(f, time) : v3{f[0], f[1], f[2]};
    const float r = moving ? f[8] : f[3];
    float t = 0.0f;
    return sphere_root(o, d, c, r, kTMin, kInf, t, inva) ? t : __builtin_nanf("");
}

// Sphere group: the object BVH over the scene's spheres (members are ObjRecs after the scan list, in leaf order)
// over float child-pair records with deferred leaf tests (as mesh_bvh_pairs, without stealing): lanes at a leaf
// queue (member, ray owner) pairs that the wave tests 64 at a time. Among spheres at the same t the sequential
// hit() keeps the highest scan order (Sphere.cu:25's inclusive test), which also wins against any other object
// at that t (Hit::finish); so one LDS minimum of (t, ~order) per ray over the accepted members is all the group
// adds to the ray's Hit. The lane whose pair set the final minimum records the member in W.src.
#ifndef RT_GROUP_MIN_TRIPS
#define RT_GROUP_MIN_TRIPS 4   // traversal trips before the wave may leave it
#endif
#ifndef RT_GROUP_EXIT_LANES
#define RT_GROUP_EXIT_LANES 8  // the wave leaves once at most this many lanes still traverse
#endif
// kResume (the sphere-group-only kernel, no media: select_variant): once at most RT_GROUP_EXIT_LANES lanes still
// traverse (after RT_GROUP_MIN_TRIPS trips) the wave tests its queued pairs and leaves; unfinished lanes keep their
// state in `gl`, skip shading and resume next trip beside the new segments. A resumed lane re-scans the objects
// before the group (the same closestSoFar) and prunes against its kept minimum: the single pass's result.
template <bool kResume>
__device__ __forceinline__ void sphere_group_batched(const ObjRec* __restrict__ objs,
                                                     const BvhNode* __restrict__ nodes, uint32_t root,
                                                     bool live, const Ray& ray, v3 inv, float inva, Hit& h,
                                                     uint32_t* wstack, WaveLdsCore& W, int lane, Counters& cnt,
                                                     int cap, GroupLds* gl RT_TM_PARAM) {
    if (__ballot(live) == 0) return;
    unsigned long long* K = kResume ? gl->key : W.key;
    int32_t* SRC = kResume ? gl->src : W.src;
    const uint32_t st0 = kResume ? gl->st[lane] : 0u;
    const bool resume = kResume && live && (st0 >> 31) != 0u;
    if (live && !resume) key_reset(K[lane]);
    const v3 o = ray.o;
    float best = h.t;  // pruning bound: the ray's closestSoFar, then its best member so far
    if (resume) best = fminf(best, __uint_as_float((uint32_t)(K[lane] >> 32)));
    uint32_t cur = resume ? gl->cur[lane] : root;  // pair index or leaf reference (root: the group's root pair)
    bool has = resume ? ((st0 >> 8) & 1u) != 0u : live;
    int sp = resume ? (int)(st0 & 0xFFu) : 0;
    uint32_t qtail = 0, qdone = 0;
    constexpr uint32_t kQ = (uint32_t)kMaxRun * 64u;
    __builtin_amdgcn_wave_barrier();
    auto batch = [&](uint32_t count) {
        const bool act = (uint32_t)lane < count;
        const uint32_t e = act ? W.slot[(qdone + (uint32_t)lane) & (kQ - 1)] : 0u;
        const uint32_t k = e >> 6;
        const int own = (int)(e & 63u);
        const v3 po{lane_read(ray.o.x, own), lane_read(ray.o.y, own), lane_read(ray.o.z, own)};
        const v3 pd{lane_read(ray.d.x, own), lane_read(ray.d.y, own), lane_read(ray.d.z, own)};
        const float ptime = lane_read(ray.time, own), pt0 = lane_read(h.t, own);
        const float pinva = lane_read(inva, own);  // the owner's 1 / dot(d, d)
        unsigned long long mine = ~0ull;
        if (act) {
            const ObjRec ob = load_obj(objs, (int)k);
            cnt.grp += ob.type == kObjMovingSphere ? 0x10000u : 1u;
            const float t = sphere_candidate(ob, po, pd, ptime, pinva);
            if (t <= pt0) {
                mine = ((unsigned long long)__float_as_uint(t) << 32) | (unsigned long long)(~ob.order);
                atomicMin(&K[own], mine);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (mine != ~0ull && K[own] == mine) SRC[own] = (int32_t)k;  // (t, order) is unique
        qdone += count;
        __builtin_amdgcn_wave_barrier();
    };
    for (int trip = 0;; ++trip) {
        const uint64_t bm = __ballot(has || sp > 0);
        if (bm == 0) break;
        if (kResume && trip >= RT_GROUP_MIN_TRIPS && __popcll(bm) <= RT_GROUP_EXIT_LANES) break;
        RT_TRIP_COUNT(has || sp > 0);
        {  // pop as lane selects (the read of slot 0 by lanes that do not pop is discarded)
            const bool pop = !has && sp > 0;
            const uint32_t v = wstack[(pop ? sp - 1 : 0) * 64 + lane];
            cur = pop ? v : cur;
            sp -= pop ? 1 : 0;
            has = has || pop;
        }
        if (has && !(cur & kLeafRef)) {
            const BvhNode nl = nodes[2 * (size_t)cur], nr = nodes[2 * (size_t)cur + 1];
            cnt.node_visits += 2;
            float tl, tr;
            const bool hl = node_hit(nl, o, inv, best, tl);
            const bool hr = node_hit(nr, o, inv, best, tr);
            // as lane selects; a lane that does not push writes the spare slot `cap` (never read)
            const bool both = hl && hr, lf = tl <= tr;
            const bool ovf = both && sp + 1 > cap;
            if (__builtin_expect(__ballot(ovf) != 0, 0))
                if (ovf) cnt.overflow();
            const bool push = both && !ovf;
            wstack[(push ? sp : cap) * 64 + lane] = lf ? nr.a : nl.a;
            sp = ovf ? 0 : sp + (push ? 1 : 0);
            cur = both ? (lf ? nl.a : nr.a) : (hl ? nl.a : nr.a);
            has = (hl || hr) && !ovf;
        }
        uint32_t lk = 0, ln = 0;
        {
            const bool leaf = has && (cur & kLeafRef);
            const uint32_t nt = ((cur >> 27) & 15u) + 1u;
            lk = cur & 0x07FFFFFFu;
            ln = leaf ? (nt < 3u ? nt : 3u) : 0u;
            cur = leaf && nt > 3u ? (kLeafRef | ((nt - 4u) << 27) | (lk + 3u)) : cur;
            has = has && !(leaf && nt <= 3u);
        }
        const uint64_t b1 = __ballot(ln >= 1u), b2 = __ballot(ln >= 2u), b3 = __ballot(ln >= 3u);
        if (b1) {
            const uint32_t at = qtail + (uint32_t)(lane_rank(b1) + lane_rank(b2) + lane_rank(b3));
            for (uint32_t j = 0; j < ln; ++j) W.slot[(at + j) & (kQ - 1)] = ((lk + j) << 6) | (uint32_t)lane;
            qtail += (uint32_t)(__popcll(b1) + __popcll(b2) + __popcll(b3));
            __builtin_amdgcn_wave_barrier();
            if (qtail - qdone >= (uint32_t)RT_GROUP_BATCH_MIN) {
                while (qtail - qdone >= 64u) batch(64u);
                if ((uint32_t)RT_GROUP_BATCH_MIN < 64u && qtail - qdone >= (uint32_t)RT_GROUP_BATCH_MIN) batch(qtail - qdone);  // an early partial batch
                if (has || sp > 0) best = fminf(best, __uint_as_float((uint32_t)(K[lane] >> 32)));
            }
        }
    }
    if (qtail > qdone) batch(qtail - qdone);
    __builtin_amdgcn_wave_barrier();
    bool pend = false;
    if constexpr (kResume) {
        pend = live && (has || sp > 0);
        gl->cur[lane] = cur;
        gl->st[lane] = pend ? (0x80000000u | ((uint32_t)has << 8) | (uint32_t)sp) : 0u;
    }
    if (live && !pend) {
        const unsigned long long key = K[lane];
        if (key != ~0ull) {
            const int32_t k = SRC[lane];
            h.merge(__uint_as_float((uint32_t)(key >> 32)), ~(uint32_t)(key & 0xFFFFFFFFu), true, k, -1);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Constant medium bounded by a cube (rt_constant_medium, rtmi.h; "Ray Tracing: The Next Week"'s ConstantMedium::hit
// with the boundary = createCube's six two-sided faces, kernels.h:139-154, each tested like Plane::hit). A ray that
// crosses the boundary draws its free-flight uniform from the sample's stream; the scan visits media in slot
// order, so the draw order is the sequential hit()'s. Returns the scattering distance t, or NaN.
__device__ __forceinline__ float medium_candidate(const ObjRec& ob, v3 o, v3 d, v3 inv, Rng& rng) {
    const float* f = ob.f;
    // blo = center - extend, bhi = center + extend (rt_scene.cpp, the restatement's p.a -/+ e.a):
    // faces at blo.x, bhi.x, bhi.y, blo.y, bhi.z, blo.z in createCube's order (kernels.h:139-154)
    const v3 blo{f[0], f[1], f[2]}, bhi{f[3], f[4], f[5]};
    float tf[6];
    bool ok[6];
    // face k: the axis a = k / 2 and its plane coordinate, in createCube's order
    auto face = [&](int k, float& da, float& num, float& ia) {
        const int a = k >> 1;
        const bool high = (k == 1) | (k == 2) | (k == 4);
        da = a == 0 ? d.x : (a == 1 ? d.y : d.z);
        const float oa = a == 0 ? o.x : (a == 1 ? o.y : o.z);
        const float pa = a == 0 ? (high ? bhi.x : blo.x) : (a == 1 ? (high ? bhi.y : blo.y) : (high ? bhi.z : blo.z));
        num = pa - oa;
        ia = a == 0 ? inv.x : (a == 1 ? inv.y : inv.z);
    };
    // Plane::hit with the face's unit normal +-e_a: dot(n, d) is +-d_a and dot(p - o, n) is +-(p_a - o_a) - the
    // zero terms only decide the sign of a zero, which no test below can see (the faces count only when
    // |d_a| > tMin; ray origins and directions are finite, or all NaN) - and (-x) / (-y) = x / y, so
    // t = (p_a - o_a) / d_a is the restatement's quotient bit for bit. It is RN((p_a - o_a) / d_a) by Markstein's
    // correction with the ray's RN(1 / d_a) (rcp_exact; round 6) for |p_a - o_a| in [2^-100, 2^100) on the faces
    // that count: their |d_a| lies in (tMin, 2) (this kernel's directions are unit vectors, metal's reflection
    // plus a fuzz below 1, or isotropic draws inside the unit ball), which keeps the quotient in Markstein's
    // domain. A wave with a counting face outside it (a zero or tiny numerator: the sign of a zero t must be the
    // IEEE one) recomputes all six with the IEEE division.
    bool slow = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        float da, num, ia;
        face(k, da, num, ia);
        tf[k] = div_y(num, da, ia);
        // |num| in [2^-100, 2^100) iff bits(|num|) - bits(2^-100) < bits(2^100) - bits(2^-100) (unsigned)
        slow = slow | ((fabsf(da) > kTMin) & ((__float_as_uint(num) & 0x7FFFFFFFu) - 0x0D800000u >= 0x64000000u));
    }
    if (__builtin_expect(__ballot(slow) != 0, 0)) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            float da, num, ia;
            face(k, da, num, ia);
            tf[k] = fdiv(num, da);
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int a = k >> 1;
        const float den = a == 0 ? d.x : (a == 1 ? d.y : d.z);
        const float t = tf[k];
        const v3 q = add(o, scale(d, t));
        bool in;
        if (k < 2)  // YZ faces
            in = (q.y > blo.y) & (q.y < bhi.y) & (q.z > blo.z) & (q.z < bhi.z);
        else if (k < 4)  // XZ faces
            in = (q.x > blo.x) & (q.x < bhi.x) & (q.z > blo.z) & (q.z < bhi.z);
        else  // XY faces
            in = (q.x > blo.x) & (q.x < bhi.x) & (q.y > blo.y) & (q.y < bhi.y);
        ok[k] = (fabsf(den) > kTMin) & in;
    }
    // rec1 = boundary.hit(-inf, inf); rec2 = boundary.hit(rec1.t + 0.0001, inf)
    bool f1 = false, f2 = false;
    float t1 = kInf, t2 = kInf;
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (ok[k] && tf[k] < t1) {
            t1 = tf[k];
            f1 = true;
        }
    if (!f1) return __builtin_nanf("");
    const float lo = t1 + 0.0001f;
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (ok[k] && tf[k] >= lo && tf[k] < t2) {
            t2 = tf[k];
            f2 = true;
        }
    if (!f2) return __builtin_nanf("");
    float t1c = t1 < kTMin ? kTMin : t1;
    if (t1c >= t2) return __builtin_nanf("");
    const float len = fsqrt(dot(d, d));
    const float inside = (t2 - t1c) * len;
    const float u = rng.next();
#ifdef RT_ABL_FLOATLOG  // ablation only: float log (results differ)
    const float hd = f[6] * __logf(u);
#else
    const float hd = f[6] * (float)ln_pos_d(u);
#endif
    if (hd > inside) return __builtin_nanf("");
    return t1c + fdiv(hd, len);
}

// hit() over the flattened object table (main.cu:43-57), called with the whole wave active (`live` masks lanes
// without a path); records are fetched one object ahead and the per-object tests are branch-free candidates
// merged with Hit's tie rule. kMed (scenes with media): no record prefetch (the long medium test would keep the
// next record's SGPRs live) and one merge per object; both measured slower elsewhere. kParts (BVH
// kernels): 1 = BVH meshes, 2 = sphere groups; the other traversal is not compiled in.
template <int K>
__device__ __forceinline__ float axis(v3 v) {
    return K == 0 ? v.x : K == 1 ? v.y : v.z;
}

// Plane::hit (Plane.cu:4-52) for a kObjPlaneAxial record: n = +-1 on the normal axis K, +-0 on the in-plane axes
// A, B. Plane.cu's den = dot(n, d) and num = dot(p - o, n) are exactly n_K d_K and (p_K - o_K) n_K when non-zero,
// so t is the same float; a zero den or num fails |den| > tMin or t >= tMin in both forms, and where the full dot
// products are NaN (NaN or inf on A or B) the hit point's A or B coordinate fails the bounds test in both forms.
template <int K, int A, int B>
__device__ __forceinline__ float plane_axial(const ObjRec& ob, v3 o, v3 d, v3 inv) {
    const float* f = ob.f;
    const float nk = f[3 + K];
    const float den = nk * axis<K>(d);
    // t = ((p_K - o_K) n_K) / (n_K d_K) is (p_K - o_K) / d_K exactly (IEEE division and Markstein's correction
    // are odd in the signs of both operands), and rcp_exact already holds RN(1 / d_K): no reciprocal per plane
    // (round 6). t matters only where |den| > tMin; a wave with |num| or |den| >= 2^100 takes the IEEE division.
    const float num = f[K] - axis<K>(o);
    float t = div_y(num, axis<K>(d), axis<K>(inv));
    if (__builtin_expect(__ballot(!(fmaxf(fabsf(num), fabsf(den)) < 0x1p100f)) != 0, 0)) t = fdiv(num, axis<K>(d));
    const float pa = axis<A>(o) + axis<A>(d) * t;
    const float pb = axis<B>(o) + axis<B>(d) * t;
    // The six conditions as one compare: proceed (twoSide ? |den| > tMin : den > tMin, with u1 = the bits of 1.0f
    // or 0: max(|den| u1, den)), t >= tMin (t > the float below it) and the four open bounds are differences that
    // are > 0 exactly when they hold, so the candidate stands iff their minimum is > 0 - no lane-mask ANDs (scalar
    // instructions). den is finite, so the proceed term is a number: where it is <= 0 so is the
    // minimum; where it is > 0 the quotient and pa, pb are finite.
    const float p1 = fmaxf(fabsf(den) * __uint_as_float(ob.u1), den) - kTMin;
    const float m = fminf(fminf(fminf(pa - f[6], f[7] - pa), fminf(pb - f[8], f[9] - pb)),
                          fminf(p1, t - 0x1.0624dcp-10f /* the float below kTMin */));
    return m > 0.0f ? t : __builtin_nanf("");
}

template <bool kBvh, bool kMed = false, bool kSph = true, int kParts = 3>
__device__ __forceinline__ Hit closest_hit(const SceneArgs& S, const Ray& ray, v3 inv, bool live,
                                           Rng& rng, WaveLdsCore& W, uint16_t* ring, uint32_t* stack, int lane,
                                           Counters& cnt, int skip, GroupLds* gl
#ifdef RT_STAMPS
                                           , uint64_t* tm
#endif
                                           ) {
    Hit h{kInf, -1, -1, 0xFFFFFFFFu, -1, 0u};
    const v3 o = ray.o, d = ray.d;
    // the spheres' 1 / dot(d, d), once per ray (only the variants that test spheres)
    const float inva = (kSph || kMed) ? sphere_inva(d) : 0.0f;
    const int n = S.n_objs;
    constexpr bool kPf = !kMed;
    // no sphere groups: merges come in scan order (the media variant measured slower with it)
    constexpr bool kOrd = !kBvh && !kMed;
    auto visit = [&](const ObjRec& ob, const int i) {
        const float* f = ob.f;
        float tc = __builtin_nanf("");  // kMed: this object's candidate, merged once below
        bool tsph = false;
        auto cand = [&](float t, bool sphere) {
            if constexpr (kMed) {
                tc = t;
                tsph = sphere;
            } else {
                h.merge_seq<kOrd>(t, ob.order, sphere, i, -1);
            }
        };
        // wave-uniform dispatch on the record type; the reference's scenes are mostly axial planes
        const uint32_t ty = ob.type;
        auto is = [&](uint32_t k) { return ty == k; };
        if (is(kObjPlaneAxial + 2)) {
            cand(plane_axial<1, 0, 2>(ob, o, d, inv), false);  // XZ
        } else if (is(kObjPlaneAxial + 1)) {
            cand(plane_axial<0, 1, 2>(ob, o, d, inv), false);  // YZ
        } else if (is(kObjPlaneAxial)) {
            cand(plane_axial<2, 0, 1>(ob, o, d, inv), false);  // XY
        } else if (is_plane(ob.type)) {
            // Plane::hit (Plane.cu:4-52); t is only used when `proceed` holds.
            const v3 nrm{f[3], f[4], f[5]};
            const float den = dot(nrm, d);
            const bool proceed = ob.u1 ? (fabsf(den) > kTMin) : (den > kTMin);
            const float num = dot(sub(v3{f[0], f[1], f[2]}, o), nrm);
            // t matters only where `proceed` holds, i.e. |den| > tMin, and then only through
            // t >= tMin and the comparisons after it. Markstein's quotient is exact for |num|, |den| in
            // [2^-100, 2^100) and |t| >= 2^-121; a smaller |num| or |t| is below tMin either way. A
            // wave with a proceeding lane whose |num| or |den| is >= 2^100, inf or NaN takes the
            // IEEE division.
            float t = div_y(num, den, rcp_nr(den));
            if (__builtin_expect(__ballot(proceed && !(fmaxf(fabsf(num), fabsf(den)) < 0x1p100f)) != 0, 0))
                t = fdiv(num, den);
            // the hit point's two in-plane coordinates (ray.at(t) per component), tested
            // against the bounds rt_scene.cpp precomputed with Plane::hit's float ops
            float pa, pb;
            if (ob.u0 == 0u) {
                pa = o.x + d.x * t;
                pb = o.y + d.y * t;
            } else if (ob.u0 == 1u) {
                pa = o.y + d.y * t;
                pb = o.z + d.z * t;
            } else {
                pa = o.x + d.x * t;
                pb = o.z + d.z * t;
            }
            const bool in = (pa > f[6]) & (pa < f[7]) & (pb > f[8]) & (pb < f[9]);
            const bool ok = proceed & (t >= kTMin) & in;
            cand(ok ? t : __builtin_nanf(""), false);
        } else if ((kSph || kMed) && (ob.type == kObjSphere || ob.type == kObjMovingSphere)) {
            cand(sphere_candidate(ob, o, d, ray.time, inva), true);
        } else if (ob.type == kObjMesh) {
            // TriangleMesh::hit (TriangleMesh.cu:34-117): the AABB early-out
            // gates the triangle scan exactly as in the reference.
            const uint32_t root = ob.u2;  // wave-uniform (scalar record)
            if (!kBvh || root == kNoBvh) {
                const uint32_t g = __float_as_uint(ob.f[7]);  // run length (0: inside a run)
                RT_STAMP(t_m0);
                if (g != 0u)
                    mesh_run<kOrd, !kBvh>(S.objs, S.tris, i, g, ob.u1, __float_as_uint(ob.f[6]), live, o, d, inv, h, cnt, W,
                                   ring, lane, skip);
                RT_STAMP(t_m1);
                RT_ACC(3, t_m0, t_m1);
            } else if constexpr ((kParts & 1) != 0) {
                const bool want = live && box_hit(f, o, inv);
                constexpr bool kDef = kMeshDefer<kBvh, kParts>();
                // W.grp_s bit 0: this lane's ray was deferred last trip (its re-scan counts no box test again);
                // bit 1: deferred in this trip
                const bool again = kDef && (W.grp_s[lane] & 1u) != 0u;
                cnt.box_tests += (uint32_t)__popcll(__ballot(live && !again));
                if constexpr (kDef) {
                    const int nw = __popcll(__ballot(want));
                    if ((__float_as_uint(ob.f[9]) & 2u) != 0u && nw > 0 && nw < RT_DEFER_MIN &&
                        __ballot(again) == 0) {
                        if (want) W.grp_s[lane] |= 2u;
                        return;  // (this object's visit: the rest of the scan goes on)
                    }
                }
                mesh_bvh_pairs(S.tris, S.tri_orig, S.nodes, __float_as_uint(ob.f[8]), __float_as_uint(ob.f[6]), ob.u0,
                               want, o, d, inv, h, i,
                               ob.order, stack - lane, W, lane, cnt, S.stack_cap RT_TM_ARG);
            }
        } else if ((kMed || (kBvh && kSph)) && ob.type == kObjMedium) {
            // (the general linear-scan kernel never sees a medium: launch_render sends scenes with
            // media to the kMed variant, so its register allocation need not cover this test)
            cand(live ? medium_candidate(ob, o, d, inv, rng) : __builtin_nanf(""), false);
        } else if (kBvh && (kParts & 2) != 0) {  // kObjSphereGroup
            sphere_group_batched<kBvh && kParts == 2>(S.objs, S.nodes, __float_as_uint(ob.f[8]), live,
                                                                         ray, inv, inva, h, stack - lane, W, lane, cnt,
                                                                         S.stack_cap, gl RT_TM_ARG);
        }
        if constexpr (kMed) h.merge_seq<kOrd>(tc, ob.order, tsph, i, -1);  // NaN: no candidate
    };
    if constexpr (kPf) {
        // Records prefetched one object ahead, in two alternating register sets (the scan unrolled by
        // two): each load lands in the registers of a record already visited, so no record is copied
        // between scalar registers per object (a single prefetched record costs 14 s_mov per object,
        // and the scalar unit, shared by the CU's four SIMDs, is as loaded as the VALU in this kernel).
        // The record after the last one is read but not visited (rt_capi.cpp allocates the table with one
        // record of padding).
        ObjRec ra = load_obj(S.objs, 0);
        for (int i = 0; i < n; i += 2) {
            const ObjRec rb = load_obj(S.objs, i + 1);
            visit(ra, i);
            if (i + 1 >= n) break;
            ra = load_obj(S.objs, i + 2);
            visit(rb, i + 1);
        }
    } else {
        for (int i = 0; i < n; ++i) visit(load_obj(S.objs, i), i);
    }
    h.finish();
    return h;
}

// renderKernel sample loop body (main.cu:179-185) + Camera::getRay (Camera.h:151-168): starts sample s's stream
// and returns its camera ray. The camera record is re-read at each sample start, not held in 21 SGPRs (their
// spills take VGPR lanes): scalar_record's empty asm makes the pointer opaque (no hoisting) and puts it in the
// constant address space, so the loads are wave-uniform s_loads (K$ hits). Through a generic pointer they were
// per-lane FLAT loads whose first use waited for every outstanding vector-memory operation (round 6).
template <typename T>
__device__ __forceinline__ T scalar_record(const T* p) {
    static_assert(sizeof(T) % 4 == 0, "whole words");
    const __attribute__((address_space(4))) uint32_t* w = (const __attribute__((address_space(4))) uint32_t*)p;
    asm volatile("" : "+s"(w));
    uint32_t buf[sizeof(T) / 4];
#pragma unroll
    for (size_t i = 0; i < sizeof(T) / 4; ++i) buf[i] = w[i];
    T r;
    __builtin_memcpy(&r, buf, sizeof(T));
    return r;
}

// normalize(a) (LinearAlgebra.h:69-72) by Markstein quotients (round 6, the camera's ray): RN(c / n) for every
// component c that is +0 or at least 2^-100 in magnitude when the norm n lies in [2^-100, 2^20) (the quotient
// is then in Markstein's domain; +0 / n gives +0 as IEEE does). A wave with a lane outside - a -0 component
// (Markstein's correction would return +0), a tiny one, or an extreme norm - takes the IEEE divisions.
__device__ __forceinline__ v3 normalize_mk(v3 a) {
    const float n = fsqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    const float y = rcp_nr(n);
    v3 r{div_y(a.x, n, y), div_y(a.y, n, y), div_y(a.z, n, y)};
    const uint32_t bx = __float_as_uint(a.x), by = __float_as_uint(a.y), bz = __float_as_uint(a.z);
    // |c| in (0, 2^-100) iff bits(|c|) - 1 < bits(2^-100) - 1 (unsigned; +0 wraps); c = -0 iff bits ^ sign = 0
    const uint32_t tiny = __builtin_elementwise_min(
        __builtin_elementwise_min((bx & 0x7FFFFFFFu) - 1u, (by & 0x7FFFFFFFu) - 1u), (bz & 0x7FFFFFFFu) - 1u);
    const uint32_t mz = __builtin_elementwise_min(__builtin_elementwise_min(bx ^ 0x80000000u, by ^ 0x80000000u),
                                                  bz ^ 0x80000000u);
    const bool ieee = (tiny < 0x0D7FFFFFu) | (mz == 0u) | !((n >= 0x1p-100f) & (n < 0x1p20f));
    if (__builtin_expect(__ballot(ieee) != 0, 0))
        if (ieee) r = normalize(a);
    return r;
}

// kMk: the camera ray normalized by normalize_mk (the linear-scan kernels, whose camera pass runs batched from
// the camera slots; in the traversal kernels the extra live values spilled the sphere-group kernel).
template <bool kMk = false>
__device__ __forceinline__ Ray camera_sample(const CamRec* camp, const RenderLaunch& L, Rng& rng,
                                             uint32_t pixel, int px, int y, int s, float fw, float fh) {
    const CamRec cam = scalar_record(camp);
    rng.begin(L.seed, pixel, L.sample_offset + (uint32_t)s);
    const float rx = rng.next();
    const float ry = rng.next();
    // (px + rx) / (W - 1): the numerator is in [2^-33, 2^31] (rx is a u01 draw), the divisor an
    // integer in [1, 2^31], so the quotient is >= 2^-64: Markstein's domain, exact without a guard
    const float dx = div_y((float)px + rx, fw, rcp_nr(fw));
    const float dy = div_y((float)y + ry, fh, rcp_nr(fh));
    const v3 disk = random_in_unit_disk(rng);
    const v3 rnd = scale(disk, cam.lens_radius);
    const v3 offset = add(scale(cam.right, rnd.x), scale(cam.true_up, rnd.y));
    const v3 norig = add(cam.origin, offset);
    v3 dir = sub(add(add(cam.lower_left, scale(cam.horizontal, dx)), scale(cam.vertical, dy)), norig);
    dir = kMk ? normalize_mk(dir) : normalize(dir);
    const float tm = random_range(rng, cam.time0, cam.time1);
    return Ray{add(cam.origin, offset), dir, tm};
}

// The Ray ctor's inverse direction (Ray.h:10-16), 1.0f / d per component, correctly rounded: rcp_nr is RN(1/x)
// for every 2^-126 <= |x| < 2^126 (3 VALU instead of the IEEE division's 11); a wave with a component outside
// that range (zero, subnormal, huge, inf, NaN) takes the IEEE division. Called by the whole wave.
__device__ __forceinline__ v3 rcp_exact(v3 d) {
    v3 r{rcp_nr(d.x), rcp_nr(d.y), rcp_nr(d.z)};
    const float lo = fminf(fminf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    const float hi = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    const bool ok = lo >= 0x1p-126f && hi < 0x1p126f;  // false for NaN (fminf / fmaxf skip NaNs:
    const bool nan = (d.x != d.x) | (d.y != d.y) | (d.z != d.z);  // checked on their own)
    if (__builtin_expect(__ballot(!ok || nan) != 0, 0))
        if (!ok || nan) r = rcp(d);
    return r;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace

// Occupancy per kernel (waves per SIMD; VGPR budget 512 / waves), each measured on the same box:
// the general BVH kernel 4, the sphere-group and mesh-BVH kernels 5, the bunny's simple-scene mesh kernel 6
// (round 6: slim LDS), the linear-scan kernels 6, CornellBox1's sphere-free one 7, pathTrace 6.
// -DRT_WAVES_PER_EU=k forces all to k.
#ifndef RT_BVH_WAVES
#define RT_BVH_WAVES 4
#endif
#ifndef RT_SCAN_WAVES
#define RT_SCAN_WAVES 6
#endif
#ifndef RT_MED_WAVES
#define RT_MED_WAVES 6
#endif
#ifndef RT_NOSPH_WAVES
#define RT_NOSPH_WAVES 7
#endif
#ifndef RT_BVH_MESH_WAVES
#define RT_BVH_MESH_WAVES 5  // the mesh-BVH-only kernel with the full material set (Suzanne; 96 VGPRs fit 5)
#endif
#ifndef RT_GROUP_WAVES
#define RT_GROUP_WAVES 5
#endif
#ifndef RT_BVH_SIMPLE_WAVES
#define RT_BVH_SIMPLE_WAVES 6  // the bunny box: six 4-wave blocks fit since round 6 (slim LDS); 9 VGPRs spill outside the traversal
#endif
#ifndef RT_PT_WAVES
#define RT_PT_WAVES 6
#endif
#ifdef RT_WAVES_PER_EU
#undef RT_BVH_WAVES
#undef RT_SCAN_WAVES
#undef RT_MED_WAVES
#undef RT_NOSPH_WAVES
#undef RT_GROUP_WAVES
#undef RT_BVH_SIMPLE_WAVES
#undef RT_BVH_MESH_WAVES
#undef RT_PT_WAVES
#define RT_BVH_WAVES RT_WAVES_PER_EU
#define RT_SCAN_WAVES RT_WAVES_PER_EU
#define RT_MED_WAVES RT_WAVES_PER_EU
#define RT_NOSPH_WAVES RT_WAVES_PER_EU
#define RT_GROUP_WAVES RT_WAVES_PER_EU
#define RT_BVH_SIMPLE_WAVES RT_WAVES_PER_EU
#define RT_BVH_MESH_WAVES RT_WAVES_PER_EU
#define RT_PT_WAVES RT_WAVES_PER_EU
#endif
template <bool kBvh, bool kMed = false, bool kSph = true, int kParts = 3>
constexpr int render_waves() {
    return kBvh ? (kParts == 2 ? RT_GROUP_WAVES
                               : (kSph ? (kParts == 1 ? RT_BVH_MESH_WAVES : RT_BVH_WAVES) : RT_BVH_SIMPLE_WAVES))
                : (kMed ? RT_MED_WAVES : (kSph ? RT_SCAN_WAVES : RT_NOSPH_WAVES));
}

// Canvas::gamma (Canvas.h:198-200) with clamp = fmaxf(a, fminf(f, b)).
__device__ __forceinline__ uint8_t gamma_u8(float c) {
    const float v = fmaxf(0.0f, fminf(fsqrt(c), 0.999f));
    return (uint8_t)(uint32_t)(255.99f * v);
}

// writePixel / accumulatePixel (Canvas.h:58-98) for one pixel's sample sum.
__device__ __forceinline__ void write_pixel(const RenderLaunch& L, float* __restrict__ out, size_t o,
                                            v3 sum, float fs) {
    if (L.accumulate) {
        const v3 acc{out[o + 0] + sum.x, out[o + 1] + sum.y, out[o + 2] + sum.z};
        out[o + 0] = acc.x;
        out[o + 1] = acc.y;
        out[o + 2] = acc.z;
        if (L.u8) {
            L.u8[o + 0] = gamma_u8(acc.x * L.accum_scale);
            L.u8[o + 1] = gamma_u8(acc.y * L.accum_scale);
            L.u8[o + 2] = gamma_u8(acc.z * L.accum_scale);
        }
    } else {
        const v3 m{sum.x / fs, sum.y / fs, sum.z / fs};
        out[o + 0] = m.x;
        out[o + 1] = m.y;
        out[o + 2] = m.z;
        if (L.u8) {
            L.u8[o + 0] = gamma_u8(m.x);
            L.u8[o + 1] = gamma_u8(m.y);
            L.u8[o + 2] = gamma_u8(m.z);
        }
    }
}

// Partial sums are stored item-major, [pixel][c][3] (an item's index is pixel << sp_log2 | c): the lanes of a
// wave that dequeued together hold consecutive items, so their stores land in a few contiguous lines, and
// a pixel's S slots, written within a few loop trips of each other, fill whole lines in L2 before they are
// written back (round 5's sub-stream-major [c][pixel][3] spread a wave's 64 stores over 64 lines: WRITE_SIZE
// 4.1x the partial-sum bytes on the bunny). combine_kernel reads a pixel's S slots in the fixed order.
__device__ __forceinline__ void store_partial(const RenderLaunch& L, uint32_t item, v3 sum) {
    float* p = L.partial + (size_t)item * 3;
    p[0] = sum.x;
    p[1] = sum.y;
    p[2] = sum.z;
}

// Work-queue item -> (sub-stream, frame column, local row); false for items past the
// window's or the shard's edge.
__device__ __forceinline__ bool queue_item(const RenderLaunch& L, uint32_t item, int& c, int& px,
                                           int& lrow) {
    const int SP = L.lanes_per_pixel;
    c = (int)(item & (uint32_t)(SP - 1));
    const uint32_t pl = item >> L.sp_log2;
    const uint32_t tile = pl >> 6, w = pl & 63u;
    const uint32_t trow = udiv(tile, L.tiles_x_div);
    const int lpx = (int)(tile - trow * (uint32_t)L.tiles_x) * 8 + (int)(w & 7u);  // column in the window
    px = L.col0 + lpx;
    lrow = (int)trow * 8 + (int)(w >> 3);
    return lpx < L.cols && lrow < L.local_rows;
}

// Work-queue shards: the item range is split into kQueueShards contiguous
// chunks, each with its own head on its own 128 B line (one device word
// saturates near 90 dequeues/us, MI355X_MICROARCH.md). A wave starts on
// shard blockIdx % kQueueShards and moves on when its shard runs dry.
#ifndef RT_QUEUE_SHARDS
#define RT_QUEUE_SHARDS 8
#endif
constexpr int kQueueShards = RT_QUEUE_SHARDS;
static_assert(kQueueShards * 32 <= kQueueHeadWords, "queue heads");
constexpr int kQueueStride = 32;  // u32 words between heads
// Idle lanes that trigger a refill (or all lanes idle): L.refill, chosen per launch
// by the host (rt_capi.cpp launch(): 4 for long items (>= 16 samples each), else 8;
// reported as rt_render_stats.refill);
// -DRT_QUEUE_REFILL=k fixes it
// for A/B builds.
#ifdef RT_QUEUE_REFILL
#define RT_REFILL_AT(L) (RT_QUEUE_REFILL)
#else
#define RT_REFILL_AT(L) ((L).refill)
#endif

// Wave-wide dequeue from shard `sh`: every lane in `need` gets the item index of its group's
// first sub-stream, or ~0u if the shard ran out (one atomic per wave).
__device__ __forceinline__ uint32_t queue_take(const RenderLaunch& L, int sh, uint64_t need, int lane) {
    const uint32_t lo = (uint32_t)(((uint64_t)L.n_qitems * (uint64_t)sh) / kQueueShards);
    const uint32_t hi = (uint32_t)(((uint64_t)L.n_qitems * (uint64_t)(sh + 1)) / kQueueShards);
    const int first = __builtin_ctzll(need);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(L.q_counter + sh * kQueueStride, (unsigned)__popcll(need));
    base = (uint32_t)lane_read((int)base, first);
    const uint32_t it = lo + base + (uint32_t)lane_rank(need);
    if (it >= hi) return ~0u;
    // group it -> (pixel, first sub-stream c < S'): item = pixel << sp_log2 | c
    const uint32_t gs = (uint32_t)(L.sp_log2 - L.grp_log2);
    return ((it >> gs) << L.sp_log2) | (it & ((1u << gs) - 1u));
}

// The next sub-stream of an item's group after c (S' = S >> grp_log2 apart), or -1.
__device__ __forceinline__ int next_member(const RenderLaunch& L, int c, int SP) {
    const int cn = c + (SP >> L.grp_log2);
    return cn < SP ? cn : -1;
}

// Partial sums of the group members from c on that have no samples (c >= spp, possible when
// S > spp): their slots hold zero.
__device__ __forceinline__ void zero_members(const RenderLaunch& L, uint32_t item, int SP) {
    const float z = fresh_f32(0.0f);
    for (int c = (int)(item & (uint32_t)(SP - 1)); c >= 0; c = next_member(L, c, SP))
        store_partial(L, (item & ~(uint32_t)(SP - 1)) | (uint32_t)c, v3{z, z, z});
}

// Refill of a wave's idle lanes (wave-uniform: called by all 64 lanes). A lane
// that wants work and gets an item calls start(item); `exhausted` is set once
// every shard ran dry.
template <typename Start, typename Flush>
__device__ __forceinline__ void queue_refill(const RenderLaunch& L, int lane, bool alive, bool& exhausted,
                                             int& shard, int& tried, Start&& start, Flush&& flush) {
    const bool want = !alive && !exhausted;
    const uint64_t need = __ballot(want);
    if (need && (__popcll(need) >= RT_REFILL_AT(L) || __ballot(alive) == 0)) {
        flush();
        const uint32_t it = queue_take(L, shard, need, lane);
        if (__ballot(want && it == ~0u)) {  // this shard ran dry: move on
            ++tried;
            shard = (shard + 1) % kQueueShards;
            if (tried >= kQueueShards) exhausted = true;
        }
        if (want && it != ~0u) start(it);
    }
}

// Queue mode's second pass: the S partial sums of each pixel in the fixed
// order ((p0 + p1) + p2) + ... (the static layout's shuffle order), then the
// pixel write (mean, accumulate, u8) of write_pixel.
__global__ __launch_bounds__(256) void combine_kernel(RenderLaunch L, float* __restrict__ out) {
    const uint32_t pl = blockIdx.x * 256u + threadIdx.x;
    const int SP = L.lanes_per_pixel;
    int c, px, lrow;
    if (pl * (uint32_t)SP >= L.n_items || !queue_item(L, pl * (uint32_t)SP, c, px, lrow)) return;
    const float* p = L.partial + (size_t)pl * (size_t)SP * 3;  // the pixel's S slots, item-major
    v3 acc{p[0], p[1], p[2]};
    for (int j = 1; j < SP; ++j) {
        p += 3;
        acc = add(acc, v3{p[0], p[1], p[2]});
    }
    write_pixel(L, out, ((size_t)lrow * (size_t)L.cols + (size_t)(px - L.col0)) * 3, acc, (float)L.spp);
}

#ifndef RT_CAM_BATCH
#define RT_CAM_BATCH 32  // lanes lacking a prepared next sample that start a camera pass on their own
#endif
// The camera slot's spare word (linear-scan kernels): the path depth (bits 0-19) and the convex-shell skip
// (bits 20-31).
constexpr uint32_t kDepthMask = (1u << 20) - 1u;  // (max_depth < 2^20 for these kernels: rt_capi.cpp validate)

// Camera slots: bit 31 of a lane's work-queue item is set while its slot holds the lane's next
// sample (s if need_cam, else s + SP or the first sample of its group's next member): a flag in a VGPR already live, not a lane mask in SGPRs (the
// megakernels' scarce registers). Item indices stay below 2^31 (rt_capi.cpp caps them).
constexpr uint32_t kPrepared = 0x80000000u;

// End (exclusive) of sub-stream c's sample sequence c, c + SP, ... < spp.
__device__ __forceinline__ int sub_end(int spp, int c, int SP, int sp_log2) {
    return spp > c ? c + (((spp - c + SP - 1) >> sp_log2) << sp_log2) : c;
}

// A sample's path finished with radiance `contrib`. Owners fold it into the
// item's sum in sample order (((p0 + p1) + p2) + ...); a thief holds it in `thr`
// until its owner folds it in (tail_steal).
// `item` may carry kPrepared; at the end of a group member's samples the owner stores its partial
// sum and goes on with the next member (tail stealing happens only in the last member).
__device__ __forceinline__ void sample_done(const RenderLaunch& L, v3 contrib, int SP, uint32_t& item, int& own_end,
                                            int& s, v3& sum, v3& thr, bool& alive, bool& need_cam, int towner,
                                            bool& held, bool& waiting, uint32_t tl_pack) {
    need_cam = true;
    if (towner >= 0) {
        thr = contrib;
        held = true;
        alive = false;
        return;
    }
    sum = add(sum, contrib);
    s += SP;
    if (s >= own_end) {
        const int cn = L.queue ? next_member(L, (int)(item & (uint32_t)(SP - 1)), SP) : -1;
        if (cn >= 0) {
            store_partial(L, item & ~kPrepared, sum);
            item += (uint32_t)(SP >> L.grp_log2);  // kPrepared (bit 31) is kept: the slot may hold s = cn
            s = cn;
            own_end = sub_end(L.spp, cn, SP, L.sp_log2);
            const float z = fresh_f32(0.0f);
            sum = v3{z, z, z};
            if (cn >= L.spp) {
                zero_members(L, item & ~kPrepared, SP);
                alive = false;
            }
            return;
        }
        alive = false;
        if (L.queue) {
            if (tl_pack) waiting = true;  // its last samples were taken by other lanes
            else store_partial(L, item & ~kPrepared, sum);
        }
    }
}

// Tail stealing (work-queue launches, once the queue is dry; wave-uniform). The
// sample sum of a sub-stream is a sequential fold, but the samples themselves are
// independent (random-access RNG keyed by pixel and sample). An idle lane takes
// the LAST unstarted sample of a lane that still has two or more to go, traces it
// and holds its radiance; the owner, once its own samples are done, folds the
// held values in sample order and writes the partial sum. The partial sums are
// therefore bit-identical; only the tail of the launch gets shorter.
__device__ __forceinline__ void tail_steal(const RenderLaunch& L, WaveLdsCore& W, int lane, int SP, bool& alive,
                                           bool& waiting, bool& held, int& towner, uint32_t& tl_pack,
                                           int& own_end, int& s, uint32_t& item, v3& sum, v3& thr,
                                           bool& need_cam) {
    const int c = (int)(item & (uint32_t)(SP - 1));  // the item's sub-stream
    // 1. owners whose stolen samples are all held fold them in and write the partial
    if (__ballot(waiting || held) != 0) {
        bool ready = true;
        v3 vals[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int src = (int)((tl_pack >> (8 * k)) & 0xFFu) - 1;
            const int sl = waiting && src >= 0 ? src : lane;
            vals[k] = v3{lane_read(thr.x, sl), lane_read(thr.y, sl), lane_read(thr.z, sl)};
            const bool hd = lane_read((int)held, sl) != 0;
            if (waiting && src >= 0) ready = ready && hd;
        }
        if (waiting && ready) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((tl_pack >> (8 * k)) & 0xFFu) sum = add(sum, vals[k]);  // positions ascend with samples
            store_partial(L, item & ~kPrepared, sum);
            waiting = false;
            tl_pack = 0;
        }
        // thieves whose owner has folded their value are free again
        const uint32_t otp = (uint32_t)lane_read((int)tl_pack, towner >= 0 ? towner : lane);
        if (held && otp == 0u) {
            held = false;
            towner = -1;
        }
    }
    // 2. pair the r-th idle lane with the r-th lane that has a spare (unstarted, not
    //    current) sample; items of at most 4 samples (one byte per position in tl_pack)
    const bool idle = !alive && !waiting && !held;
    const bool spare = alive && towner < 0 && s + SP < own_end && sub_end(L.spp, c, SP, L.sp_log2) - c <= 4 * SP &&
                       next_member(L, c, SP) < 0;  // the group's last member
    const uint64_t im = __ballot(idle), vm = __ballot(spare);
    if (im == 0 || vm == 0) return;
    const int nv = __popcll(vm), ni = __popcll(im);
    const int ri = lane_rank(im), rv = lane_rank(vm);
    if (spare) W.src[rv] = lane;
    if (idle) W.slot[ri] = (uint32_t)lane;
    __builtin_amdgcn_wave_barrier();
    const bool thief = idle && ri < nv;
    const int vic = thief ? W.src[ri] : lane;
    const int v_end = lane_read(own_end, vic);
    const uint32_t v_item = (uint32_t)lane_read((int)item, vic) & ~kPrepared;
    if (spare && rv < ni) {  // robbed: its last unstarted sample goes to the thief of the same rank
        own_end -= SP;
        const int pos = (own_end - c) >> L.sp_log2;
        tl_pack |= (W.slot[rv] + 1u) << (8 * pos);
        if ((item & kPrepared) && (need_cam ? s : s + SP) >= own_end) item &= ~kPrepared;  // the taken one was prepared
    }
    if (thief) {  // the thief's own item is finished: it carries the victim's (pixel, sub-stream)
        towner = vic;
        item = v_item;
        s = v_end - SP;
        alive = true;
        need_cam = true;
    }
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int global_row_of(const RenderLaunch& L, int lr) {
    const int lb = (int)udiv((uint32_t)lr, L.row_block_div);
    return (lb * L.row_world + L.row_rank) * L.row_block + (lr - lb * L.row_block);
}

// Lambertian::scatter's direction (Material.cu:3-19): normalize(n + normalize(rp)) of a randomInUnitSphere
// draw rp, with the reference's degenerate-direction fallback to n, by Markstein quotients where exact.
__device__ __forceinline__ v3 lambert_dir(v3 n, v3 rp) {
    v3 nd;
    // normalize(rp) of a randomInUnitSphere draw: each component is 2u - 1 of a u01 draw, so
    // +0 or at least 2^-24 in magnitude, and |rp| < 1: inside Markstein's domain (a +0
    // component gives +0, as the IEEE division does) unless rp = 0 (all three draws 1/2,
    // p = 2^-72), which takes the IEEE division
    const float nrp = fsqrt(rp.x * rp.x + rp.y * rp.y + rp.z * rp.z);
    const float yrp = rcp_nr(nrp);
    v3 u{div_y(rp.x, nrp, yrp), div_y(rp.y, nrp, yrp), div_y(rp.z, nrp, yrp)};
    if (__builtin_expect(__ballot(!(nrp > 0.0f)) != 0, 0))
        if (!(nrp > 0.0f)) u = normalize(rp);
    v3 sd = add(n, u);
    const bool degen = (fabsf(sd.x) < 1e-8f) && (fabsf(sd.y) < 1e-8f) && (fabsf(sd.z) < 1e-8f);
    if (degen) sd = n;
    {
        // normalize(sd) by Markstein quotients. Outside the degenerate case |sd| >= 1e-8 (and <= 2), so
        // the norm is in the domain; a component is in it when it is +0 (sd = n + u is never -0: u has
        // no -0 components, n + u cancels to +0) or at least 2^-100 in magnitude (its quotient then at
        // least 2^-101). A wave with a degenerate lane (sd = n may hold -0) or a component in
        // (0, 2^-100) takes the IEEE divisions.
        const float ns = fsqrt(sd.x * sd.x + sd.y * sd.y + sd.z * sd.z);
        const float ys = rcp_nr(ns);
        nd = v3{div_y(sd.x, ns, ys), div_y(sd.y, ns, ys), div_y(sd.z, ns, ys)};
        // |c| in (0, 2^-100) iff bits(|c|) - 1 < bits(2^-100) - 1 (unsigned; +0 wraps)
        const uint32_t tiny = __builtin_elementwise_min(
            __builtin_elementwise_min((__float_as_uint(sd.x) & 0x7FFFFFFFu) - 1u,
                                      (__float_as_uint(sd.y) & 0x7FFFFFFFu) - 1u),
            (__float_as_uint(sd.z) & 0x7FFFFFFFu) - 1u);
        const bool ieee = degen || tiny < 0x0D7FFFFFu;
        if (__builtin_expect(__ballot(ieee) != 0, 0))
            if (ieee) nd = normalize(sd);
    }
    return nd;
}

// kSph = false: the variant for simple scenes (CornellBox1; with kBvh the bunny box): planes and
// meshes with Lambertian and emissive materials only - neither the sphere test, the sphere
// normals, media nor the metal / dielectric / isotropic scatter is compiled in (rt_capi.cpp
// picks it).
template <bool kBvh, bool kQueue, bool kMed = false, bool kSph = true, int kParts = 3>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(render_waves<kBvh, kMed, kSph, kParts>()))) void render_kernel(
    RenderLaunch L, const ObjRec* __restrict__ objs, const TriRec* __restrict__ tris,
    const MatRec* __restrict__ mats, const BvhNode* __restrict__ nodes,
    const uint32_t* __restrict__ tri_orig, int n_objs, const CamRec* __restrict__ cam,
    float* __restrict__ out, unsigned long long* __restrict__ counters) {
    const SceneArgs S{objs, tris, mats, nodes, tri_orig, n_objs, 0, kBvh, L.stack_depth};
    constexpr int kBW = block_waves(kQueue);
    // the mesh-BVH-only kernels keep the core tables only (WaveLdsCore)
    constexpr bool kSlim = kBvh && kParts == 1;
    __shared__ std::conditional_t<kSlim, WaveLdsCore, WaveLds> lds[kBW];
    // camera slots: the linear-scan kernels only (the traversal kernels' LDS holds their stacks)
    constexpr bool kCamPf = !kBvh;
    // resumable sphere-group traversal (the sphere-group-only kernel)
    constexpr bool kResume = kBvh && kParts == 2;
    constexpr bool kDef = kMeshDefer<kBvh, kParts>();  // deferrable mesh traversal (W.grp_s bits 0-1)
    __shared__ GroupLds glds[kResume ? kBW : 1];
    __shared__ CamSlots cslots[kCamPf ? kBW : 1];
    // traversal stacks (kBvh): kBW x L.stack_depth x 64 lanes, sized per scene at launch
    extern __shared__ uint32_t dyn_stacks[];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    WaveLdsCore& W = lds[wave];
    if (kBvh) {  // sphere groups exist only in BVH scenes
        W.grp_s[lane] = 0;
        if constexpr (!kSlim) lds[wave].grp_m[lane] = 0;
    }
    if (kResume) glds[wave].st[lane] = 0u;
    uint32_t* const wstack0 = kBvh ? dyn_stacks + (size_t)wave * (L.stack_depth + stack_spare<kParts>()) * 64 : nullptr;
    uint32_t* stack = kBvh ? wstack0 + lane : nullptr;
    // the brute-force compaction's cull ring: in the slim kernels the first level of the wave's stacks (256 B)
    uint16_t* ring;
    if constexpr (kSlim) ring = reinterpret_cast<uint16_t*>(wstack0);
    else ring = lds[wave].ring;

    // Lane layout: SP = lanes_per_pixel adjacent lanes share one pixel and split
    // its samples (sub-lane c takes samples c, c+SP, c+2SP, ...). A wave covers
    // 64/SP pixels as a tw x th tile; a 4-wave workgroup covers 2tw x 2th.
    const int SP = L.lanes_per_pixel;
    int c = lane & (SP - 1);
    const int pix = lane / SP;
    const int tw = L.tile_w, th = L.tile_h;
    int px = L.col0 + blockIdx.x * (2 * tw) + (wave & 1) * tw + (pix % tw);
    int lrow = blockIdx.y * (2 * th) + (wave >> 1) * th + (pix / tw);
    // Row tiling: local row -> global row (y = 0 is the bottom row).
    int y = global_row_of(L, lrow);
    bool valid = !kQueue && (px - L.col0 < L.cols) && (lrow < L.local_rows) && (y < L.height);
    uint32_t pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;
    uint32_t item = 0;
    bool exhausted = false;
    int shard = (int)(blockIdx.x % kQueueShards), shards_tried = 0;  // wave-uniform

    v3 sum{0.0f, 0.0f, 0.0f};
    Counters cnt{0, 0, 0, 0, 0, 0, counters + 4};
    int s = c;
    bool alive = valid && s < L.spp;
    // the sub-stream's samples are c, c + SP, ... < own_end; at the end of the queue
    // other lanes of the wave may take the last unstarted ones (tail stealing)
    int own_end = sub_end(L.spp, c, SP, L.sp_log2);
    uint32_t tl_pack = 0;  // owner: thief lane + 1 per stolen item position (8 bits each)
    int towner = -1;       // thief: the lane whose sample it traces
    bool held = false;     // thief: finished, its sample's radiance waits in `thr`
    bool waiting = false;  // owner: own samples done, stolen ones not yet folded in
    bool need_cam = true;
    int depth = 0;
    Ray ray{{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 1.0f}, 0.0f};
    v3 thr{1.0f, 1.0f, 1.0f};
    Rng rng{1u, 0u, 0u, 0u};

#ifdef RT_STAMPS
    uint64_t tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    for (;;) {
        const RenderLaunch& L = launch_args();  // this trip's view of the launch parameters
        const int SP = L.lanes_per_pixel;
        RT_STAMP(t_q);
        if (kQueue) {
            // lanes without work take the next items once enough lanes are idle
            // (queue mode keeps only `item` across the loop: the pixel and sub-stream are
            // derived from it where needed, which keeps four VGPRs out of the traversal)
            queue_refill(L, lane, alive, exhausted, shard, shards_tried, [&](uint32_t it) {
                int ic, ipx, ilr;
                if (!queue_item(L, it, ic, ipx, ilr)) return;  // past the frame edge: ask again
                item = it;
                s = ic;
                const float z = fresh_f32(0.0f);
                sum = v3{z, z, z};
                alive = s < L.spp;
                own_end = sub_end(L.spp, ic, SP, L.sp_log2);
                // sub-streams with no samples (S > spp) still own their partial-sum slots
                if (!alive) zero_members(L, item, SP);
                need_cam = true;
            }, [&]() {
                // the wave-uniform event counts are 32-bit: at a dequeue, flush them to the 64-bit
                // device counters before they can wrap (a brute-force mesh adds up to 64 x its
                // triangles per trip)
                if ((cnt.segs | cnt.box_tests | cnt.tri_wave) >= 0x40000000u) {
                    if (lane == 0) {
                        atomicAdd(&counters[0], (unsigned long long)cnt.segs);
                        atomicAdd(&counters[1], (unsigned long long)cnt.tri_wave);
                        atomicAdd(&counters[2], (unsigned long long)cnt.box_tests);
                    }
                    cnt.segs = cnt.box_tests = cnt.tri_wave = 0;
                }
            });
        }
        if (kQueue && exhausted)
            tail_steal(L, W, lane, SP, alive, waiting, held, towner, tl_pack, own_end, s, item, sum, thr, need_cam);
        if (__ballot(alive || waiting || held || (kQueue && !exhausted)) == 0) break;  // wave-uniform exit
        RT_STAMP(t_a);
        RT_ACC(7, t_q, t_a);
        if constexpr (kCamPf) {
            // Camera slots. A lane starting a sample takes it from its slot when it was prepared;
            // the camera pass (Philox seeding, getRay's draws and arithmetic) runs when some lane
            // must start a sample that is not prepared, or once RT_CAM_BATCH lanes lack a prepared
            // next sample - and then for all of those lanes at once: a lane that is tracing
            // prepares its item's next sample into the slot. Each sample's ray and stream are the
            // same whichever pass computes them (the stream is keyed by pixel and sample).
            CamSlots& C = cslots[wave];
            const bool now = alive && need_cam && !(item & kPrepared);
            // the lane's next sample: the member's next one, or the first of the group's next member
            int ns = s + SP;
            if (ns >= own_end) {
                const int cn = towner < 0 ? next_member(L, (int)(item & (uint32_t)(SP - 1)), SP) : -1;
                ns = cn >= 0 && cn < L.spp ? cn : -1;
            }
            const bool nxt = alive && !need_cam && !(item & kPrepared) && towner < 0 && ns >= 0;
            if (__ballot(now) != 0 || __popcll(__ballot(nxt)) >= RT_CAM_BATCH) {
                if (now || nxt) {
                    if (kQueue) {
                        int ic, ilr;
                        queue_item(L, item, ic, px, ilr);
                        y = global_row_of(L, ilr);
                        pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;
                    }
                    Rng r2{1u, 0u, 0u, 0u};
                    const Ray cr = camera_sample<true>(cam, L, r2, pixel, px, y, now ? s : ns, (float)(L.width - 1),
                                                 (float)(L.height - 1));
                    C.a[lane] = float4{cr.o.x, cr.o.y, cr.o.z, cr.d.x};
                    C.b[lane] = float4{cr.d.y, cr.d.z, cr.time, __uint_as_float(r2.s0)};
                    // (.w holds the lane's path depth, which a tracing lane still needs)
                    uint32_t* cw = reinterpret_cast<uint32_t*>(&C.c[lane]);
                    cw[0] = r2.s1;
                    cw[1] = r2.s2;
                    cw[2] = r2.s3;
                    item |= kPrepared;
                }
            }
            const bool started = alive && need_cam && (item & kPrepared);  // prepared earlier or by this pass
            if (started) {
                const float4 a = C.a[lane], b = C.b[lane];
                const uint4 e = C.c[lane];
                ray = Ray{{a.x, a.y, a.z}, {a.w, b.x, b.y}, b.z};
                rng = Rng{__float_as_uint(b.w), e.x, e.y, e.z};
                item &= ~kPrepared;
                need_cam = false;
                thr = v3{1.0f, 1.0f, 1.0f};
                depth = 0;
                reinterpret_cast<uint32_t*>(&C.c[lane])[3] = fresh_u32(0u);
                if (L.max_depth <= 0)  // rayColor with BOUNCES = 0 returns black
                    sample_done(L, v3{0.0f, 0.0f, 0.0f}, SP, item, own_end, s, sum, thr, alive, need_cam,
                                towner, held, waiting, tl_pack);
            }
        } else if (alive && need_cam) {
            if (kQueue) {
                int ic, ilr;
                queue_item(L, item, ic, px, ilr);
                y = global_row_of(L, ilr);
                pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;
            }
            ray = camera_sample(cam, L, rng, pixel, px, y, s, (float)(L.width - 1), (float)(L.height - 1));
            thr = v3{1.0f, 1.0f, 1.0f};
            if constexpr (kDef) W.grp_s[lane] &= 3u;  // the path depth (bits 2-31)
            else depth = 0;
            need_cam = false;
            if (L.max_depth <= 0)  // rayColor with BOUNCES = 0 returns black
                sample_done(L, v3{0.0f, 0.0f, 0.0f}, SP, item, own_end, s, sum, thr, alive, need_cam, towner,
                            held, waiting, tl_pack);
        }
        // the camera slot's spare word (linear-scan kernels): path depth, convex-shell skip
        uint32_t cw = 0u;
        if constexpr (kCamPf) cw = reinterpret_cast<const uint32_t*>(&cslots[wave].c[lane])[3];
        const bool live = alive && !need_cam;
        if constexpr (kDef) W.grp_s[lane] = (W.grp_s[lane] & ~3u) | ((W.grp_s[lane] >> 1) & 1u);  // bit 0: deferred last trip
        RT_STAMP(t_b);
        RT_ACC(0, t_a, t_b);
#ifdef RT_STAMPS
        tm[4] += 1;                                  // loop trips (per wave)
        tm[5] += (uint64_t)__popcll(__ballot(live));  // lanes tracing a segment this trip
        if (!kBvh) tm[6] += (uint64_t)__popcll(__ballot(valid)); // lanes that own a pixel (BVH kernels: slot 6 counts traversal lanes)
#endif

        const v3 inv = rcp_exact(ray.d);
        // convex-shell skip: the convex mesh this segment starts on and leaves (shading below), kept beside the
        // path depth in the camera slot's spare word: bits 20-31 = its object index + 1
        const int skip = kCamPf ? (int)(cw >> 20) - 1 : -1;
        const Hit h = closest_hit<kBvh, kMed, kSph, kParts>(S, ray, inv, live, rng, W, ring, stack, lane, cnt, skip,
                                                            kResume ? &glds[wave] : nullptr
#ifdef RT_STAMPS
                                        , tm
#endif
        );
        RT_STAMP(t_c);
        RT_ACC(1, t_b, t_c);
        // a lane whose sphere-group traversal continues next trip (kResume) neither counts nor shades yet
        const bool pend = (kResume && live && (glds[kResume ? wave : 0].st[lane] >> 31) != 0u) ||
                          (kDef && live && (W.grp_s[lane] & 2u) != 0u);
        cnt.segs += (uint32_t)__popcll(__ballot(live && !pend));
        if (kBvh && !kDef && __ballot(cnt.grp != 0)) {  // drain the 16-bit sphere-group counts
            W.grp_s[lane] += cnt.grp & 0xFFFFu;
            if constexpr (!kSlim) lds[wave].grp_m[lane] += cnt.grp >> 16;
            cnt.grp = 0;
        }
        if (!live || pend) continue;

        bool done;
        v3 contrib;
        if (h.obj >= 0) {
            const ObjRec& ob = S.objs[h.obj];
            const float* f = ob.f;
            v3 p = add(ray.o, scale(ray.d, h.t));  // ray.at(t)
            v3 outward;
            constexpr bool kAnySph = kSph || kMed;
            if ((kMed || (kBvh && kSph)) && ob.type == kObjMedium) {
                outward = v3{1.0f, 0.0f, 0.0f};  // arbitrary; isotropic scatter ignores it
            } else if (is_plane(ob.type)) {
                outward = v3{f[3], f[4], f[5]};
            } else if (kAnySph && ob.type == kObjSphere) {
                outward = divs(sub(p, v3{f[0], f[1], f[2]}), f[3]);
            } else if (kAnySph && ob.type == kObjMovingSphere) {
                outward = divs(sub(p, moving_center(f, ray.time)), f[8]);
            } else {
                const TriRec& tr = S.tris[h.tri];
                outward = v3{tr.nx, tr.ny, tr.nz};
            }
            // HitResult::setFaceNormal (HitResult.h:15-18).
            const bool front = dot(ray.d, outward) < kFltEpsilon;
            const v3 n = front ? outward : neg(outward);
            const MatRec m = S.mats[ob.material];
            v3 att;
            bool scattered;
            v3 nd;
            // randomInUnitSphere is the first draw of Lambertian, Metal and isotropic scatter alike:
            // drawn here once for all three, each lane's draw sequence is unchanged, and a wave whose
            // lanes hit two of these materials runs one rejection loop instead of two
            v3 rp{0.0f, 0.0f, 0.0f};
            if (m.type == 0u || (kSph && (m.type == 1u || m.type == 4u))) rp = random_in_unit_sphere(rng);
            if (m.type == 0u) {
                // Lambertian::scatter (Material.cu:3-19).
                nd = lambert_dir(n, rp);
                att = v3{m.a0, m.a1, m.a2};
                scattered = true;
            } else if (kSph && m.type == 1u) {
                // Metal::scatter (Material.h:45-51).
                v3 refl = reflect(normalize(ray.d), n);
                nd = add(refl, scale(rp, m.p0));
                scattered = dot(nd, n) > 0.0f;
                att = scale(v3{m.a0, m.a1, m.a2}, scattered ? 1.0f : 0.0f);
            } else if (kSph && m.type == 2u) {
                // Dieletric::scatter + reflectance (Material.h:65-109).
                att = v3{1.0f, 1.0f, 1.0f};
                const float ratio = front ? (1.0f / m.p0) : m.p0;
                v3 ud = normalize(ray.d);
                float cs = fminf(dot(neg(ud), n), 1.0f);
                float sn = sqrtf(1.0f - cs * cs);
                bool refl;
                if (ratio * sn > 1.0f) {
                    refl = true;
                } else {
                    float r0 = (1.0f - ratio) / (1.0f + ratio);
                    r0 = r0 * r0;
                    float R = r0 + (1.0f - r0) * pow5(1.0f - cs);
                    refl = R > rng.next();
                }
                v3 dir = refl ? reflect(ud, n) : refract(ud, n, ratio);
                nd = normalize(dir);
                scattered = true;
            } else if (kSph && m.type == 4u) {
                // isotropic::scatter: Ray(p, randomInUnitSphere(), time), attenuation = albedo.
                nd = rp;
                att = v3{m.a0, m.a1, m.a2};
                scattered = true;
            } else {
                // Emission::scatter (Material.h:120-123): albedo * intensity, stop.
                att = v3{m.a0, m.a1, m.a2};
                scattered = false;
                nd = ray.d;
            }
            // convex-shell skip: a ray that leaves a convex brute-force mesh (rt_scene.cpp convex_shell) outward from a
            // point well inside a face cannot be accepted by any of its triangles: the next segment
            // skips that mesh. Margins: the hit at least 1e-3 (barycentric) inside its triangle's three edges,
            // the new direction at least 1e-3 (cosine) off the face's plane. Only a skip is decided here; the
            // triangles of every other object are tested as before.
            uint32_t self_bits = 0u;
            if constexpr (kCamPf) {
                const bool cand = scattered && h.tri >= 0 && h.obj < 4094 && ob.type == kObjMesh &&
                                  (__float_as_uint(f[9]) & 1u) != 0u;
                if (__ballot(cand) != 0) {
                    const TriRec& tr = S.tris[cand ? h.tri : 0];
                    const v3 e1{tr.e1x, tr.e1y, tr.e1z}, e2{tr.e2x, tr.e2y, tr.e2z};
                    const v3 sv = sub(ray.o, v3{tr.v0x, tr.v0y, tr.v0z});
                    const v3 s1 = cross(ray.d, e2), s2 = cross(sv, e1);
                    const float ic = __builtin_amdgcn_rcpf(dot(s1, e1));  // (a margin test: 1 ulp is plenty)
                    const float b1 = ic * dot(s1, sv), b2 = ic * dot(s2, ray.d);
                    const bool ok = cand & (b1 >= 1e-3f) & (b2 >= 1e-3f) & (1.0f - b1 - b2 >= 1e-3f) &
                                    (dot(nd, outward) > 1e-3f);
                    self_bits = ok ? (uint32_t)h.obj + 1u : 0u;
                }
            }
            if (scattered) {
                thr = mul(thr, att);
                ray = Ray{p, nd, ray.time};
                if constexpr (kCamPf) {
                    // the linear-scan kernels keep the path depth in the camera slot's spare word (LDS)
                    // instead of a VGPR of the persistent loop (at 7 waves/SIMD the CB1 kernel spilled it)
                    uint32_t* dw = reinterpret_cast<uint32_t*>(&cslots[wave].c[lane]) + 3;
                    const uint32_t dn = (*dw & kDepthMask) + 1u;  // (max_depth < 2^20: rt_capi.cpp validate)
                    *dw = dn | (self_bits << 20);
                    done = (int)dn >= L.max_depth;
                } else if constexpr (kDef) {
                    // the mesh-BVH-only kernels keep the path depth in bits 2-31 of W.grp_s (a VGPR was spilled
                    // and reloaded every scatter at their occupancy; max_depth < 2^30: rt_capi.cpp validate)
                    const uint32_t g = W.grp_s[lane] + 4u;
                    W.grp_s[lane] = g;
                    done = (int)(g >> 2) >= L.max_depth;
                } else {
                    ++depth;
                    done = depth >= L.max_depth;
                }
                contrib = v3{0.0f, 0.0f, 0.0f};  // exceeded recursion (main.cu:93)
            } else {
                done = true;
                contrib = mul(thr, att);
            }
        } else {
            // Sky gradient (main.cu:86-89).
            v3 ud = normalize(ray.d);
            float t = 0.5f * (ud.y + 1.0f);
            v3 bg = add(scale(v3{1.0f, 1.0f, 1.0f}, 1.0f - t), scale(v3{0.5f, 0.7f, 1.0f}, t));
            contrib = mul(thr, bg);
            done = true;
        }
        if (done)
            sample_done(L, contrib, SP, item, own_end, s, sum, thr, alive, need_cam, towner, held, waiting,
                        tl_pack);
#ifdef RT_STAMPS
        {
            RT_STAMP(t_d);
            RT_ACC(2, t_c, t_d);
        }
#endif
    }

    // Fixed-order combination of the SP partial sums: ((p0 + p1) + p2) + ...
    // (queue mode: combine_kernel does it from the partial buffer)
    if (!kQueue && SP > 1) {
        const int base = lane - c;
        v3 acc = sum;
        for (int j = 1; j < SP; ++j) {
            v3 pj{lane_read(sum.x, base + j), lane_read(sum.y, base + j), lane_read(sum.z, base + j)};
            acc = add(acc, pj);
        }
        sum = acc;
    }

    if (!kQueue && valid && c == 0) {
        const float fs = (float)L.spp;
        write_pixel(L, out, ((size_t)lrow * (size_t)L.cols + (size_t)(px - L.col0)) * 3, sum, fs);
    }

    const uint64_t ws = cnt.segs;
    const uint64_t wt = wave_sum_u64(cnt.tri_tests) + cnt.tri_wave;
    const uint64_t wb = cnt.box_tests;
    const uint64_t wn = wave_sum_u64(cnt.node_visits);
    const uint64_t wgs = kBvh && !kDef ? wave_sum_u64(W.grp_s[lane] + (cnt.grp & 0xFFFFu)) : 0;
    uint64_t wgm = 0;
    if constexpr (kBvh && !kSlim) wgm = wave_sum_u64(lds[wave].grp_m[lane] + (cnt.grp >> 16));
#ifdef RT_STAMPS
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&counters[8 + k], (unsigned long long)tm[k]);
#endif
    if (lane == 0) {
        atomicAdd(&counters[0], (unsigned long long)ws);
        atomicAdd(&counters[1], (unsigned long long)wt);
        atomicAdd(&counters[2], (unsigned long long)wb);
        if (wn) atomicAdd(&counters[3], (unsigned long long)wn);
        if (wgs) atomicAdd(&counters[5], (unsigned long long)wgs);
        if (wgm) atomicAdd(&counters[6], (unsigned long long)wgm);
    }
}

// ===========================================================================
// pathTrace integrator (CUDAPathTracer.cu:358-622, wired by main.cu:187): the
// smallpt-style material model over the Kuchkuda-triangle BVH of the loaded
// PLY meshes plus the six built-in spheres (CUDAPathTracer.cu:94-121).
// ===========================================================================
namespace {

enum : uint32_t { kDiffuse = 0, kMetalPhong = 1, kSpecular = 2, kRefraction = 3, kCoat = 4 };
// `2 * M_PI` with CUDAPathTracer.cu:38's float M_PI: an exact float product.
constexpr float kPtTwoPi = 2.0f * 3.14159265358979323846f;

struct PtSphere {
    float rad;
    float pos[3], emi[3], col[3];
    uint32_t type;
};
// CUDAPathTracer.cu:94-121 (double literals rounded to float as in the reference).
__constant__ PtSphere kPtSpheres[6] = {
    {1.6f, {0.0f, 2.8f, 0.0f}, {6.0f, 4.0f, 2.0f}, {0.0f, 0.0f, 0.0f}, kDiffuse},
    {10000.0f, {50.0f, 40.8f, -1060.0f}, {0.51f, 0.51f, 0.51f}, {0.175f, 0.175f, 0.25f}, kDiffuse},
    {100000.0f, {0.0f, -100001.1f, 0.0f}, {0.0f, 0.0f, 0.0f}, {0.5f, 0.0f, 0.0f}, kCoat},
    {100000.0f, {0.0f, -100001.2f, 0.0f}, {0.0f, 0.0f, 0.0f}, {0.3f, 0.3f, 0.3f}, kDiffuse},
    {110000.0f, {50.0f, -110048.5f, 0.0f}, {3.6f, 2.0f, 0.2f}, {0.0f, 0.0f, 0.0f}, kDiffuse},
    {1.1f, {1.6f, 0.0f, 1.0f}, {0.0f, 0.0f, 0.0f}, {0.9f, 0.9f, 0.9f}, kSpecular},
};

// Sphere::intersect (CUDAPathTracer.cu:66-79): distance, 0 if no hit.
__device__ __forceinline__ float pt_sphere_hit(int i, v3 o, v3 d) {
    const PtSphere& sp = kPtSpheres[i];
    const v3 op = sub(v3{sp.pos[0], sp.pos[1], sp.pos[2]}, o);
    const float b = dot(op, d);
    float disc = b * b - dot(op, op) + sp.rad * sp.rad;
    if (disc < 0.0f) return 0.0f;
    disc = fsqrt(disc);
    float t;
    return (t = b - disc) > 0.01f ? t : ((t = b + disc) > 0.01f ? t : 0.0f);
}

// RayIntersectsBox (CUDAPathTracer.cu:124-181), exact; also returns Tnear.
__device__ __forceinline__ bool pt_box(const CFNode& n, v3 o, v3 d, float& tnear) {
    float tn = -3.40282347e+38f, tf = 3.40282347e+38f;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float lo = n.bottom[c], hi = n.top[c];
        if (dd[c] == 0.0f) {
            if (oo[c] < lo) return false;
            if (oo[c] > hi) return false;
        } else {
            float t1 = fdiv(lo - oo[c], dd[c]);
            float t2 = fdiv(hi - oo[c], dd[c]);
            if (t1 > t2) {
                const float tmp = t1;
                t1 = t2;
                t2 = tmp;
            }
            if (t1 > tn) tn = t1;
            if (t2 < tf) tf = t2;
            if (tn > tf) return false;
            if (tf < 0.0f) return false;
        }
    }
    tnear = tn;
    return true;
}

// Per-segment ray data for the pathTrace traversal.
struct PtRay {
    v3 o, d;
    v3 inv;        // v_rcp_f32(d) per axis (1 ulp)
    float eps;     // pruning margin: eps * |inv| widens each slab (computed at each use: no VGPRs held)
    bool exact;    // a direction component is tiny but non-zero: always divide
};

// Exact-decision box test: the same accept/reject as RayIntersectsBox (pt_box). The slab parameters come from
// the reciprocal (relative error < 2^-21 against the correctly rounded quotient); the decision reduces to
// `tnear > tfar || tfar < 0` (the early-outs are monotone), the signs are exact, and only a tnear/tfar gap
// inside the rounding band falls back to the divisions. `tn` is a lower bound of the entry parameter of the box
// widened by eps (pruning only); `order` is the unwidened entry (child ordering).
__device__ __forceinline__ bool pt_box_decide(const CFNode& n, const PtRay& r, float& tn_prune,
                                              float& order) {
    float tn = -3.40282347e+38f, tf = 3.40282347e+38f, tw = -3.40282347e+38f;
    bool miss = false;
    const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z};
    const float iv[3] = {r.inv.x, r.inv.y, r.inv.z};
    const float pt[3] = {r.eps * fabsf(r.inv.x), r.eps * fabsf(r.inv.y), r.eps * fabsf(r.inv.z)};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float lo = n.bottom[c], hi = n.top[c];
        if (dd[c] == 0.0f) {
            miss |= (oo[c] < lo) | (oo[c] > hi);
        } else {
            const float t1 = (lo - oo[c]) * iv[c];
            const float t2 = (hi - oo[c]) * iv[c];
            const float tnear_c = fminf(t1, t2);
            tn = fmaxf(tn, tnear_c);
            tf = fminf(tf, fmaxf(t1, t2));
            tw = fmaxf(tw, tnear_c - pt[c]);
        }
    }
    tn_prune = tw;
    order = tn;
    if (miss) return false;
    const float m = fmaxf(fabsf(tn), fabsf(tf));
    if (!r.exact && m < 1e30f && fabsf(tn - tf) > 4e-6f * m) return tn <= tf && !(tf < 0.0f);
    float tx;
    return pt_box(n, r.o, r.d, tx);
}

// A child of a pair record: pt_box_decide for an inner child; for a leaf's box (n.u1), which the
// reference never box-tests, only the entry bounds that order and prune (none in exact mode). One pass
// without divergent branches (round 4: the traversal's exec-mask bookkeeping loaded the CU's scalar
// unit): the slab values are shared, and the exact fallback (pt_box's divisions) runs behind a
// wave-uniform test for the rare inner-box lanes inside the rounding band. Same decisions and bounds.
__device__ __forceinline__ bool pt_child(const CFNode& n, const PtRay& r, float& tn_prune, float& order) {
    float tn = -3.40282347e+38f, tf = 3.40282347e+38f, tw = -3.40282347e+38f;
    bool miss = false;
    const float oo[3] = {r.o.x, r.o.y, r.o.z}, dd[3] = {r.d.x, r.d.y, r.d.z};
    const float iv[3] = {r.inv.x, r.inv.y, r.inv.z};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float lo = n.bottom[c], hi = n.top[c];
        const bool z = dd[c] == 0.0f;
        miss |= z & ((oo[c] < lo) | (oo[c] > hi));
        const float t1 = (lo - oo[c]) * iv[c];
        const float t2 = (hi - oo[c]) * iv[c];
        const float tnear_c = fminf(t1, t2);
        tn = z ? tn : fmaxf(tn, tnear_c);
        tf = z ? tf : fminf(tf, fmaxf(t1, t2));
        tw = z ? tw : fmaxf(tw, tnear_c - r.eps * fabsf(iv[c]));
    }
    const bool leaf = n.u1 != 0u;
    // a leaf's bounds: none in exact mode
    tn_prune = leaf && r.exact ? -3.40282347e+38f : tw;
    order = leaf && r.exact ? -3.40282347e+38f : tn;
    const float m = fmaxf(fabsf(tn), fabsf(tf));
    const bool fast = !r.exact && m < 1e30f && fabsf(tn - tf) > 4e-6f * m;
    bool res = !miss && tn <= tf && !(tf < 0.0f);
    const bool need = !leaf && !miss && !fast;
    if (__builtin_expect(__ballot(need) != 0, 0))
        if (need) {
            float tx;
            res = pt_box(n, r.o, r.d, tx);
        }
    return leaf || res;
}

struct PtBest {
    float hz;      // distancesq of the best hit
    float dist;    // sqrtf(hz)
    int i;         // position in the DFS triangle list (tie-break)
    int idx;       // triangle index
    v3 hit;
};

// BVH_IntersectTriangles (CUDAPathTracer.cu:192-352) as a cooperative ordered traversal over child-pair
// records (rt_bvh.cpp cf_child_pairs): the minimum over (distance^2, DFS list position) of the triangles in the
// leaves the reference reaches. Inner boxes get the reference's exact decision (pt_box_decide), leaf boxes are
// never box-tested, and a subtree is skipped only when its eps-widened box lies beyond the best hit. Idle lanes
// steal pending subtrees (as mesh_bvh_pairs); leaves queue (list position, owner) pairs, and the wave runs the
// Kuchkuda test (CUDAPathTracer.cu:258-345) on 64 at once, merging into each ray's LDS minimum - the
// reference's first-in-DFS tie rule.
__device__ __forceinline__ void pt_traverse_coop_batched(const KTri* __restrict__ ktris,
                                                         const CFNode* __restrict__ nodes, uint32_t* wstack,
                                                         unsigned long long* keys, int32_t* vlist, uint32_t* queue,
                                                         int lane, bool want, const PtRay& ray, int avoid_in,
                                                         float len_in, float eps_in, PtBest& out, Counters& cnt,
                                                         int cap, uint32_t root_ref) {
    const uint64_t wm = __ballot(want);
    if (wm == 0) return;
    key_reset(keys[lane]);
    int owner = lane;
    PtRay r = ray;
    float len_d = len_in;
    (void)eps_in;  // = ray.eps
    float bhz = 3.40282347e+38f, bdist = 3.40282347e+38f;  // the current ray's best (pruning bound)
    auto pruned = [&](float tw) { return tw > 0.0f && tw * len_d > bdist * 1.0001f + r.eps; };
    auto refresh = [&]() {  // the ray's best over all lanes (NaN while none)
        const float g = __uint_as_float((uint32_t)(keys[owner] >> 32));
        if (g < bhz) {
            bhz = g;
            // a pruning bound only: v_sqrt_f32 (<= 1 ulp) widened by 2^-20 stays >= the IEEE root, so no
            // subtree the exact bound keeps is pruned
            bdist = __builtin_amdgcn_sqrtf(g) * 1.000001f;
        }
    };
    uint32_t cur = root_ref;  // pair index or leaf reference
    bool has = want;
    if (want) {
        ++cnt.node_visits;
        const CFNode root = nodes[0];
        if (!(root.u0 & 0x80000000u)) {
            float tw, od;
            has = pt_box_decide(root, r, tw, od);
        }
    }
    int sp = 0, bot = 0;
    uint32_t qtail = 0, qdone = 0;  // wave-uniform positions in `queue` (256 entries)
    __builtin_amdgcn_wave_barrier();
    auto batch = [&](uint32_t count) {
        const bool act = (uint32_t)lane < count;
        const uint32_t e = act ? queue[(qdone + (uint32_t)lane) & 255u] : 0u;
        const uint32_t i = e >> 6;
        const int own = (int)(e & 63u);
        const v3 po{lane_read(ray.o.x, own), lane_read(ray.o.y, own), lane_read(ray.o.z, own)};
        const v3 pd{lane_read(ray.d.x, own), lane_read(ray.d.y, own), lane_read(ray.d.z, own)};
        const int pav = lane_read(avoid_in, own);
        {
            // the Kuchkuda test for list position i (CUDAPathTracer.cu:258-345) as lane selects: lanes past
            // `count` test list position 0 (valid) and every test is evaluated, so no divergent branches
            // (their exec-mask saves and restores are scalar instructions, this kernel's co-bound). The
            // acceptance keeps the reference's comparisons, NaN cases included: the edge tests are
            // `!(e < 0)`, which holds for NaN; the key of a rejected pair is ~0, a no-op for atomicMin.
            // the record of list position i (rt_capi.cpp stores the triangles in list order, the triangle's
            // index beside its material): one load round trip, no cudaTriIdxList indirection
            const float4* T = reinterpret_cast<const float4*>(ktris + (act ? i : 0u));
            const float4 q0 = T[0], q1 = T[1], q2 = T[2], q3 = T[3], q4 = T[4];
            const int idx = __float_as_int(q4.y);
            const v3 nn{q0.x, q0.y, q0.z};
            const float k = dot(nn, pd);
            const float sd = fdiv(q0.w - dot(nn, po), k);
            const v3 hit = add(scale(pd, sd), po);
            // the three edge tests !(e < 0) as one: fminf drops a NaN e, which passes its own test, and the
            // minimum of the others is < 0 iff one of them fails (all NaN: NaN, which passes)
            const float emin = fminf(fminf(dot(v3{q1.x, q1.y, q1.z}, hit) - q1.w, dot(v3{q2.x, q2.y, q2.z}, hit) - q2.w),
                                     dot(v3{q3.x, q3.y, q3.z}, hit) - q3.w);
            const bool ok = act && (pav != idx) && (k != 0.0f) && (sd > 1e-3f) && !(emin < 0.0f);  // NUDGE_FACTOR (sd > 0 implied)
            const v3 df = sub(po, hit);
            const float hz = df.x * df.x + df.y * df.y + df.z * df.z;  // distancesq
            const unsigned long long key = ((unsigned long long)__float_as_uint(hz) << 32) | i;
            atomicMin(&keys[own], ok ? key : ~0ull);
        }
        qdone += count;
        __builtin_amdgcn_wave_barrier();
    };
    for (;;) {
        if (__ballot(has || sp > bot) == 0) break;
        const bool idle = !has && sp == bot;
        const bool spare = sp - bot >= (has ? 1 : 2);
        const uint64_t im = __ballot(idle), vm = __ballot(spare);
        if (im != 0 && vm != 0) {
            const int nv = __popcll(vm), ni = __popcll(im);
            if (spare) vlist[lane_rank(vm)] = lane;
            __builtin_amdgcn_wave_barrier();
            const bool thief = idle && lane_rank(im) < nv;
            int vic = lane;
            if (thief) vic = vlist[lane_rank(im)];
            const int vb = lane_read(bot, vic);
            auto take = [&](float& x) {
                const float v = lane_read(x, vic);
                if (thief) x = v;
            };
            {
                const int v_owner = lane_read(owner, vic);
                const int v_exact = lane_read((int)r.exact, vic);
                if (thief) {
                    owner = v_owner;
                    r.exact = v_exact != 0;
                }
            }
            take(r.o.x); take(r.o.y); take(r.o.z);
            take(r.d.x); take(r.d.y); take(r.d.z);
            take(r.inv.x); take(r.inv.y); take(r.inv.z);
            take(len_d); take(r.eps); take(bhz); take(bdist);
            if (thief) {
                const uint32_t entry = wstack[vb * 64 + vic];
                refresh();
                sp = bot = 0;
                cur = entry;
                has = true;
            }
            if (spare && lane_rank(vm) < ni) ++bot;  // robbed
            __builtin_amdgcn_wave_barrier();
        }
        if (!has && sp > bot) {
            cur = wstack[(--sp) * 64 + lane];
            refresh();
            has = true;
        }
        if (!has && sp == bot) sp = bot = 0;
        if (has && !(cur & kLeafRef)) {
            const CFNode c0 = nodes[2 * (size_t)cur], c1 = nodes[2 * (size_t)cur + 1];
            cnt.node_visits += 2;
            float w0, o0, w1, o1;
            bool h0, h1;
            h0 = pt_child(c0, r, w0, o0);
            h1 = pt_child(c1, r, w1, o1);
            h0 = h0 && !pruned(w0);
            h1 = h1 && !pruned(w1);
            if (h0 && h1) {
                if (sp + 1 > cap) {
                    cnt.overflow();
                    has = false;
                    sp = bot = 0;
                } else {
                    const bool first0 = o0 <= o1;
                    wstack[(sp++) * 64 + lane] = first0 ? c1.u0 : c0.u0;
                    cur = first0 ? c0.u0 : c1.u0;
                }
            } else if (h0) {
                cur = c0.u0;
            } else if (h1) {
                cur = c1.u0;
            } else {
                has = false;
            }
        }
        uint32_t lk = 0, ln = 0;  // this trip's leaf pairs: list positions lk .. lk + ln - 1
        if (has && (cur & kLeafRef)) {
            const uint32_t nt = ((cur >> 27) & 15u) + 1u;
            lk = cur & 0x07FFFFFFu;
            ln = nt < 3u ? nt : 3u;
            if (nt > 3u)  // a larger leaf keeps this lane for more trips
                cur = kLeafRef | ((nt - 4u) << 27) | (lk + 3u);
            else
                has = false;
            cnt.tri_tests += ln;
        }
        const uint64_t b1 = __ballot(ln >= 1u), b2 = __ballot(ln >= 2u), b3 = __ballot(ln >= 3u);
        if (b1) {
            const uint32_t at = qtail + (uint32_t)(lane_rank(b1) + lane_rank(b2) + lane_rank(b3));
            for (uint32_t j = 0; j < ln; ++j) queue[(at + j) & 255u] = ((lk + j) << 6) | (uint32_t)owner;
            qtail += (uint32_t)(__popcll(b1) + __popcll(b2) + __popcll(b3));
            __builtin_amdgcn_wave_barrier();
            if (qtail - qdone >= (uint32_t)RT_PT_BATCH_MIN) {
                while (qtail - qdone >= 64u) batch(64u);
                if ((uint32_t)RT_PT_BATCH_MIN < 64u && qtail - qdone >= (uint32_t)RT_PT_BATCH_MIN) batch(qtail - qdone);  // an early partial batch
                if (has || sp > bot) refresh();
            }
        }
    }
    if (qtail > qdone) batch(qtail - qdone);
    __builtin_amdgcn_wave_barrier();
    if (want) {
        const unsigned long long key = keys[lane];
        if (key != ~0ull) {
            // the winner's hit point with the batch test's operations on the owner's ray
            const int i = (int)(uint32_t)(key & 0xFFFFFFFFu);
            const float4* T = reinterpret_cast<const float4*>(ktris + i);
            const float4 q0 = T[0];
            const int idx = __float_as_int(T[4].y);
            const v3 nn{q0.x, q0.y, q0.z};
            const float k = dot(nn, ray.d);
            const float sd = fdiv(q0.w - dot(nn, ray.o), k);
            const float hz = __uint_as_float((uint32_t)(key >> 32));
            out.hz = hz;
            out.dist = fsqrt(hz);
            out.i = i;
            out.idx = idx;
            out.hit = add(scale(ray.d, sd), ray.o);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

}  // namespace

template <bool kQueue>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_PT_WAVES))) void pathtrace_kernel(
    RenderLaunch L, const KTri* __restrict__ ktris, const CFNode* __restrict__ nodes,
    const CamRec* __restrict__ cam, float* __restrict__ out,
    unsigned long long* __restrict__ counters) {
    constexpr int kBW = block_waves(kQueue);
    extern __shared__ uint32_t dyn_stacks[];  // kBW x L.stack_depth x 64, sized at launch
    __shared__ unsigned long long pt_keys[kBW][64];  // per-ray minima (cooperative traversal)
    __shared__ int32_t pt_vlist[kBW][64];            // victims of a steal round
    __shared__ uint32_t pt_queue[kBW][256];          // deferred leaf pairs
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    uint32_t* stack = dyn_stacks + (size_t)wave * L.stack_depth * 64 + lane;

    const int SP = L.lanes_per_pixel;
    int c = lane & (SP - 1);
    const int pix = lane / SP;
    const int tw = L.tile_w, th = L.tile_h;
    int px = L.col0 + blockIdx.x * (2 * tw) + (wave & 1) * tw + (pix % tw);
    int lrow = blockIdx.y * (2 * th) + (wave >> 1) * th + (pix / tw);
    int y = global_row_of(L, lrow);
    const bool valid = !kQueue && (px - L.col0 < L.cols) && (lrow < L.local_rows) && (y < L.height);
    uint32_t pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;
    uint32_t item = 0;
    bool exhausted = false;
    int shard = (int)(blockIdx.x % kQueueShards), shards_tried = 0;  // wave-uniform

    v3 sum{0.0f, 0.0f, 0.0f};
    Counters cnt{0, 0, 0, 0, 0, 0, counters + 4};
    int s = c;
    bool alive = valid && s < L.spp;
    bool need_cam = true;
    int bounce = 0;
    int avoid = -1;
    v3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f};
    v3 mask{1.0f, 1.0f, 1.0f}, accu{0.0f, 0.0f, 0.0f};
    Rng rng{1u, 0u, 0u, 0u};

    for (;;) {
        const RenderLaunch& L = launch_args();  // this trip's view of the launch parameters
        const int SP = L.lanes_per_pixel;
        const bool has_mesh = L.pt_has_mesh != 0;
        if (kQueue) {
            queue_refill(L, lane, alive, exhausted, shard, shards_tried, [&](uint32_t it) {
                // only `item` is kept across the traversal: the pixel is derived from it at the
                // camera (as render_kernel does), which frees four VGPRs for the traversal
                int ic, ipx, ilr;
                if (!queue_item(L, it, ic, ipx, ilr)) return;  // past the frame edge: ask again
                item = it;
                s = ic;
                alive = s < L.spp;
                const float z = fresh_f32(0.0f);  // materialised here, not kept live (and spilled)
                sum = v3{z, z, z};
                // sub-streams with no samples (S > spp) still own their partial-sum slots
                if (!alive) zero_members(L, item, SP);
                need_cam = true;
            }, []() {});
        }
        if (__ballot(alive || (kQueue && !exhausted)) == 0) break;
        if (alive && need_cam) {
            if (kQueue) {
                int ic, ilr;
                queue_item(L, item, ic, px, ilr);
                y = global_row_of(L, ilr);
                pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;
            }
            const Ray r = camera_sample(cam, L, rng, pixel, px, y, s, (float)(L.width - 1), (float)(L.height - 1));
            o = r.o;
            d = r.d;
            mask = v3{1.0f, 1.0f, 1.0f};
            accu = v3{0.0f, 0.0f, 0.0f};
            avoid = -1;  // renderKernel passes avoidSelf = -1 (main.cu:187)
            bounce = 0;
            need_cam = false;
        }
        // BVH_IntersectTriangles (CUDAPathTracer.cu:192-352). Candidates merge on
        // (distance^2, position in the DFS triangle list): the reference's
        // first-in-DFS-order tie rule, so subtrees can be pruned once their
        // entry distance exceeds the best hit without changing the result.
        // Every lane enters: lanes without a path help the others (pt_traverse_coop).
        PtBest best{3.40282347e+38f, 3.40282347e+38f, 0x7FFFFFFF, -1, v3{0.0f, 0.0f, 0.0f}};
        if (has_mesh) {
            PtRay r;
            r.o = o;
            r.d = d;
            const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
            r.exact = (ax > 0.0f && ax < 1e-30f) || (ay > 0.0f && ay < 1e-30f) || (az > 0.0f && az < 1e-30f);
            r.inv = v3{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y), __builtin_amdgcn_rcpf(d.z)};
            // eps: a bound on how far an accepted Kuchkuda hit point can sit
            // outside its triangle's box (rounding at the scale of the
            // coordinates involved), with a 10x margin.
            const float eps = 1e-5f * (1.0f + fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) + L.pt_scale);
            r.eps = eps;
            pt_traverse_coop_batched(ktris, nodes, stack - lane, pt_keys[wave], pt_vlist[wave], pt_queue[wave],
                                     lane, alive, r, avoid, fsqrt(dot(d, d)), eps, best, cnt, L.stack_depth,
                                     L.pt_root_ref);
        }
        cnt.segs += (uint32_t)__popcll(__ballot(alive));
        if (!alive) continue;
        const int best_idx = best.idx;
        const v3 best_hit = best.hit;
        const uint32_t best_mat = best_idx >= 0 ? (uint32_t)ktris[best.i].material : kDiffuse;
        const float hitdistance = best_idx >= 0 ? best.dist : 1e20f;

        // the six spheres, scanned i = 5 .. 0 (CUDAPathTracer.cu:400-404)
        float scene_t = 1e20f;
        int sphere_id = -1, geom = -1;
        for (int i = 5; i >= 0; --i) {
            const float dist = pt_sphere_hit(i, o, d);
            if (dist != 0.0f && dist < scene_t) {
                scene_t = dist;
                sphere_id = i;
                geom = 1;
            }
        }
        avoid = best_idx;  // avoidSelf = pBestTriIdx (CUDAPathTracer.cu:408)
        if (hitdistance < scene_t && hitdistance > 0.002f) {
            scene_t = hitdistance;
            geom = 2;
        }

        bool done = false;
        v3 contrib{0.0f, 0.0f, 0.0f};
        if (geom < 0 || scene_t > 1e20f) {
            done = true;  // escaped: black (CUDAPathTracer.cu:417)
        } else {
            v3 hitp, normal, oriented, f;
            uint32_t rt;
            if (geom == 1) {
                const PtSphere& sp = kPtSpheres[sphere_id];
                hitp = add(o, scale(d, scene_t));
                normal = normalize(sub(hitp, v3{sp.pos[0], sp.pos[1], sp.pos[2]}));
                oriented = dot(normal, d) < 0.0f ? normal : scale(normal, -1.0f);
                f = v3{sp.col[0], sp.col[1], sp.col[2]};
                rt = sp.type;
                accu = add(accu, mul(mask, v3{sp.emi[0], sp.emi[1], sp.emi[2]}));
            } else {
                const KTri& T = ktris[best.i];
                hitp = best_hit;
                normal = normalize(v3{T.n[0], T.n[1], T.n[2]});
                oriented = dot(normal, d) < 0.0f ? normal : scale(normal, -1.0f);
                f = v3{0.9f, 0.3f, 0.0f};  // hard-coded triangle colour (CUDAPathTracer.cu:444)
                rt = best_mat;
                accu = add(accu, mul(mask, v3{0.0f, 0.0f, 0.0f}));
            }
            v3 next = d, point = hitp;
            auto hemisphere = [&](v3 w, float phi, float r2) {
                // orthonormal frame + cosine-weighted direction (CUDAPathTracer.cu:462-469)
                const v3 a = ((double)fabsf(w.x) > 0.1) ? v3{0.0f, 1.0f, 0.0f} : v3{1.0f, 0.0f, 0.0f};
                const v3 uu = normalize(cross(a, w));
                const v3 vv = cross(w, uu);
                const float r2s = fsqrt(r2);
                float sp, cp;
                pt_sincosf(phi, &sp, &cp);
                const v3 dir = add(add(scale(scale(uu, cp), r2s), scale(scale(vv, sp), r2s)),
                                   scale(w, fsqrt(1.0f - r2)));
                return normalize(dir);
            };
            const v3 mirror = sub(d, scale(scale(normal, 2.0f), dot(normal, d)));
            if (rt == kDiffuse) {
                const float phi = kPtTwoPi * rng.next();
                const float r2 = rng.next();
                const v3 w = normalize(oriented);
                next = hemisphere(w, phi, r2);
                point = add(hitp, scale(w, 0.01f));
                mask = mul(mask, f);
            } else if (rt == kMetalPhong) {
                const float phi = kPtTwoPi * rng.next();
                const float r2 = rng.next();
                const float cos_t = pt_powf(1.0f - r2, 1.0f / (20.0f + 1.0f));
                const float sin_t = fsqrt(1.0f - cos_t * cos_t);
                const v3 w = normalize(mirror);
                const v3 a = ((double)fabsf(w.x) > 0.1) ? v3{0.0f, 1.0f, 0.0f} : v3{1.0f, 0.0f, 0.0f};
                const v3 uu = normalize(cross(a, w));
                const v3 vv = cross(w, uu);
                float sp, cp;
                pt_sincosf(phi, &sp, &cp);
                next = normalize(add(add(scale(scale(uu, cp), sin_t), scale(scale(vv, sp), sin_t)),
                                     scale(w, cos_t)));
                point = add(hitp, scale(w, 0.01f));
                mask = mul(mask, f);
            } else if (rt == kSpecular) {
                next = mirror;
                point = add(hitp, scale(oriented, 0.01f));
                mask = mul(mask, f);
            } else if (rt == kCoat) {
                if (rng.next() < 0.05f) {
                    mask = mul(mask, v3{1.0f, 1.0f, 1.0f});
                    next = mirror;
                    point = add(hitp, scale(oriented, 0.01f));
                } else {
                    const float r1 = kPtTwoPi * rng.next();
                    const float r2 = rng.next();
                    next = hemisphere(normalize(oriented), r1, r2);
                    point = add(hitp, scale(oriented, 0.01f));
                    mask = mul(mask, f);
                }
            } else {  // kRefraction (CUDAPathTracer.cu:566-614)
                const bool into = dot(normal, oriented) > 0.0f;
                const float nc = 1.0f, nt = 1.5f;
                const float nnt = into ? nc / nt : nt / nc;
                const float ddn = dot(d, oriented);
                const float cos2t = 1.0f - nnt * nnt * (1.0f - ddn * ddn);
                if (cos2t < 0.0f) {
                    next = mirror;
                    point = add(hitp, scale(oriented, 0.01f));
                } else {
                    v3 tdir = scale(d, nnt);
                    tdir = sub(tdir, scale(normal, (float)(into ? 1 : -1) * (ddn * nnt + fsqrt(cos2t))));
                    tdir = normalize(tdir);
                    const float R0 = (nt - nc) * (nt - nc) / (nt + nc) * (nt + nc);  // sic
                    const float cc = 1.0f - (into ? -ddn : dot(tdir, normal));
                    const float Re = R0 + (1.0f - R0) * cc * cc * cc * cc * cc;
                    const float Tr = 1.0f - Re;
                    const float P = 0.25f + 0.5f * Re;
                    const float RP = fdiv(Re, P), TP = fdiv(Tr, 1.0f - P);
                    if (rng.next() < 0.25f) {
                        mask = scale(mask, RP);
                        next = mirror;
                        point = add(hitp, scale(oriented, 0.01f));
                    } else {
                        mask = scale(mask, TP);
                        next = tdir;
                        point = add(hitp, scale(oriented, 0.001f));
                    }
                }
            }
            o = point;
            d = next;
            if (++bounce == L.max_depth) {  // 5 in the reference (CUDAPathTracer.cu:366)
                done = true;
                contrib = accu;
            }
        }
        if (done) {
            sum = add(sum, contrib);
            need_cam = true;
            s += SP;
            if (s >= L.spp) {  // (pathTrace launches run one sub-stream per work item: grp_log2 = 0)
                alive = false;
                if (kQueue) store_partial(L, item, sum);
            }
        }
    }

    if (!kQueue && SP > 1) {
        const int base = lane - c;
        v3 acc = sum;
        for (int j = 1; j < SP; ++j) {
            v3 pj{lane_read(sum.x, base + j), lane_read(sum.y, base + j), lane_read(sum.z, base + j)};
            acc = add(acc, pj);
        }
        sum = acc;
    }
    if (!kQueue && valid && c == 0) {
        const float fs = (float)L.spp;
        write_pixel(L, out, ((size_t)lrow * (size_t)L.cols + (size_t)(px - L.col0)) * 3, sum, fs);
    }
    const uint64_t ws = cnt.segs;
    const uint64_t wt = wave_sum_u64(cnt.tri_tests);
    const uint64_t wn = wave_sum_u64(cnt.node_visits);
    if (lane == 0) {
        atomicAdd(&counters[0], (unsigned long long)ws);
        atomicAdd(&counters[1], (unsigned long long)wt);
        if (wn) atomicAdd(&counters[3], (unsigned long long)wn);
    }
}

// Dynamic LDS of a traversal kernel: the per-lane stacks of the block's `bw` waves.
// `spare`: one more slot per lane past the stack (the render kernels' traversals push there unconditionally)
static size_t stack_bytes(const RenderLaunch& L, int bw, int spare = 0) {
    return (size_t)bw * (size_t)((L.stack_depth > 0 ? L.stack_depth : 1) + spare) * 64 * sizeof(uint32_t);
}

hipError_t launch_pathtrace(const PtSceneArgs& sc, const CamRec* cam, const RenderLaunch& L,
                            float* out, unsigned long long* counters, hipStream_t stream, hipEvent_t main_done) {
    if (L.queue) {
        if (L.n_items == 0) return main_done ? hipEventRecord(main_done, stream) : hipSuccess;
        const uint32_t waves = (L.n_qitems + 63u) / 64u;  // the queue's items (grp_log2 = 0 here)
        const uint32_t blocks = std::min<uint32_t>((waves + kQueueBlockWaves - 1) / kQueueBlockWaves,
                                                   (uint32_t)L.queue);
        hipLaunchKernelGGL(pathtrace_kernel<true>, dim3(blocks), dim3(64 * kQueueBlockWaves),
                           stack_bytes(L, kQueueBlockWaves), stream, L, sc.ktris, sc.nodes, cam, out,
                           counters);
        if (main_done) (void)hipEventRecord(main_done, stream);
        const uint32_t pixels = L.n_items / (uint32_t)L.lanes_per_pixel;
        hipLaunchKernelGGL(combine_kernel, dim3((pixels + 255u) / 256u), dim3(256), 0, stream, L, out);
        return hipGetLastError();
    }
    dim3 grid((L.cols + 2 * L.tile_w - 1) / (2 * L.tile_w),
              (L.local_rows + 2 * L.tile_h - 1) / (2 * L.tile_h));
    if (grid.x == 0 || grid.y == 0) return main_done ? hipEventRecord(main_done, stream) : hipSuccess;
    hipLaunchKernelGGL(pathtrace_kernel<false>, grid, dim3(64 * kWavesPerBlock), stack_bytes(L, kWavesPerBlock),
                       stream, L, sc.ktris, sc.nodes, cam, out, counters);
    if (main_done) (void)hipEventRecord(main_done, stream);
    return hipGetLastError();
}

// A persistent grid fills the resident waves: waves per SIMD x 4 SIMDs per CU, in blocks of
// kQueueBlockWaves, capped by what fits the CU's 160 KB of LDS (the variant's static tables + the
// launch's traversal stacks): blocks beyond it would only start once others retire, after the queue
// ran dry.
int queue_blocks(int n_cu, uint32_t variant, const RenderLaunch& L) {
    const int waves = variant_waves(variant), bw = kQueueBlockWaves;
    size_t lds = 0;
    switch (variant) {
        case RT_VARIANT_PATHTRACE_QUEUE: case RT_VARIANT_PATHTRACE_STATIC:
            lds = (size_t)bw * 64 * (8 + 4 + 4 * 4) + stack_bytes(L, bw);
            break;
        case RT_VARIANT_SCAN_QUEUE: case RT_VARIANT_SCAN_STATIC: case RT_VARIANT_SCAN_MEDIA_QUEUE:
        case RT_VARIANT_SCAN_MEDIA_STATIC: case RT_VARIANT_SCAN_SIMPLE_QUEUE: case RT_VARIANT_SCAN_SIMPLE_STATIC:
            lds = (size_t)bw * (sizeof(WaveLds) + sizeof(CamSlots));
            break;
        case RT_VARIANT_BVH_MESH_QUEUE: case RT_VARIANT_BVH_MESH_SIMPLE_QUEUE:  // kParts = 1: the slim tables
            lds = (size_t)bw * sizeof(WaveLdsCore) + stack_bytes(L, bw, stack_spare<1>());
            break;
        default:
            lds = (size_t)bw * sizeof(WaveLds) + stack_bytes(L, bw, stack_spare<3>());
            // the sphere-group-only kernel also keeps its resumed traversals' state
            if (variant == RT_VARIANT_BVH_GROUP_QUEUE) lds += (size_t)bw * sizeof(GroupLds);
    }
    const int fit = (int)((size_t)160 * 1024 / (lds ? lds : 1));
    return n_cu * std::max(1, std::min(4 * waves / bw, fit));
}

// The instantiation a launch runs (rtmi.h RT_VARIANT_*). This is the only place that maps
// scene content + schedule to a kernel: launch_render / launch_pathtrace dispatch on the id,
// the queue grid is sized with variant_waves(id), and rt_render_stats.variant reports it.
uint32_t select_variant(bool pathtrace, bool queue, bool bvh, bool media, bool full, int bvh_parts) {
    if (pathtrace) return queue ? RT_VARIANT_PATHTRACE_QUEUE : RT_VARIANT_PATHTRACE_STATIC;
    if (!queue) {
        if (bvh) return RT_VARIANT_BVH_STATIC;
        if (media) return RT_VARIANT_SCAN_MEDIA_STATIC;
        if (!full) return RT_VARIANT_SCAN_SIMPLE_STATIC;
        return RT_VARIANT_SCAN_STATIC;
    }
    if (bvh && bvh_parts == 1 && !full && !media)
        return RT_VARIANT_BVH_MESH_SIMPLE_QUEUE;
    if (bvh && bvh_parts == 1) return RT_VARIANT_BVH_MESH_QUEUE;
    // the sphere-group-only kernel resumes a traversal in the next loop trip, re-scanning the objects
    // before the group: a medium there would draw again from the ray's stream, so scenes
    // with media take the general BVH kernel, which traverses each group in one pass
    if (bvh && bvh_parts == 2 && !media) return RT_VARIANT_BVH_GROUP_QUEUE;
    if (bvh) return RT_VARIANT_BVH_QUEUE;
    if (media) return RT_VARIANT_SCAN_MEDIA_QUEUE;
    if (!full) return RT_VARIANT_SCAN_SIMPLE_QUEUE;
    return RT_VARIANT_SCAN_QUEUE;
}

// Occupancy each instantiation is compiled for (waves per SIMD).
int variant_waves(uint32_t v) {
    switch (v) {
        case RT_VARIANT_SCAN_QUEUE: case RT_VARIANT_SCAN_STATIC: return render_waves<false>();
        case RT_VARIANT_SCAN_MEDIA_QUEUE: case RT_VARIANT_SCAN_MEDIA_STATIC: return render_waves<false, true>();
        case RT_VARIANT_SCAN_SIMPLE_QUEUE: case RT_VARIANT_SCAN_SIMPLE_STATIC: return render_waves<false, false, false>();
        case RT_VARIANT_BVH_QUEUE: case RT_VARIANT_BVH_STATIC: return render_waves<true>();
        case RT_VARIANT_BVH_MESH_QUEUE: return render_waves<true, false, true, 1>();
        case RT_VARIANT_BVH_MESH_SIMPLE_QUEUE: return render_waves<true, false, false, 1>();
        case RT_VARIANT_BVH_GROUP_QUEUE: return render_waves<true, false, true, 2>();
        case RT_VARIANT_PATHTRACE_QUEUE: case RT_VARIANT_PATHTRACE_STATIC: return RT_PT_WAVES;
        default: return 4;
    }
}

// The instantiation's symbol as rocprofv3 prints it (template arguments spelled out, the
// defaults included), so a profile can be matched to the variant a launch reported.
const char* variant_name(uint32_t v) {
    switch (v) {
        case RT_VARIANT_SCAN_QUEUE: return "render_kernel<false, true, false, true, 3>";
        case RT_VARIANT_SCAN_MEDIA_QUEUE: return "render_kernel<false, true, true, true, 3>";
        case RT_VARIANT_SCAN_SIMPLE_QUEUE: return "render_kernel<false, true, false, false, 3>";
        case RT_VARIANT_BVH_QUEUE: return "render_kernel<true, true, false, true, 3>";
        case RT_VARIANT_BVH_MESH_QUEUE: return "render_kernel<true, true, false, true, 1>";
        case RT_VARIANT_BVH_MESH_SIMPLE_QUEUE: return "render_kernel<true, true, false, false, 1>";
        case RT_VARIANT_BVH_GROUP_QUEUE: return "render_kernel<true, true, false, true, 2>";
        case RT_VARIANT_SCAN_STATIC: return "render_kernel<false, false, false, true, 3>";
        case RT_VARIANT_SCAN_MEDIA_STATIC: return "render_kernel<false, false, true, true, 3>";
        case RT_VARIANT_SCAN_SIMPLE_STATIC: return "render_kernel<false, false, false, false, 3>";
        case RT_VARIANT_BVH_STATIC: return "render_kernel<true, false, false, true, 3>";
        case RT_VARIANT_PATHTRACE_QUEUE: return "pathtrace_kernel<true>";
        case RT_VARIANT_PATHTRACE_STATIC: return "pathtrace_kernel<false>";
        default: return nullptr;
    }
}

// rtmi.h RT_BUILD_*: which non-shipped options this translation unit (and, through
// the shared EXTRA flags, the whole library) was compiled with.
uint32_t kernel_build_flags() {
    uint32_t f = 0;
#if defined(RT_ABL_FASTMATH) || defined(RT_ABL_NOREJECT) || defined(RT_ABL_FLOATLOG) || RT_ABL_PHILOX_ROUNDS != 10 || \
    defined(RT_XOSHIRO_SS)
    f |= 1u;  // RT_BUILD_ABLATION: results differ from the restatement
#endif
#ifdef RT_STAMPS
    f |= 2u;  // RT_BUILD_STAMPS
#endif
// the remaining knobs: occupancies, the queue's schedule and the numeric thresholds
#if defined(RT_QUEUE_REFILL) || RT_QUEUE_SHARDS != 8 || RT_QUEUE_BLOCK_WAVES != 4 || RT_CAM_BATCH != 32 || \
    defined(RT_WAVES_PER_EU) || RT_BVH_WAVES != 4 || RT_SCAN_WAVES != 6 || RT_MED_WAVES != 6 || RT_NOSPH_WAVES != 7 || \
    RT_GROUP_WAVES != 5 || RT_BVH_SIMPLE_WAVES != 6 || RT_BVH_MESH_WAVES != 5 || RT_PT_WAVES != 6 || \
    RT_GROUP_MIN_TRIPS != 4 || RT_GROUP_EXIT_LANES != 8 || RT_BATCH_MIN != 64 || RT_GROUP_BATCH_MIN != 64 || \
    RT_PT_BATCH_MIN != 64 || RT_DEFER_MIN != 32 || defined(RT_U01_MULADD)
    f |= 4u;  // RT_BUILD_AB: same results, not the shipped schedule
#endif
#if (defined(RT_FIF_ITEMS) && RT_FIF_ITEMS != 16) || (defined(RT_FIF_GROUPS) && RT_FIF_GROUPS != 1)
    f |= 4u;  // (host-side layout switches of rt_capi.cpp, passed to every TU through EXTRA)
#endif
    return f;
}

namespace {
template <bool kBvh, bool kQueue, bool kMed = false, bool kSph = true, int kParts = 3>
void launch_rk(dim3 grid, dim3 block, size_t lds, hipStream_t stream, const RenderLaunch& L, const SceneArgs& sc,
               const CamRec* cam, float* out, unsigned long long* counters) {
    hipLaunchKernelGGL((render_kernel<kBvh, kQueue, kMed, kSph, kParts>), grid, block, kBvh ? lds : 0, stream, L,
                       sc.objs, sc.tris, sc.mats, sc.nodes, sc.tri_orig, sc.n_objs, cam, out, counters);
}
}  // namespace

hipError_t launch_render(uint32_t variant, const SceneArgs& sc, const CamRec* cam, const RenderLaunch& L, float* out,
                         unsigned long long* counters, hipStream_t stream, hipEvent_t main_done) {
    const int bw = block_waves(L.queue != 0);
    const dim3 block(64 * bw);
    const bool slim = variant == RT_VARIANT_BVH_MESH_QUEUE || variant == RT_VARIANT_BVH_MESH_SIMPLE_QUEUE;
    const size_t lds = stack_bytes(L, bw, slim ? stack_spare<1>() : stack_spare<3>());
    dim3 grid;
    if (L.queue) {
        if (L.n_items == 0) return main_done ? hipEventRecord(main_done, stream) : hipSuccess;
        // what the queue hands out: groups of 2^grp_log2 sub-streams
        const uint32_t waves_needed = (L.n_qitems + 63u) / 64u;
        grid = dim3(std::min<uint32_t>((waves_needed + bw - 1) / bw, (uint32_t)L.queue), 1);
    } else {
        grid = dim3((L.cols + 2 * L.tile_w - 1) / (2 * L.tile_w), (L.local_rows + 2 * L.tile_h - 1) / (2 * L.tile_h));
        if (grid.x == 0 || grid.y == 0) return main_done ? hipEventRecord(main_done, stream) : hipSuccess;
    }
    switch (variant) {
        case RT_VARIANT_BVH_MESH_SIMPLE_QUEUE:
            launch_rk<true, true, false, false, 1>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_BVH_MESH_QUEUE:
            launch_rk<true, true, false, true, 1>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_BVH_GROUP_QUEUE:
            launch_rk<true, true, false, true, 2>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_BVH_QUEUE: launch_rk<true, true>(grid, block, lds, stream, L, sc, cam, out, counters); break;
        case RT_VARIANT_SCAN_MEDIA_QUEUE:
            launch_rk<false, true, true>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_SCAN_SIMPLE_QUEUE:
            launch_rk<false, true, false, false>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_SCAN_QUEUE: launch_rk<false, true>(grid, block, lds, stream, L, sc, cam, out, counters); break;
        case RT_VARIANT_BVH_STATIC: launch_rk<true, false>(grid, block, lds, stream, L, sc, cam, out, counters); break;
        case RT_VARIANT_SCAN_MEDIA_STATIC:
            launch_rk<false, false, true>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_SCAN_SIMPLE_STATIC:
            launch_rk<false, false, false, false>(grid, block, lds, stream, L, sc, cam, out, counters);
            break;
        case RT_VARIANT_SCAN_STATIC: launch_rk<false, false>(grid, block, lds, stream, L, sc, cam, out, counters); break;
        default: return hipErrorInvalidValue;
    }
    if (main_done) (void)hipEventRecord(main_done, stream);
    if (L.queue) {
        const uint32_t pixels = L.n_items / (uint32_t)L.lanes_per_pixel;
        hipLaunchKernelGGL(combine_kernel, dim3((pixels + 255u) / 256u), dim3(256), 0, stream, L, out);
    }
    return hipGetLastError();
}

}  // namespace rt
