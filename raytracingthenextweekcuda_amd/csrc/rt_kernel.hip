// rt_kernel.hip — the per-pixel path-tracing megakernel for gfx950 (MI355X).
//
// Replaces renderKernel (main.cu:160-206) + rayColor (main.cu:63-94) + hit
// (main.cu:43-57) + the Hitable/Material virtual calls (Sphere.cu, Plane.cu,
// Cube.cu, TriangleMesh.cu, AABBox.h, Material.h/.cu) + Camera::getRay
// (Camera.h:151-168) + cuRAND (main.cu:120-129) with one hand-written kernel.
//
// Execution model:
//  * one lane = one pixel; a 256-thread workgroup covers a 16x16 pixel tile,
//    each wave64 an 8x8 sub-tile (spatially coherent rays share scene records);
//  * path regeneration: a lane whose path terminates immediately starts its
//    next sample, so lanes stay busy until the pixel's last sample instead of
//    idling for the longest path of every sample; the wave exits when its
//    ballot of live lanes is empty;
//  * scene records are read at wave-uniform addresses in the closest-hit scan
//    (scalar loads, broadcast to 64 lanes); materials per lane;
//  * stateless Philox RNG (no init kernel, no 48 B/pixel state in HBM);
//  * per-wave popcount-free counters: lane counts reduced in-wave, one 64-bit
//    atomic per wave per counter.
//
// Numerics: compiled with -ffp-contract=off and IEEE div/sqrt; every expression
// keeps the reference's evaluation order (rt_math.h), so the output is
// bit-identical to the CPU restatement in oracle/.
#include <hip/hip_runtime.h>

#include "rt_kernel.h"

namespace rt {

namespace {

constexpr float kInf = __builtin_huge_valf();

#ifndef RT_SCREEN
#define RT_SCREEN 1  // rcp-screened plane/triangle tests (exact fallback)
#endif

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

// Sphere::hit / MovingSphere::hit root selection (Sphere.cu:3-37, 39-73).
__device__ __forceinline__ bool sphere_root(v3 o, v3 d, v3 c, float r, float tmin, float tmax,
                                            float& root) {
    v3 oc = sub(o, c);
    float a = dot(d, d);
    float hb = dot(oc, d);
    float cc = dot(oc, oc) - r * r;
    float disc = hb * hb - a * cc;
    if (!(disc > kFltEpsilon)) return false;
    float inva = 1.0f / a;
    float sq = sqrtf(disc);
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

// In-rectangle test of Plane::hit for the plane's orientation.
__device__ __forceinline__ bool plane_in_range(v3 p, const float* f, uint32_t orient) {
    if (orient == 0u)
        return (p.x > f[0] - f[6]) && (p.x < f[0] + f[6]) && (p.y > f[1] - f[7]) && (p.y < f[1] + f[7]);
    if (orient == 1u)
        return (p.y > f[1] - f[7]) && (p.y < f[1] + f[7]) && (p.z > f[2] - f[8]) && (p.z < f[2] + f[8]);
    return (p.x > f[0] - f[6]) && (p.x < f[0] + f[6]) && (p.z > f[2] - f[8]) && (p.z < f[2] + f[8]);
}

// Relative slack that bounds the error of the screening arithmetic: v_rcp_f32
// is within 1 ulp, each further rounding adds 0.5 ulp, so screened values are
// within ~4 ulp (4.8e-7 relative) of the exact ones; 1e-5 leaves > 20x room.
constexpr float kScreen = 1e-5f;

// True only if the exact Plane::hit test is certain to fail.
__device__ __forceinline__ bool plane_surely_missed(float num, float den, v3 o, v3 d, v3 pos,
                                                    const float* f, uint32_t orient, float tmax) {
    const float tq = num * __builtin_amdgcn_rcpf(den);
    const float mt = fabsf(tq) * kScreen;
    if (tq + mt < kTMin || tq - mt >= tmax) return true;
    const v3 pq = add(o, scale(d, tq));
    // |p - pq| <= |d| |t| 4.8e-7 + rounding of p: covered by slack on |d||tq| and |pq|.
    auto out = [&](float pa, float da, float lo, float hi) {
        const float m = (fabsf(da) * fabsf(tq) + fabsf(pa)) * kScreen + 1e-30f;
        return (pa + m <= lo) || (pa - m >= hi);
    };
    if (orient == 0u)
        return out(pq.x, d.x, f[0] - f[6], f[0] + f[6]) || out(pq.y, d.y, f[1] - f[7], f[1] + f[7]);
    if (orient == 1u)
        return out(pq.y, d.y, f[1] - f[7], f[1] + f[7]) || out(pq.z, d.z, f[2] - f[8], f[2] + f[8]);
    return out(pq.x, d.x, f[0] - f[6], f[0] + f[6]) || out(pq.z, d.z, f[2] - f[8], f[2] + f[8]);
}

// True only if the exact TriangleMesh::hit acceptance test is certain to fail.
// NaN/inf screened values compare false and fall through to the exact path.
__device__ __forceinline__ bool tri_surely_missed(float det, float n_t, float n_b1, float n_b2,
                                                  float tmax) {
    if (!(fabsf(det) > 1e-30f)) return false;
    const float cq = __builtin_amdgcn_rcpf(det);
    const float tq = cq * n_t, b1 = cq * n_b1, b2 = cq * n_b2;
    const float mt = fabsf(tq) * kScreen;
    if (tq + mt < kTMin || tq - mt >= tmax) return true;
    const float m1 = fabsf(b1) * kScreen, m2 = fabsf(b2) * kScreen;
    if (b1 + m1 < kFltEpsilon || b2 + m2 < kFltEpsilon) return true;
    const float r = 1.0f - b1 - b2;
    return r + (m1 + m2 + 4e-7f) < kFltEpsilon;
}

struct Hit {
    float t;
    int32_t obj;   // object table index of the closest hit (-1: none)
    int32_t tri;   // triangle index for meshes
};

// hit() over the flattened object table (main.cu:43-57): closest so far is
// passed as tMax to each object, each object's own comparison rule is kept.
__device__ __forceinline__ Hit closest_hit(const ObjRec* __restrict__ objs, int n_objs,
                                           const TriRec* __restrict__ tris, const Ray& ray,
                                           v3 inv, uint32_t& tri_tests, uint32_t& box_tests) {
    Hit h{kInf, -1, -1};
    const v3 o = ray.o, d = ray.d;
    for (int i = 0; i < n_objs; ++i) {
        const uint32_t type = objs[i].type;
        const float* f = objs[i].f;
        if (type == kObjPlane) {
            // Plane::hit (Plane.cu:4-52).
            v3 n{f[3], f[4], f[5]};
            float den = dot(n, d);
            bool proceed = objs[i].u1 ? (fabsf(den) > kTMin) : (den > kTMin);
            if (proceed) {
                v3 pos{f[0], f[1], f[2]};
                float num = dot(sub(pos, o), n);
                // Screening with v_rcp_f32 (<= 1 ulp): only lanes that are not
                // clearly rejected evaluate the IEEE division, so every accepted
                // hit and every close call is decided by the exact arithmetic.
                if (!RT_SCREEN || !plane_surely_missed(num, den, o, d, pos, f, objs[i].u0, h.t)) {
                    float t = num / den;
                    v3 p = add(o, scale(d, t));
                    if ((t >= kTMin) && (t < h.t) && plane_in_range(p, f, objs[i].u0)) {
                        h.t = t;
                        h.obj = i;
                    }
                }
            }
        } else if (type == kObjSphere) {
            float t;
            if (sphere_root(o, d, v3{f[0], f[1], f[2]}, f[3], kTMin, h.t, t)) {
                h.t = t;
                h.obj = i;
            }
        } else if (type == kObjMovingSphere) {
            float t;
            if (sphere_root(o, d, moving_center(f, ray.time), f[8], kTMin, h.t, t)) {
                h.t = t;
                h.obj = i;
            }
        } else {
            // TriangleMesh::hit (TriangleMesh.cu:34-117): AABB early-out, then
            // every triangle with the strict t < closestSoFar rule.
            ++box_tests;
            if (box_hit(f, o, inv)) {
                const uint32_t b = objs[i].u0, e = b + objs[i].u1;
                tri_tests += e - b;
                for (uint32_t k = b; k < e; ++k) {
                    const TriRec& tr = tris[k];
                    v3 n{tr.nx, tr.ny, tr.nz};
                    if (dot(d, n) > kFltEpsilon) continue;  // backface cull
                    v3 e1{tr.e1x, tr.e1y, tr.e1z}, e2{tr.e2x, tr.e2y, tr.e2z};
                    v3 s = sub(o, v3{tr.v0x, tr.v0y, tr.v0z});
                    v3 s1 = cross(d, e2);
                    v3 s2 = cross(s, e1);
                    const float det = dot(s1, e1);
                    const float n_t = dot(s2, e2), n_b1 = dot(s1, s), n_b2 = dot(s2, d);
                    if (RT_SCREEN && tri_surely_missed(det, n_t, n_b1, n_b2, h.t)) continue;
                    float coef = 1.0f / det;
                    float t = coef * n_t;
                    float b1 = coef * n_b1;
                    float b2 = coef * n_b2;
                    if (((t >= kFltEpsilon) && ((t >= kTMin) && (t < h.t))) &&
                        (b1 >= kFltEpsilon) && (b2 >= kFltEpsilon) &&
                        ((1.0f - b1 - b2) >= kFltEpsilon)) {
                        h.t = t;
                        h.obj = i;
                        h.tri = (int32_t)k;
                    }
                }
            }
        }
    }
    return h;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace

__global__ __launch_bounds__(256) void render_kernel(
    const ObjRec* __restrict__ objs, const TriRec* __restrict__ tris,
    const MatRec* __restrict__ mats, int n_objs, CamRec cam, RenderLaunch L,
    float* __restrict__ out, unsigned long long* __restrict__ counters) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // Lane layout: S = lanes_per_pixel adjacent lanes share one pixel and split
    // its samples (sub-lane c takes samples c, c+S, c+2S, ...). A wave covers
    // 64/S pixels as a tw x th tile; a 4-wave workgroup covers 2tw x 2th.
    const int S = L.lanes_per_pixel;
    const int c = lane & (S - 1);
    const int pix = lane / S;
    const int tw = L.tile_w, th = L.tile_h;
    const int px = blockIdx.x * (2 * tw) + (wave & 1) * tw + (pix % tw);
    const int lrow = blockIdx.y * (2 * th) + (wave >> 1) * th + (pix / tw);
    // Row tiling: local row -> global row (y = 0 is the bottom row).
    const int lb = lrow / L.row_block;
    const int y = (lb * L.row_world + L.row_rank) * L.row_block + (lrow - lb * L.row_block);
    const bool valid = (px < L.width) && (lrow < L.local_rows) && (y < L.height);
    const uint32_t pixel = (uint32_t)y * (uint32_t)L.width + (uint32_t)px;

    v3 sum{0.0f, 0.0f, 0.0f};
    uint32_t segs = 0, tri_tests = 0, box_tests = 0;
    int s = c;
    bool alive = valid && s < L.spp;
    bool need_cam = true;
    int depth = 0;
    Ray ray{};
    v3 thr{1.0f, 1.0f, 1.0f};
    Rng rng;
    const float fw = (float)(L.width - 1), fh = (float)(L.height - 1);

    while (alive) {
        if (need_cam) {
            // renderKernel sample loop body (main.cu:179-185) + getRay (Camera.h:151-168).
            rng.begin(L.seed, pixel, L.sample_offset + (uint32_t)s);
            float rx = rng.next();
            float ry = rng.next();
            float dx = ((float)px + rx) / fw;
            float dy = ((float)y + ry) / fh;
            v3 disk = random_in_unit_disk(rng);
            v3 rnd = scale(disk, cam.lens_radius);
            v3 offset = add(scale(cam.right, rnd.x), scale(cam.true_up, rnd.y));
            v3 norig = add(cam.origin, offset);
            v3 dir = sub(add(add(cam.lower_left, scale(cam.horizontal, dx)),
                             scale(cam.vertical, dy)),
                         norig);
            dir = normalize(dir);
            float tm = random_range(rng, cam.time0, cam.time1);
            ray = Ray{add(cam.origin, offset), dir, tm};
            thr = v3{1.0f, 1.0f, 1.0f};
            depth = 0;
            need_cam = false;
            if (L.max_depth <= 0) {  // rayColor with BOUNCES = 0 returns black
                need_cam = true;
                s += S;
                if (s >= L.spp) alive = false;
                continue;
            }
        }

        const v3 inv = rcp(ray.d);
        Hit h = closest_hit(objs, n_objs, tris, ray, inv, tri_tests, box_tests);
        ++segs;

        bool done;
        v3 contrib;
        if (h.obj >= 0) {
            const ObjRec& ob = objs[h.obj];
            const float* f = ob.f;
            v3 p = add(ray.o, scale(ray.d, h.t));  // ray.at(t)
            v3 outward;
            if (ob.type == kObjPlane) {
                outward = v3{f[3], f[4], f[5]};
            } else if (ob.type == kObjSphere) {
                outward = divs(sub(p, v3{f[0], f[1], f[2]}), f[3]);
            } else if (ob.type == kObjMovingSphere) {
                outward = divs(sub(p, moving_center(f, ray.time)), f[8]);
            } else {
                const TriRec& tr = tris[h.tri];
                outward = v3{tr.nx, tr.ny, tr.nz};
            }
            // HitResult::setFaceNormal (HitResult.h:15-18).
            const bool front = dot(ray.d, outward) < kFltEpsilon;
            const v3 n = front ? outward : neg(outward);
            const MatRec m = mats[ob.material];
            v3 att;
            bool scattered;
            v3 nd;
            if (m.type == 0u) {
                // Lambertian::scatter (Material.cu:3-19).
                v3 u = normalize(random_in_unit_sphere(rng));
                v3 sd = add(n, u);
                if ((fabsf(sd.x) < 1e-8f) && (fabsf(sd.y) < 1e-8f) && (fabsf(sd.z) < 1e-8f)) sd = n;
                nd = normalize(sd);
                att = v3{m.a0, m.a1, m.a2};
                scattered = true;
            } else if (m.type == 1u) {
                // Metal::scatter (Material.h:45-51).
                v3 refl = reflect(normalize(ray.d), n);
                nd = add(refl, scale(random_in_unit_sphere(rng), m.p0));
                scattered = dot(nd, n) > 0.0f;
                att = scale(v3{m.a0, m.a1, m.a2}, scattered ? 1.0f : 0.0f);
            } else if (m.type == 2u) {
                // Dieletric::scatter + reflectance (Material.h:65-109).
                att = v3{1.0f, 1.0f, 1.0f};
                const float ratio = front ? (1.0f / m.p0) : m.p0;
                v3 ud = normalize(ray.d);
                float c = fminf(dot(neg(ud), n), 1.0f);
                float sn = sqrtf(1.0f - c * c);
                bool cannot = ratio * sn > 1.0f;
                bool refl;
                if (cannot) {
                    refl = true;
                } else {
                    float r0 = (1.0f - ratio) / (1.0f + ratio);
                    r0 = r0 * r0;
                    float R = r0 + (1.0f - r0) * pow5(1.0f - c);
                    refl = R > rng.next();
                }
                v3 dir = refl ? reflect(ud, n) : refract(ud, n, ratio);
                nd = normalize(dir);
                scattered = true;
            } else {
                // Emission::scatter (Material.h:120-123): albedo * intensity, stop.
                att = v3{m.a0, m.a1, m.a2};
                scattered = false;
                nd = ray.d;
            }
            if (scattered) {
                thr = mul(thr, att);
                ray = Ray{p, nd, ray.time};
                ++depth;
                done = depth >= L.max_depth;
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
        if (done) {
            sum = add(sum, contrib);
            need_cam = true;
            s += S;
            if (s >= L.spp) alive = false;
        }
    }

    // Fixed-order combination of the S partial sums: ((p0 + p1) + p2) + ...
    if (S > 1) {
        const int base = lane - c;
        v3 acc = sum;
        for (int j = 1; j < S; ++j) {
            v3 pj{__shfl(sum.x, base + j, 64), __shfl(sum.y, base + j, 64), __shfl(sum.z, base + j, 64)};
            acc = add(acc, pj);
        }
        sum = acc;
    }

    if (valid && c == 0) {
        const float fs = (float)L.spp;
        const size_t o = ((size_t)lrow * (size_t)L.width + (size_t)px) * 3;
        out[o + 0] = sum.x / fs;
        out[o + 1] = sum.y / fs;
        out[o + 2] = sum.z / fs;
    }

    uint64_t ws = wave_sum_u64(segs);
    uint64_t wt = wave_sum_u64(tri_tests);
    uint64_t wb = wave_sum_u64(box_tests);
    if (lane == 0) {
        atomicAdd(&counters[0], (unsigned long long)ws);
        atomicAdd(&counters[1], (unsigned long long)wt);
        atomicAdd(&counters[2], (unsigned long long)wb);
    }
}

hipError_t launch_render(const KernelScene& sc, const CamRec& cam, const RenderLaunch& L,
                         float* out, unsigned long long* counters, hipStream_t stream) {
    dim3 block(256);
    dim3 grid((L.width + 2 * L.tile_w - 1) / (2 * L.tile_w),
              (L.local_rows + 2 * L.tile_h - 1) / (2 * L.tile_h));
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    hipLaunchKernelGGL(render_kernel, grid, block, 0, stream, sc.objs, sc.tris, sc.mats,
                       sc.n_objs, cam, L, out, counters);
    return hipGetLastError();
}

}  // namespace rt
