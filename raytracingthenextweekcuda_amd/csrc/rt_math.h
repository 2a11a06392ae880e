// rt_math.h — float3 arithmetic and the counter-based RNG used by the render
// kernel and by the host-side scene preparation.
//
// Every operation keeps the reference's evaluation order so that results are
// bit-identical to a literal restatement of the reference (LinearAlgebra.h
// Vector3Df, Utils.h helpers). The whole library is compiled with
// -ffp-contract=off and IEEE division/sqrt (no fast-math), which is what makes
// host and device results identical.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define RT_HD inline
#endif

namespace rt {

constexpr float kFltEpsilon = 1.19209290e-07f;  // FLT_EPSILON (HitResult.h:16, TriangleMesh.cu:72)
constexpr float kTMin = 0.001f;                 // Math::epsilon (Constants.h:23), rayColor tMin (main.cu:69)

// IEEE division / square root. RT_ABL_FASTMATH (timing ablation builds only,
// never shipped: results differ) swaps in v_rcp_f32 / v_sqrt_f32.
#if defined(__HIP_DEVICE_COMPILE__) && defined(RT_ABL_FASTMATH)
RT_HD float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
RT_HD float fsqrt(float a) { return __builtin_amdgcn_sqrtf(a); }
#else
RT_HD float fdiv(float a, float b) { return a / b; }
RT_HD float fsqrt(float a) { return sqrtf(a); }
#endif

struct v3 {
    float x, y, z;
};

RT_HD v3 mk(float x, float y, float z) { return v3{x, y, z}; }
// Vector3Df operators (LinearAlgebra.h:26-45): component-wise, left to right.
RT_HD v3 add(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD v3 sub(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD v3 mul(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
// v * s and s * v are both evaluated as (v.x*s, v.y*s, v.z*s) (LinearAlgebra.h:35,61-63).
RT_HD v3 scale(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
RT_HD v3 divs(v3 a, float s) { return v3{fdiv(a.x, s), fdiv(a.y, s), fdiv(a.z, s)}; }
RT_HD v3 neg(v3 a) { return v3{-a.x, -a.y, -a.z}; }
// float + Vector3Df -> (b.x + a, ...) (LinearAlgebra.h:65-67, 39).
RT_HD v3 adds(v3 a, float s) { return v3{a.x + s, a.y + s, a.z + s}; }
RT_HD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RT_HD float lengthsq(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
RT_HD v3 cross(v3 a, v3 b) {
    return v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// normalize(v): norm = sqrtf(x*x+y*y+z*z); (x/norm, y/norm, z/norm) (LinearAlgebra.h:69-72).
RT_HD v3 normalize(v3 a) {
    float n = fsqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return v3{fdiv(a.x, n), fdiv(a.y, n), fdiv(a.z, n)};
}
RT_HD v3 rcp(v3 a) { return v3{fdiv(1.0f, a.x), fdiv(1.0f, a.y), fdiv(1.0f, a.z)}; }
RT_HD float minf_(float a, float b) { return a < b ? a : b; }
RT_HD float maxf_(float a, float b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------
// RNG, replacing cuRAND XORWOW (curand_init main.cu:127, curand_uniform
// Utils.h:44-51). Counter-based at sample granularity: Philox4x32-10 (Salmon
// et al., SC'11; Random123 constants) with key = (seed, pixel) and counter =
// (sample, 0, 0, 0) yields 128 bits that seed a xoshiro128+ 1.0 stream
// (Blackman & Vigna) for that sample's draws. Every (pixel, sample) stream is
// random-access and independent of launch geometry; a draw costs 8 full-rate
// integer ops, so divergent call sites (rejection loops) stay cheap. Uniforms
// use curand's (0, 1] mapping x * 2^-32 + 2^-33, which keeps the output's upper 24
// bits - the bits the authors recommend xoshiro128+ for (float generation). Round 5
// replaced xoshiro128** (whose output scrambler, rotl(s1 * 5, 7) * 9, cost three more
// instructions per draw; RT_XOSHIRO_SS keeps it for A/B timing builds, which then
// no longer match the restatement).
// ---------------------------------------------------------------------------
constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;

struct u4 {
    uint32_t x, y, z, w;
};

RT_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

// a ^ b ^ c as one gfx950 v_bitop3_b32 (truth table 0x96); the compiler leaves such chains as two-input xors
// (in xoshiro's update because a two-input term is shared, in Philox's round because a key is a scalar)
RT_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a ^ b ^ c;
#endif
}
// the same with a wave-uniform third operand, read from its SGPR (Philox's k0 = the launch seed)
RT_HD uint32_t xor3_uniform(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(__builtin_amdgcn_readfirstlane(k)));
    return r;
#else
    return a ^ b ^ k;
#endif
}

RT_HD u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIPCC__)
#pragma unroll
#endif
#ifndef RT_ABL_PHILOX_ROUNDS
#define RT_ABL_PHILOX_ROUNDS 10  // ablation builds only
#endif
    for (int r = 0; r < RT_ABL_PHILOX_ROUNDS; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(kPhiloxM0, c.x, hi0, lo0);
        mulhilo(kPhiloxM1, c.z, hi1, lo1);
#if defined(__HIP_DEVICE_COMPILE__)
        c = u4{xor3_uniform(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
#else
        c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
#endif
        k0 += kPhiloxW0;
        k1 += kPhiloxW1;
    }
    return c;
}

// curand's _curand_uniform: x * CURAND_2POW32_INV + CURAND_2POW32_INV/2 -> (0, 1].
RT_HD float u01(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RT_U01_MULADD)  // RT_U01_MULADD: A/B builds only
    // RN(RN(x) 2^-32 + 2^-33) = RN(RN(x) + 0.5) 2^-32 (power-of-two scaling commutes with
    // rounding; no subnormals): the same bits from an add with the inline constant 0.5 and
    // an exact ldexp, with no 32-bit literal constants to keep in registers
    return __builtin_ldexpf((float)x + 0.5f, -32);
#else
    const float inv = 2.3283064e-10f;  // 2^-32
    return (float)x * inv + (inv / 2.0f);
#endif
}

RT_HD uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

// Per-lane stream state (4 registers).
struct Rng {
    uint32_t s0, s1, s2, s3;

    RT_HD void begin(uint32_t seed, uint32_t pixel, uint32_t sample) {
        u4 b = philox4x32_10(u4{sample, 0u, 0u, 0u}, seed, pixel);
        s0 = b.x;
        s1 = b.y;
        s2 = b.z;
        s3 = b.w;
        if ((s0 | s1 | s2 | s3) == 0u) s0 = kPhiloxW0;  // xoshiro's all-zero state is invalid
    }
    RT_HD uint32_t next_u32() {
#ifdef RT_XOSHIRO_SS
        const uint32_t r = rotl32(s1 * 5u, 7) * 9u;
#else
        const uint32_t r = s0 + s3;
#endif
        // s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t (t = s1 << 9); s3 = rotl(s3, 11)
        const uint32_t t = s1 << 9, s3a = s3 ^ s1;
        const uint32_t n1 = xor3(s1, s2, s0), n2 = xor3(s2, s0, t);
        s0 ^= s3a;
        s1 = n1;
        s2 = n2;
        s3 = rotl32(s3a, 11);
        return r;
    }
    RT_HD float next() { return u01(next_u32()); }
};

// Utils::random(min,max) = min + (max - min) * u (Utils.h:49-51).
RT_HD float random_range(Rng& r, float lo, float hi) { return lo + (hi - lo) * r.next(); }

// 2u - 1 for the next draw u = RN(RN(x) 2^-32 + 2^-33) (u01). Scaling by 2 is exact,
// so 2u = RN(RN(x) 2^-31 + 2^-32), and since RN(x) 2^-31 is exact that is one FMA:
// the same bits as (u * 2) + (-1) and as -1 + (1 - -1) * u, in fewer instructions.
RT_HD float two_u_minus_one(Rng& r) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmaf((float)r.next_u32(), 4.6566129e-10f /* 2^-31 */, 2.3283064e-10f /* 2^-32 */) + -1.0f;
#else
    return r.next() * 2.0f + -1.0f;
#endif
}

// randomInUnitSphere (Utils.h:69-78): x, y, z drawn in order, each 2u + (-1)
// (randomVector(min,max) = min + (max-min)*v, Utils.h:64-66 -> v*(2) + (-1)).
RT_HD v3 random_in_unit_sphere(Rng& r) {
    for (;;) {
        const float px = two_u_minus_one(r);
        const float py = two_u_minus_one(r);
        const float pz = two_u_minus_one(r);
        v3 p{px, py, pz};
#ifndef RT_ABL_NOREJECT  // timing ablation builds only (results differ)
        if (lengthsq(p) >= 1.0f) continue;
#endif
        return p;
    }
}

// randomInUnitDisk (Utils.h:96-104). The reference's argument evaluation order
// is unspecified; this build pins x before y.
RT_HD v3 random_in_unit_disk(Rng& r) {
    for (;;) {
        // random_range(r, -1, 1) = -1 + 2u: the same bits as 2u + (-1)
        float x = two_u_minus_one(r);
        float y = two_u_minus_one(r);
        v3 p = v3{x, y, 0.0f};
        if (lengthsq(p) >= 1.0f) continue;
        return p;
    }
}

// reflect (Utils.h:112-114): v - 2*dot(v,n)*n, i.e. v - n*((2*dot(v,n))).
RT_HD v3 reflect(v3 v, v3 n) { return sub(v, scale(n, 2.0f * dot(v, n))); }

// refract (Utils.h:116-121).
RT_HD v3 refract(v3 uv, v3 n, float eta) {
    float c = fminf(dot(neg(uv), n), 1.0f);
    v3 perp = scale(add(uv, scale(n, c)), eta);
    v3 par = scale(n, -sqrtf(fabsf(1.0f - lengthsq(perp))));
    return add(perp, par);
}

// pow(x, 5.0f) in Dieletric::reflectance (Material.h:108). The reference
// compiled it with --use_fast_math (__powf); this build evaluates the exact
// product chain ((x*x)*(x*x))*x on host and device alike.
RT_HD float pow5(float x) {
    float x2 = x * x;
    return (x2 * x2) * x;
}

// ---------------------------------------------------------------------------
// Transcendentals of the pathTrace integrator: cosf/sinf/powf at
// CUDAPathTracer.cu:468,486,496,553 (the reference built them with
// --use_fast_math, i.e. __cosf/__sinf/__powf, which are not reproducible).
// Here they are evaluated in IEEE double with fixed polynomial kernels and
// exact frexp/ldexp, so host and device produce the same bits; results are
// within ~1 ulp of the correctly rounded float functions.
// ---------------------------------------------------------------------------
#if defined(__HIPCC__)
#define RT_HD_NOINLINE __host__ __device__
#else
#define RT_HD_NOINLINE static
#endif

// sin / cos of x (|x| up to ~1e6): Cody-Waite reduction by pi/2, Taylor
// polynomials to degree 17 / 16 on [-pi/4, pi/4].
RT_HD void sincos_d(double x, double* s, double* c) {
    const double two_over_pi = 0.63661977236758134308;
    const double pio2_hi = 1.57079632673412561417;      // first 33 bits of pi/2
    const double pio2_lo = 6.07710050650619224932e-11;  // pi/2 - pio2_hi
    const double k = floor(x * two_over_pi + 0.5);
    const double r = (x - k * pio2_hi) - k * pio2_lo;
    const double r2 = r * r;
    double ps = 1.0 / 355687428096000.0;                 // 1/17!
    ps = ps * r2 - 1.0 / 1307674368000.0;                // 1/15!
    ps = ps * r2 + 1.0 / 6227020800.0;
    ps = ps * r2 - 1.0 / 39916800.0;
    ps = ps * r2 + 1.0 / 362880.0;
    ps = ps * r2 - 1.0 / 5040.0;
    ps = ps * r2 + 1.0 / 120.0;
    ps = ps * r2 - 1.0 / 6.0;
    const double sn = r + (r * r2) * ps;
    double pc = 1.0 / 20922789888000.0;                  // 1/16!
    pc = pc * r2 - 1.0 / 87178291200.0;
    pc = pc * r2 + 1.0 / 479001600.0;
    pc = pc * r2 - 1.0 / 3628800.0;
    pc = pc * r2 + 1.0 / 40320.0;
    pc = pc * r2 - 1.0 / 720.0;
    pc = pc * r2 + 1.0 / 24.0;
    pc = pc * r2 - 0.5;
    const double cs = 1.0 + r2 * pc;
    const long q = ((long)k) & 3;
    *s = q == 0 ? sn : q == 1 ? cs : q == 2 ? -sn : -cs;
    *c = q == 0 ? cs : q == 1 ? -sn : q == 2 ? -cs : sn;
}

RT_HD float pt_sinf(float x) {
    double s, c;
    sincos_d((double)x, &s, &c);
    return (float)s;
}
RT_HD float pt_cosf(float x) {
    double s, c;
    sincos_d((double)x, &s, &c);
    return (float)c;
}

// x^y for x >= 0 (powf at CUDAPathTracer.cu:486): exp(y * ln x) with an atanh
// series for ln on [sqrt(1/2), sqrt(2)) and a Taylor exp after reduction by ln 2.
// sinf and cosf of one argument from one reduction (same values as pt_sinf / pt_cosf).
RT_HD void pt_sincosf(float x, float* sf, float* cf) {
    double s, c;
    sincos_d((double)x, &s, &c);
    *sf = (float)s;
    *cf = (float)c;
}

// ln x for a positive float x, in double: exact frexp split, atanh series on
// [sqrt(1/2), sqrt(2)), ln 2 in two parts.
RT_HD double ln_pos_d(float xf) {
    int e;
    double m = frexp((double)xf, &e);  // exact: m in [0.5, 1)
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e = e - 1;
    }
    const double t = (m - 1.0) / (m + 1.0), t2 = t * t;
    double p = 1.0 / 23.0;
    p = p * t2 + 1.0 / 21.0;
    p = p * t2 + 1.0 / 19.0;
    p = p * t2 + 1.0 / 17.0;
    p = p * t2 + 1.0 / 15.0;
    p = p * t2 + 1.0 / 13.0;
    p = p * t2 + 1.0 / 11.0;
    p = p * t2 + 1.0 / 9.0;
    p = p * t2 + 1.0 / 7.0;
    p = p * t2 + 1.0 / 5.0;
    p = p * t2 + 1.0 / 3.0;
    p = p * t2 + 1.0;
    const double ln_m = 2.0 * t * p;
    const double de = (double)e;
    return (de * 6.93147180369123816490e-01 + ln_m) + de * 1.90821492927058770002e-10;  // ln 2 hi, lo
}

RT_HD float pt_powf(float xf, float yf) {
    if (!(xf > 0.0f)) return xf == 0.0f ? (yf > 0.0f ? 0.0f : 1.0f) : __builtin_nanf("");
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double lnx = ln_pos_d(xf);
    const double z = (double)yf * lnx;
    const double n = floor(z * 1.44269504088896338700 + 0.5);
    const double r = (z - n * ln2_hi) - n * ln2_lo;
    double q = 1.0 / 6227020800.0;  // 1/13!
    q = q * r + 1.0 / 479001600.0;
    q = q * r + 1.0 / 39916800.0;
    q = q * r + 1.0 / 3628800.0;
    q = q * r + 1.0 / 362880.0;
    q = q * r + 1.0 / 40320.0;
    q = q * r + 1.0 / 5040.0;
    q = q * r + 1.0 / 720.0;
    q = q * r + 1.0 / 120.0;
    q = q * r + 1.0 / 24.0;
    q = q * r + 1.0 / 6.0;
    q = q * r + 0.5;
    q = q * r + 1.0;
    q = q * r + 1.0;
    return (float)ldexp(q, (int)n);
}

}  // namespace rt
