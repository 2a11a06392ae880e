// div_check.hip — GPU check of a shared-reciprocal, correctly rounded division
// (v_rcp_f32 + one Newton step + Markstein's correction) measured as a replacement for
// the kernels' IEEE a / b (bit-identical, but slower there, not shipped).
//
//  1. exhaustive: for every float b with 2^-126 <= |b| < 2^126 (every mantissa of every
//     binade, both signs), y1 = fma(fma(-b, y0, 1), y0, y0) with y0 = v_rcp_f32(b) must equal the
//     correctly rounded 1 / b (IEEE division);
//  2. random: N pseudo-random (a, b) pairs, |a|, |b| in [2^-100, 2^101), |a/b| in [2^-121, 2^125):
//     q1 = fma(fma(-b, q0, a), y1, q0), q0 = a * y1, must equal a / b.
// Prints one JSON line; any mismatch is listed (first 8).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ float rcp_nr(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

__device__ __forceinline__ float div_r(float a, float b, float y1) {
    const float q0 = a * y1;
    const float r = __builtin_fmaf(-b, q0, a);
    return __builtin_fmaf(r, y1, q0);
}

__device__ unsigned long long g_bad[2];
__device__ uint32_t g_first[16];

__global__ void recip_all(int exp_off, int sign) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const uint32_t bits = ((uint32_t)sign << 31) | ((uint32_t)(127 + exp_off) << 23) | m;
    const float b = __uint_as_float(bits);
    const float y1 = rcp_nr(b);
    const float ref = 1.0f / b;
    if (__float_as_uint(y1) != __float_as_uint(ref)) {
        const unsigned long long k = atomicAdd(&g_bad[0], 1ull);
        if (k < 8) g_first[k] = bits;
    }
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void div_random(uint32_t seed, int emax) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h1 = mix(i * 2u + seed), h2 = mix(i * 2u + 1u + seed * 0x9E3779B9u);
    const uint32_t h3 = mix(h1 ^ h2);
    // exponents in [-emax, emax], full random mantissas and signs; pairs outside div_rn's
    // domain (|a/b| in [2^-121, 2^125)) are skipped
    const int ea = (int)(h3 % (uint32_t)(2 * emax + 1)) - emax;
    const int eb = (int)((h3 >> 16) % (uint32_t)(2 * emax + 1)) - emax;
    if (ea - eb < -120 || ea - eb > 124) return;
    const float a = __uint_as_float((h1 & 0x80000000u) | ((uint32_t)(127 + ea) << 23) | (h1 & 0x7FFFFFu));
    const float b = __uint_as_float((h2 & 0x80000000u) | ((uint32_t)(127 + eb) << 23) | (h2 & 0x7FFFFFu));
    const float q = div_r(a, b, rcp_nr(b));
    const float ref = a / b;
    if (__float_as_uint(q) != __float_as_uint(ref)) {
        const unsigned long long k = atomicAdd(&g_bad[1], 1ull);
        if (k < 4) {
            g_first[8 + 2 * k] = __float_as_uint(a);
            g_first[9 + 2 * k] = __float_as_uint(b);
        }
    }
}

int main(int argc, char** argv) {
    const int batches = argc > 1 ? atoi(argv[1]) : 64;  // x 2^24 random pairs
    // every binade of the guarded domain 2^-126 <= |b| < 2^126 , both signs
    int n_exp = 0;
    for (int e = -126; e < 126; ++e, ++n_exp)
        for (int s = 0; s < 2; ++s) recip_all<<<(1u << 23) / 256, 256>>>(e, s);
    for (int k = 0; k < batches; ++k) div_random<<<(1u << 24) / 256, 256>>>(0x1234u + (uint32_t)k, 100);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("{\"error\": \"kernel failed\"}\n");
        return 1;
    }
    unsigned long long bad[2];
    uint32_t first[16];
    (void)hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof bad);
    (void)hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof first);
    printf("{\"recip_checked\": %llu, \"recip_bad\": %llu, \"div_pairs_drawn\": %llu, \"div_bad\": %llu, \"first\": [",
           (unsigned long long)n_exp * 2ull * (1ull << 23), bad[0],
           (unsigned long long)batches << 24, bad[1]);
    for (int k = 0; k < 16; ++k) printf("%s\"%08x\"", k ? ", " : "", first[k]);
    printf("]}\n");
    return (bad[0] || bad[1]) ? 2 : 0;
}
