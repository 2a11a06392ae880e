// tools/valu_probe.hip — calibration of the VALU-issue roofline.
//
// A kernel whose VALU work is known exactly: each wave runs `iters` trips of 8
// independent v_fma_f32 chains (inline asm, so nothing is folded). Two runs that
// differ only in `iters` differ by exactly waves x 8 x d_iters VALU wave-instructions,
// which calibrates rocprofv3's SQ_INSTS_VALU (is it the whole chip? per XCD?), and the
// timed run gives the chip's sustained VALU issue rate against the spec peak
// (1024 SIMDs x 2.4 GHz / 2 cycles per wave64 v_fma_f32, MI355X_MICROARCH.md).
// With active_lanes < 64 only lanes [0, active_lanes) of each wave run the loop: the same
// instruction count at a known lane utilisation (active_lanes / 64), which calibrates the
// lane-utilisation counter ratio SQ_THREAD_CYCLES_VALU / 64 / SQ_ACTIVE_INST_VALU.
// Mode 2 runs 8 independent s_add_u32 chains per trip instead (the scalar unit's issue rate: one
// scalar ALU per CU, shared by its four SIMDs), mode 3 both streams (8 v_fma_f32 + 8 s_add_u32 per trip:
// do the CU's VALU and SALU issue overlap?).
//   ./valu_probe [iters=20000] [waves_per_simd=4] [mode=0: VGPR operands, 1: inline constants, 2: SALU,
//                 3: VALU + SALU] [active_lanes=64]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void valu_probe(float* out, int iters, int active) {
    if ((int)(threadIdx.x & 63) >= active) iters = 0;
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float x = 0.999f, y = 1e-4f;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_fma_f32 %0, %8, %9, %0\n\t"
            "v_fma_f32 %1, %8, %9, %1\n\t"
            "v_fma_f32 %2, %8, %9, %2\n\t"
            "v_fma_f32 %3, %8, %9, %3\n\t"
            "v_fma_f32 %4, %8, %9, %4\n\t"
            "v_fma_f32 %5, %8, %9, %5\n\t"
            "v_fma_f32 %6, %8, %9, %6\n\t"
            "v_fma_f32 %7, %8, %9, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(x), "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// The same count with inline-constant operands: each v_fma_f32 reads ONE VGPR (no
// register-bank pressure from shared source operands), the issue-rate ceiling.
__global__ __launch_bounds__(256) void valu_probe_k(float* out, int iters, int active) {
    if ((int)(threadIdx.x & 63) >= active) iters = 0;
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_fma_f32 %0, %0, 0.5, 1.0\n\t"
            "v_fma_f32 %1, %1, 0.5, 1.0\n\t"
            "v_fma_f32 %2, %2, 0.5, 1.0\n\t"
            "v_fma_f32 %3, %3, 0.5, 1.0\n\t"
            "v_fma_f32 %4, %4, 0.5, 1.0\n\t"
            "v_fma_f32 %5, %5, 0.5, 1.0\n\t"
            "v_fma_f32 %6, %6, 0.5, 1.0\n\t"
            "v_fma_f32 %7, %7, 0.5, 1.0"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 8 independent scalar add chains per trip (wave-uniform values in SGPRs)
__global__ __launch_bounds__(256) void salu_probe(float* out, int iters, int active) {
    uint32_t s0 = __builtin_amdgcn_readfirstlane(threadIdx.x), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    uint32_t s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "s_add_u32 %0, %0, 3\n\t"
            "s_add_u32 %1, %1, 3\n\t"
            "s_add_u32 %2, %2, 3\n\t"
            "s_add_u32 %3, %3, 3\n\t"
            "s_add_u32 %4, %4, 3\n\t"
            "s_add_u32 %5, %5, 3\n\t"
            "s_add_u32 %6, %6, 3\n\t"
            "s_add_u32 %7, %7, 3"
            : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)::"scc");
    }
    (void)active;
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7);
}

// both: 8 v_fma_f32 and 8 s_add_u32 per trip
__global__ __launch_bounds__(256) void mixed_probe(float* out, int iters, int active) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t s0 = __builtin_amdgcn_readfirstlane(threadIdx.x), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    uint32_t s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_fma_f32 %0, %0, 0.5, 1.0\n\t"
            "s_add_u32 %8, %8, 3\n\t"
            "v_fma_f32 %1, %1, 0.5, 1.0\n\t"
            "s_add_u32 %9, %9, 3\n\t"
            "v_fma_f32 %2, %2, 0.5, 1.0\n\t"
            "s_add_u32 %10, %10, 3\n\t"
            "v_fma_f32 %3, %3, 0.5, 1.0\n\t"
            "s_add_u32 %11, %11, 3\n\t"
            "v_fma_f32 %4, %4, 0.5, 1.0\n\t"
            "s_add_u32 %12, %12, 3\n\t"
            "v_fma_f32 %5, %5, 0.5, 1.0\n\t"
            "s_add_u32 %13, %13, 3\n\t"
            "v_fma_f32 %6, %6, 0.5, 1.0\n\t"
            "s_add_u32 %14, %14, 3\n\t"
            "v_fma_f32 %7, %7, 0.5, 1.0\n\t"
            "s_add_u32 %15, %15, 3"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
              "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)::"scc");
    }
    (void)active;
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const int wps = argc > 2 ? atoi(argv[2]) : 4;
    const int konst = argc > 3 ? atoi(argv[3]) : 0;  // mode: 1 inline constants, 2 SALU, 3 VALU + SALU
    const int active = argc > 4 ? atoi(argv[4]) : 64;  // lanes per wave that run the loop
    auto kern = konst == 3 ? mixed_probe : konst == 2 ? salu_probe : konst ? valu_probe_k : valu_probe;
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1;
    const int blocks = n_cu * wps;  // 4 waves per block: wps waves per SIMD
    float* out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, nullptr, out, iters, active);  // warm-up
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, nullptr, out, iters, active);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double waves = (double)blocks * 4;
    const double insts = waves * 8.0 * iters;  // loop body only; the prologue/epilogue add a few per wave
    // VALU: 4 SIMDs per CU, 2 cycles per wave64 instruction; SALU: one scalar unit per CU, 1 per cycle
    const double peak = konst == 2 ? (double)n_cu * 2.4e9 : (double)n_cu * 4 * 2.4e9 / 2.0;
    printf("{\"kernel\": \"%s\", \"iters\": %d, \"active_lanes\": %d, \"waves_per_simd\": %d, \"cus\": %d, \"waves\": %.0f, \"loop_valu_insts\": %.6g, \"best_ms\": %.4f, "
           "\"inst_per_s\": %.6g, \"spec_peak_inst_per_s\": %.6g, \"frac_of_spec\": %.4f, \"launches\": 6}\n",
           konst == 3 ? "mixed_probe (8 VALU + 8 SALU per trip)" : konst == 2 ? "salu_probe (8 s_add_u32 per trip; peak = 1 per CU per cycle)" : konst ? "valu_probe_k (inline constants)" : "valu_probe (VGPR operands)", iters, active, wps, n_cu, waves, insts, best, insts / (best * 1e-3), peak, insts / (best * 1e-3) / peak);
    hipFree(out);
    return 0;
}
