// rt_rows.hip — assembly of a row-sharded frame on the gather's root device
// (SURVEY §8(e)). Rank k of n owns row blocks k, k + n, ... of `row_block` rows;
// the gather delivers the tiles rank-major, each padded to `max_rows` rows. One
// pass streams the staging buffer into frame order (HBM-bound: 2 x 12 B per pixel).
#include <hip/hip_runtime.h>

#include "rt_kernel.h"

namespace rt {

namespace {

// One thread per 16 B of a frame row (rows are 3 * width floats; a trailing
// remainder of 1-3 floats is copied by scalar lanes).
__global__ __launch_bounds__(256) void assemble_rows_kernel(const float* __restrict__ staging,
                                                            float* __restrict__ frame, int32_t width,
                                                            int32_t height, int32_t row_block, int32_t world,
                                                            int32_t max_rows) {
    const size_t row_floats = (size_t)width * 3;
    const size_t vec_per_row = (row_floats + 3) / 4;
    const size_t total = vec_per_row * (size_t)height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int32_t y = (int32_t)(i / vec_per_row);
        const size_t v = i - (size_t)y * vec_per_row;
        const int32_t b = y / row_block;           // global row block
        const int32_t rank = b % world;            // its owner
        const int32_t lb = b / world;              // the owner's local block
        const int32_t j = lb * row_block + (y - b * row_block);  // the owner's local row
        const float* src = staging + ((size_t)rank * (size_t)max_rows + (size_t)j) * row_floats;
        float* dst = frame + (size_t)y * row_floats;
        const size_t f = v * 4;
        if (f + 4 <= row_floats && ((row_floats & 3) == 0)) {
            *reinterpret_cast<float4*>(dst + f) = *reinterpret_cast<const float4*>(src + f);
        } else {
            for (size_t k = f; k < f + 4 && k < row_floats; ++k) dst[k] = src[k];
        }
    }
}

}  // namespace

hipError_t launch_assemble_rows(const float* staging, float* frame, int32_t width, int32_t height,
                                int32_t row_block, int32_t world, int32_t max_rows, hipStream_t stream) {
    const size_t vec = ((size_t)width * 3 + 3) / 4 * (size_t)height;
    const size_t want = (vec + 255) / 256;
    const unsigned blocks = (unsigned)(want < 8192 ? (want ? want : 1) : 8192);
    hipLaunchKernelGGL(assemble_rows_kernel, dim3(blocks), dim3(256), 0, stream, staging, frame, width, height,
                       row_block, world, max_rows);
    return hipGetLastError();
}

}  // namespace rt
