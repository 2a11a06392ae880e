// examples/materialball.cpp — the reference's committed renderKernel setup:
// pathTrace (main.cu:187) over materialball.ply loaded as COAT and placed by
// processTriangleData(Vector3Df(0.1f, 0.0f, -1.0f)) (prepareCUDAscene,
// main.cu:430-432), seen through cornellbox2.yaml's camera (main.cu:629-638),
// written against the C++ facade include/rtmi.hpp. Renders to materialball.ppm.
//   ./materialball [device=0] [width=512] [height=512] [spp=32]
//   device -1: load and process the mesh only (no GPU), print the census and exit.
//   With a device the BVH is built by the GPU builder (rt_set_bvh_builder).
#include <cstdio>
#include <cstdlib>

#include "rtmi.hpp"

using rtmi::Vector3Df;

int main(int argc, char** argv) {
    const int device = argc > 1 ? atoi(argv[1]) : 0;
    const int width = argc > 2 ? atoi(argv[2]) : 512, height = argc > 3 ? atoi(argv[3]) : 512;
    const int spp = argc > 4 ? atoi(argv[4]) : 32;
    try {
        rtmi::Context ctx(device);
        Vector3Df eye(0, 0, 1), center(0, 0, -1), up(0, 1, 0);  // cornellbox2.yaml
        rtmi::Camera camera(eye, center, up, float(width) / height, 60.0f, 0.0f, 2.0f, 0.0f, 1.0f);
        ctx.setCamera(camera);

        // on a GPU context the BVH is built on the device (byte-identical to the host build)
        if (device >= 0) ctx.setBVHBuilder(RT_BVH_GPU);
        ctx.loadObject(RTMI_ASSETS "/models/materialball/materialball.ply", RT_PT_COAT);
        int32_t info[4];
        const Vector3Df offset(0.1f, 0.0f, -1.0f);
        ctx.check(rt_process_triangle_data(ctx.raw(), offset.data(), 1.0f, info));
        std::printf("pathTrace scene: %d triangles, %d BVH nodes, depth %d; BVH build %.2f ms (%s)\n", info[0],
                    info[1], info[3], ctx.lastBVHBuildMs(), device >= 0 ? "GPU" : "host");
        if (device < 0) return 0;

        rtmi::Canvas canvas(width, height);
        ctx.pathTraceFrame(canvas, spp);  // 5 bounces, as CUDAPathTracer.cu:366
        rt_render_stats st;
        ctx.check(rt_sync_stats(ctx.raw(), &st));
        canvas.writeToPPM("materialball.ppm");
        std::printf("%dx%d, %d spp: %.3f ms, %.1f Mrays/s\n", width, height, spp, st.kernel_ms,
                    st.segments / (st.kernel_ms * 1e3));
    } catch (const rtmi::Error& e) {
        std::fprintf(stderr, "rtmi error %d: %s\n", e.status, e.what());
        return 1;
    }
    return 0;
}
