// examples/rtmi_render.cpp — the reference's offline main() (main.cu:945) as a
// native program over librtmi.so: read a scene YAML (initialize(), main.cu:623-786),
// render one frame (pathTracing(), main.cu:875-898) and write the image
// (Canvas::writeToPNG / writeToPPM, Canvas.h:116-154).
//   ./rtmi_render SCENE.yaml [--width 512] [--height 512] [--spp 32] [--depth 10]
//       [--seed 1984] [--lanes 0] [--device 0] [--bvh gpu|host] [--models DIR]
//       [--out render.png]
// --lanes 0 lets the library pick the sub-stream layout (as bench.py does); 1 is
// the reference's sequential per-pixel sum. --device -1 builds the scene only
// and prints its census and digest (no GPU needed).
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "rtmi.hpp"

#ifndef RTMI_ASSETS
#define RTMI_ASSETS "assets"
#endif

static int usage() {
    std::fprintf(stderr,
                 "usage: rtmi_render SCENE.yaml [--width W] [--height H] [--spp S] [--depth D] [--seed N]\n"
                 "       [--lanes L] [--device G] [--bvh gpu|host] [--models DIR] [--out FILE.png|.ppm]\n");
    return 2;
}

int main(int argc, char** argv) {
    if (argc < 2 || argv[1][0] == '-') return usage();
    std::string scene = argv[1], models = RTMI_ASSETS "/models", out = "render.png", bvh = "gpu";
    int width = 512, height = 512, spp = 32, depth = 10, lanes = 0, device = 0;
    uint32_t seed = 1984;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (i + 1 >= argc) return usage();
        const char* v = argv[++i];
        if (a == "--width") width = atoi(v);
        else if (a == "--height") height = atoi(v);
        else if (a == "--spp") spp = atoi(v);
        else if (a == "--depth") depth = atoi(v);
        else if (a == "--seed") seed = (uint32_t)strtoul(v, nullptr, 10);
        else if (a == "--lanes") lanes = atoi(v);
        else if (a == "--device") device = atoi(v);
        else if (a == "--bvh") bvh = v;
        else if (a == "--models") models = v;
        else if (a == "--out") out = v;
        else return usage();
    }
    const bool png = out.size() > 4 && out.compare(out.size() - 4, 4, ".png") == 0;
    const bool ppm = out.size() > 4 && out.compare(out.size() - 4, 4, ".ppm") == 0;
    if (width < 2 || height < 2 || spp < 1 || depth < 0 || (!png && !ppm) || (bvh != "gpu" && bvh != "host"))
        return usage();
    try {
        rtmi::Context ctx(device);
        if (device >= 0) ctx.setBVHBuilder(bvh == "gpu" ? RT_BVH_GPU : RT_BVH_HOST);
        ctx.loadYAMLScene(scene, models, width, height);
        ctx.commit();
        int32_t info[8];
        ctx.check(rt_scene_info(ctx.raw(), info));
        std::printf("scene %s: %d planes, %d spheres, %d meshes, %d triangles, %d BVH nodes, digest %016" PRIx64 "\n",
                    scene.c_str(), info[0], info[1] + info[2], info[3], info[4], info[6], ctx.sceneDigest());
        if (device < 0) return 0;

        rtmi::Canvas canvas(width, height);
        rt_render_params p{width, height, spp, depth, seed, 0, 1, 0, 1, lanes, RT_INTEGRATOR_RAYCOLOR, 0};
        ctx.check(rt_render(ctx.raw(), &p, canvas.data()));
        canvas.gammaFromRadiance();  // writePixel's gamma (Canvas.h:63-67)
        rt_render_stats st;
        ctx.check(rt_sync_stats(ctx.raw(), &st));
        if (png) canvas.writeToPNG(out);
        else canvas.writeToPPM(out);
        std::printf("%dx%d spp=%d depth=%d: kernel %.3f ms, %.1f Mrays/s -> %s\n", width, height, spp, depth,
                    st.kernel_ms, st.segments / (st.kernel_ms * 1e3), out.c_str());
    } catch (const rtmi::Error& e) {
        std::fprintf(stderr, "rtmi error %d: %s\n", e.status, e.what());
        return 1;
    }
    return 0;
}
