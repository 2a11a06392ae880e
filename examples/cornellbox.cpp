// examples/cornellbox.cpp — CornellBox1 (resources/scenes/cornellbox1.yaml)
// written the way the reference's initialize() builds scenes (main.cu:623-786),
// against the C++ facade include/rtmi.hpp. Renders to cornellbox.ppm.
//   ./cornellbox [device=0] [width=512] [height=512] [spp=32] [bounces=10]
//   device -1: build the scene only (no GPU), print the census and exit.
#include <cstdio>
#include <cstdlib>

#include "rtmi.hpp"

using rtmi::Vector3Df;

int main(int argc, char** argv) {
    const int device = argc > 1 ? atoi(argv[1]) : 0;
    const int width = argc > 2 ? atoi(argv[2]) : 512, height = argc > 3 ? atoi(argv[3]) : 512;
    const int spp = argc > 4 ? atoi(argv[4]) : 32, bounces = argc > 5 ? atoi(argv[5]) : 10;
    try {
        rtmi::Context ctx(device);
        rtmi::Material** materials = ctx.materials(9);
        rtmi::Hitable** spheres = ctx.objects(10);

        Vector3Df eye(0, 0, 1), center(0, 0, -1), up(0, 1, 0);
        rtmi::Camera camera(eye, center, up, float(width) / height, 60.0f, 0.0f, 2.0f, 0.0f, 1.0f);
        ctx.setCamera(camera);

        // main.cu:643-651 pre-seeded materials
        createLambertianMaterial(materials, 0, Vector3Df(1.0f, 0.0f, 0.0f));
        createLambertianMaterial(materials, 1, Vector3Df(0.0f, 1.0f, 0.0f));
        createLambertianMaterial(materials, 2, Vector3Df(0.0f, 0.0f, 1.0f));
        createLambertianMaterial(materials, 3, Vector3Df(1.0f, 1.0f, 1.0f));
        createLambertianMaterial(materials, 4, Vector3Df(0.75f, 0.25f, 0.25f));
        createLambertianMaterial(materials, 5, Vector3Df(0.25f, 0.25f, 0.75f));
        createMetalMaterial(materials, 6, Vector3Df(1.0f, 1.0f, 1.0f), 0.0f);
        createDieletricMaterial(materials, 7, 1.5f);
        createEmissionMaterial(materials, 8, Vector3Df(1.0f, 1.0f, 1.0f), 5.0f);
        if (materials[9 - 1] == nullptr) return 2;  // the nullptr guards read as in main.cu:714

        using O = rtmi::PlaneOrientation;
        const Vector3Df half(0.5f, 0.5f, 0.5f);
        createPlane(spheres, 0, {0, 0.5f, 0}, {0, 1, 0}, half, materials[3], O::XZ, true);    // top
        createPlane(spheres, 1, {0, -0.5f, 0}, {0, -1, 0}, half, materials[3], O::XZ, true);  // bottom
        createPlane(spheres, 2, {-0.5f, 0, 0}, {-1, 0, 0}, half, materials[4], O::YZ, true);  // left
        createPlane(spheres, 3, {0.5f, 0, 0}, {1, 0, 0}, half, materials[5], O::YZ, true);    // right
        createPlane(spheres, 4, {0, 0, -0.5f}, {0, 0, -1}, half, materials[3], O::XY, true);  // back
        createPlane(spheres, 5, {0, 0.49f, 0}, {0, 1, 0}, {0.125f, 0.125f, 0.125f}, materials[8], O::XZ, false);
        const char* cube = RTMI_ASSETS "/models/cube/cube_small.obj";
        createMeshFromOBJ(spheres, 6, cube, {0.5f, 1.0f, 0.5f}, {0, 30, 0}, {-0.25f, -0.25f, -0.25f}, materials[3]);
        createMeshFromOBJ(spheres, 7, cube, {0.5f, 0.5f, 0.5f}, {0, -30, 0}, {0.25f, -0.375f, -0.25f}, materials[3]);
        ctx.commit();

        int32_t info[8];
        ctx.check(rt_scene_info(ctx.raw(), info));
        std::printf("scene: %d planes, %d meshes, %d triangles\n", info[0], info[3], info[4]);
        if (device < 0) return 0;

        rtmi::Canvas canvas(width, height);
        ctx.pathTracing(canvas, spp, bounces);
        rt_render_stats st;
        ctx.check(rt_sync_stats(ctx.raw(), &st));
        canvas.writeToPPM("cornellbox.ppm");
        canvas.writeToPNG("cornellbox.png");
        std::printf("rendered %dx%d spp=%d: %.3f ms, %.1f Mrays/s\n", width, height, spp, st.kernel_ms,
                    st.segments / (st.kernel_ms * 1e3));
    } catch (const rtmi::Error& e) {
        std::fprintf(stderr, "rtmi error %d: %s\n", e.status, e.what());
        return 1;
    }
    return 0;
}
