// examples/main_driver.cpp — a frontend written against the reference's main.h
// (initialize / clearBackBuffers / pathTracing / cleanup + globals, main.h:22-35),
// driving librtmi.so through include/rtmi_main.hpp. It mirrors the offline main()
// (main.cu:940-954) and, with --realtime, OpenGLFrontend.cpp's frame loop
// (pathTracing() once per displayed frame, the image read from imageData).
//   ./main_driver SCENE.yaml [--width W] [--height H] [--spp S] [--depth D]
//       [--frames F] [--realtime] [--camera] [--move-at K] [--device G] [--out FILE.ppm]
// --camera sets an explicit camera (the `camera` global) over the scene's; --move-at K
// moves it before frame K (walk + yaw, Camera.h:40-67), which clears the accumulation
// (camera->isDirty(), main.cu:877-881).
// --device -1 runs initialize()/cleanup() only (scene build, no GPU).
// --save FILE.pfm writes the realtime accumulation and counters after the last frame
// (Canvas::writeAccumulation); --resume FILE.pfm restores them after initialize(), so the
// frames continue the sample sequence where the saved run stopped.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "rtmi_main.hpp"

#ifndef RTMI_ASSETS
#define RTMI_ASSETS "assets"
#endif

namespace H = rtmi::host;

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: main_driver SCENE.yaml [--width W] [--height H] [--spp S] [--depth D] "
                             "[--frames F] [--realtime] [--camera] [--move-at K] [--device G] [--out FILE.ppm]\n");
        return 2;
    }
    int w = 64, h = 48, frames = 1, moveAt = -1;
    bool explicitCamera = false;
    std::string out = "main_driver.ppm", save, resume;
    H::sceneFile = argv[1];
    H::modelsDir = RTMI_ASSETS "/models";
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--realtime") { H::realtime = true; continue; }
        if (a == "--camera") { explicitCamera = true; continue; }
        if (i + 1 >= argc) return 2;
        const char* v = argv[++i];
        if (a == "--width") w = atoi(v);
        else if (a == "--height") h = atoi(v);
        else if (a == "--spp") H::samplesPerFrame = atoi(v);
        else if (a == "--depth") H::maxDepth = atoi(v);
        else if (a == "--frames") frames = atoi(v);
        else if (a == "--move-at") moveAt = atoi(v);
        else if (a == "--device") H::device = atoi(v);
        else if (a == "--out") out = v;
        else if (a == "--save") save = v;
        else if (a == "--resume") resume = v;
        else return 2;
    }
    rtmi::Camera cam({0.0f, 0.0f, 1.25f}, {0.0f, 0.0f, -1.0f}, {0.0f, 1.0f, 0.0f}, (float)w / (float)h, 60.0f,
                     0.0f, 1.0f);
    if (explicitCamera) H::camera = &cam;
    try {
        H::initialize(w, h);
        std::printf("initialized %dx%d, %d channels\n", H::imageData->width, H::imageData->height,
                    H::imageData->channels);
        if (H::device < 0) {
            H::cleanup();
            return 0;
        }
        if (!resume.empty()) {
            // the saved camera view: nothing to clear on the first frame
            H::camera->updateViewMatrix();
            H::camera->resetDiryFlag();
            H::canvas->readAccumulation(resume, H::context->raw());
        }
        for (int f = 0; f < frames; ++f) {
            if (f == moveAt) {
                H::camera->walk(-0.05f);
                H::camera->yaw(0.03f);
            }
            const auto t0 = std::chrono::steady_clock::now();
            H::pathTracing();
            H::frameTime = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
        }
        if (!save.empty()) H::canvas->writeAccumulation(save);
        std::printf("frames %d samples %u\n", frames,
                    H::realtime ? H::canvas->getSampleCount() * (uint32_t)H::samplesPerFrame
                                : (uint32_t)H::samplesPerFrame);
        FILE* fp = std::fopen(out.c_str(), "wb");
        if (!fp) return 1;
        std::fprintf(fp, "P6\n%d %d\n255\n", w, h);  // top row first (Canvas::writeToPPM)
        for (int y = h - 1; y >= 0; --y) std::fwrite(H::imageData->data + (size_t)y * w * 3, 1, (size_t)w * 3, fp);
        std::fclose(fp);
        H::cleanup();
    } catch (const rtmi::Error& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
