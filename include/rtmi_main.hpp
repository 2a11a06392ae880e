// rtmi_main.hpp — the reference's host driver shape (main.h:9-35, main.cu:555-936)
// over the C++ facade: globals `imageData`, `camera`, `canvas`, `width`, `height`,
// `frameTime` and the four entry points initialize / clearBackBuffers / pathTracing /
// cleanup, so a frontend written against main.h (OpenGLFrontend.cpp's loop) links
// against librtmi.so unchanged apart from the namespace.
//
// Two modes, as the reference's GPU_REALTIME switch (main.cu:867-897):
//  - offline (default): pathTracing() renders one frame of `samplesPerFrame` samples
//    (renderKernel's sequential-sum-equivalent output) into `canvas`; imageData->data
//    points at its gamma'd RGB8 (top row last, like Canvas's pixel buffer).
//  - realtime (`realtime = true` before initialize(); needs librtmi's rt_accumulate and
//    HIP for the device buffers, so build with -DRTMI_REALTIME and link amdhip64):
//    every pathTracing() adds `samplesPerFrame` fresh samples per pixel to a device
//    accumulation buffer (Canvas::accumulatePixel, Canvas.h:73-98) and refreshes
//    imageData->data; a camera change clears the buffers first (camera->isDirty(),
//    main.cu:869-873), detected by comparing `*camera` with the one last applied.
//
// The scene: initialize() loads `sceneFile` (initialize()'s SCENE == 1 YAML path,
// main.cu:623-786) when set, otherwise it calls `buildScene(context, width, height)`
// (the create* factories of the compiled-in scenes, main.cu:243-402).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "rtmi.hpp"

#ifdef RTMI_REALTIME
#include <hip/hip_runtime_api.h>
#endif

namespace rtmi {
namespace host {

// ImageData (main.h:9-20): the frontend's view of the current frame.
struct ImageData {
    uint8_t* data = nullptr;
    int32_t size = 0;
    int32_t width = 0;
    int32_t height = 0;
    int32_t channels = 0;
};

// main.h:22-30 globals (C++17 inline variables: one definition across translation units)
inline std::shared_ptr<ImageData> imageData;
inline Camera* camera = nullptr;  // optional: when set, applied at initialize and watched in realtime mode
inline Canvas* canvas = nullptr;
inline int32_t width = 512;
inline int32_t height = 512;
inline float frameTime = 0.0f;  // seconds of the last frame, as the frontend's loop measures it

// Driver settings that the reference fixes at compile time (SCENE, SAMPLES_PER_PIXEL,
// MAX_DEPTH in main.cu / Constants.h).
inline int32_t device = 0;
inline std::string sceneFile;  // scene YAML; empty = buildScene
inline std::string modelsDir = "assets/models";
inline std::function<void(Context&, int32_t, int32_t)> buildScene;
inline int32_t samplesPerFrame = 1;
inline int32_t maxDepth = 8;
inline uint32_t seed = 1984;
inline int32_t integrator = RT_INTEGRATOR_RAYCOLOR;
inline bool realtime = false;

// Canvas counters (Canvas.h incrementSampleCount / incrementRenderingTime)
inline uint32_t sampleCount = 0;
inline float renderingTime = 0.0f;  // ms

inline Context* context = nullptr;

namespace detail {
inline std::vector<uint8_t>& hostPixels() {
    static std::vector<uint8_t> px;
    return px;
}
inline Camera& appliedCamera() {
    static Camera c;
    return c;
}
inline bool sameCamera(const Camera& a, const Camera& b) {
    return std::memcmp(a.eye.data(), b.eye.data(), 3 * sizeof(float)) == 0 &&
           std::memcmp(a.center.data(), b.center.data(), 3 * sizeof(float)) == 0 &&
           std::memcmp(a.up.data(), b.up.data(), 3 * sizeof(float)) == 0 && a.aspectRatio == b.aspectRatio &&
           a.fov == b.fov && a.aperture == b.aperture && a.focusDistance == b.focusDistance &&
           a.time0 == b.time0 && a.time1 == b.time1;
}
inline void applyCamera() {
    context->setCamera(*camera);
    appliedCamera() = *camera;
}
#ifdef RTMI_REALTIME
inline float*& accumDevice() {
    static float* p = nullptr;
    return p;
}
inline uint8_t*& pixelsDevice() {
    static uint8_t* p = nullptr;
    return p;
}
inline void hipCheck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw Error(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#endif
inline rt_render_params params(uint32_t offset) {
    return rt_render_params{width, height, samplesPerFrame, maxDepth, seed, offset, 1, 0, 1, 0, integrator, 0};
}
}  // namespace detail

// initialize (main.cu:855-865 with the scene setup of 623-853): context on `device`,
// scene, camera, canvas, imageData.
inline void initialize(int32_t w, int32_t h) {
    if (context) throw Error(RT_ERR_STATE, "initialize: already initialized (call cleanup first)");
    if (w < 1 || h < 1 || samplesPerFrame < 1) throw Error(RT_ERR_INVALID, "initialize: bad size or spp");
#ifndef RTMI_REALTIME
    if (realtime) throw Error(RT_ERR_INVALID, "initialize: realtime mode needs a build with -DRTMI_REALTIME");
#endif
    width = w;
    height = h;
    context = new Context(device);
    if (!sceneFile.empty())
        context->loadYAMLScene(sceneFile, modelsDir, w, h);
    else if (buildScene)
        buildScene(*context, w, h);
    else
        throw Error(RT_ERR_INVALID, "initialize: set sceneFile or buildScene");
    if (camera) detail::applyCamera();
    context->commit();
    canvas = new Canvas(w, h);
    imageData = std::make_shared<ImageData>();
    imageData->width = w;
    imageData->height = h;
    imageData->channels = 3;
    imageData->size = w * h * 3;
    detail::hostPixels().assign((size_t)w * h * 3, 0);
    imageData->data = detail::hostPixels().data();
#ifdef RTMI_REALTIME
    if (realtime && device >= 0) {
        detail::hipCheck(hipMalloc((void**)&detail::accumDevice(), (size_t)w * h * 3 * sizeof(float)), "hipMalloc");
        detail::hipCheck(hipMalloc((void**)&detail::pixelsDevice(), (size_t)w * h * 3), "hipMalloc");
    }
#endif
    sampleCount = 0;
    renderingTime = 0.0f;
}

// clearBackBuffers (main.cu:867-873): zero the accumulation, reset the counters.
inline void clearBackBuffers() {
    if (!canvas) throw Error(RT_ERR_STATE, "clearBackBuffers: not initialized");
    std::memset(canvas->data(), 0, (size_t)width * height * 3 * sizeof(float));
#ifdef RTMI_REALTIME
    if (detail::accumDevice())
        detail::hipCheck(hipMemset(detail::accumDevice(), 0, (size_t)width * height * 3 * sizeof(float)),
                         "hipMemset");
#endif
    sampleCount = 0;
    renderingTime = 0.0f;
}

// pathTracing (main.cu:875-898)
inline void pathTracing() {
    if (!context) throw Error(RT_ERR_STATE, "pathTracing: not initialized");
    if (camera && !detail::sameCamera(*camera, detail::appliedCamera())) {
        clearBackBuffers();
        detail::applyCamera();
    }
    if (!realtime) {
        rt_render_params p = detail::params(0);
        context->commit();
        context->check(rt_render(context->raw(), &p, canvas->data()));
        sampleCount = (uint32_t)samplesPerFrame;
        detail::hostPixels() = canvas->pixels();
        imageData->data = detail::hostPixels().data();
        return;
    }
#ifdef RTMI_REALTIME
    context->commit();
    const uint32_t offset = sampleCount;
    sampleCount += (uint32_t)samplesPerFrame;
    renderingTime += frameTime * 1000.0f;
    rt_render_params p = detail::params(offset);
    context->check(rt_accumulate(context->raw(), &p, detail::accumDevice(), sampleCount, detail::pixelsDevice(),
                                 nullptr));
    detail::hipCheck(hipMemcpy(detail::hostPixels().data(), detail::pixelsDevice(), (size_t)width * height * 3,
                               hipMemcpyDeviceToHost),
                     "hipMemcpy");
    imageData->data = detail::hostPixels().data();
#endif
}

// cleanup (main.cu:900-936)
inline void cleanup() {
#ifdef RTMI_REALTIME
    if (detail::accumDevice()) (void)hipFree(detail::accumDevice());
    if (detail::pixelsDevice()) (void)hipFree(detail::pixelsDevice());
    detail::accumDevice() = nullptr;
    detail::pixelsDevice() = nullptr;
#endif
    delete canvas;
    canvas = nullptr;
    delete context;
    context = nullptr;
    imageData.reset();
    detail::hostPixels().clear();
    sampleCount = 0;
    renderingTime = 0.0f;
}

}  // namespace host
}  // namespace rtmi
