// rtmi_main.hpp — the reference's host driver shape (main.h:9-35, main.cu:555-936) over the
// C++ facade: globals `imageData`, `camera`, `canvas`, `width`, `height`, `frameTime` and the
// four entry points initialize / clearBackBuffers / pathTracing / cleanup, so a frontend
// written against main.h - OpenGLFrontend.cpp's loop, which calls camera->walk / strafe /
// raise / yaw / pitch / updateViewMatrix, writes through camera->getAperture() / getFOV() /
// getMovingSpeed() and reads canvas->getSampleCount() / getRenderingTime() - compiles against
// these names (namespace rtmi::host) and links against librtmi.so alone (no HIP headers).
//
// Two modes, as the reference's GPU_REALTIME switch (main.cu:875-898):
//  - offline (default): pathTracing() renders one frame of `samplesPerFrame` samples
//    (renderKernel's offline output) into `canvas`; imageData->data points at its gamma'd
//    RGB8 pixel buffer (row 0 = the bottom row, like Canvas's pixel buffer).
//  - realtime (`realtime = true`): pathTracing() follows main.cu:876-888 - if the camera is
//    dirty: clearBackBuffers(), camera->updateViewMatrix(), camera->resetDiryFlag(); then
//    canvas->incrementSampleCount(), canvas->incrementRenderingTime(frameTime * 1000), and one
//    frame of `samplesPerFrame` fresh samples (the reference: 1) accumulated on the device
//    (Canvas::accumulatePixel, Canvas.h:82-98); imageData->data = canvas->getPixelBuffer().
//
// The scene: initialize() loads `sceneFile` (initialize()'s SCENE == 1 YAML path,
// main.cu:623-786) when set, otherwise it calls `buildScene(context, width, height)` (the
// create* factories of the compiled-in scenes, main.cu:243-402). `camera` is the scene's
// camera after initialize() unless the frontend set its own before.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>

#include "rtmi.hpp"

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
inline Camera* camera = nullptr;  // the scene's camera after initialize(), unless set before it
inline Canvas* canvas = nullptr;
inline int32_t width = 512;
inline int32_t height = 512;
inline float frameTime = 0.0f;  // seconds of the last frame, as the frontend's loop measures it

// Driver settings that the reference fixes at compile time (SCENE, samplesPerPixel,
// BOUNCES in main.cu / Constants.h).
inline int32_t device = 0;
inline std::string sceneFile;  // scene YAML; empty = buildScene
inline std::string modelsDir = "assets/models";
inline std::function<void(Context&, int32_t, int32_t)> buildScene;
inline int32_t samplesPerFrame = 1;
inline int32_t maxDepth = 8;
inline uint32_t seed = 1984;
inline int32_t integrator = RT_INTEGRATOR_RAYCOLOR;
inline bool realtime = false;

inline Context* context = nullptr;

namespace detail {
inline std::unique_ptr<Camera>& ownCamera() {  // the scene's camera when the frontend set none
    static std::unique_ptr<Camera> c;
    return c;
}
}  // namespace detail

// initialize (main.cu:555-865): context on `device`, scene, camera, canvas, imageData.
inline void initialize(int32_t w, int32_t h) {
    if (context) throw Error(RT_ERR_STATE, "initialize: already initialized (call cleanup first)");
    if (w < 2 || h < 2 || samplesPerFrame < 1) throw Error(RT_ERR_INVALID, "initialize: bad size or spp");
    width = w;
    height = h;
    context = new Context(device);
    if (!sceneFile.empty())
        context->loadYAMLScene(sceneFile, modelsDir, w, h);
    else if (buildScene)
        buildScene(*context, w, h);
    else
        throw Error(RT_ERR_INVALID, "initialize: set sceneFile or buildScene");
    if (!camera) {
        detail::ownCamera().reset(new Camera(context->getCamera()));
        camera = detail::ownCamera().get();
    }
    context->setCamera(*camera);
    if (integrator == RT_INTEGRATOR_RAYCOLOR) context->commit();
    canvas = new Canvas(w, h);
    imageData = std::make_shared<ImageData>();
    imageData->width = w;
    imageData->height = h;
    imageData->channels = 3;
    imageData->size = w * h * 3;
    imageData->data = canvas->getPixelBuffer();
}

// clearBackBuffers (main.cu:866-873)
inline void clearBackBuffers() {
    if (!canvas) throw Error(RT_ERR_STATE, "clearBackBuffers: not initialized");
    canvas->clearAccumulationBuffer();
    canvas->resetSampleCount();
    canvas->resetRenderingTime();
}

// pathTracing (main.cu:875-898)
inline void pathTracing() {
    if (!context) throw Error(RT_ERR_STATE, "pathTracing: not initialized");
    if (realtime) {
        if (camera->isDirty()) {
            clearBackBuffers();
            camera->updateViewMatrix();
            camera->resetDiryFlag();
        }
        canvas->incrementSampleCount();
        canvas->incrementRenderingTime(frameTime * 1000.0f);
        context->setCamera(*camera);  // renderKernel reads the camera object at each launch
        context->accumulate(*canvas, samplesPerFrame, maxDepth, seed, integrator);
    } else {
        canvas->incrementSampleCount();
        context->setCamera(*camera);
        if (integrator == RT_INTEGRATOR_PATHTRACE)
            context->pathTraceFrame(*canvas, samplesPerFrame, maxDepth, seed);
        else
            context->pathTracing(*canvas, samplesPerFrame, maxDepth, seed);
    }
    imageData->data = canvas->getPixelBuffer();
}

// cleanup (main.cu:900-936)
inline void cleanup() {
    delete canvas;  // its device buffers before the context
    canvas = nullptr;
    delete context;
    context = nullptr;
    if (camera == detail::ownCamera().get()) camera = nullptr;
    detail::ownCamera().reset();
    imageData.reset();
}

}  // namespace host
}  // namespace rtmi
