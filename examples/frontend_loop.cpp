// examples/frontend_loop.cpp — OpenGLFrontend.cpp's frame loop without GLFW / ImGui / GL: the
// same calls on the `camera` and `canvas` globals of main.h (include/rtmi_main.hpp), driven by
// a scripted input sequence instead of a window. Per frame, as OpenGLFrontend.cpp:538-557:
// input callbacks (scroll -> onScrollCallback :387-394, mouse move -> onMouseMoveCallback
// :396-412 with the right / middle button held), the settings window's sliders (:189-197:
// aperture / FOV written through camera->getAperture() / getFOV() then setDirty(), camera speed
// through getMovingSpeed()), processInput (:576-612: W/A/S/D/Q/E keys, then
// camera->updateViewMatrix()), then pathTracing() (main.cu:875-898) and the frame statistics
// (:226-228 getSampleCount / getRenderingTime).
//   ./frontend_loop SCENE.yaml [--width W] [--height H] [--frames F] [--still S] [--depth D]
//       [--device G] [--out FILE.ppm]
// The first F frames replay the script below; the last S frames have no input, so the
// accumulation after the last camera change covers exactly S frames. --device -1 replays the
// camera script without rendering. Prints the camera's state after the loop (hex floats).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "rtmi_main.hpp"

#ifndef RTMI_ASSETS
#define RTMI_ASSETS "assets"
#endif

namespace H = rtmi::host;
using rtmi::host::camera;
using rtmi::host::canvas;
using rtmi::host::frameTime;

namespace {

// Math::radians (Constants.h:29-31)
float radians(float degree) { return 3.1415926535897932f / 180.0f * degree; }

// OpenGLFrontend.cpp state
bool bRightMouseButtonDown = false;
bool bMiddleMouseButtonDown = false;
struct { float x = 0.0f, y = 0.0f; } lastMousePosition;
float rotateSpeed = 5.0f;
bool keyW = false, keyA = false, keyS = false, keyD = false, keyQ = false, keyE = false;

void onScrollCallback(double, double yOffset) {  // :387-394
    camera->walk(static_cast<float>(yOffset / 8.0f));
}

void onMouseMoveCallback(double x, double y) {  // :396-412
    double dx = (lastMousePosition.x - x) * frameTime;
    double dy = (lastMousePosition.y - y) * frameTime;
    if (bRightMouseButtonDown) {
        camera->yaw(radians(static_cast<float>(dx * rotateSpeed)));
        camera->pitch(radians(static_cast<float>(dy * rotateSpeed)));
    }
    if (bMiddleMouseButtonDown) {
        camera->strafe(static_cast<float>(-dx / 4.0f));
        camera->raise(static_cast<float>(dy / 4.0f));
    }
    lastMousePosition.x = static_cast<float>(x);
    lastMousePosition.y = static_cast<float>(y);
}

void settingsWindow(const float* aperture, const float* fov, const float* speed) {  // :189-197
    if (aperture) {  // ImGui::SliderFloat("Aperture", &camera->getAperture(), 0.0f, 2.0f) changed
        camera->getAperture() = *aperture;
        camera->setDirty();
    }
    if (fov) {  // ImGui::SliderFloat("FOV", &camera->getFOV(), 20.0f, 90.0f) changed
        camera->getFOV() = *fov;
        camera->setDirty();
    }
    if (speed) camera->getMovingSpeed() = *speed;  // "Camera Speed" (no setDirty)
}

void processInput() {  // :576-612
    if (keyA) camera->strafe(-frameTime);
    if (keyD) camera->strafe(frameTime);
    if (keyW) camera->walk(frameTime);
    if (keyS) camera->walk(-frameTime);
    if (keyQ) camera->raise(frameTime);
    if (keyE) camera->raise(-frameTime);
    camera->updateViewMatrix();
}

// The scripted input of frame f (tests/test_camera.py replays the same camera calls on the
// restatement's Camera).
void scriptedInput(int f) {
    bRightMouseButtonDown = bMiddleMouseButtonDown = false;
    keyW = keyA = keyS = keyD = keyQ = keyE = false;
    switch (f) {
        case 0: onScrollCallback(0.0, 1.0); break;  // scroll up: walk(1/8)
        case 1:                                     // right drag: yaw + pitch
            bRightMouseButtonDown = true;
            lastMousePosition = {100.0f, 100.0f};
            onMouseMoveCallback(94.0, 103.0);
            break;
        case 2:  // middle drag: strafe + raise
            bMiddleMouseButtonDown = true;
            lastMousePosition = {50.0f, 50.0f};
            onMouseMoveCallback(53.0, 48.0);
            break;
        case 3: {  // sliders
            const float aperture = 0.05f, fov = 55.0f, speed = 2.0f;
            settingsWindow(&aperture, &fov, &speed);
            break;
        }
        case 4: keyW = keyD = true; break;  // W + D held
        case 5: keyS = keyQ = true; break;  // S + Q held
        case 6: keyA = keyE = true; break;  // A + E held
        default: break;
    }
}

void printVec(const char* name, const float* v) {
    std::printf("%s %a %a %a\n", name, v[0], v[1], v[2]);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: frontend_loop SCENE.yaml [--width W] [--height H] [--frames F] [--still S] "
                             "[--depth D] [--device G] [--out FILE.ppm]\n");
        return 2;
    }
    int w = 64, h = 48, frames = 7, still = 3;
    std::string out = "frontend_loop.ppm";
    H::sceneFile = argv[1];
    H::modelsDir = RTMI_ASSETS "/models";
    H::realtime = true;  // GPU_REALTIME: one sample per pixel per frame (main.cu:165-169)
    H::samplesPerFrame = 1;
    for (int i = 2; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        const char* v = argv[i + 1];
        if (a == "--width") w = atoi(v);
        else if (a == "--height") h = atoi(v);
        else if (a == "--frames") frames = atoi(v);
        else if (a == "--still") still = atoi(v);
        else if (a == "--depth") H::maxDepth = atoi(v);
        else if (a == "--device") H::device = atoi(v);
        else if (a == "--out") out = v;
        else return 2;
    }
    try {
        const bool gpu = H::device >= 0;
        if (!gpu) H::device = -1;
        H::initialize(w, h);
        for (int f = 0; f < frames + still; ++f) {
            frameTime = 1.0f / 60.0f;  // a fixed frame time keeps the script deterministic
            scriptedInput(f);
            processInput();
            if (gpu) H::pathTracing();
        }
        const rt_camera_state& s = camera->state();
        printVec("eye", s.eye);
        printVec("center", s.center);
        printVec("forward", s.forward);
        printVec("right", s.right);
        printVec("origin", s.origin);
        printVec("lower_left", s.lower_left);
        printVec("horizontal", s.horizontal);
        printVec("vertical", s.vertical);
        std::printf("lens_radius %a fov %a moving_speed %a dirty %d\n", s.lens_radius, s.fov, s.moving_speed, s.dirty);
        if (gpu) {
            std::printf("sample count %u rendering time %.3f ms\n", canvas->getSampleCount(),
                        canvas->getRenderingTime());
            FILE* fp = std::fopen(out.c_str(), "wb");
            if (!fp) return 1;
            std::fprintf(fp, "P6\n%d %d\n255\n", w, h);  // top row first (Canvas::writeToPPM)
            for (int y = h - 1; y >= 0; --y)
                std::fwrite(H::imageData->data + (size_t)y * w * 3, 1, (size_t)w * 3, fp);
            std::fclose(fp);
        }
        H::cleanup();
    } catch (const rtmi::Error& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
