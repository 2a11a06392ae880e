// rtmi.hpp — header-only C++ facade over the C ABI (rtmi.h) that keeps the
// reference's host-side scene API, so scene code written against
// RayTracingTheNextWeekCUDA's kernels.h / Camera.h / Canvas.h ports with the
// same call shapes:
//
//   rtmi::Context ctx(0);                                   // initialize()
//   Material** materials = ctx.materials();                // createObjectPtrArray<Material*>
//   Hitable** spheres = ctx.objects();
//   createLambertianMaterial(materials, 0, Vector3Df(1, 0, 0));        // kernels.h:54
//   createSphere(spheres, 0, {-1, 0, -1}, 0.5f, materials[0]);        // kernels.h:103
//   Camera camera(eye, center, up, float(w) / h, 60.0f, 0.0f, 2.0f, 0.0f, 1.0f);
//   camera.walk(0.1f); camera.updateViewMatrix();              // Camera.h:40-44, 86-103
//   ctx.setCamera(camera);
//   Canvas canvas(w, h);
//   ctx.pathTracing(canvas, spp, bounces);                  // main.cu:875-898
//   canvas.writeToPPM("render.ppm");                        // Canvas.h:116-139
//
// `materials[i]` is nullptr until slot i is created (the reference's
// `materials[id] == nullptr` guards, main.cu:714-744). Material* / Hitable*
// are opaque non-null handles; the device data lives behind the C ABI.
// Errors throw rtmi::Error (the reference exits the process instead).
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "rtmi.h"

namespace rtmi {

struct Vector3Df {
    float x = 0, y = 0, z = 0;
    Vector3Df() = default;
    Vector3Df(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
    const float* data() const { return &x; }
};

struct Error : std::runtime_error {
    rt_status status;
    Error(rt_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

enum class PlaneOrientation : uint8_t { XY = RT_PLANE_XY, YZ = RT_PLANE_YZ, XZ = RT_PLANE_XZ };

class Context;

// The context that the reference-shaped factories act on: set by
// Context::materials() / objects() (the tables the factories receive).
inline Context*& table_owner() {
    static thread_local Context* owner = nullptr;
    return owner;
}

// Opaque device-object handles (stand-ins for the reference's device pointers).
struct Handle {
    Context* ctx;
    int32_t index;
};
using Material = Handle;
using Hitable = Handle;

// Camera (Camera.h:12-196): the reference's fields (rt_camera_state) and methods, restated
// by the library with the reference's float operations (rtmi.h rt_camera_*), so a frontend's
// moves - walk/strafe/raise/yaw/pitch from OpenGLFrontend.cpp:393-407 and 586-611, the
// aperture/FOV/speed sliders of 189-197 - give the reference's floats. Context::setCamera
// hands the current view (what getRay reads) to the renderer.
class Camera {
public:
    Camera() = default;
    Camera(const Vector3Df& e, const Vector3Df& c, const Vector3Df& u, float aspect, float fov_ = 90.0f,
           float aperture_ = 2.0f, float focus = 1.0f, float t0 = 0.0f, float t1 = 0.0f) {
        initialize(e, c, u, aspect, fov_, aperture_, focus, t0, t1);
    }
    explicit Camera(const rt_camera_state& s) : s_(s) {}
    void initialize(const Vector3Df& e, const Vector3Df& c, const Vector3Df& u, float aspect,
                    float fov_ = 90.0f, float aperture_ = 2.0f, float focus = 1.0f, float t0 = 0.0f,
                    float t1 = 0.0f) {
        check(rt_camera_initialize(&s_, e.data(), c.data(), u.data(), aspect, fov_, aperture_, focus, t0, t1));
    }
    void walk(float delta) { check(rt_camera_walk(&s_, delta)); }
    void strafe(float delta) { check(rt_camera_strafe(&s_, delta)); }
    void raise(float delta) { check(rt_camera_raise(&s_, delta)); }
    void yaw(float delta) { check(rt_camera_yaw(&s_, delta)); }
    void pitch(float delta) { check(rt_camera_pitch(&s_, delta)); }
    void orbit(const Vector3Df& target) { check(rt_camera_orbit(&s_, target.data())); }
    void updateViewMatrix() { check(rt_camera_update_view_matrix(&s_)); }
    void setAperture(float a) { check(rt_camera_set_aperture(&s_, a)); }
    void updateLensRadius() { check(rt_camera_set_aperture(&s_, s_.aperture)); }
    // Camera.h:115-137: references, so an ImGui::SliderFloat can write through them
    // (followed by setDirty(), OpenGLFrontend.cpp:189-197)
    float& getAperture() { return s_.aperture; }
    const float& getAperture() const { return s_.aperture; }
    float& getFOV() { return s_.fov; }
    const float& getFOV() const { return s_.fov; }
    float& getMovingSpeed() { return s_.moving_speed; }
    const float& getMovingSpeed() const { return s_.moving_speed; }
    void setDirty() { s_.dirty = 1; }
    bool isDirty() const { return s_.dirty != 0; }
    void resetDiryFlag() { s_.dirty = 0; }  // the reference's spelling (Camera.h:147)
    Vector3Df getEye() const { return {s_.eye[0], s_.eye[1], s_.eye[2]}; }
    Vector3Df getCenter() const { return {s_.center[0], s_.center[1], s_.center[2]}; }
    const rt_camera_state& state() const { return s_; }

private:
    static void check(rt_status st) {
        if (st != RT_OK) throw Error(st, "camera: invalid argument");
    }
    rt_camera_state s_{};
};

// Canvas (Canvas.h:20-200): float radiance of the last offline frame (row 0 = bottom), the
// gamma'd 8-bit pixel buffer, and the realtime accumulation on the device (a librtmi
// rt_canvas, created by the first Context::accumulate). Counters as Canvas.h:162-189.
class Canvas {
public:
    Canvas(int32_t w, int32_t h) { initialize(w, h); }
    ~Canvas() { rt_canvas_destroy(device_); }
    Canvas(const Canvas&) = delete;
    Canvas& operator=(const Canvas&) = delete;
    // Canvas::initialize (Canvas.h:27-40)
    void initialize(int32_t w, int32_t h) {
        rt_canvas_destroy(device_);
        device_ = nullptr;
        width = w;
        height = h;
        radiance.assign((size_t)w * h * 3, 0.0f);
        pixelBuffer.assign((size_t)w * h * 3, 0);
        sampleCount = 0;
        scale = 0.0f;
        renderingTime = 0.0f;
    }
    int32_t getWidth() const { return width; }
    int32_t getHeight() const { return height; }
    float* data() { return radiance.data(); }
    const float* data() const { return radiance.data(); }
    // getPixelBuffer (Canvas.h:105-107): the last frame written or accumulated
    uint8_t* getPixelBuffer() { return pixelBuffer.data(); }
    std::vector<uint8_t> pixels() const { return pixelBuffer; }
    // clearAccumulationBuffer (Canvas.h:162-164), to zero (the reference's memset(1) is a bug)
    void clearAccumulationBuffer() {
        std::fill(radiance.begin(), radiance.end(), 0.0f);
        if (device_ && rt_canvas_clear_accumulation(device_) != RT_OK)
            throw Error(RT_ERR_HIP, "clearAccumulationBuffer failed");
    }
    // Canvas.h:166-189
    void incrementSampleCount() {
        sampleCount++;
        scale = 1.0f / sampleCount;
    }
    void resetSampleCount() { sampleCount = 0; }
    void resetRenderingTime() { renderingTime = 0.0f; }
    uint32_t getSampleCount() const { return sampleCount; }
    float getRenderingTime() const { return renderingTime; }
    void incrementRenderingTime(float amount = 16.0f) { renderingTime += amount; }

    // the offline frame's radiance -> pixel buffer (writePixel's gamma, Canvas.h:63-67)
    void gammaFromRadiance() {
        rt_status s = rt_gamma_u8(radiance.data(), (int64_t)radiance.size(), pixelBuffer.data());
        if (s != RT_OK) throw Error(s, "rt_gamma_u8");
    }
    rt_canvas* device(rt_ctx* ctx) {
        if (!device_) {
            rt_status s = rt_canvas_create(ctx, width, height, &device_);
            if (s != RT_OK) throw Error(s, rt_last_error(ctx));
        }
        return device_;
    }
    // Checkpoint / resume of a progressive render (the reference loses its
    // accumulation on exit): the accumulation sums as a little-endian PFM (bottom row first,
    // the buffer's own order) and `<path>.json` with the counters. With a device canvas the
    // device buffer is saved / restored; resuming continues the sample sequence where it stopped.
    void writeAccumulation(const std::string& path) {
        std::vector<float> acc = radiance;
        if (device_ && rt_canvas_read_accumulation(device_, acc.data()) != RT_OK)
            throw Error(RT_ERR_HIP, "writeAccumulation: device read failed");
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) throw Error(RT_ERR_IO, "cannot write " + path);
        std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
        const bool ok = std::fwrite(acc.data(), sizeof(float), acc.size(), f) == acc.size();
        std::fclose(f);
        FILE* j = std::fopen((path + ".json").c_str(), "w");
        if (!ok || !j) throw Error(RT_ERR_IO, "cannot write " + path);
        std::fprintf(j, "{\"sampleCount\": %u, \"renderingTime\": %.9g, \"width\": %d, \"height\": %d}\n",
                     sampleCount, renderingTime, width, height);
        std::fclose(j);
    }
    void readAccumulation(const std::string& path, rt_ctx* ctx = nullptr) {
        FILE* f = std::fopen(path.c_str(), "rb");
        if (!f) throw Error(RT_ERR_IO, "cannot read " + path);
        int w = 0, h = 0;
        float endian = 0.0f;
        const bool head = std::fscanf(f, "PF %d %d %f", &w, &h, &endian) == 3 && std::fgetc(f) == '\n';
        if (!head || w != width || h != height || endian >= 0.0f) {
            std::fclose(f);
            throw Error(RT_ERR_IO, path + ": not a little-endian RGB PFM of this canvas's size");
        }
        std::vector<float> acc(radiance.size());
        const bool ok = std::fread(acc.data(), sizeof(float), acc.size(), f) == acc.size();
        std::fclose(f);
        FILE* j = std::fopen((path + ".json").c_str(), "r");
        unsigned n = 0;
        float t = 0.0f;
        const bool meta = j && std::fscanf(j, " { \"sampleCount\": %u, \"renderingTime\": %f", &n, &t) == 2;
        if (j) std::fclose(j);
        if (!ok || !meta) throw Error(RT_ERR_IO, "cannot read " + path + " / its .json");
        radiance = acc;
        if (ctx && rt_canvas_write_accumulation(device(ctx), acc.data()) != RT_OK)
            throw Error(RT_ERR_HIP, "readAccumulation: device write failed");
        sampleCount = n;
        scale = n ? 1.0f / n : 0.0f;
        renderingTime = t;
    }
    // writeToPPM (Canvas.h:116-139): top row first.
    void writeToPPM(const std::string& path) const {
        const std::vector<uint8_t>& px = pixelBuffer;
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) throw Error(RT_ERR_IO, "cannot write " + path);
        std::fprintf(f, "P6\n%d %d\n255\n", width, height);
        for (int32_t y = height - 1; y >= 0; --y) std::fwrite(&px[(size_t)y * width * 3], 1, (size_t)width * 3, f);
        std::fclose(f);
    }
    // writeToPNG (Canvas.h:141-154, stbi_write_png with the rows flipped): RGB8, top row
    // first, zlib stream of stored (uncompressed) deflate blocks - no codec dependency.
    void writeToPNG(const std::string& path) const {
        const std::vector<uint8_t>& px = pixelBuffer;
        std::vector<uint8_t> raw;  // filter byte 0 + one top-down row
        raw.reserve((size_t)height * ((size_t)width * 3 + 1));
        for (int32_t y = height - 1; y >= 0; --y) {
            raw.push_back(0);
            raw.insert(raw.end(), px.begin() + (size_t)y * width * 3, px.begin() + (size_t)(y + 1) * width * 3);
        }
        std::vector<uint8_t> z{0x78, 0x01};
        for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
            const size_t n = std::min<size_t>(65535, raw.size() - off);
            z.push_back(off + n >= raw.size() ? 1 : 0);  // BFINAL, BTYPE = 00 (stored)
            z.push_back((uint8_t)(n & 0xFF));
            z.push_back((uint8_t)(n >> 8));
            z.push_back((uint8_t)(~n & 0xFF));
            z.push_back((uint8_t)((~n >> 8) & 0xFF));
            z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
            if (n == 0) break;
        }
        uint32_t a = 1, b = 0;  // Adler-32 of the uncompressed data
        for (uint8_t v : raw) {
            a = (a + v) % 65521u;
            b = (b + a) % 65521u;
        }
        for (int k = 3; k >= 0; --k) z.push_back((uint8_t)(((b << 16) | a) >> (8 * k)));
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) throw Error(RT_ERR_IO, "cannot write " + path);
        static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
        std::fwrite(sig, 1, 8, f);
        auto be32 = [](uint8_t* o, uint32_t v) {
            for (int k = 0; k < 4; ++k) o[k] = (uint8_t)(v >> (24 - 8 * k));
        };
        auto chunk = [&](const char* tag, const std::vector<uint8_t>& data) {
            uint8_t hdr[8];
            be32(hdr, (uint32_t)data.size());
            std::memcpy(hdr + 4, tag, 4);
            std::fwrite(hdr, 1, 8, f);
            if (!data.empty()) std::fwrite(data.data(), 1, data.size(), f);
            uint32_t crc = 0xFFFFFFFFu;  // CRC-32 over tag + data
            auto upd = [&](uint8_t v) {
                crc ^= v;
                for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
            };
            for (int k = 0; k < 4; ++k) upd((uint8_t)tag[k]);
            for (uint8_t v : data) upd(v);
            uint8_t c[4];
            be32(c, crc ^ 0xFFFFFFFFu);
            std::fwrite(c, 1, 4, f);
        };
        std::vector<uint8_t> ihdr(13, 0);
        be32(ihdr.data(), (uint32_t)width);
        be32(ihdr.data() + 4, (uint32_t)height);
        ihdr[8] = 8;  // bit depth
        ihdr[9] = 2;  // colour type RGB
        chunk("IHDR", ihdr);
        chunk("IDAT", z);
        chunk("IEND", {});
        std::fclose(f);
    }

private:
    int32_t width = 0, height = 0;
    std::vector<float> radiance;
    std::vector<uint8_t> pixelBuffer;
    uint32_t sampleCount = 0;
    float scale = 0.0f;
    float renderingTime = 0.0f;
    rt_canvas* device_ = nullptr;
};

class Context {
public:
    explicit Context(int32_t device = 0) {
        rt_status s = rt_create(device, &ctx_);
        if (s != RT_OK) throw Error(s, "rt_create failed");
    }
    ~Context() {
        if (table_owner() == this) table_owner() = nullptr;
        rt_destroy(ctx_);
    }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;

    rt_ctx* raw() const { return ctx_; }
    void check(rt_status s) const {
        if (s != RT_OK) throw Error(s, rt_last_error(ctx_));
    }

    // Pointer tables (createObjectPtrArray<Material*> / <Hitable*>, kernels.h:26-31).
    Material** materials(int32_t n = 4096) {
        table_owner() = this;
        return table(mat_slots_, mat_ptrs_, n, true);
    }
    Hitable** objects(int32_t n = 4096) {
        table_owner() = this;
        return table(obj_slots_, obj_ptrs_, n, false);
    }

    // the renderer reads the camera's current view, as renderKernel reads the managed Camera
    void setCamera(const Camera& c) { check(rt_camera_apply(ctx_, &c.state())); }
    // the context's Camera object (a scene file's camera after loadYAMLScene)
    Camera getCamera() const {
        rt_camera_state s{};
        check(rt_get_camera(ctx_, &s));
        return Camera(s);
    }
    void commit() { check(rt_commit(ctx_)); }
    // initialize() for SCENE == 1 (main.cu:623-786): camera, pre-seeded materials
    // and objects of a scene YAML; model paths relative to modelsDir. The
    // materials()/objects() tables are not updated: query rt_material_defined.
    void loadYAMLScene(const std::string& path, const std::string& modelsDir, int32_t width, int32_t height) {
        check(rt_load_yaml_scene(ctx_, path.c_str(), modelsDir.c_str(), width, height));
    }
    uint64_t sceneDigest() const {
        uint64_t h = 0;
        check(rt_scene_digest(ctx_, &h));
        return h;
    }
    // BVH builds of commit() / processTriangleData(): RT_BVH_HOST (Recurse on the host,
    // BVH.cpp:94-497) or RT_BVH_GPU (its byte-identical GPU restatement).
    void setBVHBuilder(int32_t builder) { check(rt_set_bvh_builder(ctx_, builder)); }
    // UpdateBoundingVolumeHierarchy's `.bvh` cache (BVH.cpp:500-554): RT_BVH_CACHE_READ |
    // RT_BVH_CACHE_WRITE is the reference's read-if-fresh / write-after-build behaviour.
    void setBVHCache(int32_t mode) { check(rt_set_bvh_cache(ctx_, mode)); }
    double lastBVHBuildMs() const {
        double ms = 0.0;
        check(rt_bvh_build_stats(ctx_, &ms, nullptr));
        return ms;
    }

    // pathTracing (main.cu:875-898): one frame of `spp` samples into the canvas,
    // with rayColor over the create* scene.
    void pathTracing(Canvas& canvas, int32_t spp, int32_t bounces, uint32_t seed = 1984,
                     uint32_t sampleOffset = 0) {
        commit();
        rt_render_params p{canvas.getWidth(), canvas.getHeight(), spp, bounces, seed, sampleOffset,
                           1, 0, 1, 0, RT_INTEGRATOR_RAYCOLOR, 0};
        check(rt_render(ctx_, &p, canvas.data()));
        canvas.gammaFromRadiance();
    }

    // One GPU_REALTIME frame (main.cu:876-888 after incrementSampleCount): `spp` fresh samples
    // per pixel (the reference: 1) added to the canvas's device accumulation, its pixel buffer
    // = gamma(acc * (1 / samples so far)). The canvas's sample count is the frame count, as the
    // reference's (one incrementSampleCount per frame).
    void accumulate(Canvas& canvas, int32_t spp, int32_t bounces, uint32_t seed = 1984,
                    int32_t integrator = RT_INTEGRATOR_RAYCOLOR) {
        if (canvas.getSampleCount() == 0) throw Error(RT_ERR_STATE, "accumulate: call incrementSampleCount first");
        if (integrator == RT_INTEGRATOR_RAYCOLOR) commit();
        const uint32_t frames = canvas.getSampleCount();
        rt_render_params p{canvas.getWidth(), canvas.getHeight(), spp, bounces, seed, (frames - 1) * (uint32_t)spp,
                           1, 0, 1, 0, integrator, 0};
        rt_canvas* d = canvas.device(ctx_);
        check(rt_canvas_accumulate(d, &p, frames * (uint32_t)spp));
        check(rt_canvas_read_pixels(d, canvas.getPixelBuffer()));
    }

    // prepareCUDAscene (main.cu:404-553): loadObject(...) per PLY, then
    // processTriangleData(offset) builds the BVH and uploads it.
    void loadObject(const std::string& file, int32_t reflectionType) {
        check(rt_load_object(ctx_, file.c_str(), reflectionType));
    }
    void processTriangleData(Vector3Df offset, float maxCoord = 1.0f) {
        check(rt_process_triangle_data(ctx_, offset.data(), maxCoord, nullptr));
    }
    // renderKernel's committed pathTrace call (main.cu:187; 5 bounces there).
    void pathTraceFrame(Canvas& canvas, int32_t spp, int32_t bounces = 5, uint32_t seed = 1984,
                        uint32_t sampleOffset = 0) {
        rt_render_params p{canvas.getWidth(), canvas.getHeight(), spp, bounces, seed, sampleOffset,
                           1, 0, 1, 0, RT_INTEGRATOR_PATHTRACE, 0};
        check(rt_render(ctx_, &p, canvas.data()));
        canvas.gammaFromRadiance();
    }

    // called by the factories below
    void markMaterial(int32_t i) { slot(mat_slots_, mat_ptrs_, i, true); }
    void markObject(int32_t i) { slot(obj_slots_, obj_ptrs_, i, false); }

private:
    Material** table(std::vector<std::unique_ptr<Material>>& slots, std::vector<Material*>& ptrs,
                     int32_t n, bool) {
        if ((int32_t)ptrs.size() < n) {
            ptrs.resize(n, nullptr);
            slots.resize(n);
        }
        return ptrs.data();
    }
    void slot(std::vector<std::unique_ptr<Material>>& slots, std::vector<Material*>& ptrs, int32_t i, bool) {
        // Tables are fixed-size once handed out (growing them would invalidate
        // the caller's Material** / Hitable**), like createObjectPtrArray(n).
        if (i < 0 || i >= (int32_t)ptrs.size()) throw Error(RT_ERR_INVALID, "slot index beyond table size");
        if (!slots[i]) slots[i].reset(new Material{this, i});
        ptrs[i] = slots[i].get();
    }

    rt_ctx* ctx_ = nullptr;
    std::vector<std::unique_ptr<Material>> mat_slots_, obj_slots_;
    std::vector<Material*> mat_ptrs_, obj_ptrs_;
};

// pathTracing over several GPUs from one process: contexts[k] renders the
// row tiles of rank k (same scene on each, committed here), one ncclGather brings them to
// contexts[0]'s device, where the rows are de-interleaved; the frame lands in `canvas`.
inline void pathTracingMulti(const std::vector<Context*>& contexts, Canvas& canvas, int32_t spp,
                             int32_t bounces, int32_t rowBlock = 2, uint32_t seed = 1984) {
    if (contexts.empty()) throw Error(RT_ERR_INVALID, "no contexts");
    std::vector<rt_ctx*> raw;
    for (Context* c : contexts) {
        c->commit();
        raw.push_back(c->raw());
    }
    rt_render_params p{canvas.getWidth(), canvas.getHeight(), spp, bounces, seed, 0,
                       rowBlock, 0, 1, 0, RT_INTEGRATOR_RAYCOLOR, 0};
    contexts[0]->check(rt_render_multi(raw.data(), (int32_t)raw.size(), &p, canvas.data()));
    canvas.gammaFromRadiance();
}

namespace detail {
inline int32_t mat_index(Material* m) {
    if (!m) throw Error(RT_ERR_INVALID, "material is nullptr");
    return m->index;
}
}  // namespace detail

// ---- kernels.h factories (same names and argument order) ----
// They act on the context whose tables were handed out last (table_owner()).

inline void createLambertianMaterial(Material** materials, int32_t index, Vector3Df albedo, float absorb = 1.0f) {
    Context& c = *table_owner();
    c.check(rt_material_lambertian(c.raw(), index, albedo.data(), absorb));
    c.markMaterial(index);
    (void)materials;
}
inline void createMetalMaterial(Material** materials, int32_t index, Vector3Df albedo, float fuzz = 1.0f) {
    Context& c = *table_owner();
    c.check(rt_material_metal(c.raw(), index, albedo.data(), fuzz));
    c.markMaterial(index);
    (void)materials;
}
inline void createDieletricMaterial(Material** materials, int32_t index, float indexOfRefraction = 1.5f) {
    Context& c = *table_owner();
    c.check(rt_material_dielectric(c.raw(), index, indexOfRefraction));
    c.markMaterial(index);
    (void)materials;
}
inline void createEmissionMaterial(Material** materials, int32_t index, Vector3Df albedo, float intensity = 1.0f) {
    Context& c = *table_owner();
    c.check(rt_material_emission(c.raw(), index, albedo.data(), intensity));
    c.markMaterial(index);
    (void)materials;
}
// Build extensions for participating media (rtmi.h rt_material_isotropic /
// rt_constant_medium; the reference has no media).
inline void createIsotropicMaterial(Material** materials, int32_t index, Vector3Df albedo) {
    Context& c = *table_owner();
    c.check(rt_material_isotropic(c.raw(), index, albedo.data()));
    c.markMaterial(index);
    (void)materials;
}
inline void createSphere(Hitable** spheres, int32_t index, Vector3Df center, float radius, Material* material,
                         bool bShading = true) {
    Context& c = *table_owner();
    c.check(rt_sphere(c.raw(), index, center.data(), radius, detail::mat_index(material), bShading));
    c.markObject(index);
    (void)spheres;
}
inline void createMovingSphere(Hitable** spheres, int32_t index, Vector3Df center0, Vector3Df center1, float time0,
                               float time1, float radius, Material* material) {
    Context& c = *table_owner();
    c.check(rt_moving_sphere(c.raw(), index, center0.data(), center1.data(), time0, time1, radius,
                             detail::mat_index(material)));
    c.markObject(index);
    (void)spheres;
}
inline void createPlane(Hitable** planes, int32_t index, const Vector3Df& position, const Vector3Df& normal,
                        const Vector3Df& extend, Material* material, PlaneOrientation orientation,
                        bool bTwoSide = true) {
    Context& c = *table_owner();
    c.check(rt_plane(c.raw(), index, position.data(), normal.data(), extend.data(), detail::mat_index(material),
                     (int32_t)orientation, bTwoSide));
    c.markObject(index);
    (void)planes;
}
inline void createCube(Hitable** cubes, int32_t index, const Vector3Df& center, const Vector3Df& extend,
                       Material* material) {
    Context& c = *table_owner();
    c.check(rt_cube(c.raw(), index, center.data(), extend.data(), detail::mat_index(material)));
    c.markObject(index);
    (void)cubes;
}
inline void createConstantMedium(Hitable** objects, int32_t index, const Vector3Df& center,
                                 const Vector3Df& extend, float density, Material* material) {
    Context& c = *table_owner();
    c.check(rt_constant_medium(c.raw(), index, center.data(), extend.data(), density,
                               detail::mat_index(material)));
    c.markObject(index);
    (void)objects;
}
// createTriangleMeshData + createMesh (main.cu:384-401, kernels.h:126-133) from
// world-space triangle vertices (loadModel(...).vertices, 3 per triangle).
inline void createMesh(Hitable** meshes, int32_t index, const std::vector<Vector3Df>& vertices,
                       Material* material) {
    Context& c = *table_owner();
    c.check(rt_mesh(c.raw(), index, vertices.empty() ? nullptr : &vertices[0].x, (int32_t)(vertices.size() / 3),
                    detail::mat_index(material)));
    c.markObject(index);
    (void)meshes;
}
// loadModel(file, scale, rotate, offset) + createMesh in one call.
inline void createMeshFromOBJ(Hitable** meshes, int32_t index, const std::string& path, Vector3Df scale,
                              Vector3Df rotate, Vector3Df offset, Material* material) {
    Context& c = *table_owner();
    c.check(rt_mesh_obj(c.raw(), index, path.c_str(), scale.data(), rotate.data(), offset.data(),
                        detail::mat_index(material)));
    c.markObject(index);
    (void)meshes;
}

}  // namespace rtmi
