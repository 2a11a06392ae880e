// rt_camera.cpp — the reference's Camera object (Camera.h:12-196) on the host: its fields in
// rt_camera_state and its methods with the reference's float operations, in the order it
// evaluates them. Compiled with -ffp-contract=off like the rest of the library, so a frontend's
// camera moves (OpenGLFrontend.cpp:393-407, 586-611) land on the same floats as the
// reference's, and rt_camera_apply hands the view that Camera::getRay reads to a context.
#include <math.h>

#include "../../include/rtmi.h"
#include "rt_ctx.h"
#include "rt_math.h"

namespace {

using rt::v3;

v3 get(const float* a) { return v3{a[0], a[1], a[2]}; }
void put(float* a, v3 v) {
    a[0] = v.x;
    a[1] = v.y;
    a[2] = v.z;
}
bool finite3(const float* a) { return std::isfinite(a[0]) && std::isfinite(a[1]) && std::isfinite(a[2]); }

// Math::radians (Constants.h:29-31): pi / 180.0f * degree.
float radians(float deg) { return 3.1415926535897932f / 180.0f * deg; }

// rotateY (LinearAlgebra.h:84-87) with CUDATypes.h's float cos / sin.
v3 rotate_y(v3 v, float r) { return v3{v.x * cosf(r) + v.z * sinf(r), v.y, -v.x * sinf(r) + v.z * cosf(r)}; }

// rotate (LinearAlgebra.h:94-109): the axis-angle matrix, row by row, left to right.
v3 rotate(v3 v, v3 axis, float r) {
    const float c = cosf(r), s = sinf(r);
    const float n1 = axis.x, n2 = axis.y, n3 = axis.z;
    const float r00 = n1 * n1 * (1.0f - c) + c, r01 = n1 * n2 * (1.0f - c) - n3 * s,
                r02 = n1 * n3 * (1.0f - c) + n2 * s;
    const float r10 = n1 * n2 * (1.0f - c) + n3 * s, r11 = n2 * n2 * (1.0f - c) + c,
                r12 = n2 * n3 * (1.0f - c) - n1 * s;
    const float r20 = n1 * n3 * (1.0f - c) - n2 * s, r21 = n2 * n3 * (1.0f - c) + n1 * s,
                r22 = n3 * n3 * (1.0f - c) + c;
    return v3{r00 * v.x + r01 * v.y + r02 * v.z, r10 * v.x + r11 * v.y + r12 * v.z,
              r20 * v.x + r21 * v.y + r22 * v.z};
}

// Camera::updateLensRadius (Camera.h:110-113).
void update_lens_radius(rt_camera_state* c) {
    c->dirty = 1;
    c->lens_radius = c->aperture / 2.0f;
}

// eye += forward * movingSpeed * delta; center likewise (Camera.h:40-56, one axis each).
void move(rt_camera_state* c, const float* axis, float delta) {
    const v3 step = rt::scale(rt::scale(get(axis), c->moving_speed), delta);
    put(c->eye, rt::add(get(c->eye), step));
    put(c->center, rt::add(get(c->center), step));
    c->dirty = 1;
}

}  // namespace

extern "C" {

// Camera::updateViewMatrix (Camera.h:86-103): only while dirty; it leaves the flag set
// (updateLensRadius sets it), so pathTracing's isDirty() sees the change (main.cu:877-881).
rt_status rt_camera_update_view_matrix(rt_camera_state* c) {
    if (!c) return RT_ERR_INVALID;
    if (!c->dirty) return RT_OK;
    c->scale = tanf(radians(c->fov / 2.0f));
    c->viewport_height = 2.0f * c->scale;
    c->viewport_width = c->viewport_height * c->aspect_ratio;
    const v3 forward = rt::normalize(rt::sub(get(c->center), get(c->eye)));
    const v3 right = rt::normalize(rt::cross(forward, get(c->up)));
    const v3 true_up = rt::cross(right, forward);
    put(c->forward, forward);
    put(c->right, right);
    put(c->true_up, true_up);
    put(c->origin, get(c->eye));
    const v3 horizontal = rt::scale(rt::scale(right, c->viewport_width), c->focus_distance);
    const v3 vertical = rt::scale(rt::scale(true_up, c->viewport_height), c->focus_distance);
    put(c->horizontal, horizontal);
    put(c->vertical, vertical);
    put(c->lower_left, rt::add(rt::sub(rt::sub(get(c->eye), rt::divs(horizontal, 2.0f)), rt::divs(vertical, 2.0f)),
                               rt::scale(forward, c->focus_distance)));
    update_lens_radius(c);
    return RT_OK;
}

// Camera::initialize (Camera.h:19-34).
rt_status rt_camera_initialize(rt_camera_state* c, const float eye[3], const float center[3], const float up[3],
                               float aspect_ratio, float fov, float aperture, float focus_distance, float time0,
                               float time1) {
    if (!c || !eye || !center || !up || !finite3(eye) || !finite3(center) || !finite3(up) ||
        !std::isfinite(aspect_ratio) || !std::isfinite(fov) || !std::isfinite(aperture) ||
        !std::isfinite(focus_distance) || !std::isfinite(time0) || !std::isfinite(time1))
        return RT_ERR_INVALID;
    *c = rt_camera_state{};
    put(c->eye, get(eye));
    put(c->center, get(center));
    put(c->up, get(up));
    c->aspect_ratio = aspect_ratio;
    c->fov = fov;
    c->aperture = aperture;
    c->focus_distance = focus_distance;
    c->moving_speed = 1.5f;
    c->time0 = time0;
    c->time1 = time1;
    c->dirty = 1;
    return rt_camera_update_view_matrix(c);
}

rt_status rt_camera_walk(rt_camera_state* c, float delta) {  // Camera.h:40-44
    if (!c) return RT_ERR_INVALID;
    move(c, c->forward, delta);
    return RT_OK;
}

rt_status rt_camera_strafe(rt_camera_state* c, float delta) {  // Camera.h:46-50
    if (!c) return RT_ERR_INVALID;
    move(c, c->right, delta);
    return RT_OK;
}

rt_status rt_camera_raise(rt_camera_state* c, float delta) {  // Camera.h:52-56
    if (!c) return RT_ERR_INVALID;
    move(c, c->up, delta);
    return RT_OK;
}

// Camera::yaw (Camera.h:58-67): forward and right turn about +y; center = eye + forward.
rt_status rt_camera_yaw(rt_camera_state* c, float delta) {
    if (!c) return RT_ERR_INVALID;
    const v3 forward = rt::normalize(rotate_y(get(c->forward), delta));
    put(c->forward, forward);
    put(c->right, rt::normalize(rotate_y(get(c->right), delta)));
    put(c->center, rt::add(get(c->eye), forward));
    c->dirty = 1;
    return RT_OK;
}

// Camera::pitch (Camera.h:69-76): forward turns about right; center = eye + forward.
rt_status rt_camera_pitch(rt_camera_state* c, float delta) {
    if (!c) return RT_ERR_INVALID;
    const v3 forward = rt::normalize(rotate(get(c->forward), get(c->right), delta));
    put(c->forward, forward);
    put(c->center, rt::add(get(c->eye), forward));
    c->dirty = 1;
    return RT_OK;
}

// Camera::orbit (Camera.h:78-84): eye turns 0.01 rad about the vertical through `target`.
rt_status rt_camera_orbit(rt_camera_state* c, const float target[3]) {
    if (!c || !target) return RT_ERR_INVALID;
    const float x = c->eye[0], z = c->eye[2];
    c->eye[0] = (x - target[0]) * cosf(0.01f) - (z - target[2]) * sinf(0.01f) + target[0];
    c->eye[2] = (x - target[0]) * sinf(0.01f) + (z - target[2]) * cosf(0.01f) + target[2];
    c->dirty = 1;
    return RT_OK;
}

// Camera::setAperture (Camera.h:105-108).
rt_status rt_camera_set_aperture(rt_camera_state* c, float aperture) {
    if (!c) return RT_ERR_INVALID;
    c->aperture = aperture;
    update_lens_radius(c);
    return RT_OK;
}

// The fields Camera::getRay reads (Camera.h:151-168) as the context's camera: the view of the
// last updateViewMatrix, whatever has moved since (the reference's kernel reads the managed
// Camera the same way).
rt_status rt_camera_apply(rt_ctx* ctx, const rt_camera_state* c) {
    if (!ctx) return RT_ERR_INVALID;
    if (!c) return rtc::fail(ctx, RT_ERR_INVALID, "camera_apply: null camera");
    rt::CamRec r;
    r.origin = get(c->origin);
    r.lower_left = get(c->lower_left);
    r.horizontal = get(c->horizontal);
    r.vertical = get(c->vertical);
    r.right = get(c->right);
    r.true_up = get(c->true_up);
    r.lens_radius = c->lens_radius;
    r.time0 = c->time0;
    r.time1 = c->time1;
    const float* all[] = {c->origin, c->lower_left, c->horizontal, c->vertical, c->right, c->true_up};
    for (const float* a : all)
        if (!finite3(a)) return rtc::fail(ctx, RT_ERR_INVALID, "camera_apply: non-finite view");
    if (!std::isfinite(c->lens_radius) || !std::isfinite(c->time0) || !std::isfinite(c->time1))
        return rtc::fail(ctx, RT_ERR_INVALID, "camera_apply: non-finite view");
    ctx->scene.camera = r;
    ctx->scene.has_camera = true;
    ctx->cam_state = *c;
    return RT_OK;
}

}  // extern "C"
