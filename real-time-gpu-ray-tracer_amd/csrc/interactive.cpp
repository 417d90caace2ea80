// interactive.cpp — the host half of the reference's interactive frame loop, without a window
// (SURVEY §8f row 4): camera control from key / mouse input and the frame limiter.
//
// Restates, on caller-supplied input instead of SDL events:
//   SDL_OpenGLWindow::getOperateArgs        include/Global/SDL_OpenGLWindow.cuh:63-74
//   SDL_OpenGLWindow::calculateNewPosition  src/Global/SDL_OpenGLWindow.cu:182-256
//   the loop's camera / move-speed steps    src/Global/Renderer.cu:236-262
//   the 120-fps limiter                     src/Global/Renderer.cu:327-337
// Vector arithmetic follows Vec3 / Point3 (include/Basic/Vec3.cuh:57-160, Point3.cuh:45-84) in the same
// evaluation order (compiled with -ffp-contract=off), so a scripted input sequence moves the camera through
// the same float values the reference's loop computes.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <string>
#include <thread>

#include "../../include/rt.h"
#include "host_math.hpp"

void rtamd_set_error(const std::string &msg);   // rt_api.cpp

using namespace rtamd::hm;

namespace {

// Vec3::rotate (Vec3.cuh:140-159): Rodrigues' formula about unit(axis)
V3 rotate(V3 v, V3 axis, float angle) {
    const V3 k = unit(axis);
    const float c = std::cos(angle), s = std::sin(angle);
    const V3 part1 = v * c;
    const V3 part2 = cross(k, v) * s;
    const V3 part3 = k * dot(k, v) * (1.0f - c);
    return part1 + part2 + part3;
}

rt_vec3 to_rt(V3 a) { return rt_vec3{a.x, a.y, a.z}; }

}  // namespace

extern "C" {

rt_status rt_camera_control_init(rt_camera_control *ctl, float fps_limit, float mouse_sensitivity, float pitch_limit_degree,
                                 uint32_t move_speed_n_steps, float move_speed_change_step) {
    if (!ctl) { rtamd_set_error("null argument"); return RT_ERR_INVALID_ARGUMENT; }
    if (!(fps_limit > 0.0f)) { rtamd_set_error("fps_limit must be > 0 (INFINITY: no cap)"); return RT_ERR_INVALID_ARGUMENT; }
    *ctl = rt_camera_control{};
    ctl->mouse_sensitivity = mouse_sensitivity;
    // .pitchLimitDegree = PI / MathHelper::degreeToRadian(pitchLimitDegree) (SDL_OpenGLWindow.cuh:66):
    // kept as the reference computes it (80 degrees -> 2.25, beyond asin's range, so the clamp never fires)
    ctl->pitch_limit = PI / (pitch_limit_degree * PI / 180.0f);
    ctl->move_speed = static_cast<float>(move_speed_n_steps) * move_speed_change_step;
    ctl->move_speed_change_step = move_speed_change_step;
    ctl->fps_limit = fps_limit;
    ctl->restrict_frame_count = fps_limit != INFINITY ? 1u : 0u;
    ctl->target_frame_us = static_cast<int64_t>(1000000.0f / fps_limit);
    ctl->sleep_margin_us = 2000;
    ctl->relative_mouse = 1;                          // SDL_SetRelativeMouseMode(SDL_TRUE) (Renderer.cu:230)
    return RT_OK;
}

rt_status rt_camera_move(rt_camera_input *camera, rt_camera_control *ctl, const rt_input_state *in, uint32_t *moved) {
    if (!camera || !ctl || !in) { rtamd_set_error("null argument"); return RT_ERR_INVALID_ARGUMENT; }
    // mouse motion is accumulated only while relative mode is on (SDL_OpenGLWindow.cu:173-176); the click
    // toggles the mode after this frame's events were read (Renderer.cu:239-241)
    const int32_t mdx = ctl->relative_mouse ? in->dx : 0, mdy = ctl->relative_mouse ? in->dy : 0;
    if (in->mouse_click) ctl->relative_mouse ^= 1u;

    // the camera frame calculateCameraProperties derived from this camera (RenderPin.cu:84-86)
    const V3 center = of(camera->center), target = of(camera->target), up = of(camera->up);
    const V3 cW = unit(target - center);
    const V3 cU = unit(cross(cW, up));
    const V3 cV = unit(cross(cU, cW));

    V3 ret_center = center, ret_target = target;
    bool is_moved = false;
    if (mdx != 0 || mdy != 0) {                                          // SDL_OpenGLWindow.cu:192-231
        is_moved = true;
        const V3 view = target - center;                                 // Point3::constructVector
        V3 W = unit(cW);
        const V3 U = unit(cU);
        const V3 V = unit(cV);
        const float yaw = -static_cast<float>(mdx) * ctl->mouse_sensitivity;
        W = rotate(W, V, yaw);
        const float pitch = -static_cast<float>(mdy) * ctl->mouse_sensitivity;
        W = rotate(W, U, pitch);
        float new_pitch = std::asin(W.y);
        bool correct = false;
        if (new_pitch > ctl->pitch_limit) { new_pitch = ctl->pitch_limit; correct = true; }
        else if (new_pitch < -ctl->pitch_limit) { new_pitch = -ctl->pitch_limit; correct = true; }
        if (correct) {
            const V3 horizontal = unit(v3(W.x, 0.0f, W.z));
            const float mag = std::cos(new_pitch);
            W = horizontal * mag + v3(0.0f, std::sin(new_pitch), 0.0f);
        }
        ret_target = center + W * length(view);
    }
    // keys: movement in the horizontal plane / along up (SDL_OpenGLWindow.cu:234-252)
    V3 dir = v3(0.0f, 0.0f, 0.0f);
    const V3 fwd = unit(v3(cW.x, 0.0f, cW.z));
    if (in->key_w) dir = dir + fwd;
    if (in->key_s) dir = dir - fwd;
    if (in->key_d) dir = dir + cU;
    if (in->key_a) dir = dir - cU;
    if (in->key_space) dir = dir + up;
    if (in->key_lshift) dir = dir - up;
    if (dot(dir, dir) > 0.0f) {
        is_moved = true;
        const V3 t = unit(dir) * ctl->move_speed;
        ret_center = ret_center + t;
        ret_target = ret_target + t;
    }
    if (is_moved) {                                                      // Renderer.cu:247-251
        camera->center = to_rt(ret_center);
        camera->target = to_rt(ret_target);
    }
    if (in->d_speed != 0) {                                              // Renderer.cu:252-258
        if (in->d_speed > 0) ctl->move_speed += ctl->move_speed_change_step;
        else ctl->move_speed = ctl->move_speed < ctl->move_speed_change_step ? 0.0f
                                                                              : ctl->move_speed - ctl->move_speed_change_step;
    }
    if (moved) *moved = is_moved ? 1u : 0u;
    return RT_OK;
}

int64_t rt_clock_ns(void) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int64_t rt_frame_pace(const rt_camera_control *ctl, int64_t frame_start_ns) {
    if (!ctl) return 0;
    const int64_t target = ctl->target_frame_us * 1000, margin = ctl->sleep_margin_us * 1000;
    const int64_t t0 = rt_clock_ns();
    const int64_t work = t0 - frame_start_ns;
    if (work >= target) return 0;
    const int64_t wait = target - work;                                  // Renderer.cu:328-336
    if (wait > margin) std::this_thread::sleep_for(std::chrono::nanoseconds(wait - margin));
    while (rt_clock_ns() - frame_start_ns < target) {}
    return rt_clock_ns() - t0;
}

}  // extern "C"
