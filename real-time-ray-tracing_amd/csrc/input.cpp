// input.cpp — the RayTracer input surface (inputControl.cu) behind the C-ABI: a windowing host
// forwards its key / cursor events here and rt_draw applies the movement once per frame.
//
//   keyboardUpdate       inputControl.cu:29-52   (WASD/C/X movement, shift = slow, ctrl+C / ctrl+V
//                                                 save / load the camera file)
//   cursorPosUpdate      inputControl.cu:54-76   (yaw / pitch from the cursor delta, pitch clamp)
//   scrollUpdate         inputControl.cu:78-81   (no-op)
//   mouseButtenUpdate    inputControl.cu:83-86   (no-op)
//   InputControlUpdate   inputControl.cu:88-113  (pos += moveDir * deltaTime * moveSpeed)
//
// The reference keeps this state in one global (InputControl inputControl); here every context
// has its own.  Key, action and modifier values are GLFW's.
#include <math.h>

#include "context.h"

namespace {

constexpr int kKeyA = 65, kKeyC = 67, kKeyD = 68, kKeyS = 83, kKeyV = 86, kKeyW = 87, kKeyX = 88;
constexpr int kKeyLeftShift = 340;
constexpr int kRelease = 0, kPress = 1;
constexpr int kModControl = 0x0002;
constexpr float kPiOver2 = 1.5707963267948966192313216916397514420985f;  // linearMath.h:12

void set_flag(bool& flag, int action) {
    if (action == kPress) flag = true;
    else if (action == kRelease) flag = false;
}

float clampf(float a, float lo, float hi) { return a < lo ? lo : a > hi ? hi : a; }  // linearMath.h:479

}  // namespace

// InputControlUpdate (inputControl.cu:88-113), called by rt_draw after the dynamic-resolution
// step with the frame's deltaTime.  camera.dir is Camera::update's (rt_camera_update).
void rt_input_control_update(rt_context* ctx, float deltaTime) {
    InputState& in = ctx->input;
    if (!(in.moveW || in.moveS || in.moveA || in.moveD || in.moveC || in.moveX)) return;
    HostCamera hc;
    rt_camera_update(ctx->camera, ctx->renderW, ctx->renderH, hc);
    const float* d = hc.dir;
    // strafeDir = cross(camera.dir, Float3(0, 1, 0)).normalize(): the dop-based cross reduces to
    // these products exactly (the zero terms are exact)
    auto dop = [](float a, float b, float c, float e) {
        const float ce = c * e;
        const float err = fmaf(-c, e, ce);
        const float dp = fmaf(a, b, -ce);
        return dp + err;
    };
    float s[3] = {dop(d[1], 0.0f, d[2], 1.0f), dop(d[2], 0.0f, d[0], 0.0f), dop(d[0], 1.0f, d[1], 0.0f)};
    const float n = sqrtf(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    s[0] /= n; s[1] /= n; s[2] /= n;
    float m[3] = {0.0f, 0.0f, 0.0f};
    for (int k = 0; k < 3; ++k) {
        if (in.moveW) m[k] += d[k];
        if (in.moveS) m[k] -= d[k];
        if (in.moveA) m[k] -= s[k];
        if (in.moveD) m[k] += s[k];
    }
    if (in.moveC) m[1] += 1.0f;
    if (in.moveX) m[1] -= 1.0f;
    // camera.pos += movingDir * deltaTime * moveSpeed (two roundings per component)
    for (int k = 0; k < 3; ++k) ctx->camera.pos[k] += (m[k] * deltaTime) * in.moveSpeed;
}

extern "C" {

int rt_keyboard_update(rt_context* ctx, int key, int scancode, int action, int mods) {
    (void)scancode;
    if (!ctx) return RT_ERR_ARG;
    InputState& in = ctx->input;
    if (mods == kModControl) {
        int rc = RT_OK;
        if (key == kKeyC && action == kPress) rc = rt_save_camera(ctx, ctx->cameraSaveFileName.c_str());
        if (key == kKeyV && action == kPress) rc = rt_load_camera(ctx, ctx->cameraSaveFileName.c_str());
        return rc;
    }
    if (key == kKeyW) set_flag(in.moveW, action);
    if (key == kKeyS) set_flag(in.moveS, action);
    if (key == kKeyA) set_flag(in.moveA, action);
    if (key == kKeyD) set_flag(in.moveD, action);
    if (key == kKeyC) set_flag(in.moveC, action);
    if (key == kKeyX) set_flag(in.moveX, action);
    if (key == kKeyLeftShift) {
        if (action == kPress) in.moveSpeed = 0.001f;
        else if (action == kRelease) in.moveSpeed = 0.01f;
    }
    return RT_OK;
}

int rt_cursor_pos_update(rt_context* ctx, double xpos, double ypos) {
    if (!ctx) return RT_ERR_ARG;
    InputState& in = ctx->input;
    if (in.cursorReset) {
        in.cursorReset = false;
        in.xpos = xpos;
        in.ypos = ypos;
        return RT_OK;
    }
    in.deltax = (float)(xpos - in.xpos);
    in.deltay = (float)(ypos - in.ypos);
    in.xpos = xpos;
    in.ypos = ypos;
    rt_camera& c = ctx->camera;
    c.yaw -= in.deltax * in.cursorMoveSpeed;
    c.pitch -= in.deltay * in.cursorMoveSpeed;
    c.pitch = clampf(c.pitch, -kPiOver2 + 0.1f, kPiOver2 - 0.1f);
    return RT_OK;
}

int rt_scroll_update(rt_context* ctx, double xoffset, double yoffset) {
    (void)xoffset;
    (void)yoffset;
    return ctx ? RT_OK : RT_ERR_ARG;
}

int rt_mouse_button_update(rt_context* ctx, int button, int action, int mods) {
    (void)button;
    (void)action;
    (void)mods;
    return ctx ? RT_OK : RT_ERR_ARG;
}

int rt_set_cursor_reset(rt_context* ctx, int reset) {
    if (!ctx) return RT_ERR_ARG;
    ctx->input.cursorReset = reset != 0;
    return RT_OK;
}

}  // extern "C"
