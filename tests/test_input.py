"""Input surface (inputControl.cu:29-113) over the C-ABI: cursor -> yaw / pitch, key flags,
ctrl+C / ctrl+V camera save / load (CPU), and the per-frame InputControlUpdate movement that
rt_draw applies (GPU).  Expected values restate the reference's float arithmetic in numpy
float32; the camera direction uses the oracle's rt_sinf / rt_cosf (the renderer's own)."""
import numpy as np
import pytest

KEY_A, KEY_C, KEY_D, KEY_S, KEY_V, KEY_W, KEY_X, KEY_SHIFT = 65, 67, 68, 83, 86, 87, 88, 340
RELEASE, PRESS, REPEAT = 0, 1, 2
MOD_CONTROL = 2
f32 = np.float32


def make(rtx, tmp_path, extra_file=""):
    cfg = rtx.write_config(str(tmp_path / "c.toml"), 64, 36)
    if extra_file:
        text = open(cfg).read().replace("[file]\nloadCameraAtInit = false\n",
                                        '[file]\nloadCameraAtInit = false\ncameraSaveFileName = "%s"\n' % extra_file)
        open(cfg, "w").write(text)
    return rtx.RayTracer(64, 36, cfg)


def test_cursor_turns_camera(rtx, tmp_path):
    rt = make(rtx, tmp_path)
    c0 = rt.camera
    rt.cursor_pos_update(100.0, 50.0)          # first event after a cursor reset: position only
    c1 = rt.camera
    assert (c1.yaw, c1.pitch) == (c0.yaw, c0.pitch)
    rt.cursor_pos_update(130.5, 20.25)         # dx = 30.5, dy = -29.75
    c2 = rt.camera
    assert c2.yaw == f32(f32(c0.yaw) - f32(30.5) * f32(0.001))
    assert c2.pitch == f32(f32(c0.pitch) - f32(-29.75) * f32(0.001))
    rt.cursor_pos_update(130.5, -5000.0)       # pitch clamped to pi/2 - 0.1
    assert rt.camera.pitch == f32(f32(1.5707963267948966) - f32(0.1))
    rt.set_cursor_reset(True)
    rt.cursor_pos_update(0.0, 0.0)             # re-anchored, no turn
    assert rt.camera.pitch == f32(f32(1.5707963267948966) - f32(0.1))
    rt.scroll_update(1.0, 2.0)                 # no-ops in the reference
    rt.mouse_button_update(0, PRESS, 0)
    rt.cleanup()


def test_ctrl_c_ctrl_v_save_and_load_camera(rtx, tmp_path):
    path = str(tmp_path / "cam.bin")
    rt = make(rtx, tmp_path, extra_file=path)
    cam = rt.camera
    cam.pos[:] = (1.0, 2.0, 3.0)
    cam.yaw = 0.5
    rt.camera = cam
    rt.keyboard_update(KEY_C, 0, PRESS, MOD_CONTROL)        # save
    cam.pos[:] = (9.0, 9.0, 9.0)
    cam.yaw = -1.0
    rt.camera = cam
    rt.keyboard_update(KEY_V, 0, PRESS, MOD_CONTROL)        # load
    got = rt.camera
    assert list(got.pos) == [1.0, 2.0, 3.0] and got.yaw == f32(0.5)
    rt.keyboard_update(KEY_C, 0, RELEASE, MOD_CONTROL)      # release with ctrl: nothing
    rt.cleanup()


def expected_moves(oracle, cam, keys, dt, speed):
    """InputControlUpdate (inputControl.cu:88-113) in float32."""
    sin = lambda v: f32(oracle.lib().orc_rtmath(0, float(v), 0.0))
    cos = lambda v: f32(oracle.lib().orc_rtmath(1, float(v), 0.0))
    cp = cos(cam.pitch)
    d = np.array([sin(cam.yaw) * cp, sin(cam.pitch), cos(cam.yaw) * cp], f32)
    s = np.array([-d[2], 0.0, d[0]], f32)                   # cross(dir, (0, 1, 0))
    n = np.sqrt(f32(s[0] * s[0] + s[1] * s[1]) + s[2] * s[2], dtype=f32)
    s = (s / n).astype(f32)
    m = np.zeros(3, f32)
    if KEY_W in keys: m = m + d
    if KEY_S in keys: m = m - d
    if KEY_A in keys: m = m - s
    if KEY_D in keys: m = m + s
    if KEY_C in keys: m[1] += f32(1.0)
    if KEY_X in keys: m[1] -= f32(1.0)
    return (np.array(cam.pos, f32) + (m * f32(dt)).astype(f32) * f32(speed)).astype(f32)


@pytest.mark.gpu
def test_draw_applies_held_keys(rtx, oracle, tmp_path):
    rt = make(rtx, tmp_path).init()
    rt.set_delta_time(16.667)
    cam = rt.camera
    cam.yaw, cam.pitch = 0.4, -0.3
    rt.camera = cam
    rt.keyboard_update(KEY_W, 0, PRESS, 0)
    rt.keyboard_update(KEY_D, 0, PRESS, 0)
    rt.keyboard_update(KEY_C, 0, PRESS, 0)
    before = rt.camera
    rt.draw()
    after = rt.camera
    assert np.array_equal(np.array(after.pos, f32), expected_moves(oracle, before, {KEY_W, KEY_D, KEY_C}, 16.667, 0.01))
    rt.keyboard_update(KEY_SHIFT, 0, PRESS, 0)              # slow movement
    rt.keyboard_update(KEY_W, 0, RELEASE, 0)
    rt.keyboard_update(KEY_D, 0, REPEAT, 0)                 # repeat keeps the flag
    rt.set_delta_time(20.0)
    before = rt.camera
    rt.draw()
    after = rt.camera
    assert np.array_equal(np.array(after.pos, f32), expected_moves(oracle, before, {KEY_D, KEY_C}, 20.0, 0.001))
    for k in (KEY_D, KEY_C, KEY_SHIFT):
        rt.keyboard_update(k, 0, RELEASE, 0)
    before = rt.camera
    rt.draw()
    assert list(rt.camera.pos) == list(before.pos)         # nothing held: no movement
    rt.cleanup()
