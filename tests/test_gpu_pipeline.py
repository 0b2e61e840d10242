"""Frame pipelining (rt_set_post_stream): the denoise/post chain of frame f on a second
stream, overlapping the trace of frame f+1 into the other G-buffer set.  Every output after
a 6-frame moving-camera sequence, and the RGBA8 image of every frame, must be identical to
the serial order (and to each other frame-by-frame)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 320, 180, 6


def hip_stream():
    """A HIP stream made through the HIP runtime directly (the renderer has initialised HIP by
    the time this runs; torch's own lazy init is not needed for the C-ABI)."""
    import ctypes
    import os

    # the HIP runtime the renderer is bound to: whichever libamdhip64 the process loaded first
    # (torch's bundled copy when torch came first) -- a second copy would not link
    loaded = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln]
    path = loaded[0] if loaded else os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libamdhip64.so")
    hip = ctypes.CDLL(path)
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    return hip, s


def run(rtx, tmp_path, pipelined, per_frame):
    cfg = rtx.write_config(str(tmp_path / ("p%d%d.toml" % (pipelined, per_frame))), W, H, spp=2)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    hip, post = hip_stream() if pipelined else (None, None)
    if pipelined:
        rt.set_post_stream(post.value)
    cam0 = rt.camera
    images = []
    for f in range(1, FRAMES + 1):
        cam = rt.camera
        cam.yaw = cam0.yaw + 0.01 * f
        cam.pos[0] = cam0.pos[0] + 0.05 * f
        rt.camera = cam
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
        if per_frame:
            images.append(rt.download("RGBA8", np.uint8).copy())
    out = {k: rt.download(k, np.uint8).copy() for k in ("RGBA8", "EXPOSURE")}
    for b in ("RENDER_COLOR", "ACCUMULATION", "HISTORY_COLOR", "HISTORY_DEPTH", "SCALED_COLOR", "NORMAL", "DEPTH"):
        out[b] = rt.get_buffer(b).copy()
    sets = rt.info().gbufferSet
    rt.cleanup()
    if pipelined:
        hip.hipStreamDestroy(post)
    return out, images, sets


def test_pipelined_frames_match_serial(rtx, tmp_path):
    ref, ref_imgs, s0 = run(rtx, tmp_path, False, True)
    got, _, s1 = run(rtx, tmp_path, True, False)
    assert s0 == 0 and s1 == FRAMES % rtx.GBUFFER_SETS
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k
    _, imgs, _ = run(rtx, tmp_path, True, True)
    for f, (a, b) in enumerate(zip(ref_imgs, imgs)):
        assert np.array_equal(a, b), "frame %d" % (f + 1)
