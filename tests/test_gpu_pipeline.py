"""Frame pipelining (rt_set_post_stream): the denoise/post chain of frame f on a second
stream, overlapping the trace of frame f+1 into the other G-buffer set.  Every output after
a 6-frame moving-camera sequence, and the RGBA8 image of every frame, must be identical to
the serial order (and to each other frame-by-frame)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 320, 180, 6


def post_stream():
    """The post stream, made by torch as bench.py makes it: torch and the renderer share one HIP
    runtime in this process, so torch's stream handle is valid for rt_set_post_stream."""
    import torch

    return torch.cuda.Stream(device=0)


def run(rtx, tmp_path, pipelined, per_frame):
    cfg = rtx.write_config(str(tmp_path / ("p%d%d.toml" % (pipelined, per_frame))), W, H, spp=2)
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    post = post_stream() if pipelined else None
    if pipelined:
        rt.set_post_stream(post.cuda_stream)
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
