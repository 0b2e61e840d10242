"""Frame pipelining (rt_set_post_stream): the denoise/post chain of frame f on a second
stream, overlapping the trace of frame f+1 into the next G-buffer set.  Every output after a
9-frame moving-camera sequence (each of the RT_GBUFFER_SETS = 4 sets reused at least once), and
the RGBA8 image of every frame, must be identical to the serial order (and to each other
frame-by-frame)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 320, 180, 9


def post_stream():
    """The post stream, made by torch as bench.py makes it: torch and the renderer share one HIP
    runtime in this process, so torch's stream handle is valid for rt_set_post_stream."""
    import torch

    return torch.cuda.Stream(device=0)


def run(rtx, tmp_path, pipelined, per_frame, tuning=None):
    cfg = rtx.write_config(str(tmp_path / ("p%d%d.toml" % (pipelined, per_frame))), W, H, spp=2,
                           tuning=tuning or {})
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


@pytest.mark.parametrize("chain", ["always", "off"])
def test_pipelined_chain_modes_match_serial(rtx, tmp_path, chain):
    """The bounce chain as one launch (k_pt_chain: what serial frames run) and as four kernels
    (what pipelined frames run), each pipelined ([tuning] chain), against serial frames
    (k_pt_chain): identical outputs."""
    ref, _, _ = run(rtx, tmp_path, False, False)
    got, _, _ = run(rtx, tmp_path, True, False, tuning={"chain": chain})
    for k in ref:
        assert np.array_equal(ref[k], got[k]), k


@pytest.mark.parametrize("tuning", [{"dnFold": 1}, {"dnSplit": 2}, {"dnSplit": 2, "dnFold": 1}],
                         ids=["fold", "split", "split-fold"])
def test_denoise_list_variants_match_default(rtx, tmp_path, tuning):
    """The a-trous list passes at two threads per pixel ([tuning] dnSplit, k_spatial5_list2 /
    k_spatial7_list2) and the folded chain ([tuning] dnFold: the last pass over list 1 only, its
    other tiles written by the first) against the default kernels: identical outputs, serial and
    pipelined."""
    ref, _, _ = run(rtx, tmp_path, False, False)
    for pipelined in (False, True):
        got, _, _ = run(rtx, tmp_path, pipelined, False, tuning=tuning)
        for k in ref:
            assert np.array_equal(ref[k], got[k]), (pipelined, k)


def test_sync_on_null_stream_then_other_stream(rtx, oracle, tmp_path, default_scene):
    """rt_sync with the renderer on the null stream (set_stream(0), torch's default stream) must
    still issue the deferred denoise and wait for every renderer stream: G-buffers bound as torch
    tensors and read on an unrelated stream right after it hold the finished frame."""
    import torch

    w, h = 160, 96
    cfg = rtx.write_config(str(tmp_path / "ns.toml"), w, h)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(16.667)
    rt.set_stream(0)
    post = post_stream()
    rt.set_post_stream(post.cuda_stream)
    bufs = [{k: torch.zeros(rt.buffer_bytes(k), dtype=torch.uint8, device="cuda:0") for k in ("NORMAL", "DEPTH")}
            for _ in range(rtx.GBUFFER_SETS)]
    for s, d in enumerate(bufs):
        for k, t in d.items():
            rt.bind_buffer(k, t.data_ptr(), t.numel(), gbuffer_set=s)
    torch.cuda.synchronize()
    other = torch.cuda.Stream(device=0)
    s, tex = oracle.sky(), oracle.textures()
    cam = oracle.default_camera(w, h)
    for f in range(1, 4):
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
        rt.sync()
        k = rt.info().gbufferSet
        with torch.cuda.stream(other):
            got = {n: t.to("cpu", non_blocking=True) for n, t in bufs[k].items()}
        other.synchronize()
        g = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, cam=cam, sky_out=s, tex=tex)
        assert np.array_equal(got["NORMAL"].numpy().view(np.uint16).reshape(-1, 4), g["normal"]), f
        assert np.array_equal(got["DEPTH"].numpy().view(np.uint16), g["depth"]), f
    rt.cleanup()


def test_post_stream_after_dynamic_resolution_shrink(rtx, oracle, tmp_path, default_scene):
    """rt_set_post_stream after dynamic resolution has shrunk the frame sizes its extra G-buffer
    sets for the largest frame: the sequence grows back and stays bit-exact vs the oracle."""
    maxw, maxh, ws, hs = 192, 108, 160, 90
    cfg = rtx.write_config(str(tmp_path / "dr.toml"), ws, hs, dynamic=True, max_size=(maxw, maxh),
                           min_size=(64, 36))
    rt = rtx.RayTracer(ws, hs, cfg).init()
    s, tex = oracle.sky(), oracle.textures()
    dn = oracle.Denoiser(maxw, maxh, ws, hs)
    rgba = np.zeros((hs, ws, 4), np.uint8)
    w, h, cam = maxw, maxh, None
    for f, dt in enumerate((16.667, 40.0, 16.667, 10.0, 5.0), start=1):
        if f > 1:
            w, h = oracle.dynamic_resolution(w, dt, 60.0, 64, maxw, maxh)
        if f == 3:  # the frame is 128x72 now: pipelining turned on at the shrunk size
            rt.set_post_stream(post_stream().cuda_stream)
        rt.set_delta_time(dt)
        rt.draw(rgba)
        assert (rt.info().renderWidth, rt.info().renderHeight) == (w, h)
        oc = oracle.default_camera(w, h)
        gb = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, cam=oc, hist_cam=cam or oc, sky_out=s, tex=tex)
        o = dn.draw(gb, f, delta_time=dt, size=(w, h))
        assert np.array_equal(rgba.reshape(-1, 4), o["rgba"]), f
        cam = oc
    assert (w, h) == (192, 108)  # grew back to the maximum
    rt.cleanup()


def test_draw_device_target_sync_and_async(rtx, oracle, tmp_path, default_scene):
    """draw(SurfObj*) (kernel.cu:259, CopyToOutput kernel.cu:26-59): the RGBA8 frame written into a
    caller-owned device buffer with a row pitch, synchronously and asynchronously (pipelined, one
    target per frame), each frame bit-exact vs the oracle; rt_download(RGBA8) reads the last target."""
    import torch

    w, h = 160, 96
    pitch = (w + 16) * 4  # padded rows: the pad bytes must stay untouched
    s, tex = oracle.sky(), oracle.textures()
    cam = oracle.default_camera(w, h)
    for asynchronous in (False, True):
        cfg = rtx.write_config(str(tmp_path / ("dd%d.toml" % asynchronous)), w, h, spp=2)
        rt = rtx.RayTracer(w, h, cfg).init()
        rt.set_delta_time(16.667)
        dn = oracle.Denoiser(w, h)
        targets = [torch.full((h * pitch,), 7, dtype=torch.uint8, device="cuda:0") for _ in range(4)]
        torch.cuda.synchronize()
        for f, t in enumerate(targets, start=1):
            rt.draw_device(t.data_ptr(), pitch, asynchronous=asynchronous)
        rt.sync()
        last = rt.download("RGBA8", np.uint8).reshape(-1, 4)
        for f, t in enumerate(targets, start=1):
            g = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, spp=2, cam=cam, sky_out=s, tex=tex)
            o = dn.draw(g, f, delta_time=16.667)
            img = t.cpu().numpy().reshape(h, pitch)
            assert np.array_equal(img[:, :w * 4].reshape(-1, 4), o["rgba"]), (asynchronous, f)
            assert (img[:, w * 4:] == 7).all()
        assert np.array_equal(last, o["rgba"])
        rt.cleanup()


def test_chain_choice_refreshes_without_sync(rtx, tmp_path):
    """Serial frames whose host never calls rt_sync still learn queue 3's length: the
    resolve kernel stores {length, frame tag} into pinned memory and the next rt_path_trace picks it
    up without waiting (frame.cpp poll_q3).  The terrain view's queue 3 (~3.9 M rays at 1080p 4 spp)
    is past the fused chain's limit, so once the first frame's length is known the frames run the
    four-kernel bounce stages (rt_info.lastChain 0) — with no host sync in between."""
    import time

    w, h = 1920, 1080
    rt = rtx.RayTracer(w, h, rtx.write_config(str(tmp_path / "q3.toml"), w, h, spp=4)).init()
    rt.set_delta_time(16.667)
    cam = rt.camera
    cam.pos[:] = (8.0, 15.0, -6.0)
    cam.yaw, cam.pitch = 0.0, -0.7
    rt.camera = cam
    chains = []
    for f in range(1, 6):
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
        chains.append(rt.info().lastChain)
        time.sleep(0.1)  # the GPU finishes the frame meanwhile; the host does not synchronise
    assert chains[0] == 1, chains  # nothing known yet: the short-queue default
    assert chains[-1] == 0, chains  # the long queue-3 length arrived without an rt_sync
    rt.sync()
    rt.cleanup()


# frames whose denoise skips the active-tile lists: SpatialFilter7x7 off (4, 8) or the a-trous
# passes off (6); the others after frame 1 run the list chain, which alternates the two
# accumulation buffers (accum / accumAlt, swapped by the host) and the list counters' parity
NO_LOCAL, NO_WIDE = (4, 8), (6,)


def test_pipelined_list_toggles_match_serial_and_oracle(rtx, oracle, tmp_path, default_scene):
    """Round-5 verdict item 8: every buffer the post stream shares across frames — the G-buffer
    sets, the two accumulation buffers the host swaps after a list frame, the list counters of
    both parities, the single colour ping-pong partner, the exposure state and the RGBA8 output —
    reused under pipelining while the denoise alternates between list and non-list frames.  The
    drop-in path (rt_draw_device, asynchronous, one device target per frame) against synchronous
    draws of the same sequence, frame by frame, and each synchronous frame against the oracle."""
    import torch

    w, h, spp, frames = 192, 112, 2, 12
    s, tex = oracle.sky(), oracle.textures()
    cam = oracle.default_camera(w, h)
    images = {}
    for asynchronous in (False, True):
        cfg = rtx.write_config(str(tmp_path / ("lt%d.toml" % asynchronous)), w, h, spp=spp)
        rt = rtx.RayTracer(w, h, cfg).init()
        rt.set_delta_time(16.667)
        targets = [torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0") for _ in range(frames)]
        torch.cuda.synchronize()
        for f in range(1, frames + 1):
            p = rt.params
            p.pass_.enableLocalSpatialFilter = 0 if f in NO_LOCAL else 1
            p.pass_.enableWideSpatialFilter = 0 if f in NO_WIDE else 1
            rt.params = p
            rt.draw_device(targets[f - 1].data_ptr(), 0, asynchronous=asynchronous)
        rt.sync()
        images[asynchronous] = [t.cpu().numpy().reshape(-1, 4) for t in targets]
        images[asynchronous].append(rt.get_buffer("ACCUMULATION").copy())
        images[asynchronous].append(rt.get_buffer("HISTORY_COLOR").copy())
        rt.cleanup()
    for f, (a, b) in enumerate(zip(images[False], images[True]), start=1):
        assert np.array_equal(a, b), "frame %d" % f if f <= frames else ("ACCUMULATION", "HISTORY_COLOR")[f - frames - 1]
    dn = oracle.Denoiser(w, h)
    for f in range(1, frames + 1):
        op = oracle.default_params()
        op.enableLocalSpatialFilter = 0 if f in NO_LOCAL else 1
        op.enableWideSpatialFilter = 0 if f in NO_WIDE else 1
        g = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, spp=spp, cam=cam, sky_out=s, tex=tex)
        o = dn.draw(g, f, params=op, delta_time=16.667)
        assert np.array_equal(images[False][f - 1], o["rgba"]), f


def test_serial_counter_blocks_across_mode_switches(rtx, tmp_path):
    """Serial frames start without a counter memset: each frame's resolve zeroes the other of two
    counter blocks for the next frame (frame.cpp syncZeroed).  Frames interleaved with what dirties
    those blocks — rt_trace_rays (block 0), a pipelined stretch (block 0 is pipelined slot 0), the
    per-kernel timing path — must equal an uninterrupted sequence of synchronous draws, frame by frame."""
    import torch

    w, h = 192, 112
    ref = draw_sequence_plain(rtx, tmp_path, "plain", w, h, 8)
    cfg = rtx.write_config(str(tmp_path / "mix.toml"), w, h, spp=2)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(16.667)
    target = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    got = []
    for f in range(1, 9):
        if f == 3:
            rt.trace_rays([[0.2, 0.2, 0.0]], [[0.0, 0.0, 1.0]])
        if f == 5:  # frames 5 and 6 pipelined, then synchronous again
            rt.set_post_stream(post_stream().cuda_stream)
        if f == 7:
            rt.set_post_stream(None)
        rt.draw_device(target.data_ptr(), 0, asynchronous=f in (5, 6))
        rt.sync()
        got.append(target.cpu().numpy().copy())
    rt.cleanup()
    for f, (a, b) in enumerate(zip(ref, got), start=1):
        assert np.array_equal(a, b), "frame %d" % f


def draw_sequence_plain(rtx, tmp_path, name, w, h, frames):
    import torch

    cfg = rtx.write_config(str(tmp_path / (name + ".toml")), w, h, spp=2)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(16.667)
    target = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
    out = []
    for _ in range(frames):
        rt.draw_device(target.data_ptr(), 0)
        out.append(target.cpu().numpy().copy())
    rt.cleanup()
    return out


def test_bound_accumulation_keeps_the_list_chain(rtx, tmp_path):
    """A caller-bound accumulation buffer (rt_bind_buffer) no longer turns the active-tile list chain
    off: the chain writes the internal buffer and copies the frame back into the caller's.  Every
    frame's RGBA8 and the caller's buffer equal a context without the binding."""
    import torch

    w, h, frames = 192, 112, 6
    outs = []
    for bound in (False, True):
        cfg = rtx.write_config(str(tmp_path / ("acc%d.toml" % bound)), w, h, spp=2)
        rt = rtx.RayTracer(w, h, cfg).init()
        rt.set_delta_time(16.667)
        acc = None
        if bound:
            acc = torch.zeros(rt.buffer_bytes("ACCUMULATION"), dtype=torch.uint8, device="cuda:0")
            rt.bind_buffer("ACCUMULATION", acc.data_ptr(), acc.numel())
        imgs = []
        rgba = np.zeros((h, w, 4), np.uint8)
        for _ in range(frames):
            rt.draw(rgba)
            imgs.append(rgba.copy())
        accum = rt.get_buffer("ACCUMULATION").copy()
        if bound:
            torch.cuda.synchronize()
            assert np.array_equal(acc.cpu().numpy()[:accum.size], accum)
        outs.append((imgs, accum))
        rt.cleanup()
    for f, (a, b) in enumerate(zip(outs[0][0], outs[1][0]), start=1):
        assert np.array_equal(a, b), "frame %d" % f
    assert np.array_equal(outs[0][1], outs[1][1])


def test_sync_draws_trace_camera_rays_ahead(rtx, tmp_path):
    """A synchronous draw traces the next frame's camera rays ahead, beside its own bounces and
    denoise (frame.cpp launch_spec_camera), and the next draw uses them only when its launch
    parameters equal theirs.  A sequence that moves the camera, changes the sky, reads a buffer,
    resets the frame index, and draws into host memory between device draws — each of which makes
    the next draw trace its camera rays again — against the same sequence with [tuning] syncSpec
    off: every frame's RGBA8, and the ray count, identical."""
    import torch

    w, h, frames = 192, 112, 12
    outs = []
    for spec in (False, True):
        cfg = rtx.write_config(str(tmp_path / ("sp%d.toml" % spec)), w, h, spp=2, tuning={"syncSpec": spec})
        rt = rtx.RayTracer(w, h, cfg).init()
        rt.set_delta_time(16.667)
        target = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
        imgs = []
        for f in range(1, frames + 1):
            if f == 3:
                cam = rt.camera
                cam.yaw += 0.05
                rt.camera = cam
            if f == 5:
                p = rt.params
                p.sky.timeOfDay += 0.02
                rt.params = p
            if f == 7:
                rt.get_buffer("DEPTH")
            if f == 9:
                rt.set_frame_index(4)
            if f == 11:
                rgba = np.zeros((h, w, 4), np.uint8)
                rt.draw(rgba)
                imgs.append(rgba.reshape(-1).copy())
                continue
            rt.draw_device(target.data_ptr(), 0)
            imgs.append(target.cpu().numpy().copy())
        rays = rt.ray_count()
        info = rt.info()
        rt.cleanup()
        outs.append((imgs, rays, info.gbufferSet))
    for f, (a, b) in enumerate(zip(outs[0][0], outs[1][0]), start=1):
        assert np.array_equal(a, b), "frame %d" % f
    assert outs[0][1] == outs[1][1]
    assert outs[0][2] == 0 and outs[1][2] in (0, 1)  # the sets alternate with the camera rays traced ahead


@pytest.mark.parametrize("material", [5, 4])
def test_sync_draws_ahead_with_glossy_materials(rtx, tmp_path, material):
    """The launches ahead of synchronous draws with the mirror (5) and microfacet (4) materials
    ([render] materialOverride: the glossy shade kernel traces inline, the bounces run as the four
    kernels), and a camera move in between: every frame equal to draws without them."""
    import torch

    w, h, frames = 160, 96, 6
    outs = []
    for spec in (False, True):
        cfg = rtx.write_config(str(tmp_path / ("g%d%d.toml" % (material, spec))), w, h, spp=2,
                               extra="materialOverride = %d\n" % material, tuning={"syncSpec": spec})
        rt = rtx.RayTracer(w, h, cfg).init()
        rt.set_delta_time(16.667)
        target = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0")
        imgs = []
        for f in range(1, frames + 1):
            if f == 4:
                cam = rt.camera
                cam.pos[1] += 0.1
                rt.camera = cam
            rt.draw_device(target.data_ptr(), 0)
            imgs.append(target.cpu().numpy().copy())
        outs.append((imgs, rt.ray_count()))
        rt.cleanup()
    for f, (a, b) in enumerate(zip(outs[0][0], outs[1][0]), start=1):
        assert np.array_equal(a, b), "frame %d" % f
    assert outs[0][1] == outs[1][1]
