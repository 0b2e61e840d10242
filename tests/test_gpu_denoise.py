"""GPU denoiser + post-processing (denoising.cu, postprocessing.cu, CopyToOutput) vs the oracle.

Multi-frame sequences with a moving camera exercise the temporal passes (reprojection through
the motion vectors, history clamping, accumulation/history buffers); every intermediate the
C-ABI exposes is compared bit-exactly: noise tiles, denoised HDR colour, history buffers,
DownScale4 chain, luminance histogram, the persistent exposure state, the tone-mapped screen
image and the dithered RGBA8 output.
"""
import numpy as np
import pytest

from test_gpu_pathtrace import make_rt, terrain_camera

pytestmark = pytest.mark.gpu

DT = 16.667


def cams(rtx, oracle, w, h, n):
    return [terrain_camera(rtx, oracle, w, h, pos=(8.0 + 0.15 * k, 15.0, -6.0 + 0.1 * k), yaw=0.02 * k,
                           pitch=-0.7 + 0.01 * k) for k in range(n)]


def gpu_state(rt, w, h, ws, hs):
    g = dict(color=rt.get_buffer("RENDER_COLOR", (w * h, 4), np.uint16),
             accum=rt.get_buffer("ACCUMULATION", (w * h, 4), np.uint16),
             hist_color=rt.get_buffer("HISTORY_COLOR", (w * h, 4), np.uint16),
             hist_depth=rt.get_buffer("HISTORY_DEPTH", (w * h,), np.uint16),
             noise8=rt.get_buffer("NOISE_LEVEL", dtype=np.uint16),
             noise16=rt.get_buffer("NOISE_LEVEL16", dtype=np.uint16),
             scaled=rt.get_buffer("SCALED_COLOR", (ws * hs, 4), np.uint16),
             c4=rt.download("COLOR4", np.uint16).reshape(-1, 4), c16=rt.download("COLOR16", np.uint16).reshape(-1, 4),
             c64=rt.download("COLOR64", np.uint16).reshape(-1, 4), histogram=rt.download("HISTOGRAM", np.uint32),
             exposure=rt.download("EXPOSURE", np.float32), rgba=rt.download("RGBA8", np.uint8).reshape(-1, 4))
    return g


def assert_state(g, o, dn):
    pairs = [("color", o["color"]), ("accum", dn.accum), ("hist_color", dn.hist_color),
             ("hist_depth", dn.hist_depth), ("noise8", o["noise8"]), ("noise16", o["noise16"]),
             ("scaled", o["scaled"]), ("c4", o["c4"]), ("c16", o["c16"]), ("c64", o["c64"]),
             ("histogram", o["histogram"]), ("rgba", o["rgba"])]
    for k, ref in pairs:
        a = g[k]
        assert a.shape == ref.shape, (k, a.shape, ref.shape)
        bad = np.nonzero((a != ref).reshape(a.shape[0], -1).any(axis=1))[0]
        assert bad.size == 0, "%s differs at %d entries, first %s: gpu %s oracle %s" % (
            k, bad.size, bad[:5], a[bad[:2]], ref[bad[:2]])
    assert np.array_equal(g["exposure"].view(np.uint32), o["exposure"].view(np.uint32)), (g["exposure"], o["exposure"])


def run_sequence(rtx, oracle, tmp_path, default_scene, w, h, frames, spp=1, extra="", params_fn=None, ws=None,
                 hs=None, dynamic=False, cam_list=None, expect_flare=None):
    ws, hs = ws or w, hs or h
    s, tex = oracle.sky(), oracle.textures()
    if dynamic:
        cfg = rtx.write_config(str(tmp_path / "c.toml"), ws, hs, dynamic=True, spp=spp, extra=extra,
                               max_size=(w, h))
        rt = rtx.RayTracer(ws, hs, cfg).init()
        rt.build_bvh()
    else:
        rt = make_rt(rtx, tmp_path, w, h, spp=spp, extra=extra)
    rt.set_delta_time(DT)
    op = oracle.default_params()
    if params_fn:
        p = rt.params
        params_fn(p, op)
        rt.params = p
    dn = oracle.Denoiser(w, h, ws, hs)
    cs = cam_list or cams(rtx, oracle, w, h, frames)
    for f in range(1, frames + 1):
        oc, rc = cs[f - 1]
        rt.camera = rc
        rt.build_bvh()
        rt.path_trace(f)
        rt.denoise_post(f)
        rt.sync()
        g = gpu_state(rt, w, h, ws, hs)
        hist_cam = cs[f - 2][0] if f > 1 else oc
        gb = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, spp=spp, cam=oc, hist_cam=hist_cam,
                              sky_out=s, tex=tex)
        o = dn.draw(gb, f, params=op, delta_time=DT, cam=oc, sun_dir=s["sun_dir"])
        if expect_flare is not None:  # the predicate held and the sun's texel is sky (the pass ran)
            assert o["lens_flare"] == expect_flare
            ux, uy = o["sun_uv"]
            assert gb["depth"].reshape(h, w)[uy, ux] == 0x7C00
        assert_state(g, o, dn)
    rt.cleanup()
    return g


def test_denoise_post_sequence(rtx, oracle, tmp_path, default_scene):
    g = run_sequence(rtx, oracle, tmp_path, default_scene, 160, 96, 3)
    assert g["rgba"][:, 3].min() == 1


def test_denoise_post_odd_size_spp2(rtx, oracle, tmp_path, default_scene):
    """Sizes that are not multiples of the 8/16/64 tiles (clamped reads at every level)."""
    run_sequence(rtx, oracle, tmp_path, default_scene, 150, 86, 2, spp=2)


def test_denoise_post_settings(rtx, oracle, tmp_path, default_scene):
    """Fixed exposure, noise-level visualisation and no sharpening."""
    def tweak(p, op):
        p.pass_.enableAutoExposure = 0
        p.pass_.enableNoiseLevelVisualize = 1
        p.pass_.enableSharpening = 0
        p.post.exposure = 3.5
        op.enableAutoExposure = 0
        op.enableNoiseLevelVisualize = 1
        op.enableSharpening = 0
        op.exposure = 3.5
    run_sequence(rtx, oracle, tmp_path, default_scene, 128, 72, 2, params_fn=tweak)


def test_denoise_post_scaled_output(rtx, oracle, tmp_path, default_scene):
    """Render size != screen size (dynamic-resolution configuration): BicubicScale resamples."""
    run_sequence(rtx, oracle, tmp_path, default_scene, 192, 108, 2, ws=160, hs=90, dynamic=True)


def test_draw_1080p_4spp(rtx, oracle, tmp_path, default_scene):
    """BASELINE config 3 (1080p, 4 spp, SVGF, tone map) through rt_draw, two frames."""
    w, h = 1920, 1080
    cfg = rtx.write_config(str(tmp_path / "c.toml"), w, h, spp=4)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(DT)
    (oc1, rc1), (oc2, rc2) = cams(rtx, oracle, w, h, 2)
    rgba = np.zeros((h, w, 4), np.uint8)
    hdr = np.zeros((h, w, 4), np.float32)
    s, tex = oracle.sky(), oracle.textures()
    dn = oracle.Denoiser(w, h)
    for f, (oc, rc), hc in ((1, (oc1, rc1), oc1), (2, (oc2, rc2), oc1)):
        rt.camera = rc
        rt.draw(rgba, hdr)
        gb = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, spp=4, cam=oc, hist_cam=hc, sky_out=s, tex=tex)
        o = dn.draw(gb, f, delta_time=DT)
        assert np.array_equal(rgba.reshape(-1, 4), o["rgba"])
        ref = o["color"][:, :3].view(np.float16).astype(np.float32)
        got = hdr.reshape(-1, 4)[:, :3]
        assert np.array_equal(got, ref)  # bit-exact (the north-star bar is 1e-3 relative L2)
    rt.cleanup()


def test_draw_dynamic_resolution(rtx, oracle, tmp_path, default_scene):
    """useDynamicResolution through rt_draw (UpdateFrame, kernel.cu:77-100): frame times outside
    the targetFps band resize the render size frame to frame; the temporal passes read their
    history at the previous frame's size (historyDim) and BicubicScale resamples to the screen."""
    maxw, maxh, ws, hs = 192, 108, 160, 90
    cfg = rtx.write_config(str(tmp_path / "c.toml"), ws, hs, dynamic=True, max_size=(maxw, maxh), min_size=(64, 36))
    rt = rtx.RayTracer(ws, hs, cfg).init()
    s, tex = oracle.sky(), oracle.textures()
    dn = oracle.Denoiser(maxw, maxh, ws, hs)
    rgba = np.zeros((hs, ws, 4), np.uint8)
    hdr = np.zeros((maxw * maxh, 4), np.float32)
    w, h, prev, sizes = maxw, maxh, None, []
    for f, dt in enumerate((16.667, 40.0, 10.0, 25.0, 16.4), start=1):
        if f > 1:
            w, h = oracle.dynamic_resolution(w, dt, 60.0, 64, maxw, maxh)
        sizes.append((w, h))
        oc, rc = terrain_camera(rtx, oracle, w, h, pos=(8.0 + 0.15 * f, 15.0, -6.0 + 0.1 * f), yaw=0.02 * f,
                                pitch=-0.7 + 0.01 * f)
        rt.camera = rc
        rt.set_delta_time(dt)
        rt.draw(rgba, hdr)
        info = rt.info()
        assert (info.renderWidth, info.renderHeight) == (w, h)
        gb = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, cam=oc, hist_cam=prev or oc, sky_out=s, tex=tex)
        o = dn.draw(gb, f, delta_time=dt, size=(w, h))
        assert np.array_equal(rgba.reshape(-1, 4), o["rgba"]), f
        ref = o["color"][:, :3].view(np.float16).astype(np.float32)
        assert np.array_equal(hdr[:w * h, :3], ref), f
        prev = oc
    rt.cleanup()
    assert sizes == [(192, 108), (128, 72), (160, 90), (128, 72), (128, 72)]


@pytest.mark.parametrize("tm", [0, 1, 2])
def test_denoise_post_tone_mappers(rtx, oracle, tmp_path, default_scene, tm):
    """ToneMappingType Uncharted (0, NaN by construction in the reference), ACES1 (1, ACESFitted
    with the sRGB->AP1 matrices), ACES2 (2, ACESFilm); Reinhard (3) is the default everywhere else."""
    def tweak(p, op):
        p.post.toneMappingType = tm
        op.toneMappingType = tm
    run_sequence(rtx, oracle, tmp_path, default_scene, 128, 72, 2, params_fn=tweak)


def sun_cams(rtx, oracle, w, h, n):
    """Cameras above the terrain looking just below the sun, so it sits in the upper half of the view."""
    import math
    sd = oracle.sky()["sun_dir"].astype(np.float64)
    yaw, pitch = math.atan2(sd[0], sd[2]), math.asin(sd[1]) - 0.25
    return [terrain_camera(rtx, oracle, w, h, pos=(8.0 + 0.1 * k, 15.0, -6.0), yaw=yaw + 0.01 * k, pitch=pitch)
            for k in range(n)]


def test_denoise_post_bloom_lens_flare(rtx, oracle, tmp_path, default_scene):
    """The off-by-default post passes: BloomGuassian on the 1/4 and 1/16 chains + Bloom, and the
    lens flare (host sun projection + LensFlarePred's depth test at the sun's texel)."""
    def tweak(p, op):
        p.pass_.enableBloomEffect = 1
        p.pass_.enableLensFlare = 1
        op.enableBloomEffect = 1
        op.enableLensFlare = 1
    w, h = 160, 96
    run_sequence(rtx, oracle, tmp_path, default_scene, w, h, 2, params_fn=tweak, cam_list=sun_cams(rtx, oracle, w, h, 2),
                 expect_flare=1)


def test_offscreen_dumps_and_camera_at_init(rtx, oracle, tmp_path, default_scene):
    """The presentation stand-in: PPM of the RGBA8 frame and PFM of the denoised HDR colour, read
    back and compared with the downloads; a camera saved to file is loaded by rt_init
    (loadCameraAtInit, init.cu:433-435) and renders the same frame."""
    w, h = 96, 64
    cfg = rtx.write_config(str(tmp_path / "a.toml"), w, h)
    a = rtx.RayTracer(w, h, cfg).init()
    a.set_delta_time(DT)
    _, rc = terrain_camera(rtx, oracle, w, h)
    a.camera = rc
    rgba = np.zeros((h, w, 4), np.uint8)
    a.draw(rgba)
    ppm, pfm, camf = str(tmp_path / "f.ppm"), str(tmp_path / "f.pfm"), str(tmp_path / "cam.bin")
    a.save_image(ppm, rtx.IMAGE_PPM_RGBA8)
    a.save_image(pfm, rtx.IMAGE_PFM_HDR)
    a.save_camera(camf)
    raw = open(ppm, "rb").read()
    head = b"P6\n%d %d\n255\n" % (w, h)
    assert raw.startswith(head)
    assert np.array_equal(np.frombuffer(raw[len(head):], np.uint8).reshape(h, w, 3), rgba[:, :, :3])
    raw = open(pfm, "rb").read()
    head = b"PF\n%d %d\n-1.0\n" % (w, h)
    assert raw.startswith(head)
    hdr = np.frombuffer(raw[len(head):], np.float32).reshape(h, w, 3)[::-1]
    col = a.get_buffer("RENDER_COLOR", (h, w, 4), np.uint16)[:, :, :3].astype(np.uint16).view(np.float16)
    assert np.array_equal(hdr, col.astype(np.float32))
    b = rtx.RayTracer(w, h, rtx.write_config(str(tmp_path / "b.toml"), w, h, camera_file=camf)).init()
    b.set_delta_time(DT)
    assert list(b.camera.pos) == list(rc.pos) and b.camera.pitch == rc.pitch
    rgba2 = np.zeros_like(rgba)
    b.draw(rgba2)
    assert np.array_equal(rgba, rgba2)
    a.cleanup()
    b.cleanup()
