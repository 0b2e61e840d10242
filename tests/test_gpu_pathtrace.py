"""GPU path tracer (PathTrace, pathtrace.cuh:11-128) and sky/sun generation vs the CPU oracle.

Everything here is bit-exact: the sky/sun images and their CDFs, and every G-buffer the path
tracer writes (demodulated half colour + material mask, shading normal, albedo, depth, motion
vectors) plus the per-pixel count of traced rays.  Cases cover the reference's default
material (Lambertian + triplanar soil textures, sky/sun MIS), the glossy materials reachable
through the material table (mirror, glass, microfacet) via [render] materialOverride, a
moving camera (motion vectors against the history camera), spp > 1 and screen strips.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def terrain_camera(rtx, oracle, w, h, pos=(8.0, 15.0, -6.0), yaw=0.0, pitch=-0.7):
    """A camera looking down on the default terrain (half the pixels hit geometry)."""
    c = oracle.default_camera(w, h)
    c.pos[:] = pos
    c.yaw = yaw
    c.pitch = pitch
    r = rtx.Camera()
    r.pos[:] = pos
    r.yaw, r.pitch, r.focal, r.aperture, r.fovX = yaw, pitch, c.focal, c.aperture, c.fovX
    return c, r


@pytest.fixture(scope="module")
def sky_tex(oracle):
    return oracle.sky(), oracle.textures()


def gpu_gbuffers(rt, w, h):
    P = w * h
    return dict(color=rt.get_buffer("RENDER_COLOR", (P, 4), np.uint16),
                normal=rt.get_buffer("NORMAL", (P, 4), np.uint16),
                albedo=rt.get_buffer("ALBEDO", (P, 4), np.uint16),
                depth=rt.get_buffer("DEPTH", (P,), np.uint16),
                motion=rt.get_buffer("MOTION", (P, 2), np.uint16),
                rays=rt.download("RAYS", np.uint32)[:P])


def assert_gbuffers_equal(g, o, rows=None):
    sl = slice(None) if rows is None else rows
    for k in ("color", "normal", "albedo", "depth", "motion", "rays"):
        a, b = g[k][sl], o[k][sl]
        bad = np.nonzero(np.any((a != b).reshape(a.shape[0], -1), axis=1))[0]
        assert bad.size == 0, "%s differs at %d pixels, first %s: gpu %s oracle %s" % (
            k, bad.size, bad[:5], a[bad[:2]], b[bad[:2]])


def make_rt(rtx, tmp_path, w, h, spp=1, extra=""):
    cfg = rtx.write_config(str(tmp_path / "c.toml"), w, h, spp=spp, extra=extra)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.build_bvh()
    return rt


def test_sky_and_sun_bit_exact(rtx, oracle, tmp_path, sky_tex):
    s, _ = sky_tex
    rt = make_rt(rtx, tmp_path, 64, 36)
    rt.path_trace(1)
    rt.sync()
    sky = rt.get_buffer("SKY", (256, 512, 4), np.float32)
    sun = rt.get_buffer("SUN", (32, 32, 4), np.float32)
    u = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    assert np.array_equal(u(sky), u(s["sky"]))
    assert np.array_equal(u(sun), u(s["sun"]))
    assert np.array_equal(u(rt.download("SKY_PDF", np.float32)), u(s["sky_pdf"]))
    assert np.array_equal(u(rt.download("SKY_CDF", np.float32)), u(s["sky_cdf"]))
    assert np.array_equal(u(rt.download("SUN_PDF", np.float32)), u(s["sun_pdf"]))
    assert np.array_equal(u(rt.download("SUN_CDF", np.float32)), u(s["sun_cdf"]))
    sd = rt.download("SUN_DIR", np.float32)
    assert np.array_equal(u(sd[:3]), u(s["sun_dir"]))
    assert np.array_equal(u(sd[3:4]), u(np.array([s["cos_theta_max"]], np.float32)))
    rt.cleanup()


def test_sky_regenerates_on_param_change(rtx, oracle, tmp_path):
    rt = make_rt(rtx, tmp_path, 32, 18)
    p = rt.params
    p.sky.timeOfDay = 0.4
    p.sky.sunAxisAngle = 30.0
    p.sky.sunAngle = 0.8
    rt.params = p
    rt.path_trace(1)
    rt.sync()
    s = oracle.sky(dict(timeOfDay=0.4, sunAxisAngle=30.0, sunAngle=0.8))
    u = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    assert np.array_equal(u(rt.get_buffer("SKY", (256, 512, 4), np.float32)), u(s["sky"]))
    assert np.array_equal(u(rt.download("SUN_CDF", np.float32)), u(s["sun_cdf"]))
    rt.cleanup()


@pytest.mark.parametrize("w,h,frame,cam_kind", [(160, 90, 1, "default"), (192, 108, 1, "terrain"),
                                                (97, 61, 5, "terrain")])
def test_pathtrace_bit_exact(rtx, oracle, tmp_path, default_scene, sky_tex, w, h, frame, cam_kind):
    s, tex = sky_tex
    rt = make_rt(rtx, tmp_path, w, h)
    if cam_kind == "terrain":
        ocam, rcam = terrain_camera(rtx, oracle, w, h)
        rt.camera = rcam
    else:
        ocam = oracle.default_camera(w, h)
    rt.path_trace(frame, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rays = rt.ray_count()
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=frame, cam=ocam, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o)
    assert rays == int(o["rays"].sum())
    if cam_kind == "terrain":
        assert (o["color"][:, 3] == 3).mean() > 0.3  # material 3 (Lambertian) on the terrain


def test_pathtrace_1m_scene_deep_stack(rtx, oracle, tmp_path):
    """The camera kernel keeps 10 of the 16 traversal-stack entries in LDS and the deepest six in
    registers (traverse.h trav_step_t<10>).  The default scene's rays hold at most 11 entries; the
    1M-triangle scene's (BASELINE config 4, BLAS depth up to 19) reach 15, so this frame runs the
    register entries 10..14 for thousands of rays, and its G-buffers and per-pixel ray counts stay
    bit-exact."""
    w, h, frame = 1280, 720, 2
    v, i, n = oracle.scene(4)
    bvh = oracle.build_bvh(v, i, n, oracle.smooth_normals(v, i))
    rays, _ = oracle.primary_rays(w, h, frame)
    depth = oracle.intersect(bvh, rays)["maxDepth"]
    assert (depth >= 11).sum() > 1000 and (depth >= 15).sum() > 0  # deep stacks occur in this view
    cfg = rtx.write_config(str(tmp_path / "c.toml"), w, h, chunk_dim=4)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.build_bvh()
    rt.path_trace(frame, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(bvh, w, h, frame_num=frame, cam=oracle.default_camera(w, h), sky_out=oracle.sky(),
                         tex=oracle.textures())
    assert_gbuffers_equal(g, o)


@pytest.mark.parametrize("dist", [1e3, 1e4, 1e5])
def test_pathtrace_distant_camera_cull(rtx, oracle, tmp_path, default_scene, sky_tex, dist):
    """The camera kernel's scene cull (`root_surely_missed`, a slab test of the root box grown by
    0.01 + 1 % of the scene extent) far from the scene: a narrow field of view from 10^3 .. 10^5
    units away keeps the terrain in the image, so culled and traced rays sit side by side, and the
    G-buffers stay bit-exact with the oracle, which traces every ray."""
    import math
    s, tex = sky_tex
    w, h = 96, 54
    centre = np.array([8.0, 8.0, 8.0])  # the default scene spans [-0.5, 16.5] x [5, 11] x [-0.5, 16.5]
    off = np.array([0.6, 0.35, -0.72])
    off /= np.linalg.norm(off)
    pos = centre + dist * off
    d = -off
    ocam, rcam = terrain_camera(rtx, oracle, w, h, pos=tuple(np.float32(pos)), yaw=float(np.float32(math.atan2(d[0], d[2]))),
                                pitch=float(np.float32(math.asin(d[1]))))
    fov = np.float32(2.0 * math.atan(9.0 / dist))
    ocam.fovX = fov
    rcam.fovX = fov
    rt = make_rt(rtx, tmp_path, w, h)
    rt.camera = rcam
    rt.path_trace(1, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    culled = int(rt.download("PT_QUEUE", np.uint32)[22])
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=1, cam=ocam, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o)
    surface = (o["depth"] != 0x7C00).mean()  # sky depth: half infinity
    assert 0 < culled < w * h, culled  # both the culled and the traversed branch ran
    if dist <= 1e4:  # (at 10^5 the traversed rays miss the terrain, on both sides alike)
        assert 0.05 < surface < 0.95, surface


def test_pathtrace_motion_vectors(rtx, oracle, tmp_path, default_scene, sky_tex):
    """Frame 2 after a camera move: motion vectors come from the frame-1 (history) camera."""
    s, tex = sky_tex
    w, h = 128, 72
    rt = make_rt(rtx, tmp_path, w, h)
    c1, r1 = terrain_camera(rtx, oracle, w, h)
    c2, r2 = terrain_camera(rtx, oracle, w, h, pos=(8.3, 15.1, -5.8), yaw=0.05, pitch=-0.68)
    rt.camera = r1
    rt.path_trace(1)
    rt.camera = r2
    rt.path_trace(2, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=2, cam=c2, hist_cam=c1, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o)
    mv = o["motion"].view(np.float16).astype(np.float32)
    assert np.abs(mv - 0.5).max() > 1e-3  # the camera moved


@pytest.mark.parametrize("material", [1, 4, 5])
def test_pathtrace_glossy_materials(rtx, oracle, tmp_path, default_scene, sky_tex, material):
    """Glass (1), microfacet (4) and mirror (5) from the reference material table."""
    s, tex = sky_tex
    w, h = 96, 54
    rt = make_rt(rtx, tmp_path, w, h, extra="materialOverride = %d\n" % material)
    ocam, rcam = terrain_camera(rtx, oracle, w, h)
    rt.camera = rcam
    rt.path_trace(1, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=1, cam=ocam, sky_out=s, tex=tex,
                         material_override=material)
    assert_gbuffers_equal(g, o)


def test_pathtrace_spp4_bit_exact(rtx, oracle, tmp_path, default_scene, sky_tex):
    s, tex = sky_tex
    w, h = 128, 72
    rt = make_rt(rtx, tmp_path, w, h, spp=4)
    ocam, rcam = terrain_camera(rtx, oracle, w, h)
    rt.camera = rcam
    rt.path_trace(3, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=3, spp=4, cam=ocam, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o)


def test_pathtrace_strip(rtx, oracle, tmp_path, default_scene, sky_tex):
    """A screen strip (the multi-GPU split) renders exactly the rows of the full frame."""
    s, tex = sky_tex
    w, h, y0, rows = 128, 96, 40, 24
    rt = make_rt(rtx, tmp_path, w, h, extra="stripY0 = %d\nstripRows = %d\n" % (y0, rows))
    ocam, rcam = terrain_camera(rtx, oracle, w, h)
    rt.camera = rcam
    rt.path_trace(1, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=1, cam=ocam, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o, rows=slice(y0 * w, (y0 + rows) * w))


def test_pathtrace_interleaved_strip(rtx, oracle, tmp_path, default_scene, sky_tex):
    """Interleaved strips (stripCount / stripIndex, the multi-GPU load balance): the context
    renders exactly its 16-row blocks of the full frame, deferred samples included (spp 2)."""
    from rtx.dist import strip_blocks

    s, tex = sky_tex
    w, h, n, r = 128, 100, 3, 1
    rt = make_rt(rtx, tmp_path, w, h, spp=2, extra="stripCount = %d\nstripIndex = %d\n" % (n, r))
    ocam, rcam = terrain_camera(rtx, oracle, w, h)
    rt.camera = rcam
    rt.path_trace(1, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=1, spp=2, cam=ocam, sky_out=s, tex=tex)
    owned = np.concatenate([np.arange(y0 * w, (y0 + rows) * w) for y0, rows in strip_blocks(h, n, r)])
    assert owned.size == 2 * 16 * w
    assert_gbuffers_equal(g, o, rows=owned)
    assert (g["rays"][np.setdiff1d(np.arange(w * h), owned)] == 0).all()  # nothing outside its blocks


def test_pathtrace_1080p_bit_exact(rtx, oracle, tmp_path, default_scene, sky_tex):
    s, tex = sky_tex
    w, h = 1920, 1080
    rt = make_rt(rtx, tmp_path, w, h)
    ocam, rcam = terrain_camera(rtx, oracle, w, h)
    rt.camera = rcam
    rt.path_trace(1, detail=True)
    rt.sync()
    g = gpu_gbuffers(rt, w, h)
    rt.cleanup()
    o = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=1, cam=ocam, sky_out=s, tex=tex)
    assert_gbuffers_equal(g, o)
