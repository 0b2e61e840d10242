"""C-ABI boundary checks that need no GPU: librtx.so loads, exports every entry point the
public header declares, and the host-side lifecycle/config handling behaves."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtx_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text)))


def test_dist_header_symbols_exported_and_bound(rtx):
    """include/rtx_dist.h (the C-ABI multi-GPU split) is exported by librtx.so and mirrored by rtx.cdist."""
    from rtx.cdist import DIST_SIGNATURES, lib

    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "rtx_dist.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(rtd_[a-z_0-9]+)\s*\(", text)))
    L = lib()
    assert syms and not [s for s in syms if not hasattr(L, s)]
    assert set(syms) == set(DIST_SIGNATURES)


def test_gbuffer_set_constants_match_the_header(rtx):
    """RT_GBUFFER_SETS / RT_BUF_SET1..3 (frame pipelining) and their Python mirrors agree."""
    text = open(HEADER).read()
    consts = {k: int(v, 0) for k, v in re.findall(r"#define\s+(RT_GBUFFER_SETS|RT_BUF_SET\d)\s+(\w+)", text)}
    assert consts["RT_GBUFFER_SETS"] == rtx.GBUFFER_SETS
    for k in range(1, rtx.GBUFFER_SETS):
        assert consts["RT_BUF_SET%d" % k] == k << 8 == getattr(rtx, "BUF_SET%d" % k)


def test_header_declares_the_renderer_api():
    syms = declared_symbols()
    for s in ("rt_create", "rt_init", "rt_draw", "rt_destroy", "rt_build_bvh", "rt_trace_primary",
              "rt_get_buffer", "rt_set_params", "rt_set_camera"):
        assert s in syms


def test_library_exports_every_declared_symbol(rtx):
    lib = rtx.load_library()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python mirror binds all of them
    assert set(declared_symbols()) == set(rtx.SIGNATURES)


def test_create_reads_config(rtx, tmp_path):
    cfg = rtx.write_config(str(tmp_path / "c.toml"), 320, 200, dynamic=False, chunk_dim=2, spp=4)
    rt = rtx.RayTracer(0, 0, cfg)
    info = rt.info()
    assert (info.screenWidth, info.screenHeight, info.renderWidth, info.renderHeight) == (320, 200, 320, 200)
    assert info.spp == 4
    p = rt.params
    assert p.post.maxWhite == pytest.approx(7.0) and p.sky.timeOfDay == pytest.approx(0.25)
    cam = rt.camera
    assert list(cam.pos) == [-2.0, 2.0, -2.0] and cam.focal == 5.0
    rt.cleanup()


def test_dynamic_resolution_renders_at_max(rtx, tmp_path):
    cfg = rtx.write_config(str(tmp_path / "c.toml"), 1920, 1080, dynamic=True)
    rt = rtx.RayTracer(1920, 1080, cfg)
    info = rt.info()
    assert (info.renderWidth, info.renderHeight) == (3840, 2160)  # init.cu:58-62
    rt.cleanup()


def test_bad_config_is_an_error_not_an_exit(rtx, tmp_path):
    with pytest.raises(rtx.RtError):
        rtx.RayTracer(64, 64, str(tmp_path / "missing.toml"))
    bad = tmp_path / "bad.toml"
    bad.write_text("[resolution\nwidth = 3\n")
    with pytest.raises(rtx.RtError):
        rtx.RayTracer(64, 64, str(bad))


def test_stage_calls_before_init_fail_cleanly(rtx):
    rt = rtx.RayTracer(64, 64, None)
    lib = rt.lib
    assert lib.rt_build_bvh(rt.h) == -4
    assert lib.rt_trace_primary(rt.h, 1, 0) == -4
    rt.cleanup()


def test_init_without_gpu_reports_no_device(rtx, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cfg = rtx.write_config(str(tmp_path / "c.toml"), 64, 64)
    rt = rtx.RayTracer(64, 64, cfg)
    with pytest.raises(rtx.RtError, match="RT_ERR_NO_DEVICE"):
        rt.init()
    rt.cleanup()


def test_camera_file_round_trip(rtx, tmp_path):
    """SaveCameraToFile / LoadCameraFromFile (inputControl.cu:115-149): the reference's 176-byte
    Camera record, pos/pitch/dir/focal/left/aperture/up/yaw/resolution/... in struct order."""
    import numpy as np
    cfg = rtx.write_config(str(tmp_path / "c.toml"), 320, 180)
    a = rtx.RayTracer(320, 180, cfg)
    cam = a.camera
    cam.pos[:] = (1.5, 7.25, -3.0)
    cam.yaw, cam.pitch, cam.focal, cam.aperture, cam.fovX = 0.3, -0.2, 4.0, 0.01, 1.2
    a.camera = cam
    path = str(tmp_path / "camera.bin")
    a.save_camera(path)
    rec = np.fromfile(path, np.float32)
    assert rec.size == 44
    assert list(rec[0:3]) == [1.5, 7.25, -3.0] and rec[3] == np.float32(-0.2)  # pos, pitch
    assert rec[7] == np.float32(4.0) and rec[11] == np.float32(0.01) and rec[15] == np.float32(0.3)
    assert list(rec[16:18]) == [320.0, 180.0] and rec[20] == np.float32(1.2)  # resolution, fov.x
    d = rec[4:7]  # Camera::update: dir = (sin yaw cos pitch, sin pitch, cos yaw cos pitch)
    assert np.allclose(d, [np.sin(0.3) * np.cos(-0.2), np.sin(-0.2), np.cos(0.3) * np.cos(-0.2)], atol=1e-6)
    b = rtx.RayTracer(320, 180, cfg)
    b.load_camera(path)
    cb = b.camera
    assert list(cb.pos) == list(cam.pos) and (cb.yaw, cb.pitch, cb.focal, cb.aperture, cb.fovX) == (
        cam.yaw, cam.pitch, cam.focal, cam.aperture, cam.fovX)
    with pytest.raises(rtx.RtError, match="RT_ERR_IO"):
        b.load_camera(str(tmp_path / "nope.bin"))
    a.cleanup()
    b.cleanup()


def test_rccl_communicator_library_exports():
    """lib/librtx_rccl.so (include/rtx_dist_rccl.h) loads and exports its four entry points."""
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "rtx_dist_rccl.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(rtd_[a-z_0-9]+)\s*\(", text)))
    L = C.CDLL(os.path.join(ROOT, "real-time-ray-tracing_amd", "lib", "librtx_rccl.so"))
    assert len(syms) == 4 and all(hasattr(L, s) for s in syms)


def test_hook_stage_mask_requires_histogram_and_rows(rtx):
    """rt_set_hook_stages: HISTOGRAM and ROWS are mandatory for a strip-local denoise; the mask only opts
    into GBUFFERS (a mask without them would leave ranks with their own exposure and stale peer rows)."""
    rt = rtx.RayTracer(64, 64, None)
    L = rt.lib
    assert L.rt_set_hook_stages(rt.h, 0) == -1
    assert L.rt_set_hook_stages(rt.h, 1 << 2) == -1          # GBUFFERS alone
    assert L.rt_set_hook_stages(rt.h, (1 << 0) | (1 << 2)) == -1  # no ROWS
    assert L.rt_set_hook_stages(rt.h, 8) == -1                # unknown stage
    assert L.rt_set_hook_stages(rt.h, 3) == 0
    assert L.rt_set_hook_stages(rt.h, 7) == 0
    rt.cleanup()


def test_bvh_threads_config_is_checked(rtx, tmp_path):
    """[render] bvhThreads picks the LBVH workgroup shape: 0 (by batch count), 512 or 1024."""
    for v in (0, 512, 1024):
        rtx.RayTracer(64, 64, rtx.write_config(str(tmp_path / ("t%d.toml" % v)), 64, 64,
                                               extra="bvhThreads = %d\n" % v)).cleanup()
    with pytest.raises(rtx.RtError):
        rtx.RayTracer(64, 64, rtx.write_config(str(tmp_path / "bad.toml"), 64, 64, extra="bvhThreads = 256\n"))
