"""The exact path bench.py times (rtx.frames.FramePipeline: torch streams with priorities, the
renderer on the high-priority one, denoise/post pipelined on a low-priority post stream, the
next frame's LBVH build + camera rays on the renderer's side stream), on the default scene,
camera and sky, checked bit for bit against the CPU oracle:

* BASELINE config 3 (1920x1080, 4 spp, 4 frames) — the bench workload itself;
* config 5's frame (3840x2160, 4 spp) — the size at which Histogram2's one 32x32 workgroup sees
  only 32x32 of the 60x34 texels of the 1/64 image while AutoExposure still divides by all
  2,040 (postprocessing.cu:37-49);
* the parity metric of SURVEY.md §8d against the oracle built on host libm (liboracle_libm.so),
  and on host libm with nvcc-style multiply-add contraction (liboracle_libm_fma.so): relative L2
  of the raw and the final HDR and the fraction of pixels whose path diverged, frames 2 and 4.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = 16.667


def pipeline_frames(rtx, tmp_path, w, h, spp, frames, per_frame=None):
    import torch

    from rtx.frames import FramePipeline

    cfg = rtx.write_config(str(tmp_path / ("bp%dx%d.toml" % (w, h))), w, h, dynamic=False, spp=spp)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(DT)
    prev = torch.cuda.current_stream(0)
    fp = FramePipeline(rt, torch.device("cuda", 0), pipelined=True)
    try:
        for f in range(1, frames + 1):
            fp.frame(f)
            if per_frame:
                per_frame(rt, f)
        fp.finish()
        out = dict(rgba=rt.download("RGBA8", np.uint8).reshape(-1, 4).copy(),
                   color=rt.get_buffer("RENDER_COLOR", (w * h, 4), np.uint16).copy(),
                   exposure=rt.download("EXPOSURE", np.float32).copy(),
                   histogram=rt.download("HISTOGRAM", np.uint32).copy())
    finally:
        rt.cleanup()
        torch.cuda.set_stream(prev)
    return out


def oracle_frames(oracle, scene, w, h, spp, frames):
    s, tex = oracle.sky(), oracle.textures()
    cam = oracle.default_camera(w, h)
    dn = oracle.Denoiser(w, h)
    for f in range(1, frames + 1):
        g = oracle.pathtrace(scene["bvh"], w, h, frame_num=f, spp=spp, cam=cam, hist_cam=cam, sky_out=s, tex=tex)
        o = dn.draw(g, f, delta_time=DT)
    return o, g


def assert_frame(got, o):
    for k in ("rgba", "color", "histogram"):
        bad = np.nonzero((got[k] != o[k]).reshape(len(got[k]), -1).any(1))[0]
        assert bad.size == 0, "%s differs at %d entries (first %s)" % (k, bad.size, bad[:4])
    assert np.array_equal(got["exposure"].view(np.uint32), o["exposure"].view(np.uint32))


def test_bench_path_1080p_4spp(rtx, oracle, tmp_path, default_scene):
    """bench.py's workload: 4 pipelined frames at 1920x1080, 4 spp, the last one vs the oracle."""
    got = pipeline_frames(rtx, tmp_path, 1920, 1080, 4, 4)
    o, _ = oracle_frames(oracle, default_scene, 1920, 1080, 4, 4)
    assert_frame(got, o)
    assert got["histogram"].sum() == 30 * 17  # the whole 1/64 image (30x17) at 1080p


def test_bench_path_4k_histogram_quirk(rtx, oracle, tmp_path, default_scene):
    """Config 5's frame on one GPU: 2 pipelined frames at 3840x2160, 4 spp, vs the oracle."""
    got = pipeline_frames(rtx, tmp_path, 3840, 2160, 4, 2)
    o, _ = oracle_frames(oracle, default_scene, 3840, 2160, 4, 2)
    assert_frame(got, o)
    # Histogram2 counts the top-left 32x32 texels of the 60x34 1/64 image only ...
    assert got["histogram"].sum() == 32 * 32
    # ... and AutoExposure normalises by the full 60*34 area, so the bins sum to 1024/2040 < 1:
    # the 40 % / 90 % quantiles then fall at higher bins than a full count would put them
    full = got["histogram"].astype(np.float64) / (60 * 34)
    assert abs(full.sum() - 1024 / 2040) < 1e-12


def _hdr(a):
    return a[:, :3].astype(np.uint16).view(np.float16).astype(np.float64)


_PARITY_GPU = {}


def _gpu_parity_frames(rtx, tmp_path, frames):
    """The GPU side of the parity metric (cached per frame count: both oracle builds compare with
    the same frames): the raw PathTrace colour / albedo / ray counts of the last frame from a
    serial context, and the final HDR, which the pipelined path must reproduce."""
    if frames in _PARITY_GPU:
        return _PARITY_GPU[frames]
    w, h, spp = 1920, 1080, 4
    raw = {}
    # get_buffer(RENDER_COLOR) right after the path trace returns the G-buffer colour only while
    # the denoise of the frame is still pending; read it from a serial context instead
    cfg = rtx.write_config(str(tmp_path / "raw.toml"), w, h, spp=spp)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(DT)
    for f in range(1, frames + 1):
        rt.build_bvh()
        rt.path_trace(f, detail=f == frames)
        rt.sync()
        if f == frames:
            raw["color"] = rt.get_buffer("RENDER_COLOR", (w * h, 4), np.uint16).copy()
            raw["albedo"] = rt.get_buffer("ALBEDO", (w * h, 4), np.uint16).copy()
            raw["rays"] = rt.download("RAYS", np.uint32).copy()
        rt.denoise_post(f)
    rt.sync()
    raw["final"] = rt.get_buffer("RENDER_COLOR", (w * h, 4), np.uint16).copy()
    rt.cleanup()
    got = pipeline_frames(rtx, tmp_path, w, h, spp, frames)
    assert np.array_equal(got["color"], raw["final"])  # the pipelined path ends on the same frame
    raw["rgba"] = got["rgba"]
    _PARITY_GPU[frames] = raw
    return raw


_VARIANTS = {"libm": "oracle/_build/liboracle_libm.so (host glibc transcendentals, no contraction)",
             "libm_fma": "oracle/_build/liboracle_libm_fma.so (host glibc transcendentals, a*b+c contracted "
                         "to fused multiply-adds as nvcc's default --fmad=true does)"}


@pytest.mark.parametrize("frames", [2, 4])
@pytest.mark.parametrize("variant", ["libm", "libm_fma"])
def test_parity_metric_vs_libm_oracle(rtx, oracle, tmp_path, default_scene, variant, frames):
    """SURVEY.md §8d parity metric against evaluations that share no transcendental code with the
    product (the oracle built on glibc's sinf/expf/powf/atan2f/...), without and with nvcc-style
    multiply-add contraction (the reference is built with nvcc's defaults, CMakeLists.txt:42, so
    every a*b+c outside its explicit FMA calls, linearMath.h:71-91, may be fused): relative L2 <=
    1e-3 of the raw PathTrace colour x albedo and of the final pre-tone-map HDR, plus the fraction
    of pixels whose path decisions diverged (ray count differs, or the raw colour moved by more
    than 1 % of its magnitude) < 1e-3.  The numbers go to
    $RTX_REPORT_DIR/parity_metric_<variant>_f<frames>.json when set."""
    w, h, spp = 1920, 1080, 4
    raw = _gpu_parity_frames(rtx, tmp_path, frames)
    with oracle.libm(variant):
        o, g = oracle_frames(oracle, default_scene, w, h, spp, frames)
    ref_raw = _hdr(g["color"]) * _hdr(g["albedo"])
    gpu_raw = _hdr(raw["color"]) * _hdr(raw["albedo"])
    rel_raw = float(np.linalg.norm(gpu_raw - ref_raw) / np.linalg.norm(ref_raw))
    rel_hdr = float(np.linalg.norm(_hdr(raw["final"]) - _hdr(o["color"])) / np.linalg.norm(_hdr(o["color"])))
    moved = np.abs(gpu_raw - ref_raw).max(1) > 1e-2 * np.maximum(np.abs(ref_raw).max(1), 1e-3)
    diverged = float((moved | (raw["rays"] != g["rays"])).mean())
    rgba_equal = float((raw["rgba"] == o["rgba"]).all(1).mean())
    report = dict(config="1920x1080 4 spp, frame %d of a default-camera sequence" % frames,
                  reference=_VARIANTS[variant], rel_l2_raw_color_x_albedo=rel_raw, rel_l2_final_hdr=rel_hdr,
                  diverged_pixel_fraction=diverged, rgba8_identical_fraction=rgba_equal, bar=1e-3)
    print(json.dumps(report))
    if os.environ.get("RTX_REPORT_DIR"):
        os.makedirs(os.environ["RTX_REPORT_DIR"], exist_ok=True)
        name = "parity_metric_%s_f%d.json" % (variant, frames)
        with open(os.path.join(os.environ["RTX_REPORT_DIR"], name), "w") as fh:
            json.dump(report, fh, indent=1)
    assert rel_raw <= 1e-3 and rel_hdr <= 1e-3
    assert diverged < 1e-3
