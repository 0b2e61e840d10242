"""rtx — Python host interface of the MI355X path tracer (ctypes over librtx.so).

Mirrors the reference renderer API, ``class RayTracer`` (/root/reference/src/kernel.cuh:431-470):
``RayTracer(screen_w, screen_h, config)`` -> ``init()`` -> ``draw()`` ... -> ``cleanup()``,
plus the hot-path stages (``build_bvh``, ``trace_primary``) and array downloads used by the
parity tests and bench.  Everything runs in librtx.so (hand-written HIP for gfx950); there
is no CPU fallback: a missing or unloadable library raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "lib", "librtx.so")
DATA_DIR = os.path.join(_PKG, "data")

RT_OK = 0
ERRORS = {-1: "RT_ERR_ARG", -2: "RT_ERR_HIP", -3: "RT_ERR_IO", -4: "RT_ERR_STATE", -5: "RT_ERR_NO_DEVICE", -6: "RT_ERR_DEVICE"}

# rt_array_name (include/rtx_amd.h)
ARR = dict(VERTICES=0, INDICES=1, NORMALS=2, TRI_POS=3, AABBS=4, MORTON=5, REORDER=6, NODES=7, TLAS_AABBS=8,
           TLAS_MORTON=9, TLAS_REORDER=10, TLAS_NODES=11, TLAS_SCENE_AABB=12, BATCH_SCENE_AABBS=13, HITS=14,
           HIT_NORMALS=15, HIT_FAKE_NORMALS=16, HIT_STATS=17, TRI_NRM=18, RAYS=19, SKY_PDF=20, SKY_CDF=21,
           SUN_PDF=22, SUN_CDF=23, SUN_DIR=24, HISTOGRAM=25, EXPOSURE=26, COLOR4=27, COLOR16=28, COLOR64=29,
           RGBA8=30, PT_STATS=31, PT_QUEUE=32, PT_Q3_ORIGINS=33, PT_Q3_DIRS=34,
           PT_Q4_ORIGINS=35, PT_Q4_DIRS=36, TEX_ALBEDO_AO=37, TEX_NORMAL_ROUGHNESS=38, TEX_HEIGHT=39, HDR=40,
           BVH_ARENA=41)
TEX = dict(SOIL_ALBEDO_AO=0, SOIL_NORMAL_ROUGHNESS=1, SOIL_HEIGHT=2)  # MipmapTextureName (texture.h:5-12)
# rt_buffer_name (Buffer2DName, kernel.cuh:286-315)
BUF = dict(RENDER_COLOR=0, ACCUMULATION=1, HISTORY_COLOR=2, SCALED_COLOR=3, NORMAL=10, DEPTH=11, HISTORY_DEPTH=12,
           MOTION=13, NOISE_LEVEL=14, NOISE_LEVEL16=15, SKY=16, SUN=17, ALBEDO=18, RGBA8=19, HISTOGRAM=20)

# canonical 64-byte BVH node as a numpy record (see RT_ARR_NODES)
NODE_DTYPE = np.dtype([("lmin", "<f4", 3), ("lmax", "<f4", 3), ("rmin", "<f4", 3), ("rmax", "<f4", 3),
                       ("idxLeft", "<u4"), ("idxRight", "<u4"), ("isLeftLeaf", "<u4"), ("isRightLeaf", "<u4")])


class SkyParams(C.Structure):
    _fields_ = [("needRegenerate", C.c_int32), ("timeOfDay", C.c_float), ("sunAxisAngle", C.c_float),
                ("skyScalar", C.c_float), ("sunScalar", C.c_float), ("sunAngle", C.c_float)]


class SampleParams(C.Structure):
    _fields_ = [("sampleSurfaceVsLightUseMisWeight", C.c_int32), ("sampleSkyVsSunUseFluxWeight", C.c_int32),
                ("sampleSurfaceVsLight", C.c_float), ("sampleSkyVsSun", C.c_float)]


class RenderPassSettings(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "enableTemporalDenoising", "enableLocalSpatialFilter", "enableNoiseLevelVisualize",
        "enableWideSpatialFilter", "enableTemporalDenoising2", "enablePostProcess", "enableDownScalePasses",
        "enableHistogram", "enableAutoExposure", "enableBloomEffect", "enableLensFlare", "enableToneMapping",
        "enableSharpening")]


class PostProcessParams(C.Structure):
    _fields_ = [("toneMappingType", C.c_int32), ("exposure", C.c_float), ("gain", C.c_float),
                ("maxWhite", C.c_float), ("gamma", C.c_float)]


class DenoisingParams(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "local_denoise_sigma_normal", "local_denoise_sigma_depth", "local_denoise_sigma_material",
        "large_denoise_sigma_normal", "large_denoise_sigma_depth", "large_denoise_sigma_material",
        "temporal_denoise_sigma_normal", "temporal_denoise_sigma_depth", "temporal_denoise_sigma_material",
        "noise_threshold_local", "noise_threshold_large")]


class Params(C.Structure):
    _fields_ = [("sky", SkyParams), ("sample", SampleParams), ("pass_", RenderPassSettings),
                ("post", PostProcessParams), ("denoise", DenoisingParams)]


class Camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("yaw", C.c_float), ("pitch", C.c_float), ("focal", C.c_float),
                ("aperture", C.c_float), ("fovX", C.c_float)]


class Info(C.Structure):
    _fields_ = [("triCount", C.c_uint32), ("triCountPadded", C.c_uint32), ("batchCount", C.c_uint32),
                ("vertexCount", C.c_uint32), ("renderWidth", C.c_int32), ("renderHeight", C.c_int32),
                ("screenWidth", C.c_int32), ("screenHeight", C.c_int32), ("frameNum", C.c_int32),
                ("deviceId", C.c_int32), ("spp", C.c_uint32), ("gbufferSet", C.c_int32),
                ("denoiseRowBegin", C.c_int32), ("denoiseRowEnd", C.c_int32),
                ("gbufferRowBegin", C.c_int32), ("gbufferRowEnd", C.c_int32), ("stripLocalDenoise", C.c_int32),
                ("shadeOnSide", C.c_int32), ("lastChain", C.c_int32)]


class StripExchange(C.Structure):
    """rt_strip_exchange: what a strip-local denoise asks the host to exchange (rt_set_collective_hook)."""
    _fields_ = [("frameNum", C.c_int32), ("rowBegin", C.c_int32), ("rowEnd", C.c_int32), ("historySet", C.c_int32),
                ("gbufferSet", C.c_int32), ("stripLocal", C.c_int32)]


COLLECTIVE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(StripExchange))
HOOK_HISTOGRAM, HOOK_ROWS, HOOK_GBUFFERS = 0, 1, 2


# every entry point declared in include/rtx_amd.h, with its ctypes signature
SIGNATURES = {
    "rt_create": (C.c_int, [C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_void_p)]),
    "rt_init": (C.c_int, [C.c_void_p]),
    "rt_draw": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_draw_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "rt_destroy": (None, [C.c_void_p]),
    "rt_last_error": (C.c_char_p, [C.c_void_p]),
    "rt_get_params": (C.c_int, [C.c_void_p, C.POINTER(Params)]),
    "rt_set_params": (C.c_int, [C.c_void_p, C.POINTER(Params)]),
    "rt_get_camera": (C.c_int, [C.c_void_p, C.POINTER(Camera)]),
    "rt_set_camera": (C.c_int, [C.c_void_p, C.POINTER(Camera)]),
    "rt_set_frame_index": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_set_delta_time": (C.c_int, [C.c_void_p, C.c_float]),
    "rt_keyboard_update": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]),
    "rt_cursor_pos_update": (C.c_int, [C.c_void_p, C.c_double, C.c_double]),
    "rt_scroll_update": (C.c_int, [C.c_void_p, C.c_double, C.c_double]),
    "rt_mouse_button_update": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "rt_set_cursor_reset": (C.c_int, [C.c_void_p, C.c_int]),
    "rt_get_info": (C.c_int, [C.c_void_p, C.POINTER(Info)]),
    "rt_get_buffer": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    "rt_buffer_bytes": (C.c_size_t, [C.c_void_p, C.c_int]),
    "rt_path_trace": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "rt_denoise_post": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "rt_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_set_post_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_set_gather_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_bind_buffer": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    "rt_set_collective_hook": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_set_hook_stages": (C.c_int, [C.c_void_p, C.c_uint32]),
    "rt_get_ray_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "rt_build_bvh": (C.c_int, [C.c_void_p]),
    "rt_trace_primary": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "rt_sync": (C.c_int, [C.c_void_p]),
    "rt_time_stage": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]),
    "rt_debug_pk_math": (C.c_int, [C.c_int, C.c_void_p, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_size_t]),
    "rt_time_path_trace_kernels": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float), C.c_int]),
    "rt_time_frame_kernels": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_int]),
    "rt_trace_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(C.c_float)]),
    "rt_download": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
    "rt_array_bytes": (C.c_size_t, [C.c_void_p, C.c_int]),
    "rt_save_camera": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rt_load_camera": (C.c_int, [C.c_void_p, C.c_char_p]),
    "rt_save_image": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "rt_upload_texture": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]),
    "rt_scene_noise3d": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
    "rt_filter_kernel": (C.c_int, [C.c_int, C.c_void_p, C.c_int]),
    "rt_scan_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "rt_frame_marks_begin": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32]),
    "rt_frame_marks_read": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]),
}
IMAGE_PPM_RGBA8, IMAGE_PFM_HDR = 0, 1
DRAW_ASYNC = 1  # rt_draw_device flag
BUF_SET1, BUF_SET2, BUF_SET3 = 0x100, 0x200, 0x300  # rt_bind_buffer: further G-buffer sets (frame pipelining)
GBUFFER_SETS = 4  # G-buffer sets a pipelined context cycles through (rt_set_post_stream; RT_GBUFFER_SETS)

_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load librtx.so (RTX_LIB overrides the in-tree path, for ablation builds); raises if it is
    missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RTX_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError("librtx.so not found at %s — run `make` (or __graft_entry__.build())" % path)
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname, different path).
    # Loaded after librtx it would be a second runtime that finds no GPU, so when torch is
    # installed it is loaded first and librtx binds to it; streams then pass freely between them.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class RtError(RuntimeError):
    pass


def write_config(path: str, width: int, height: int, dynamic: bool = False, chunk_dim: int = 1, spp: int = 1,
                 extra: str = "", max_size=(3840, 2160), camera_file: str | None = None, min_size=(640, 480),
                 target_fps: float = 60.0, mesh_file: str | None = None, tuning: dict | None = None) -> str:
    """Write a config.toml with the reference's three tables (resources/config.toml) + extensions.

    `tuning`: the [tuning] table (scheduling A/B aids, include/rtx_amd.h).  When None, the
    RTX_TUNING environment variable ("key=value,key=value", e.g. "chain=off,tracePerCu=2") fills
    it: the A/B tools (tools/ab.sh) set it per variant.  The library itself reads no environment."""
    with open(path, "w") as f:
        f.write("[resolution]\nwidth = %d\nheight = %d\n\n" % (width, height))
        if camera_file:
            f.write('[file]\nloadCameraAtInit = true\ninputCameraFileName = "%s"\ncameraSaveFileName = "%s"\n\n'
                    % (camera_file, camera_file))
        else:
            f.write("[file]\nloadCameraAtInit = false\n\n")
        f.write("[optimziation]\nuseDynamicResolution = %s\ntargetFps = %r\nmaxWidth = %d\nmaxHeight = %d\n"
                "minWidth = %d\nminHeight = %d\n\n" % ("true" if dynamic else "false", float(target_fps), max_size[0],
                                                      max_size[1], min_size[0], min_size[1]))
        f.write("[scene]\nchunkDim = %d\n" % chunk_dim)
        if mesh_file:  # a meshProcessor .bin instead of the procedural terrain (init.cu:28-50)
            f.write('meshFile = "%s"\n' % mesh_file)
        f.write("\n[render]\nspp = %d\n" % spp)
        f.write(extra)
        if tuning is None:
            tuning = tuning_from_env()
        if tuning:
            f.write("\n[tuning]\n")
            for k, v in tuning.items():
                f.write("%s = %s\n" % (k, _toml_value(v)))
    return path


def _toml_value(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return repr(v)
    s = str(v)
    if s in ("true", "false") or s.lstrip("-").isdigit():
        return s
    return '"%s"' % s


def tuning_from_env() -> dict:
    """RTX_TUNING="key=value,..." as a [tuning] table (A/B tools only)."""
    out = {}
    for item in filter(None, (x.strip() for x in os.environ.get("RTX_TUNING", "").split(","))):
        k, _, v = item.partition("=")
        out[k.strip()] = v.strip()
    return out


class RayTracer:
    """The reference's RayTracer lifecycle over the C-ABI (kernel.cuh:431-470)."""

    def __init__(self, screen_width: int, screen_height: int, config: str | None = None):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.rt_create(screen_width, screen_height, config.encode() if config else None, C.byref(h))
        if rc != RT_OK:
            raise RtError("rt_create: %s %s" % (ERRORS.get(rc, rc), self.lib.rt_last_error(None).decode()))
        self.h = h

    # ---- lifecycle
    def _check(self, rc, what):
        if rc != RT_OK:
            raise RtError("%s: %s %s" % (what, ERRORS.get(rc, rc), self.lib.rt_last_error(self.h).decode()))

    def init(self):
        self._check(self.lib.rt_init(self.h), "rt_init")
        return self

    def draw(self, rgba8: np.ndarray | None = None, hdr: np.ndarray | None = None):
        self._check(self.lib.rt_draw(self.h, _ptr(rgba8), _ptr(hdr)), "rt_draw")

    def draw_device(self, device_ptr: int, pitch_bytes: int = 0, asynchronous: bool = False):
        """draw(SurfObj*): the RGBA8 frame into caller-owned device memory (e.g. a torch uint8
        tensor's data_ptr()); asynchronous=True enqueues the frame and pipelines frames."""
        self._check(self.lib.rt_draw_device(self.h, device_ptr, pitch_bytes, DRAW_ASYNC if asynchronous else 0),
                    "rt_draw_device")

    def cleanup(self):
        if getattr(self, "h", None):
            self.lib.rt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.cleanup()
        except Exception:
            pass

    # ---- parameters
    @property
    def params(self) -> Params:
        p = Params()
        self._check(self.lib.rt_get_params(self.h, C.byref(p)), "rt_get_params")
        return p

    @params.setter
    def params(self, p: Params):
        self._check(self.lib.rt_set_params(self.h, C.byref(p)), "rt_set_params")

    @property
    def camera(self) -> Camera:
        c = Camera()
        self._check(self.lib.rt_get_camera(self.h, C.byref(c)), "rt_get_camera")
        return c

    @camera.setter
    def camera(self, c: Camera):
        self._check(self.lib.rt_set_camera(self.h, C.byref(c)), "rt_set_camera")

    def set_frame_index(self, n: int):
        self._check(self.lib.rt_set_frame_index(self.h, n), "rt_set_frame_index")

    def set_delta_time(self, ms: float):
        self._check(self.lib.rt_set_delta_time(self.h, ms), "rt_set_delta_time")

    # ---- input (inputControl.cu): GLFW key / action / modifier values
    def keyboard_update(self, key: int, scancode: int, action: int, mods: int):
        self._check(self.lib.rt_keyboard_update(self.h, key, scancode, action, mods), "rt_keyboard_update")

    def cursor_pos_update(self, x: float, y: float):
        self._check(self.lib.rt_cursor_pos_update(self.h, x, y), "rt_cursor_pos_update")

    def scroll_update(self, dx: float, dy: float):
        self._check(self.lib.rt_scroll_update(self.h, dx, dy), "rt_scroll_update")

    def mouse_button_update(self, button: int, action: int, mods: int):
        self._check(self.lib.rt_mouse_button_update(self.h, button, action, mods), "rt_mouse_button_update")

    def set_cursor_reset(self, reset: bool = True):
        self._check(self.lib.rt_set_cursor_reset(self.h, int(reset)), "rt_set_cursor_reset")

    def info(self) -> Info:
        i = Info()
        self._check(self.lib.rt_get_info(self.h, C.byref(i)), "rt_get_info")
        return i

    # ---- hot-path stages
    def build_bvh(self):
        self._check(self.lib.rt_build_bvh(self.h), "rt_build_bvh")

    def trace_primary(self, frame_num: int = 1, detail: bool = False):
        self._check(self.lib.rt_trace_primary(self.h, frame_num, 1 if detail else 0), "rt_trace_primary")

    def path_trace(self, frame_num: int = 1, detail: bool = False):
        self._check(self.lib.rt_path_trace(self.h, frame_num, 1 if detail else 0), "rt_path_trace")

    def denoise_post(self, frame_num: int, hdr: bool = False):
        self._check(self.lib.rt_denoise_post(self.h, frame_num, 1 if hdr else 0), "rt_denoise_post")

    def set_stream(self, stream_ptr: int | None):
        """Enqueue on a hipStream_t handle (0: the null stream, torch's default stream); None
        restores the context's own stream (RT_OWN_STREAM)."""
        ptr = C.c_void_p(-1) if stream_ptr is None else C.c_void_p(stream_ptr)
        self._check(self.lib.rt_set_stream(self.h, ptr), "rt_set_stream")

    def set_post_stream(self, stream_ptr: int | None):
        """Run denoise + post on a second stream and alternate two G-buffer sets (frame pipelining)."""
        self._check(self.lib.rt_set_post_stream(self.h, stream_ptr), "rt_set_post_stream")

    def set_gather_stream(self, stream: int | None):
        """Stream the caller gathers G-buffers on; each later denoise also waits for it.
        0 is the null stream (torch's default stream), as in set_stream; None turns it off."""
        ptr = C.c_void_p(-2) if stream is None else C.c_void_p(stream)  # RT_STREAM_OFF
        self._check(self.lib.rt_set_gather_stream(self.h, ptr), "rt_set_gather_stream")

    def set_collective_hook(self, fn):
        """fn(stage, stream_handle, exchange) -> None, called on the host when a strip-local denoise
        needs its histogram all-reduce (HOOK_HISTOGRAM) or its rows all-gather (HOOK_ROWS) enqueued
        on stream_handle; None removes the hook (every rank then denoises the whole frame)."""
        if fn is None:
            self._hook = None
            self._check(self.lib.rt_set_collective_hook(self.h, None, None), "rt_set_collective_hook")
            return

        def tramp(arg, stage, stream, x):
            try:
                fn(stage, stream or 0, x.contents)
                return 0
            except Exception:  # reported through rt_last_error's RT_ERR_STATE
                import traceback
                traceback.print_exc()
                return 1

        self._hook = COLLECTIVE_FN(tramp)  # keep the thunk alive as long as the context
        self._check(self.lib.rt_set_collective_hook(self.h, C.cast(self._hook, C.c_void_p), None),
                    "rt_set_collective_hook")

    def set_hook_stages(self, *stages):
        """The hook stages the renderer calls (HOOK_HISTOGRAM, HOOK_ROWS, HOOK_GBUFFERS)."""
        mask = 0
        for st in stages:
            mask |= 1 << int(st)
        self._check(self.lib.rt_set_hook_stages(self.h, mask), "rt_set_hook_stages")

    def bind_buffer(self, name: str, device_ptr: int, nbytes: int, gbuffer_set: int = 0):
        what = BUF[name] | (int(gbuffer_set) << 8)  # RT_BUF_SET1 / RT_BUF_SET2 / RT_BUF_SET3
        self._check(self.lib.rt_bind_buffer(self.h, what, device_ptr, nbytes), "rt_bind_buffer")

    def buffer_bytes(self, name: str) -> int:
        return self.lib.rt_buffer_bytes(self.h, BUF[name])

    def ray_count(self, reset: bool = False) -> int:
        v = C.c_uint64()
        self._check(self.lib.rt_get_ray_count(self.h, C.byref(v), 1 if reset else 0), "rt_get_ray_count")
        return v.value

    def sync(self):
        self._check(self.lib.rt_sync(self.h), "rt_sync")

    def time_stage(self, stage: int, iters: int) -> float:
        ms = C.c_float()
        self._check(self.lib.rt_time_stage(self.h, stage, iters, C.byref(ms)), "rt_time_stage")
        return ms.value

    PT_KERNELS = ("k_pt_camera", "k_pt_shade0", "k_trace_queue<3>", "k_pt_resume<3>", "k_trace_queue<4>",
                  "k_pt_resume<4>", "k_pt_resolve")
    DN_KERNELS = ("k_temporal", "k_spatial7", "k_spatial5<3>", "k_spatial5<6>", "k_spatial5<12>", "k_temporal2",
                  "k_downscale_chain", "k_scale_post")
    FRAME_KERNELS = PT_KERNELS + DN_KERNELS

    def time_path_trace_kernels(self, iters=10):
        """Average ms of each path-trace kernel (HIP events on the context stream)."""
        ms = (C.c_float * len(self.PT_KERNELS))()
        self._check(self.lib.rt_time_path_trace_kernels(self.h, iters, ms, len(ms)), "rt_time_path_trace_kernels")
        return dict(zip(self.PT_KERNELS, (float(v) for v in ms)))

    def time_frame_kernels(self, first_frame: int, iters: int = 10):
        """Average ms of each path-trace and denoise / post kernel over `iters` whole frames run as
        the caller runs them (pipelined when a post stream is set); waits for the frames."""
        ms = (C.c_float * len(self.FRAME_KERNELS))()
        self._check(self.lib.rt_time_frame_kernels(self.h, first_frame, iters, ms, len(ms)), "rt_time_frame_kernels")
        return dict(zip(self.FRAME_KERNELS, (float(v) for v in ms)))

    def frame_marks_begin(self, frames: int, kernels=None):
        """Bracket the kernels named in `kernels` (all 15 when None) of the next `frames` frames with
        HIP events on the streams they run on."""
        names = self.FRAME_KERNELS if kernels is None else kernels
        mask = sum(1 << self.FRAME_KERNELS.index(k) for k in names)
        self._check(self.lib.rt_frame_marks_begin(self.h, frames, mask), "rt_frame_marks_begin")

    def frame_marks_read(self):
        """({kernel: average ms over the recorded frames} for the marked kernels, frames recorded); waits."""
        ms = (C.c_float * len(self.FRAME_KERNELS))()
        n = C.c_int()
        self._check(self.lib.rt_frame_marks_read(self.h, ms, len(ms), C.byref(n)), "rt_frame_marks_read")
        return {k: float(v) for k, v in zip(self.FRAME_KERNELS, ms) if v >= 0.0}, n.value

    # ---- camera file I/O and offscreen image dumps
    def save_camera(self, path: str):
        self._check(self.lib.rt_save_camera(self.h, path.encode()), "rt_save_camera")

    def load_camera(self, path: str):
        self._check(self.lib.rt_load_camera(self.h, path.encode()), "rt_load_camera")

    def save_image(self, path: str, kind: int = IMAGE_PPM_RGBA8):
        self._check(self.lib.rt_save_image(self.h, path.encode(), kind), "rt_save_image")

    def upload_texture(self, name: str, texels: np.ndarray):
        """init.cu:524-580: a 16-bit (H, W, C) level-0 image into the atlas; mips built on the device."""
        t = np.ascontiguousarray(texels, np.uint16)
        h, w = t.shape[:2]
        c = 1 if t.ndim == 2 else t.shape[2]
        self._check(self.lib.rt_upload_texture(self.h, TEX[name], t.ctypes.data, w, h, c), "rt_upload_texture")

    # ---- downloads
    def download(self, name: str, dtype=np.uint8) -> np.ndarray:
        what = ARR[name]
        n = self.lib.rt_array_bytes(self.h, what)
        buf = np.empty(n, dtype=np.uint8)
        self._check(self.lib.rt_download(self.h, what, buf.ctypes.data, n), "rt_download(%s)" % name)
        return buf.view(dtype)

    def trace_rays(self, org, dirs, want_iters=False):
        """Closest hits of n rays (RaySceneIntersect traversal) through the queue tracer.
        Returns (t, tri, u, v[, iters], kernel_ms); tri = -1 on a miss."""
        org = np.asarray(org, np.float32).reshape(-1, 3)
        dirs = np.asarray(dirs, np.float32).reshape(-1, 3)
        n = len(org)
        rays = np.zeros((n, 8), np.float32)
        rays[:, 0:3] = org
        rays[:, 4:7] = dirs
        hits = np.zeros((n, 4), np.float32)
        iters = np.zeros(n, np.uint32) if want_iters else None
        ms = C.c_float()
        self._check(self.lib.rt_trace_rays(self.h, rays.ctypes.data, n, hits.ctypes.data, _ptr(iters), C.byref(ms)),
                    "rt_trace_rays")
        out = (hits[:, 0], hits[:, 1].view(np.int32), hits[:, 2], hits[:, 3])
        return out + ((iters,) if want_iters else ()) + (ms.value,)

    def get_buffer(self, name: str, shape=None, dtype=np.uint8) -> np.ndarray:
        if shape is None:
            n = self.lib.rt_buffer_bytes(self.h, BUF[name])
            shape = (n // np.dtype(dtype).itemsize,)
        out = np.empty(shape, dtype=dtype)
        self._check(self.lib.rt_get_buffer(self.h, BUF[name], out.ctypes.data, out.nbytes), "rt_get_buffer")
        return out


def _ptr(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data
