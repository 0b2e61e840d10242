"""ORACLE — ctypes wrapper of oracle/_build/liboracle.so (CPU restatement of the reference).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / CPU baseline, never as the measured product.
See oracle/ocommon.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
# the same restatement with host-libm transcendentals (ocommon.h ORC_LIBM): the parity-metric
# reference that shares no transcendental code with the product
LIBM_PATH = os.path.join(HERE, "_build", "liboracle_libm.so")
# ... and with nvcc-style a*b+c contraction into fused multiply-adds (Makefile liboracle_libm_fma.so)
LIBM_FMA_PATH = os.path.join(HERE, "_build", "liboracle_libm_fma.so")
_PATHS = {"libm": LIBM_PATH, "libm_fma": LIBM_FMA_PATH}
DATA_DIR = os.path.join(os.path.dirname(HERE), "real-time-ray-tracing_amd", "data")

NODE_DTYPE = np.dtype([("lmin", "<f4", 3), ("lmax", "<f4", 3), ("rmin", "<f4", 3), ("rmax", "<f4", 3),
                       ("idxLeft", "<u4"), ("idxRight", "<u4"), ("isLeftLeaf", "<u4"), ("isRightLeaf", "<u4")])


class BvhIO(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("normals", C.c_void_p), ("indices", C.c_void_p),
                ("triCount", C.c_uint32), ("triCountPadded", C.c_uint32),
                ("triangles", C.c_void_p), ("aabbs", C.c_void_p), ("mortonUnsorted", C.c_void_p),
                ("mortonSorted", C.c_void_p), ("reorderIdx", C.c_void_p), ("nodes", C.c_void_p),
                ("batchSceneAabbs", C.c_void_p), ("tlasAabbs", C.c_void_p), ("tlasSceneAabb", C.c_void_p),
                ("tlasMortonUnsorted", C.c_void_p), ("tlasMortonSorted", C.c_void_p),
                ("tlasReorderIdx", C.c_void_p), ("tlasNodes", C.c_void_p)]


class Scene(C.Structure):
    _fields_ = [("triangles", C.c_void_p), ("nodes", C.c_void_p), ("tlasNodes", C.c_void_p),
                ("triCountPadded", C.c_uint32), ("batchCount", C.c_uint32)]


HIT_DTYPE = np.dtype([("t", "<f4"), ("objectIdx", "<i4"), ("u", "<f4"), ("v", "<f4"), ("normal", "<f4", 3),
                      ("fakeNormal", "<f4", 3), ("pos", "<f4", 3), ("offset", "<f4"), ("hit", "<u4"),
                      ("nodeVisits", "<u4"), ("triTests", "<u4"), ("droppedPushes", "<u4"),
                      ("iterations", "<u4"), ("intoSurface", "<u4"), ("ndr", "<f4"),
                      ("maxDepth", "<u4")])


class CameraIn(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("yaw", C.c_float), ("pitch", C.c_float), ("focal", C.c_float),
                ("aperture", C.c_float), ("fovX", C.c_float), ("resolution", C.c_float * 2)]


_libs: dict = {}
_variant = "rtmath"


@contextlib.contextmanager
def libm(variant: str = "libm"):
    """Run the oracle calls inside the block on the host-libm build (liboracle_libm.so), or with
    variant "libm_fma" on that build with a*b+c contracted to fused multiply-adds."""
    global _variant
    if variant not in _PATHS:
        raise ValueError(variant)
    old, _variant = _variant, variant
    try:
        yield
    finally:
        _variant = old


def lib() -> C.CDLL:
    path = _PATHS.get(_variant, LIB_PATH)
    if path not in _libs:
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: %s (run make)" % path)
        L = C.CDLL(path)
        L.orc_build_bvh.argtypes = [C.POINTER(BvhIO)]
        L.orc_build_bvh.restype = C.c_int
        L.orc_build_bvh_mt.argtypes = [C.POINTER(BvhIO), C.c_int]
        L.orc_build_bvh_mt.restype = C.c_int
        L.orc_morton3.argtypes = [C.c_uint32] * 3
        L.orc_morton3.restype = C.c_uint32
        L.orc_smooth_normals.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p]
        L.orc_smooth_normals.restype = None
        L.orc_intersect.argtypes = [C.POINTER(Scene), C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
        L.orc_intersect.restype = None
        L.orc_primary_rays.argtypes = [C.POINTER(CameraIn), C.c_uint32, C.c_uint32, C.c_int, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
        L.orc_primary_rays.restype = None
        L.orc_bluenoise.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]
        L.orc_bluenoise.restype = C.c_float
        L.orc_rtmath.argtypes = [C.c_int, C.c_float, C.c_float]
        L.orc_rtmath.restype = C.c_float
        L.orc_div_const_mismatches.argtypes = [C.c_float, C.c_uint32]
        L.orc_div_const_mismatches.restype = C.c_long
        L.orc_div_rcp_mismatches.argtypes = [C.c_float, C.c_uint32]
        L.orc_div_rcp_mismatches.restype = C.c_long
        L.orc_unorm16_mismatches.argtypes = []
        L.orc_unorm16_mismatches.restype = C.c_int
        L.orc_rtmath_n.argtypes = [C.c_int, C.c_void_p, C.c_float, C.c_float, C.c_void_p, C.c_size_t]
        L.orc_rtmath_n.restype = None
        L.orc_f2h_n.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_f2h_n.restype = None
        L.orc_h2f_n.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_h2f_n.restype = None
        L.orc_scene_generate.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_uint32)]
        L.orc_scene_generate.restype = C.c_int
        L.orc_scene_copy.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_scene_copy.restype = None
        _bind_frame_api(L)
        _libs[path] = L
    return _libs[path]


def scene(chunk_dim: int = 1):
    """Procedural default scene (input generator): (vertices [nv,3] f32, indices [NP,3] u32, triCount)."""
    L = lib()
    n, npad, nv = C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = L.orc_scene_generate(os.path.join(DATA_DIR, "roundcubes_l2.bin").encode(), chunk_dim, C.byref(n),
                              C.byref(npad), C.byref(nv))
    if rc != 0:
        raise RuntimeError("scene generation failed (%d)" % rc)
    v = np.empty((nv.value, 3), np.float32)
    i = np.empty((npad.value, 3), np.uint32)
    L.orc_scene_copy(v.ctypes.data, i.ctypes.data)
    return v, i, n.value


def smooth_normals(vertices: np.ndarray, indices: np.ndarray) -> np.ndarray:
    out = np.empty_like(vertices)
    lib().orc_smooth_normals(vertices.ctypes.data, vertices.shape[0], indices.ctypes.data, indices.shape[0],
                             out.ctypes.data)
    return out


def build_bvh(vertices, indices, tri_count, normals=None, threads: int = 1) -> dict:
    NP = indices.shape[0]
    B = (tri_count + 1023) // 1024
    out = dict(
        triangles=np.zeros((NP, 18), np.float32), aabbs=np.zeros((NP, 6), np.float32),
        morton_unsorted=np.zeros(B * 1024, np.uint32), morton=np.zeros(B * 1024, np.uint32),
        reorder=np.zeros(B * 1024, np.uint32), nodes=np.zeros(NP, NODE_DTYPE),
        batch_scene_aabbs=np.zeros((B, 6), np.float32), tlas_aabbs=np.zeros((B, 6), np.float32),
        tlas_scene_aabb=np.zeros(6, np.float32), tlas_morton_unsorted=np.zeros(1024, np.uint32),
        tlas_morton=np.zeros(1024, np.uint32), tlas_reorder=np.zeros(1024, np.uint32),
        tlas_nodes=np.zeros(B, NODE_DTYPE))
    io = BvhIO(vertices.ctypes.data, normals.ctypes.data if normals is not None else None, indices.ctypes.data,
               tri_count, NP, out["triangles"].ctypes.data, out["aabbs"].ctypes.data,
               out["morton_unsorted"].ctypes.data, out["morton"].ctypes.data, out["reorder"].ctypes.data,
               out["nodes"].ctypes.data, out["batch_scene_aabbs"].ctypes.data, out["tlas_aabbs"].ctypes.data,
               out["tlas_scene_aabb"].ctypes.data, out["tlas_morton_unsorted"].ctypes.data,
               out["tlas_morton"].ctypes.data, out["tlas_reorder"].ctypes.data, out["tlas_nodes"].ctypes.data)
    rc = lib().orc_build_bvh_mt(C.byref(io), threads)
    if rc < 0:
        raise RuntimeError("orc_build_bvh failed (%d)" % rc)
    out["batch_count"] = rc
    out["tri_count"] = tri_count
    return out


def intersect(bvh: dict, rays: np.ndarray, threads: int = 0) -> np.ndarray:
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = rays.shape[0]
    hits = np.zeros(n, HIT_DTYPE)
    sc = Scene(bvh["triangles"].ctypes.data, bvh["nodes"].ctypes.data, bvh["tlas_nodes"].ctypes.data,
               bvh["triangles"].shape[0], bvh["batch_count"])
    lib().orc_intersect(C.byref(sc), rays.ctypes.data, n, hits.ctypes.data, threads)
    return hits


def default_camera(width: int, height: int) -> CameraIn:
    # CameraSetup, init.cu:412-439
    c = CameraIn()
    c.pos[:] = (-2.0, 2.0, -2.0)
    c.yaw = 0.0
    c.pitch = 0.0
    c.focal = 5.0
    c.aperture = 0.001
    c.fovX = np.float32(90.0) * np.float32(0.01745329251)
    c.resolution[:] = (float(width), float(height))
    return c


def bluenoise_tables() -> np.ndarray:
    return np.fromfile(os.path.join(DATA_DIR, "bluenoise_4spp.bin"), dtype=np.uint8)


def primary_rays(width: int, height: int, frame_num: int = 1, cam: CameraIn | None = None):
    cam = cam or default_camera(width, height)
    bn = bluenoise_tables()
    rays = np.zeros((width * height, 6), np.float32)
    cone = np.zeros(width * height, np.float32)
    lib().orc_primary_rays(C.byref(cam), width, height, frame_num, bn.ctypes.data, rays.ctypes.data,
                           cone.ctypes.data)
    return rays, cone


RTMATH = dict(sin=0, cos=1, tan=2, atan=3, atan2=4, acos=5, asin=6, exp=7, exp2=8, log=9, log2=10, pow=11,
              log2_div=12, pow_div=13)  # *_div: the path tracer's log2 variant (rtmath.h log2_pair_t)


def rtmath(fn: str, x: float, y: float = 0.0) -> float:
    return lib().orc_rtmath(RTMATH[fn], x, y)


def rtmath_n(fn: int, x: np.ndarray, y: float = 0.0, c: float = 0.0) -> np.ndarray:
    """rtmath.h over a float32 array (0 pow(x, y), 1 expf(x), 2 rt_div_rcp(x, y, c))."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    lib().orc_rtmath_n(fn, x.ctypes.data, y, c, out.ctypes.data, x.size)
    return out


def f2h(f: np.ndarray) -> np.ndarray:
    """rt_f2h over a float32 array: uint16 bit patterns (round to nearest even, NaN -> sign|0x7E00)."""
    f = np.ascontiguousarray(f, np.float32)
    h = np.empty(f.shape, np.uint16)
    lib().orc_f2h_n(f.ctypes.data, h.ctypes.data, f.size)
    return h


def h2f(h: np.ndarray) -> np.ndarray:
    """rt_h2f over a uint16 array of half bit patterns: float32 (exact; NaN quieted, payload kept)."""
    h = np.ascontiguousarray(h, np.uint16)
    f = np.empty(h.shape, np.float32)
    lib().orc_h2f_n(h.ctypes.data, f.ctypes.data, h.size)
    return f


# ---------------------------------------------------------------- sky (oracle/sky.cpp)
class SkyTables(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("skyDataSets", "skyDataSetsRad", "solarDatasets",
                                          "limbDarkeningDatasets", "cieX", "cieY", "cieZ")]


class SkyParams(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("timeOfDay", "sunAxisAngle", "skyScalar", "sunScalar", "sunAngle")]


class SkyOut(C.Structure):
    _fields_ = [("sunDir", C.c_float * 3), ("skyBuffer", C.c_void_p), ("skyPdf", C.c_void_p),
                ("skyCdf", C.c_void_p), ("sunBuffer", C.c_void_p), ("sunPdf", C.c_void_p), ("sunCdf", C.c_void_p),
                ("sunArea", C.c_float), ("sunAngleCosThetaMax", C.c_float)]


class Frame(C.Structure):
    _fields_ = [("scene", Scene), ("triCount", C.c_uint32), ("materialOverride", C.c_int32), ("cam", CameraIn),
                ("histCam", CameraIn), ("frameNum", C.c_int), ("spp", C.c_uint32), ("bluenoise", C.c_void_p),
                ("texAlbedoAo", C.c_void_p), ("texNormalRough", C.c_void_p), ("skyBuffer", C.c_void_p),
                ("sunBuffer", C.c_void_p), ("skyCdf", C.c_void_p), ("sunCdf", C.c_void_p),
                ("sunDir", C.c_float * 3), ("sunAngleCosThetaMax", C.c_float)]


class GBuffer(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("color", "normal", "albedo", "depth", "motion", "rays")]


SKY_DEFAULTS = dict(timeOfDay=0.25, sunAxisAngle=45.0, skyScalar=0.01, sunScalar=0.01, sunAngle=0.6)  # settingParams.h:41-45
TEX_TEXELS = 1398101  # 11-level mip chain of a 1024^2 ushort4 texture


def _bind_frame_api(L):
    L.orc_sky.argtypes = [C.POINTER(SkyTables), C.POINTER(SkyParams), C.POINTER(SkyOut)]
    L.orc_sky.restype = None
    L.orc_sun_dir.argtypes = [C.c_float, C.c_float, C.c_void_p]
    L.orc_sun_dir.restype = None
    L.orc_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.orc_scan.restype = None
    L.orc_scan_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
    L.orc_scan_ex.restype = None
    L.orc_cpu_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.orc_cpu_scan.restype = None
    L.orc_filter_kernel.argtypes = [C.c_int, C.c_void_p]
    L.orc_filter_kernel.restype = C.c_int
    L.orc_textures.argtypes = [C.c_void_p, C.c_void_p]
    L.orc_textures.restype = None
    L.orc_mip_chain.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
    L.orc_mip_chain.restype = None
    L.orc_pathtrace.argtypes = [C.POINTER(Frame), C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.POINTER(GBuffer), C.c_int]
    L.orc_pathtrace.restype = None
    L.orc_sky_radiance.argtypes = [C.POINTER(SkyTables), C.c_float, C.c_float, C.c_void_p, C.c_void_p]
    L.orc_sky_radiance.restype = None
    L.orc_denoise_post.argtypes = [C.c_void_p]
    L.orc_denoise_post.restype = C.c_int
    L.orc_lens_flare_setup.argtypes = [C.POINTER(CameraIn), C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                       C.c_void_p]
    L.orc_lens_flare_setup.restype = C.c_int
    L.orc_dynamic_resolution.argtypes = [C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.orc_dynamic_resolution.restype = None


def sky_tables() -> list:
    raw = np.fromfile(os.path.join(DATA_DIR, "sky_tables.bin"), dtype=np.uint8)
    count = int(raw[:4].view(np.uint32)[0])
    lens = raw[4:4 + 4 * count].view(np.uint32)
    off = 4 + 4 * count
    out = []
    for n in lens:
        out.append(raw[off:off + 4 * int(n)].view(np.float32).copy())
        off += 4 * int(n)
    return out


def sky(params: dict | None = None) -> dict:
    """Sky + sun buffers, luminance pdfs and their inclusive-scan CDFs (kernel.cu:280-307)."""
    L = lib()
    p = dict(SKY_DEFAULTS, **(params or {}))
    t = sky_tables()
    tabs = SkyTables(*[a.ctypes.data for a in t])
    out = dict(sky=np.zeros((256, 512, 4), np.float32), sky_pdf=np.zeros(131072, np.float32),
               sky_cdf=np.zeros(131072, np.float32), sun=np.zeros((32, 32, 4), np.float32),
               sun_pdf=np.zeros(1024, np.float32), sun_cdf=np.zeros(1024, np.float32))
    so = SkyOut((C.c_float * 3)(), out["sky"].ctypes.data, out["sky_pdf"].ctypes.data, out["sky_cdf"].ctypes.data,
                out["sun"].ctypes.data, out["sun_pdf"].ctypes.data, out["sun_cdf"].ctypes.data, 0.0, 0.0)
    L.orc_sky(C.byref(tabs), C.byref(SkyParams(*[p[k] for k in SKY_DEFAULTS])), C.byref(so))
    out["sun_dir"] = np.array(so.sunDir[:], np.float32)
    out["sun_area"] = np.float32(so.sunArea)
    out["cos_theta_max"] = np.float32(so.sunAngleCosThetaMax)
    return out


def sky_radiance(direction, time_of_day: float = 0.25, sun_axis_angle: float = 45.0) -> np.ndarray:
    """GetSkyRadiance before skyScalar for one direction (sky.cuh:165-197)."""
    t = sky_tables()
    tabs = SkyTables(*[a.ctypes.data for a in t])
    d = np.ascontiguousarray(direction, np.float32)
    out = np.zeros(3, np.float32)
    lib().orc_sky_radiance(C.byref(tabs), time_of_day, sun_axis_angle, d.ctypes.data, out.ctypes.data)
    return out


def scan(x: np.ndarray, block: int, postfix: int = 1) -> np.ndarray:
    """Scan (scan.cuh:258-298): Blelloch blocks in tree order, block totals scanned, added."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().orc_scan_ex(x.ctypes.data, y.ctypes.data, x.size, block, postfix)
    return y


def cpu_scan(x: np.ndarray, postfix: int = 1) -> np.ndarray:
    """CpuScan (scan.cuh:235-251): the sequential float scan the reference's scan test compares with."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().orc_cpu_scan(x.ctypes.data, y.ctypes.data, x.size, postfix)
    return y


def filter_kernel(size: int) -> np.ndarray:
    """The denoiser's Gaussian table (gaussian.cuh:12-43) as the oracle's filters use it."""
    out = np.zeros(size * size, np.float32)
    assert lib().orc_filter_kernel(size, out.ctypes.data) == 0
    return out


def textures():
    a = np.zeros((TEX_TEXELS, 4), np.uint16)
    n = np.zeros((TEX_TEXELS, 4), np.uint16)
    lib().orc_textures(a.ctypes.data, n.ctypes.data)
    return a, n


def mip_chain(level0: np.ndarray) -> np.ndarray:
    """MipmapGen chain (11 levels, 1024 -> 1, concatenated) of a 1024x1024 16-bit image (H, W[, C])."""
    c = 1 if level0.ndim == 2 else level0.shape[2]
    chain = np.zeros((TEX_TEXELS, c), np.uint16)
    chain[:1024 * 1024] = np.asarray(level0, np.uint16).reshape(-1, c)
    lib().orc_mip_chain(chain.ctypes.data, 1024, 11, c)
    return chain


def pathtrace(bvh: dict, width: int, height: int, frame_num: int = 1, spp: int = 1, cam: CameraIn | None = None,
              hist_cam: CameraIn | None = None, sky_out: dict | None = None, tex=None, y0: int = 0,
              rows: int | None = None, material_override: int = -1, threads: int = 0) -> dict:
    """PathTrace G-buffers (pathtrace.cuh:11-128) for rows [y0, y0+rows): raw half/ushort bits."""
    cam = cam or default_camera(width, height)
    hist_cam = hist_cam or cam
    sky_out = sky_out or sky()
    tex = tex or textures()
    rows = height - y0 if rows is None else rows
    bn = bluenoise_tables()
    sc = Scene(bvh["triangles"].ctypes.data, bvh["nodes"].ctypes.data, bvh["tlas_nodes"].ctypes.data,
               bvh["triangles"].shape[0], bvh["batch_count"])
    f = Frame(sc, bvh["tri_count"], material_override, cam, hist_cam, frame_num, spp, bn.ctypes.data,
              tex[0].ctypes.data, tex[1].ctypes.data, sky_out["sky"].ctypes.data, sky_out["sun"].ctypes.data,
              sky_out["sky_cdf"].ctypes.data, sky_out["sun_cdf"].ctypes.data,
              (C.c_float * 3)(*sky_out["sun_dir"].tolist()), float(sky_out["cos_theta_max"]))
    P = width * height
    g = dict(color=np.zeros((P, 4), np.uint16), normal=np.zeros((P, 4), np.uint16),
             albedo=np.zeros((P, 4), np.uint16), depth=np.zeros(P, np.uint16), motion=np.zeros((P, 2), np.uint16),
             rays=np.zeros(P, np.uint32))
    gb = GBuffer(*[g[k].ctypes.data for k in ("color", "normal", "albedo", "depth", "motion", "rays")])
    lib().orc_pathtrace(C.byref(f), width, height, y0, rows, C.byref(gb), threads)
    return g


# ---------------------------------------------------------------- denoise + post (oracle/denoise.cpp)
class RtParams(C.Structure):
    """Layout of rt_params (include/rtx_amd.h) with the reference defaults (settingParams.h)."""
    _fields_ = [("sky_needRegenerate", C.c_int32)] + [(n, C.c_float) for n in (
        "timeOfDay", "sunAxisAngle", "skyScalar", "sunScalar", "sunAngle")] + [
        ("sampleSurfaceVsLightUseMisWeight", C.c_int32), ("sampleSkyVsSunUseFluxWeight", C.c_int32),
        ("sampleSurfaceVsLight", C.c_float), ("sampleSkyVsSun", C.c_float)] + [(n, C.c_int32) for n in (
        "enableTemporalDenoising", "enableLocalSpatialFilter", "enableNoiseLevelVisualize",
        "enableWideSpatialFilter", "enableTemporalDenoising2", "enablePostProcess", "enableDownScalePasses",
        "enableHistogram", "enableAutoExposure", "enableBloomEffect", "enableLensFlare", "enableToneMapping",
        "enableSharpening")] + [("toneMappingType", C.c_int32)] + [(n, C.c_float) for n in (
        "exposure", "gain", "maxWhite", "gamma",
        "local_denoise_sigma_normal", "local_denoise_sigma_depth", "local_denoise_sigma_material",
        "large_denoise_sigma_normal", "large_denoise_sigma_depth", "large_denoise_sigma_material",
        "temporal_denoise_sigma_normal", "temporal_denoise_sigma_depth", "temporal_denoise_sigma_material",
        "noise_threshold_local", "noise_threshold_large")]


def default_params() -> RtParams:
    p = RtParams()
    p.sky_needRegenerate = 1
    for k, v in SKY_DEFAULTS.items():
        setattr(p, k, v)
    p.sampleSurfaceVsLightUseMisWeight = p.sampleSkyVsSunUseFluxWeight = 1
    p.sampleSurfaceVsLight = p.sampleSkyVsSun = 0.5
    for k in ("enableTemporalDenoising", "enableLocalSpatialFilter", "enableWideSpatialFilter",
              "enableTemporalDenoising2", "enablePostProcess", "enableDownScalePasses", "enableHistogram",
              "enableAutoExposure", "enableToneMapping", "enableSharpening"):
        setattr(p, k, 1)
    p.toneMappingType = 3
    p.exposure, p.gain, p.maxWhite, p.gamma = 1.0, 40.0, 7.0, 2.2
    p.local_denoise_sigma_normal, p.local_denoise_sigma_depth, p.local_denoise_sigma_material = 100.0, 0.1, 100.0
    p.large_denoise_sigma_normal, p.large_denoise_sigma_depth, p.large_denoise_sigma_material = 100.0, 0.01, 100.0
    p.temporal_denoise_sigma_normal, p.temporal_denoise_sigma_depth = 100.0, 0.1
    p.temporal_denoise_sigma_material = 100.0
    p.noise_threshold_local = p.noise_threshold_large = 0.001
    return p


class PostState(C.Structure):
    _fields_ = [("accum", C.c_void_p), ("histColor", C.c_void_p), ("histDepth", C.c_void_p),
                ("exposure", C.c_float * 4)]


class DrawIO(C.Structure):
    _fields_ = [("W", C.c_uint32), ("H", C.c_uint32), ("Ws", C.c_uint32), ("Hs", C.c_uint32),
                ("frameNum", C.c_int), ("deltaTime", C.c_float), ("params", C.c_void_p), ("bluenoise", C.c_void_p),
                ("color", C.c_void_p), ("normal", C.c_void_p), ("albedo", C.c_void_p), ("depth", C.c_void_p),
                ("motion", C.c_void_p), ("noise8", C.c_void_p), ("noise16", C.c_void_p), ("c4", C.c_void_p),
                ("c16", C.c_void_p), ("c64", C.c_void_p), ("histogram", C.c_void_p), ("scaled", C.c_void_p),
                ("rgba", C.c_void_p), ("state", C.c_void_p), ("bloom4", C.c_void_p), ("bloom16", C.c_void_p),
                ("lensFlare", C.c_int), ("sunPos", C.c_float * 2), ("sunUv", C.c_int * 2),
                ("histW", C.c_uint32), ("histH", C.c_uint32)]


def dynamic_resolution(w: int, dt: float, target_fps: float, min_w: int, max_w: int, max_h: int):
    """UpdateFrame's dynamic-resolution step (kernel.cu:77-100): (next width, next height)."""
    ow, oh = C.c_int(), C.c_int()
    lib().orc_dynamic_resolution(w, dt, target_fps, min_w, max_w, max_h, C.byref(ow), C.byref(oh))
    return ow.value, oh.value


class Denoiser:
    """Frame-persistent oracle state for TemporalSpatialDenoising + PostProcessing."""

    def __init__(self, W: int, H: int, Ws: int | None = None, Hs: int | None = None):
        self.W, self.H = W, H
        self.hist_size = (W, H)  # render size the history buffers hold (historyDim)
        self.Ws, self.Hs = Ws or W, Hs or H
        P = W * H
        self.accum = np.zeros((P, 4), np.uint16)
        self.hist_color = np.zeros((P, 4), np.uint16)
        self.hist_depth = np.zeros(P, np.uint16)
        self.state = PostState(self.accum.ctypes.data, self.hist_color.ctypes.data, self.hist_depth.ctypes.data,
                               (C.c_float * 4)(1.0, 1.0, 1.0, 1.0))
        self.bn = bluenoise_tables()

    def draw(self, g: dict, frame_num: int, params=None, delta_time: float = 1000.0 / 60.0,
             cam: CameraIn | None = None, sun_dir=None, size: tuple[int, int] | None = None) -> dict:
        """cam / sun_dir: the frame's camera and sun direction, needed only for the lens flare.
        size: this frame's render size when dynamic resolution changed it (at most (W, H)); the
        history buffers keep the layout of the size they were written at."""
        params = params if params is not None else default_params()
        W, H = size or (self.W, self.H)
        assert W * H <= self.W * self.H
        Ws, Hs = self.Ws, self.Hs
        d = lambda n: (n + 3) // 4
        W4, H4 = d(W), d(H)
        W16, H16 = d(W4), d(H4)
        W64, H64 = d(W16), d(H16)
        out = dict(color=np.ascontiguousarray(g["color"]).copy(),
                   noise8=np.zeros(((H + 7) // 8) * ((W + 7) // 8), np.uint16),
                   noise16=np.zeros(((H + 15) // 16) * ((W + 15) // 16), np.uint16),
                   c4=np.zeros((W4 * H4, 4), np.uint16), c16=np.zeros((W16 * H16, 4), np.uint16),
                   c64=np.zeros((W64 * H64, 4), np.uint16), histogram=np.zeros(64, np.uint32),
                   scaled=np.zeros((Ws * Hs, 4), np.uint16), rgba=np.zeros((Ws * Hs, 4), np.uint8))
        src = {k: np.ascontiguousarray(g[k]) for k in ("normal", "albedo", "depth", "motion")}
        io = DrawIO(W, H, Ws, Hs, frame_num, delta_time, C.addressof(params), self.bn.ctypes.data,
                    out["color"].ctypes.data, src["normal"].ctypes.data, src["albedo"].ctypes.data,
                    src["depth"].ctypes.data, src["motion"].ctypes.data, out["noise8"].ctypes.data,
                    out["noise16"].ctypes.data, out["c4"].ctypes.data, out["c16"].ctypes.data,
                    out["c64"].ctypes.data, out["histogram"].ctypes.data, out["scaled"].ctypes.data,
                    out["rgba"].ctypes.data, C.addressof(self.state))
        out["bloom4"] = np.zeros((W4 * H4, 4), np.uint16)
        out["bloom16"] = np.zeros((W16 * H16, 4), np.uint16)
        io.bloom4, io.bloom16 = out["bloom4"].ctypes.data, out["bloom16"].ctypes.data
        if params.enableLensFlare and cam is not None and sun_dir is not None:
            sd = np.ascontiguousarray(sun_dir, np.float32)
            sp, su = np.zeros(2, np.float32), np.zeros(2, np.int32)
            io.lensFlare = lib().orc_lens_flare_setup(C.byref(cam), sd.ctypes.data, W, H, sp.ctypes.data,
                                                      su.ctypes.data)
            io.sunPos[:] = sp.tolist()
            io.sunUv[:] = su.tolist()
        io.histW, io.histH = self.hist_size
        rc = lib().orc_denoise_post(C.byref(io))
        self.hist_size = (W, H)
        out["lens_flare"] = int(io.lensFlare)
        out["sun_uv"] = (int(io.sunUv[0]), int(io.sunUv[1]))
        if rc < 0:
            raise RuntimeError("orc_denoise_post: unsupported settings")
        out["exposure"] = np.array(self.state.exposure[:], np.float32)
        return out
