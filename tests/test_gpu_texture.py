"""Texture path (init.cu:524-580, MipmapGen mipgen.cu:121-182) on the GPU: level 0 of a 16-bit
image uploaded through rt_upload_texture, the 11-level chain built by the device kernel, checked
against the oracle's restatement (oracle/texture.cpp) and an integer numpy restatement of the
same rule, then sampled by the diffuse shading of a rendered frame."""
import numpy as np
import pytest

from test_gpu_pathtrace import make_rt, terrain_camera

pytestmark = pytest.mark.gpu

LEVELS = [1024 >> l for l in range(11)]


def numpy_chain(img):
    """(a + b + c + d) / 4 in float is exact below 2^24 and truncation is floor: integer >> 2."""
    c = 1 if img.ndim == 2 else img.shape[2]
    lv = [np.asarray(img, np.int64).reshape(1024, 1024, c)]
    for n in LEVELS[1:]:
        p = lv[-1]
        lv.append((p[0::2, 0::2] + p[0::2, 1::2] + p[1::2, 0::2] + p[1::2, 1::2]) >> 2)
    return np.concatenate([a.reshape(-1, c) for a in lv]).astype(np.uint16)


def test_synthetic_pair_mips_built_on_device(rtx, oracle, tmp_path):
    rt = make_rt(rtx, tmp_path, 64, 48)
    a, n = oracle.textures()
    assert np.array_equal(rt.download("TEX_ALBEDO_AO", np.uint16).reshape(-1, 4), a)
    assert np.array_equal(rt.download("TEX_NORMAL_ROUGHNESS", np.uint16).reshape(-1, 4), n)
    assert np.array_equal(numpy_chain(a[:1024 * 1024].reshape(1024, 1024, 4)), a)
    rt.cleanup()


def test_upload_16bit_textures_and_render(rtx, oracle, tmp_path, default_scene):
    rng = np.random.default_rng(3)
    w, h = 128, 72
    rt = make_rt(rtx, tmp_path, w, h, spp=2)
    rt.set_delta_time(16.667)
    imgs = {}
    for name, c in (("SOIL_ALBEDO_AO", 4), ("SOIL_NORMAL_ROUGHNESS", 4), ("SOIL_HEIGHT", 1)):
        img = rng.integers(0, 65536, size=(1024, 1024, c) if c > 1 else (1024, 1024), dtype=np.uint16)
        img[:8, :8] = 65535  # a saturated corner: the min(65535) and the truncation at the top of the range
        rt.upload_texture(name, img)
        got = rt.download("TEX_" + name[5:], np.uint16).reshape(-1, c)
        ref = oracle.mip_chain(img)
        assert np.array_equal(got, ref), name
        assert np.array_equal(ref, numpy_chain(img)), name
        imgs[name] = ref
    with pytest.raises(rtx.RtError):
        rt.upload_texture("SOIL_ALBEDO_AO", np.zeros((512, 512, 4), np.uint16))  # the atlas is 1024^2
    oc, rc = terrain_camera(rtx, oracle, w, h)
    rt.camera = rc
    s = oracle.sky()
    tex = (imgs["SOIL_ALBEDO_AO"], imgs["SOIL_NORMAL_ROUGHNESS"])
    dn = oracle.Denoiser(w, h)
    rgba = np.zeros((h, w, 4), np.uint8)
    for f in (1, 2):
        rt.draw(rgba)
        g = oracle.pathtrace(default_scene["bvh"], w, h, frame_num=f, spp=2, cam=oc, hist_cam=oc, sky_out=s, tex=tex)
        o = dn.draw(g, f, delta_time=16.667)
        assert np.array_equal(rgba.reshape(-1, 4), o["rgba"]), f
    rt.cleanup()
