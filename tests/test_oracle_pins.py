"""Pin the CPU oracle to the reference: known answers SURVEY.md recorded from the reference's
own code and scene (tests/golden/golden.json "survey_pins"), plus regression digests."""
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
PINS = GOLD["survey_pins"]


def hit_core(h):
    """The 76-byte OrcHit prefix the digests were taken on (fields added later are excluded)."""
    return np.ascontiguousarray(h).view(np.uint8).reshape(len(h), -1)[:, :76]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def leaf_depths(nodes):
    """nodes on each root-to-leaf path, leaf included (SURVEY §0 #8c counts this way)"""
    out, st = [], [(0, 1)]
    while st:
        v, d = st.pop()
        nd = nodes[v]
        for idx, leaf in ((nd["idxLeft"], nd["isLeftLeaf"]), (nd["idxRight"], nd["isRightLeaf"])):
            if leaf:
                out.append(d + 1)
            else:
                st.append((int(idx), d + 1))
    return out


def batch_slices(b):
    B, n = b["batch_count"], b["tri_count"]
    for k in range(B):
        cnt = 1024 if k < B - 1 else n - (B - 1) * 1024
        yield k, cnt


def check_tree(nodes, n):
    """valid binary tree over n leaves: every internal node except the root has one parent."""
    parents = np.zeros(n - 1, np.int32)
    leaves = np.zeros(n, np.int32)
    for nd in nodes[:n - 1]:
        for idx, leaf in ((nd["idxLeft"], nd["isLeftLeaf"]), (nd["idxRight"], nd["isRightLeaf"])):
            if leaf:
                leaves[idx] += 1
            else:
                parents[idx] += 1
    assert parents[0] == 0 and (parents[1:] == 1).all() and (leaves == 1).all()


def test_morton3_known_answer(oracle):
    assert oracle.lib().orc_morton3(1023, 0, 0) == PINS["morton3_1023_0_0"]


@pytest.mark.parametrize("key,cd", [("default", 1), ("chunk4", 4)])
def test_scene_and_bvh_pins(oracle, key, cd):
    pin = PINS[key]
    v, i, n = oracle.scene(cd)
    assert n == pin["triCount"]
    b = oracle.build_bvh(v, i, n, oracle.smooth_normals(v, i))
    assert b["batch_count"] == pin["batchCount"]
    depths, dup = [], 0
    for k, cnt in batch_slices(b):
        keys = b["morton"][k * 1024:k * 1024 + cnt]
        dup += cnt - len(np.unique(keys))
        nodes = b["nodes"][k * 1024:k * 1024 + cnt - 1]
        check_tree(nodes, cnt)
        depths.append(max(leaf_depths(nodes)))
    assert cnt == pin["lastBatch"]
    assert dup == pin["dupKeys"]
    assert [min(depths), int(np.median(depths)), max(depths)] == pin["blasDepthMinMedMax"]
    check_tree(b["tlas_nodes"], b["batch_count"])
    assert max(leaf_depths(b["tlas_nodes"])) == pin["tlasDepth"]
    if "quirkBoxMaxXY" in pin:
        sb = b["tlas_scene_aabb"]
        assert [float(sb[3]), float(sb[4])] == pytest.approx(pin["quirkBoxMaxXY"], abs=1e-5)
        ta = b["tlas_aabbs"]
        assert [float(ta[:, 3].max()), float(ta[:, 4].max())] == pytest.approx(pin["trueBoxMaxXY"], abs=1e-5)
        c = (ta[:, 3:] + ta[:, :3]) / np.float32(2)
        u = (c - sb[:3]) / (sb[3:] - sb[:3])
        assert int(((u < 0) | (u > 1)).any(1).sum()) == pin["tlasCentresOutside"]


def test_sorted_keys_are_stable_sort_of_unsorted(default_scene):
    b = default_scene["bvh"]
    for k, cnt in batch_slices(b):
        uns = b["morton_unsorted"][k * 1024:(k + 1) * 1024]
        order = np.argsort(uns, kind="stable")
        assert (b["reorder"][k * 1024:(k + 1) * 1024] == order).all()
        assert (b["morton"][k * 1024:(k + 1) * 1024] == uns[order]).all()


def test_oracle_regression_digests(default_scene, oracle):
    g = GOLD["oracle"]["default"]
    assert sha(default_scene["vertices"]) == g["vertices_sha256"]
    assert sha(default_scene["indices"]) == g["indices_sha256"]
    assert sha(default_scene["normals"]) == g["normals_sha256"]
    b = default_scene["bvh"]
    assert sha(b["morton"]) == g["morton_sha256"]
    assert sha(b["reorder"]) == g["reorder_sha256"]
    assert sha(b["tlas_nodes"]) == g["tlas_nodes_sha256"]
    rays, _ = oracle.primary_rays(64, 64, 1)
    assert sha(rays) == g["primary64_rays_sha256"]
    assert sha(hit_core(oracle.intersect(b, rays))) == g["primary64_hits_sha256"]


def test_primary_rays_hit_terrain(default_scene, oracle):
    rays, cone = oracle.primary_rays(64, 64, 1)
    hits = oracle.intersect(default_scene["bvh"], rays)
    # default camera (-2,2,-2) looks +z from below the terrain top (y 5..11): up-left rays hit
    assert 0.05 < hits["hit"].mean() < 0.95
    assert (hits["t"][hits["hit"] == 1] < 40).all()
    assert (hits["objectIdx"][hits["hit"] == 0] == -1).all()
    nz = np.linalg.norm(hits["normal"][hits["hit"] == 1], axis=1)
    assert np.allclose(nz, 1, atol=1e-5)
    assert (cone > 0).all()


def test_sky_model_matches_reference_probe(oracle):
    """SURVEY.md §8c ran the reference's own UpdateSkyState + GetSkyRadiance for the zenith ray and
    got (12.18, 11.81, 11.38); the sun direction of that probe was not recorded.  One free
    parameter (the sun's zenith angle) must reproduce all three channels to the printed
    precision: a one-dimensional family matching a 3-vector pins the spectral model (fitted
    configs, radiances, CIE weights, XYZ->sRGB) up to the sun position."""
    import ctypes as C

    L = oracle.lib()
    t = oracle.sky_tables()
    tabs = oracle.SkyTables(*[a.ctypes.data for a in t])
    L.orc_sky_radiance_sun.argtypes = [C.POINTER(oracle.SkyTables), C.c_void_p, C.c_void_p, C.c_void_p]
    L.orc_sky_radiance_sun.restype = None
    target = np.array([12.18, 11.81, 11.38])
    zen = np.array([0.0, 1.0, 0.0], np.float32)
    best = None
    for th in np.linspace(0.30, 0.55, 2501):
        sun = np.array([np.sin(th), np.cos(th), 0.0], np.float32)
        out = np.zeros(3, np.float32)
        L.orc_sky_radiance_sun(C.byref(tabs), sun.ctypes.data, zen.ctypes.data, out.ctypes.data)
        err = np.abs(out - target).max()
        if best is None or err < best:
            best = err
    assert best < 0.005


def test_dynamic_resolution_rule(oracle):
    """UpdateFrame's dynamic-resolution step (kernel.cu:77-100) restated in float32 arithmetic:
    outside the targetFps +-2 band the width scales by sqrt(target / dt) (int *= float), snaps
    to the nearest multiple of 16 (8 rounds up), clamps to [minWidth, maxWidth]; height = w/16*9."""
    f32 = np.float32

    def rule(w, dt, fps, lo, hi, maxh):
        high, low = f32(1000.0) / f32(fps - 2), f32(1000.0) / f32(fps + 2)
        if high < f32(dt) or low > f32(dt):
            w = int(f32(w) * np.sqrt(f32(1000.0) / f32(fps) / f32(dt)))
        w = w - w % 16 if w % 16 < 8 else w + 16 - w % 16
        w = lo if w < lo else (hi if w > hi else w)
        return w, min((w // 16) * 9, maxh)

    cases = [(192, 40.0), (128, 10.0), (160, 25.0), (128, 16.4), (1920, 16.0), (1920, 13.3), (3840, 5.0),
             (1000, 1000.0), (647, 16.667), (1288, 17.5)]
    for w, dt in cases:
        assert oracle.dynamic_resolution(w, dt, 60.0, 640 if w >= 640 else 64, 3840, 2160) == \
            rule(w, dt, 60.0, 640 if w >= 640 else 64, 3840, 2160), (w, dt)
    assert oracle.dynamic_resolution(192, 40.0, 60.0, 64, 192, 108) == (128, 72)
    assert oracle.dynamic_resolution(1920, 1000.0, 60.0, 640, 3840, 2160) == (640, 360)   # clamped to minWidth
    assert oracle.dynamic_resolution(3840, 13.3, 60.0, 640, 3840, 2160) == (3840, 2160)   # 75-fps cap: grows, clamped


def _probe_hit(oracle, tmp_path, z0, z1):
    """closest hit of the ray (0.2, 0.2, 0) + t (0, 0, 1) on the two-triangle probe scene, built as
    a meshProcessor .bin through the oracle's LBVH (1 BLAS batch of 2 + padding, the B == 1 TLAS)"""
    from scene_bin import bin_bvh, probe_triangles, write_bin

    path = write_bin(str(tmp_path / "probe.bin"), probe_triangles(z0, z1))
    b, _, _, _ = bin_bvh(oracle, path)
    assert b["batch_count"] == 1
    tl = b["tlas_nodes"][0]  # buildBVH.cuh:31-38: {aabbs[0], AABB(0, 0)}, both children leaf 0
    assert (tl["isLeftLeaf"], tl["isRightLeaf"], tl["idxLeft"], tl["idxRight"]) == (1, 1, 0, 0)
    assert (tl["rmin"] == 0).all() and (tl["rmax"] == 0).all()
    return oracle.intersect(b, np.array([[0.2, 0.2, 0.0, 0.0, 0.0, 1.0]], np.float32))[0]


def test_traverse_probe_two_triangles(oracle, tmp_path):
    """SURVEY.md §8c ran the reference's TraverseBvh on a hand-built 2-triangle BLAS under a
    1-leaf TLAS and printed obj=1, t=2.99999952 (two ulps below 3: the watertight test's
    T * (1/det) rounding), geometric normal (0,0,1), uv (0.6, 0.2).  The geometry was not recorded;
    this reconstruction (unit right triangles in z = 5 and z = 3, the nearer one object 1, a +z
    ray through (0.2, 0.2)) reproduces every printed value bit for bit (t) or to the printed digits."""
    pin = PINS["traverse_probe"]
    h = _probe_hit(oracle, tmp_path, 5.0, 3.0)
    assert int(h["objectIdx"]) == pin["objectIdx"]
    assert np.float32(h["t"]).view(np.uint32) == np.float32(pin["t"]).view(np.uint32) == 0x403FFFFE
    assert round(float(h["u"]), 6) == pin["u"] and round(float(h["v"]), 6) == pin["v"]
    # RaySceneIntersect flips the geometric normal (0,0,1) to face the +z ray (traverse.cuh:192-217)
    assert list(np.abs(h["normal"])) == pin["geometricNormal"] and h["normal"][2] == -1.0


def test_triangle_probe(oracle, tmp_path):
    """RayTriangleIntersect -> t=1, u=0.6, v=0.2 (the same unit triangle at z = 1)."""
    pin = PINS["triangle_probe"]
    h = _probe_hit(oracle, tmp_path, 5.0, 1.0)
    assert float(h["t"]) == pin["t"] and int(h["objectIdx"]) == 1
    assert round(float(h["u"]), 6) == pin["u"] and round(float(h["v"]), 6) == pin["v"]


def test_padding_triangles_displace_real_ones(oracle, tmp_path):
    """the padding triangles (index 0 repeated up to a multiple of 4, init.cu:104-115)
    are Morton-coded with the rest and only the first triCount sorted keys are built, so a padding
    key can take a real triangle's place.  Two triangles at z = 1 and 5: both pads sit on vertex 0
    (the box minimum, Morton 0) and sort first, so the tree holds the two pads and the ray misses."""
    from scene_bin import bin_bvh, probe_triangles, write_bin

    b, _, _, _ = bin_bvh(oracle, write_bin(str(tmp_path / "pad.bin"), probe_triangles(1.0, 5.0)))
    assert list(b["reorder"][:2]) == [2, 3] and list(b["morton"][:2]) == [0, 0]
    h = oracle.intersect(b, np.array([[0.2, 0.2, 0.0, 0.0, 0.0, 1.0]], np.float32))[0]
    assert int(h["objectIdx"]) == -1
