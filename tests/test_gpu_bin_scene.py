"""meshProcessor .bin scenes through the GPU renderer ([scene] meshFile, init.cu:28-50): the
loader, the one-batch BLAS with padding triangles and the B == 1 TLAS special case
(buildBVH.cuh:31-38), traversal, and a full frame, against the oracle fed by the test's own
numpy reader of the same file (tests/scene_bin.py)."""
import numpy as np
import pytest

from scene_bin import bin_bvh, probe_triangles, terrain_patch, write_bin

pytestmark = pytest.mark.gpu


def make(rtx, tmp_path, path, w=64, h=48, spp=1, threads=0):
    cfg = rtx.write_config(str(tmp_path / "b.toml"), w, h, spp=spp, mesh_file=path,
                           extra="bvhThreads = %d\n" % threads)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(16.667)
    return rt


def gpu_nodes(rt, rtx, n):
    return rt.download("NODES").view(rtx.NODE_DTYPE)[:n - 1], rt.download("TLAS_NODES").view(rtx.NODE_DTYPE)[:1]


def test_probe_scene_traversal(rtx, oracle, tmp_path):
    """SURVEY §8c's two-triangle probe (tests/test_oracle_pins.py) traced by the GPU queue tracer."""
    for z0, z1, bits, obj in ((5.0, 3.0, 0x403FFFFE, 1), (5.0, 1.0, 0x3F800000, 1), (1.0, 5.0, None, -1)):
        path = write_bin(str(tmp_path / ("p%g_%g.bin" % (z0, z1))), probe_triangles(z0, z1))
        rt = make(rtx, tmp_path, path)
        info = rt.info()
        assert (info.triCount, info.triCountPadded, info.batchCount) == (2, 4, 1)
        rt.build_bvh()
        b, _, _, _ = bin_bvh(oracle, path)
        g, gt = gpu_nodes(rt, rtx, 2)
        assert g.tobytes() == b["nodes"][:1].tobytes()
        assert gt.tobytes() == b["tlas_nodes"][:1].tobytes()
        t, tri, u, v, ms = rt.trace_rays([[0.2, 0.2, 0.0]], [[0.0, 0.0, 1.0]])
        assert int(tri[0]) == obj
        if bits is not None:
            assert t[0].view(np.uint32) == bits
            assert (u[0], v[0]) == (np.float32(0.59999996), np.float32(0.19999999))
        rt.cleanup()


@pytest.mark.parametrize("ntri", [1012, 1010])
def test_bin_terrain_frame(rtx, oracle, tmp_path, ntri):
    """A 1,012 / 1,010-triangle height field (one batch; 1,010 adds two padding triangles):
    LBVH, primary hits and a 2-frame path trace + denoise + post, bit-exact vs the oracle."""
    tris = terrain_patch()[:ntri]
    path = write_bin(str(tmp_path / "t.bin"), tris)
    w, h = 96, 64
    rt = make(rtx, tmp_path, path, w, h, spp=2)
    b, _, _, n = bin_bvh(oracle, path)
    assert rt.info().triCount == n == ntri and rt.info().batchCount == 1
    cam = rtx.Camera()
    cam.pos[:] = (5.5, 4.0, -3.0)
    cam.yaw, cam.pitch, cam.focal, cam.aperture, cam.fovX = 0.0, -0.55, 5.0, 0.001, np.float32(90.0) * np.float32(0.01745329251)
    rt.camera = cam
    rt.build_bvh()
    g, gt = gpu_nodes(rt, rtx, n)
    assert g.tobytes() == b["nodes"][:n - 1].tobytes()
    assert gt.tobytes() == b["tlas_nodes"][:1].tobytes()
    assert np.array_equal(rt.download("MORTON", np.uint32)[:1024], b["morton"])
    assert np.array_equal(rt.download("REORDER", np.uint32)[:1024], b["reorder"])
    oc = oracle.default_camera(w, h)
    oc.pos[:] = (5.5, 4.0, -3.0)
    oc.pitch = -0.55
    rt.trace_primary(1)
    hits = rt.download("HITS", np.float32).reshape(-1, 4)
    rays, _ = oracle.primary_rays(w, h, 1, cam=oc)
    oh = oracle.intersect(b, rays)
    assert 0.3 < oh["hit"].mean() and np.array_equal(hits[:, 0].view(np.uint32), oh["t"].view(np.uint32))
    assert np.array_equal(hits[:, 1].view(np.int32), oh["objectIdx"])
    s, tex = oracle.sky(), oracle.textures()
    dn = oracle.Denoiser(w, h)
    rgba = np.zeros((h, w, 4), np.uint8)
    for f in (1, 2):
        rt.draw(rgba)
        gb = oracle.pathtrace(b, w, h, frame_num=f, spp=2, cam=oc, hist_cam=oc, sky_out=s, tex=tex)
        o = dn.draw(gb, f, delta_time=16.667)
        assert np.array_equal(rgba.reshape(-1, 4), o["rgba"]), f
        assert np.array_equal(rt.get_buffer("RENDER_COLOR", (w * h, 4), np.uint16), o["color"]), f
    rt.cleanup()


@pytest.mark.parametrize("threads", [0, 512])
def test_one_triangle_last_batch(rtx, oracle, tmp_path, threads):
    """N = 1,025: the last BLAS batch holds 1 real triangle and 3 padding ones (triCountArray = 1,
    init.cu:104-130), the triCount == 1 branch of BuildLBVH (buildBVH.cuh:31-38).  The reference
    writes that node to bvhNodes[0] BEFORE the per-batch offset, racing batch 0's own root and
    leaving batch 1's root unwritten; here it is written to the batch's own node 0 (DESIGN.md §5,
    deviation 12).  Batch 0 (1,024 triangles), batch 1's root, the 2-leaf TLAS, Morton codes and
    traversal hits on the lone triangle are bit-exact vs the oracle, and a full frame renders."""
    tris = terrain_patch(23, 23)[:1025]
    path = write_bin(str(tmp_path / "n1025.bin"), tris)
    w, h = 96, 64
    rt = make(rtx, tmp_path, path, w, h, threads=threads)
    info = rt.info()
    assert (info.triCount, info.triCountPadded, info.batchCount) == (1025, 1028, 2)
    b, _, _, n = bin_bvh(oracle, path)
    rt.build_bvh()
    nodes = rt.download("NODES").view(rtx.NODE_DTYPE)
    assert nodes[:1023].tobytes() == b["nodes"][:1023].tobytes()  # batch 0 keeps its own root
    root1 = nodes[1024]
    assert root1.tobytes() == b["nodes"][1024].tobytes()
    assert (int(root1["idxLeft"]), int(root1["idxRight"]), int(root1["isLeftLeaf"]), int(root1["isRightLeaf"])) == (0, 0, 1, 1)
    tl = rt.download("TLAS_NODES").view(rtx.NODE_DTYPE)[:1]
    assert tl.tobytes() == b["tlas_nodes"][:1].tobytes()
    assert np.array_equal(rt.download("MORTON", np.uint32)[:2048], b["morton"])
    assert np.array_equal(rt.download("REORDER", np.uint32)[:2048], b["reorder"])
    # rays straight down onto the centroids of the last triangles (1,024 is the lone one of batch 1)
    c = tris[1016:1025].mean(axis=1)
    org = np.stack([c[:, 0], np.full(len(c), 20.0, np.float32), c[:, 2]], axis=1).astype(np.float32)
    dirs = np.tile(np.array([0.0, -1.0, 0.0], np.float32), (len(c), 1))
    t, tri, u, v, ms = rt.trace_rays(org, dirs)
    o = oracle.intersect(b, np.concatenate([org, dirs], axis=1))
    assert int(tri[-1]) == 1024
    assert np.array_equal(tri, o["objectIdx"]) and np.array_equal(t.view(np.uint32), o["t"].view(np.uint32))
    rgba = np.zeros((h, w, 4), np.uint8)
    cam = rtx.Camera()
    cam.pos[:] = (5.5, 4.0, -3.0)
    cam.yaw, cam.pitch, cam.focal, cam.aperture, cam.fovX = 0.0, -0.55, 5.0, 0.001, np.float32(90.0) * np.float32(0.01745329251)
    rt.camera = cam
    rt.draw(rgba)
    oc = oracle.default_camera(w, h)
    oc.pos[:] = (5.5, 4.0, -3.0)
    oc.pitch = -0.55
    gb = oracle.pathtrace(b, w, h, frame_num=1, spp=1, cam=oc, hist_cam=oc, sky_out=oracle.sky(), tex=oracle.textures())
    assert np.array_equal(rgba.reshape(-1, 4), oracle.Denoiser(w, h).draw(gb, 1, delta_time=16.667)["rgba"])
    rt.cleanup()


@pytest.mark.parametrize("ntri,threads", [(2 * 1024 + 6, 0), (2 * 1024 + 6, 512), (65 * 1024 + 3, 0), (65 * 1024 + 3, 1024)])
def test_partial_last_batch_tlas(rtx, oracle, tmp_path, ntri, threads):
    """A last batch of 6 (3) real and 2 (1) padding triangles, in a 3-batch scene (one-wave TLAS) and
    a 66-batch one (workgroup TLAS): the batch's leaves are its first real-count elements in SORTED
    order, padding ones among them, so its TLAS leaf box (published to the TLAS workgroup after the
    batch's sort) and every node, Morton code and TLAS record stay bit-exact vs the oracle."""
    tris = terrain_patch(190, 180)[:ntri]
    path = write_bin(str(tmp_path / ("n%d.bin" % ntri)), tris)
    rt = make(rtx, tmp_path, path, threads=threads)
    b, _, _, n = bin_bvh(oracle, path)
    B = b["batch_count"]
    assert rt.info().triCount == n == ntri and rt.info().batchCount == B == (ntri + 1023) // 1024
    for _ in range(2):  # a rebuild reuses the launch counter
        rt.build_bvh()
    rt.sync()
    nodes = rt.download("NODES").view(rtx.NODE_DTYPE)
    for k in range(B):
        cnt = 1024 if k < B - 1 else n - (B - 1) * 1024
        assert nodes[k * 1024:k * 1024 + cnt - 1].tobytes() == b["nodes"][k * 1024:k * 1024 + cnt - 1].tobytes(), k
    assert np.array_equal(rt.download("MORTON", np.uint32)[:B * 1024], b["morton"])
    assert np.array_equal(rt.download("TLAS_AABBS", np.float32).reshape(-1, 6), b["tlas_aabbs"])
    assert np.array_equal(rt.download("TLAS_SCENE_AABB", np.float32), b["tlas_scene_aabb"])
    assert rt.download("TLAS_NODES").view(rtx.NODE_DTYPE).tobytes() == b["tlas_nodes"].tobytes()
    rt.cleanup()
