"""GPU LBVH build (one fused launch) vs the CPU oracle: bit-exact Morton codes, reorder
indices, node topology and boxes, TLAS — default scene and the ~1M-triangle variant, in both
workgroup shapes of the build kernel ([render] bvhThreads: 1024 threads with leaf boxes in LDS,
512 threads with two elements each and leaf boxes read back from the AABB array; 0 picks by the
batch count: 1024 for the default scene's 60 batches, 512 for the 1M scene's 937)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def build_gpu(rtx, tmp_path, chunk_dim, w=64, h=64, threads=0):
    cfg = rtx.write_config(str(tmp_path / ("c%d_%d.toml" % (chunk_dim, threads))), w, h, chunk_dim=chunk_dim,
                           extra="bvhThreads = %d\n" % threads)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.build_bvh()
    rt.sync()
    return rt


def as_nodes(rtx, raw):
    return raw.view(rtx.NODE_DTYPE)


@pytest.mark.parametrize("chunk_dim,threads", [(1, 0), (4, 0), (1, 512), (4, 1024), (2, 512)])
def test_bvh_bit_exact(rtx, oracle, tmp_path, chunk_dim, threads):
    v, i, n = oracle.scene(chunk_dim)
    rt = build_gpu(rtx, tmp_path, chunk_dim, threads=threads)
    info = rt.info()
    assert info.triCount == n and info.triCountPadded == i.shape[0]
    gv = rt.download("VERTICES", np.float32).reshape(-1, 3)
    gi = rt.download("INDICES", np.uint32).reshape(-1, 3)
    assert np.array_equal(gv, v) and np.array_equal(gi, i)
    gn = rt.download("NORMALS", np.float32).reshape(-1, 3)
    on = oracle.smooth_normals(v, i)
    assert np.array_equal(gn.view(np.uint32), on.view(np.uint32)), "smooth normals differ"
    ob = oracle.build_bvh(v, i, n, on)
    B = ob["batch_count"]
    assert info.batchCount == B
    assert np.array_equal(rt.download("MORTON", np.uint32), ob["morton"])
    assert np.array_equal(rt.download("REORDER", np.uint32), ob["reorder"])
    aabbs = rt.download("AABBS", np.float32).reshape(-1, 6)
    assert np.array_equal(aabbs.view(np.uint32), ob["aabbs"].view(np.uint32))
    bs = rt.download("BATCH_SCENE_AABBS", np.float32).reshape(-1, 6)
    assert np.array_equal(bs, ob["batch_scene_aabbs"])
    gnodes = as_nodes(rtx, rt.download("NODES"))
    for k in range(B):
        cnt = 1024 if k < B - 1 else n - (B - 1) * 1024
        g = gnodes[k * 1024:k * 1024 + cnt - 1]
        o = ob["nodes"][k * 1024:k * 1024 + cnt - 1]
        assert g.tobytes() == o.tobytes(), "batch %d nodes differ" % k
    assert np.array_equal(rt.download("TLAS_AABBS", np.float32).reshape(-1, 6), ob["tlas_aabbs"])
    assert np.array_equal(rt.download("TLAS_SCENE_AABB", np.float32), ob["tlas_scene_aabb"])
    assert np.array_equal(rt.download("TLAS_MORTON", np.uint32), ob["tlas_morton"])
    assert np.array_equal(rt.download("TLAS_REORDER", np.uint32), ob["tlas_reorder"])
    assert as_nodes(rtx, rt.download("TLAS_NODES")).tobytes() == ob["tlas_nodes"].tobytes()
    tp = rt.download("TRI_POS", np.float32).reshape(-1, 3, 4)[:, :, :3].reshape(-1, 9)
    assert np.array_equal(tp, ob["triangles"][:, :9])
    rt.cleanup()


@pytest.mark.parametrize("threads", [1024, 512])
def test_bvh_rebuild_is_idempotent(rtx, tmp_path, threads):
    rt = build_gpu(rtx, tmp_path, 1, threads=threads)
    first = rt.download("NODES").copy()
    tlas = rt.download("TLAS_NODES").copy()
    for _ in range(5):
        rt.build_bvh()
    rt.sync()
    assert np.array_equal(rt.download("NODES"), first)
    assert np.array_equal(rt.download("TLAS_NODES"), tlas)
    rt.cleanup()


@pytest.mark.parametrize("chunk_dim,threads", [(1, 1024), (2, 512)])
def test_tlas_wait_timeout_is_reported(rtx, tmp_path, chunk_dim, threads):
    """The TLAS workgroup's bounded wait (bvh_build.hip tlas_wait): batch 1 never publishes its leaf
    box ([debug] bvhSkipPublish fault injection), so the wait ends at its 20-ms bound.  The build
    still drains, the failure reaches the host as RT_ERR_DEVICE at the next sync with the number of
    missing batches, is reported once, and the launch counters are re-armed: the next faulty build
    again misses exactly one batch (without the re-arm its count would start one short)."""
    extra = "bvhThreads = %d\n\n[debug]\nbvhSkipPublish = 1\nbvhWaitMs = 20\n" % threads
    cfg = rtx.write_config(str(tmp_path / "fault.toml"), 64, 64, chunk_dim=chunk_dim, extra=extra)
    rt = rtx.RayTracer(64, 64, cfg).init()
    assert rt.info().batchCount > (64 if chunk_dim > 1 else 1)  # the workgroup-wide TLAS path for chunk_dim 2
    for _ in range(2):
        rt.build_bvh()
        with pytest.raises(rtx.RtError, match=r"RT_ERR_DEVICE .*for 1 batch publication"):
            rt.sync()
        rt.sync()  # reported once
    rt.build_bvh()
    time.sleep(0.5)  # the faulty build has ended (its wait is bounded at 20 ms)
    with pytest.raises(rtx.RtError, match="rt_build_bvh: RT_ERR_DEVICE"):  # a known report stops the next build
        rt.build_bvh()
    rt.sync()
    rt.cleanup()


@pytest.mark.parametrize("chunk_dim,threads", [(1, 1024), (2, 512)])
def test_build_queued_behind_timeout_reports(rtx, tmp_path, chunk_dim, threads):
    """A healthy build queued behind a faulty one on the same LBVH set, with no sync between them
    (ADVICE r5): the faulty build leaves the launch counter one below zero until the host re-arms
    it, so the second build's batches bring it only to B - 1.  tlas_wait compares signed: the
    second build waits, times out and reports too (the report names build 2), instead of taking
    the wrapped count as complete.  After the re-arm a build equals a fault-free context's."""
    base = "bvhThreads = %d\n" % threads
    extra = base + "\n[debug]\nbvhSkipPublish = 1\nbvhSkipPublishBuilds = 1\nbvhWaitMs = 20\n"
    cfg = rtx.write_config(str(tmp_path / "fault.toml"), 64, 64, chunk_dim=chunk_dim, extra=extra)
    rt = rtx.RayTracer(64, 64, cfg).init()
    rt.build_bvh()  # build 1: batch 1 never publishes
    rt.build_bvh()  # build 2: healthy, queued while build 1 still waits
    with pytest.raises(rtx.RtError, match=r"RT_ERR_DEVICE .*for 1 batch publication\(s\) \(last in build 2\)"):
        rt.sync()
    rt.build_bvh()  # build 3, after the re-arm
    rt.sync()
    tlas, nodes = rt.download("TLAS_NODES").copy(), rt.download("NODES").copy()
    rt.cleanup()
    ok = rtx.RayTracer(64, 64, rtx.write_config(str(tmp_path / "ok.toml"), 64, 64, chunk_dim=chunk_dim,
                                                 extra=base)).init()
    ok.build_bvh()
    ok.sync()
    assert np.array_equal(ok.download("TLAS_NODES"), tlas)
    assert np.array_equal(ok.download("NODES"), nodes)
    ok.cleanup()


def test_tlas_no_fault_no_report(rtx, tmp_path):
    """Healthy builds back to back with the bounded wait: no report, the TLAS equals the first one."""
    rt = build_gpu(rtx, tmp_path, 1, threads=1024)
    tlas = rt.download("TLAS_NODES").copy()
    for _ in range(20):
        rt.build_bvh()
    rt.sync()
    assert np.array_equal(rt.download("TLAS_NODES"), tlas)
    rt.cleanup()
