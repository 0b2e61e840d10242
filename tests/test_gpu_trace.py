"""GPU primary-ray traversal (BASELINE config 2) vs the CPU oracle, bit-exact per ray:
t, object index, barycentrics, normals, ray offset and the traversal counters (node
visits, triangle tests, dropped stack pushes, iterations)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(rtx, oracle, tmp_path, w, h, frame, chunk_dim=1):
    cfg = rtx.write_config(str(tmp_path / "c.toml"), w, h, chunk_dim=chunk_dim)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.build_bvh()
    rt.trace_primary(frame, detail=True)
    rt.sync()
    g = dict(hits=rt.download("HITS", np.float32).reshape(-1, 4),
             nrm=rt.download("HIT_NORMALS", np.float32).reshape(-1, 4),
             fake=rt.download("HIT_FAKE_NORMALS", np.float32).reshape(-1, 4),
             stats=rt.download("HIT_STATS", np.uint32).reshape(-1, 4))
    rt.cleanup()
    v, i, n = oracle.scene(chunk_dim)
    ob = oracle.build_bvh(v, i, n, oracle.smooth_normals(v, i))
    rays, _ = oracle.primary_rays(w, h, frame)
    o = oracle.intersect(ob, rays)
    return g, o


def assert_same(g, o):
    bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    assert np.array_equal(bits(g["hits"][:, 0]), bits(o["t"]))
    assert np.array_equal(g["hits"][:, 1].view(np.int32), o["objectIdx"])
    assert np.array_equal(bits(g["hits"][:, 2]), bits(o["u"]))
    assert np.array_equal(bits(g["hits"][:, 3]), bits(o["v"]))
    assert np.array_equal(bits(g["nrm"][:, :3]), bits(o["normal"]))
    assert np.array_equal(g["nrm"][:, 3].astype(np.uint32), o["hit"])
    assert np.array_equal(bits(g["fake"][:, :3]), bits(o["fakeNormal"]))
    assert np.array_equal(bits(g["fake"][:, 3]), bits(o["offset"]))
    assert np.array_equal(g["stats"][:, 0], o["nodeVisits"])
    assert np.array_equal(g["stats"][:, 1], o["triTests"])
    assert np.array_equal(g["stats"][:, 2], o["droppedPushes"])
    assert np.array_equal(g["stats"][:, 3], o["iterations"])


@pytest.mark.parametrize("w,h,frame", [(256, 256, 1), (97, 61, 3)])
def test_primary_bit_exact_small(rtx, oracle, tmp_path, w, h, frame):
    g, o = run(rtx, oracle, tmp_path, w, h, frame)
    assert_same(g, o)


def test_primary_bit_exact_1080p(rtx, oracle, tmp_path):
    g, o = run(rtx, oracle, tmp_path, 1920, 1080, 1)
    assert_same(g, o)
    assert o["hit"].mean() > 0.05


def test_primary_bit_exact_1m_scene(rtx, oracle, tmp_path):
    g, o = run(rtx, oracle, tmp_path, 320, 180, 2, chunk_dim=4)
    assert_same(g, o)


def test_trace_rays_queue_and_random_bit_exact(rtx, oracle, tmp_path):
    """rt_trace_rays (the persistent queue tracer) on the real incoherent bounce rays of a
    1080p 4-spp frame plus random rays (axis-parallel directions, origins outside the scene),
    vs oracle.intersect: t, triangle, barycentrics and TraverseBvh iterations."""
    w, h = 1920, 1080
    cfg = rtx.write_config(str(tmp_path / "c.toml"), w, h, spp=4)
    rt = rtx.RayTracer(w, h, cfg).init()
    rt.set_delta_time(16.667)
    rt.build_bvh()
    rt.path_trace(1)
    rt.sync()
    n3 = int(rt.download("PT_QUEUE", np.uint32)[0])
    o3 = rt.download("PT_Q3_ORIGINS", np.float32).reshape(-1, 4)[:n3, :3]
    d3 = rt.download("PT_Q3_DIRS", np.float32).reshape(-1, 4)[:n3, :3]
    rng = np.random.default_rng(7)
    m = 20000
    ro = rng.uniform(-40.0, 100.0, (m, 3)).astype(np.float32)
    rd = rng.normal(size=(m, 3)).astype(np.float32)
    rd[: m // 4, rng.integers(0, 3)] = 0.0     # axis-parallel components (safe_divide path)
    rd /= np.linalg.norm(rd, axis=1, keepdims=True).astype(np.float32)
    org = np.concatenate([o3, ro])
    dirs = np.concatenate([d3, rd])
    t, tri, u, v, iters, ms = rt.trace_rays(org, dirs, want_iters=True)
    rt.cleanup()
    assert n3 > 100000 and ms > 0.0
    vtx, idx, nt = oracle.scene(1)
    ob = oracle.build_bvh(vtx, idx, nt, oracle.smooth_normals(vtx, idx))
    o = oracle.intersect(ob, np.concatenate([org, dirs], axis=1))
    bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    assert np.array_equal(bits(t), bits(o["t"]))
    assert np.array_equal(tri, o["objectIdx"])
    assert np.array_equal(bits(u), bits(o["u"]))
    assert np.array_equal(bits(v), bits(o["v"]))
    assert np.array_equal(iters, o["iterations"])
    assert (tri >= 0).mean() > 0.05
