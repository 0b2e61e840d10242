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
