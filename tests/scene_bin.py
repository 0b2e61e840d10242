"""meshProcessor .bin scenes for the tests (tool/meshProcessor.cpp:204-209, read by
LoadTrianglesFromFile, init.cu:28-50): u32 triangle count + Triangle[count], 128 B each
(geometry.h:52-97: v1 w1 v2 w2 v3 w3 v4 w4, then n1 u1 .. n4 u4).

Written and read here with numpy alone, independently of the renderer's loader and of the
procedural scene generator both the product and the oracle link."""
import numpy as np

TRI_DTYPE = np.dtype([("v", "<f4", (4, 4)), ("n", "<f4", (4, 4))])
assert TRI_DTYPE.itemsize == 128


def write_bin(path, tris):
    """tris: [N][3][3] vertex positions; the face normal goes into n1..n3."""
    t = np.asarray(tris, np.float32).reshape(-1, 3, 3)
    rec = np.zeros(len(t), TRI_DTYPE)
    rec["v"][:, :3, :3] = t
    nrm = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
    rec["n"][:, :3, :3] = nrm[:, None, :]
    with open(path, "wb") as f:
        f.write(np.uint32(len(t)).tobytes())
        f.write(rec.tobytes())
    return path


def read_bin(path):
    """(vertices [3N,3], indices [NP,3] padded to a multiple of 4 with index 0 (init.cu:104-115),
    N): one unshared vertex per corner, as the renderer loads the file."""
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    rec = np.frombuffer(raw[4:4 + 128 * n], TRI_DTYPE)
    v = np.ascontiguousarray(rec["v"][:, :3, :3].reshape(-1, 3))
    idx = np.arange(3 * n, dtype=np.uint32).reshape(-1, 3)
    pad = (n + 3) // 4 * 4
    idx = np.concatenate([idx, np.zeros((pad - n, 3), np.uint32)])
    return v, idx, n


def bin_bvh(oracle, path):
    """Oracle BVH of a .bin scene (smooth normals of unshared corners = face normals)."""
    v, i, n = read_bin(path)
    nrm = oracle.smooth_normals(v, i)
    return oracle.build_bvh(v, i, n, nrm), v, i, n


def probe_triangles(z0, z1):
    """Two parallel unit right triangles in the planes z = z0 (object 0) and z = z1 (object 1)."""
    return [[(0, 0, z), (1, 0, z), (0, 1, z)] for z in (z0, z1)]


def terrain_patch(n_quads_x=22, n_quads_z=23, seed=7):
    """A small height-field mesh (<= 1024 triangles: one BLAS batch, the B == 1 TLAS case),
    2 * 22 * 23 = 1012 triangles (1012 % 4 == 0) by default; odd counts exercise the padding."""
    rng = np.random.default_rng(seed)
    h = rng.uniform(0.0, 1.5, size=(n_quads_z + 1, n_quads_x + 1)).astype(np.float32)
    tris = []
    for z in range(n_quads_z):
        for x in range(n_quads_x):
            a = (x, h[z, x], z)
            b = (x + 1, h[z, x + 1], z)
            c = (x + 1, h[z + 1, x + 1], z + 1)
            d = (x, h[z + 1, x], z + 1)
            tris.append([a, c, b])
            tris.append([a, d, c])
    return np.asarray(tris, np.float32) * np.float32(0.5)
