"""Screen-strip split + all-gather (rtx/dist.py) on CPU with the gloo backend, world size 2 and 3.

Each rank path traces its strip with the oracle (standing in for the GPU kernel, which is
pinned bit-exact to the oracle by the gpu tests), writes it into its chunk of the flat
G-buffer tensors, and all-gathers; every rank must then hold the full single-process frame.
"""
import os
import socket

import numpy as np
import pytest

from rtx.dist import GBUFFERS, ROW_BLOCK, StripGather, strip_blocks, strip_rows

W, H = 48, 72
ORACLE_KEYS = dict(RENDER_COLOR="color", NORMAL="normal", ALBEDO="albedo", DEPTH="depth", MOTION="motion")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def camera(O):
    c = O.default_camera(W, H)
    c.pos[:] = (8.0, 15.0, -6.0)
    c.pitch = -0.7
    return c


def worker(rank, world, port, result_dir):
    import torch
    import torch.distributed as dist

    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v, i, n = O.scene(1)
        bvh = O.build_bvh(v, i, n, O.smooth_normals(v, i))
        sg = StripGather(W, H, world, rank, torch.device("cpu"))
        for y0, rows in strip_blocks(H, world, rank):  # this rank's interleaved row blocks
            g = O.pathtrace(bvh, W, H, frame_num=2, cam=camera(O), y0=y0, rows=rows, threads=1)
            for name, bpp in GBUFFERS:
                a = np.ascontiguousarray(g[ORACLE_KEYS[name]]).view(np.uint8).reshape(-1)
                lo, hi = y0 * W * bpp, (y0 + rows) * W * bpp
                sg.tensors[name][lo:hi] = torch.from_numpy(a[lo:hi].copy())
        sg.gather()
        out = {name: sg.tensors[name][:W * H * bpp].numpy().copy() for name, bpp in GBUFFERS}
        np.savez(os.path.join(result_dir, "rank%d.npz" % rank), **out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strip_allgather_matches_full_frame(tmp_path, world, oracle):
    import torch.multiprocessing as mp

    mp.spawn(worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    v, i, n = oracle.scene(1)
    bvh = oracle.build_bvh(v, i, n, oracle.smooth_normals(v, i))
    full = oracle.pathtrace(bvh, W, H, frame_num=2, cam=camera(oracle), threads=1)
    for r in range(world):
        got = np.load(os.path.join(str(tmp_path), "rank%d.npz" % r))
        for name, _ in GBUFFERS:
            ref = np.ascontiguousarray(full[ORACLE_KEYS[name]]).view(np.uint8).reshape(-1)
            assert np.array_equal(got[name], ref), (r, name)


@pytest.mark.parametrize("h,world", [(1080, 1), (1080, 2), (1080, 8), (1081, 8), (2160, 8), (30, 2), (144, 3)])
def test_strip_blocks_cover_frame(h, world):
    """Interleaved row blocks: every row owned by exactly one rank, block b by rank b mod N."""
    covered = np.zeros(h, np.int32)
    for r in range(world):
        for y0, rows in strip_blocks(h, world, r):
            assert (y0 // ROW_BLOCK) % world == r and 1 <= rows <= ROW_BLOCK
            covered[y0:y0 + rows] += 1
    assert (covered == 1).all()


@pytest.mark.parametrize("h,world", [(1080, 1), (1080, 2), (1080, 8), (1081, 8), (2160, 8), (30, 3)])
def test_strip_rows_cover_frame(h, world):
    covered = np.zeros(h, np.int32)
    for r in range(world):
        y0, rows, per = strip_rows(h, world, r)
        assert rows >= 1 and rows <= per and y0 == r * per
        covered[y0:y0 + rows] += 1
    assert (covered == 1).all()


def test_strip_rows_rejects_too_many_ranks():
    with pytest.raises(ValueError):
        strip_rows(10, 8, 7)


def worker_sets(rank, world, port, result_dir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sg = StripGather(W, H, world, rank, torch.device("cpu"), sets=3)
        for k in range(3):  # rank r writes value 10 * k + r into its row blocks of set k
            for name, bpp in GBUFFERS:
                sg.mine(name, k).fill_(10 * k + rank)
        sg.gather(gbuffer_set=1)  # only set 1 is assembled
        out = {"%s_%d" % (name, k): sg.sets[k][name].numpy().copy() for name, _ in GBUFFERS for k in range(3)}
        np.savez(os.path.join(result_dir, "rank%d.npz" % rank), **out)
    finally:
        dist.destroy_process_group()


def test_strip_allgather_pipelined_sets(tmp_path):
    """StripGather over three bound G-buffer sets (any count works): gather(set k) assembles set k only."""
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(worker_sets, args=(world, free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    for r in range(world):
        d = np.load(tmp_path / ("rank%d.npz" % r))
        for name, bpp in GBUFFERS:
            blk = ROW_BLOCK * W * bpp
            for k in range(3):
                a = d["%s_%d" % (name, k)].reshape(-1, world, blk)  # [round, owner rank, block]
                for q in range(world):
                    # gathered set: every rank's blocks; the others: this rank's own blocks only
                    want = 10 * k + q if (k == 1 or q == r) else 0
                    assert (a[:, q] == want).all(), (r, name, k, q)


def denoise_worker(rank, world, port, result_dir):
    import torch
    import torch.distributed as dist

    from rtx.dist import StripDenoise

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        Wd, Hd = 40, (200 if world < 4 else 600)  # 4 / 10 blocks of 64 rows (the last one short)
        sd = StripDenoise(Wd, Hd, world, rank, torch.device("cpu"))
        rng = np.random.default_rng(11)
        full = dict(accum=rng.integers(0, 256, Wd * Hd * 8, dtype=np.uint8),
                    h1=rng.integers(0, 256, Wd * Hd * 8, dtype=np.uint8),
                    rgba=rng.integers(0, 256, Wd * Hd * 4, dtype=np.uint8))
        a, b = sd.a, sd.b
        # this rank computed its own rows (and stale halo rows elsewhere): only [a, b) are right
        for t, key, bpp in ((sd.accum, "accum", 8), (sd.history[1], "h1", 8), (sd.rgba, "rgba", 4)):
            t.fill_(0xEE)
            t[a * Wd * bpp:b * Wd * bpp] = torch.from_numpy(full[key][a * Wd * bpp:b * Wd * bpp].copy())
        sd.history[0].fill_(0x55)  # the other history buffer is not exchanged this frame
        sd.histogram.copy_(torch.arange(64, dtype=torch.int32) * (rank + 1))
        sd.exchange_histogram()
        sd.exchange_rows(1)
        np.savez(os.path.join(result_dir, "d%d.npz" % rank), accum=sd.accum.numpy(), h1=sd.history[1].numpy(),
                 rgba=sd.rgba.numpy(), h0=sd.history[0].numpy(), hist=sd.histogram.numpy(),
                 **{"full_" + k: v for k, v in full.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_strip_denoise_exchange(tmp_path, world):
    """StripDenoise (the strip-local denoise's collectives) with gloo on CPU: after the histogram
    all-reduce and the rows all-gather every rank holds the whole frame's accumulation, history
    (only the buffer TemporalFilter2 wrote) and RGBA8, and the summed histogram."""
    import torch.multiprocessing as mp

    from rtx.dist import denoise_rows

    assert [denoise_rows(1080, 8, r) for r in (0, 7)] == [(0, 128), (896, 1080)]
    assert sum(b - a for a, b in (denoise_rows(2160, 8, r) for r in range(8))) == 2160
    with pytest.raises(ValueError):
        denoise_rows(100, 3, 0)  # 2 blocks of 64 rows for 3 ranks
    mp.start_processes(denoise_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    for r in range(world):
        d = np.load(tmp_path / ("d%d.npz" % r))
        for k in ("accum", "h1", "rgba"):
            assert np.array_equal(d[k], d["full_" + k]), (r, k)
        assert (d["h0"] == 0x55).all()
        assert np.array_equal(d["hist"], np.arange(64) * sum(range(1, world + 1)))


def exchange_worker(rank, world, port, result_dir, He=1080):
    import torch
    import torch.distributed as dist

    from rtx.dist import gbuffer_rows

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        We = 8
        sg = StripGather(We, He, world, rank, torch.device("cpu"), sets=2)
        need = [gbuffer_rows(He, world, r) for r in range(world)]
        full = {}
        for name, bpp in GBUFFERS:
            rows = len(sg.sets[1][name]) // (We * bpp)
            v = (np.arange(rows * We * bpp, dtype=np.int64) * 7 + len(name)) % 251
            full[name] = v.astype(np.uint8)
            t = sg.sets[1][name]
            t.fill_(0xEE)
            for y0, n in strip_blocks(He, world, rank):  # this rank path traced its own blocks
                lo, hi = y0 * We * bpp, (y0 + n) * We * bpp
                t[lo:hi] = torch.from_numpy(full[name][lo:hi].copy())
            sg.sets[0][name].fill_(0x11)
        sg.exchange(need, gbuffer_set=1)
        np.savez(os.path.join(result_dir, "x%d.npz" % rank), recv=np.array(sg.exchange_bytes_per_frame(need)),
                 **{name: sg.sets[1][name].numpy() for name, _ in GBUFFERS},
                 **{"set0_" + name: sg.sets[0][name].numpy() for name, _ in GBUFFERS},
                 **{"full_" + name: full[name] for name, _ in GBUFFERS})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("He,world", [(1080, 2), (1080, 3), (1080, 4), (1080, 8), (2160, 8)])
def test_strip_exchange_delivers_the_rows_each_rank_reads(tmp_path, He, world):
    """StripGather.exchange (gloo, CPU): after the all-to-all every rank holds the whole frame's
    G-buffers in the rows gbuffer_rows says its strip-local denoise reads, its own blocks
    everywhere, and nothing else was written; the other G-buffer set is untouched; each rank
    receives well under the all-gather's (N - 1) / N of the frame.  (2160, 8) is config 5's split:
    34 denoise blocks over 8 ranks."""
    import torch.multiprocessing as mp

    from rtx.dist import gbuffer_rows

    assert gbuffer_rows(1080, 8, 0) == (0, 208) and gbuffer_rows(1080, 8, 7) == (816, 1080)
    mp.start_processes(exchange_worker, args=(world, free_port(), str(tmp_path), He), nprocs=world,
                       start_method="spawn")
    We = 8
    for r in range(world):
        d = np.load(tmp_path / ("x%d.npz" % r))
        lo, hi = gbuffer_rows(He, world, r)
        mine = np.zeros(He, bool)
        for y0, n in strip_blocks(He, world, r):
            mine[y0:y0 + n] = True
        frame_bytes = 0
        for name, bpp in GBUFFERS:
            got = d[name][:He * We * bpp].reshape(He, We * bpp)
            want = d["full_" + name][:He * We * bpp].reshape(He, We * bpp)
            frame_bytes += He * We * bpp
            rows = np.arange(He)
            exact = ((rows >= lo) & (rows < hi)) | mine
            assert np.array_equal(got[exact], want[exact]), (r, name)
            # outside its rows a rank may receive whole 16-row blocks that straddle lo / hi only
            far = (rows < (lo // ROW_BLOCK) * ROW_BLOCK) | (rows >= -(-hi // ROW_BLOCK) * ROW_BLOCK)
            assert (got[far & ~mine] == 0xEE).all(), (r, name)
            assert (d["set0_" + name] == 0x11).all()
        assert int(d["recv"]) < 0.75 * frame_bytes * (world - 1) / world, (r, int(d["recv"]))
