"""include/rtx_dist.h (the C-ABI multi-GPU split in librtx.so) on CPU: every rank a thread of this
process over host memory (rtx.cdist.ThreadComm, an in-process fake communicator), no GPU.

* The C++ layout and exchange plan equal rtx/dist.py's (denoise strips, G-buffer rows, the rounds
  each rank sends to and receives from every peer, bytes per frame).
* rtd_exchange_gbuffers delivers the rows each rank's strip-local denoise reads (or the whole frame)
  and writes nothing else; rtd_exchange_rows / rtd_exchange_histogram leave every rank with the whole
  frame's accumulation / history / RGBA8 and the summed histogram — the same postconditions
  tests/test_dist_strips.py checks for the Python exchanges over gloo."""
import ctypes as C
import threading

import numpy as np
import pytest
import torch

from rtx.cdist import GB_NAMES, Strips, ThreadComm
from rtx.dist import GBUFFERS, ROW_BLOCK, StripDenoise, StripGather, denoise_rows, gbuffer_rows, strip_blocks

BPP = dict(GBUFFERS)


def run_ranks(world, fn):
    errs = []

    def body(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs


@pytest.mark.parametrize("W,H,world", [(8, 1080, 2), (8, 1080, 3), (8, 1080, 8), (8, 2160, 8), (24, 200, 2)])
def test_layout_and_plan_match_python(W, H, world):
    hub = ThreadComm(world)
    for r in range(world):
        s = Strips(W, H, world, r, hub.rank(r))
        try:
            for q in range(world):
                assert s.denoise_rows(q) == denoise_rows(H, world, q)
                assert s.gbuffer_rows(q) == gbuffer_rows(H, world, q)
            sg = StripGather(W, H, world, r, torch.device("cpu"))
            for name, bpp in GBUFFERS:
                assert s.gbuffer_bytes(name) == sg.sets[0][name].numel()
            need = [gbuffer_rows(H, world, q) for q in range(world)]
            assert s.recv_bytes(2, True) == sg.exchange_bytes_per_frame(need)
            # the whole frame: every peer's blocks inside the frame (the all-gather also moves padding)
            blk_all = sum(ROW_BLOCK * W * bpp for _, bpp in GBUFFERS)
            whole = sum(len(strip_blocks(H, world, q)) for q in range(world) if q != r) * blk_all
            assert s.recv_bytes(2, False) == whole <= sg.bytes_per_frame()
            sd_rows = max(b - a for a, b in (denoise_rows(H, world, q) for q in range(world)))
            assert s.recv_bytes(1) == (world - 1) * sd_rows * W * 20
            assert s.recv_bytes(0) == 256
        finally:
            s.destroy()


@pytest.mark.parametrize("W,H,world,strip_local", [(8, 1080, 2, True), (8, 1080, 3, True), (8, 2160, 8, True),
                                                    (8, 520, 3, False)])
def test_gbuffer_exchange(W, H, world, strip_local):
    hub = ThreadComm(world)
    out = {}

    def rank(r):
        s = Strips(W, H, world, r, hub.rank(r))
        bufs, full = {}, {}
        for name in GB_NAMES:
            n = s.gbuffer_bytes(name)
            full[name] = ((np.arange(n, dtype=np.int64) * 7 + len(name)) % 251).astype(np.uint8)
            b = np.full(n, 0xEE, np.uint8)
            for y0, rows in strip_blocks(H, world, r):  # this rank traced its own blocks
                lo, hi = y0 * W * BPP[name], (y0 + rows) * W * BPP[name]
                b[lo:hi] = full[name][lo:hi]
            bufs[name] = b
        s.exchange_gbuffers({k: v.ctypes.data for k, v in bufs.items()}, strip_local)
        out[r] = (bufs, full)
        s.destroy()

    run_ranks(world, rank)
    for r in range(world):
        bufs, full = out[r]
        lo, hi = gbuffer_rows(H, world, r) if strip_local else (0, H)
        mine = np.zeros(H, bool)
        for y0, n in strip_blocks(H, world, r):
            mine[y0:y0 + n] = True
        rows = np.arange(H)
        exact = ((rows >= lo) & (rows < hi)) | mine
        far = (rows < (lo // ROW_BLOCK) * ROW_BLOCK) | (rows >= -(-hi // ROW_BLOCK) * ROW_BLOCK)
        for name in GB_NAMES:
            got = bufs[name][:H * W * BPP[name]].reshape(H, -1)
            want = full[name][:H * W * BPP[name]].reshape(H, -1)
            assert np.array_equal(got[exact], want[exact]), (r, name)
            assert (got[far & ~mine] == 0xEE).all(), (r, name)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_denoise_exchanges(world):
    """rtd_exchange_rows / rtd_exchange_histogram vs rtx.dist.StripDenoise's contract."""
    W, H = 40, 200 if world < 4 else 600
    hub = ThreadComm(world)
    rng = np.random.default_rng(11)
    full = dict(accum=rng.integers(0, 256, W * H * 8, dtype=np.uint8),
                hist=rng.integers(0, 256, W * H * 8, dtype=np.uint8),
                rgba=rng.integers(0, 256, W * H * 4, dtype=np.uint8))
    out = {}

    def rank(r):
        s = Strips(W, H, world, r, hub.rank(r))
        a, b = s.denoise_rows(r)
        bufs = {}
        for key, bpp in (("accum", 8), ("hist", 8), ("rgba", 4)):
            t = np.full(W * H * bpp, 0xEE, np.uint8)
            t[a * W * bpp:b * W * bpp] = full[key][a * W * bpp:b * W * bpp]
            bufs[key] = t
        h = (np.arange(64, dtype=np.int32) * (r + 1)).astype(np.int32)
        s.exchange_histogram(h.ctypes.data)
        s.exchange_rows(bufs["accum"].ctypes.data, bufs["hist"].ctypes.data, bufs["rgba"].ctypes.data)
        out[r] = (bufs, h)
        s.destroy()

    run_ranks(world, rank)
    sd = StripDenoise(W, H, world, 0, torch.device("cpu"), group=object())  # layout only, no collectives
    for r in range(world):
        bufs, h = out[r]
        for key in ("accum", "hist", "rgba"):
            assert np.array_equal(bufs[key], full[key]), (r, key)
        assert np.array_equal(h, np.arange(64) * sum(range(1, world + 1)))
    assert sd.bytes_per_frame() == (world - 1) * sd.max_rows * W * 20
