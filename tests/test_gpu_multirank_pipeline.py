"""The bench's own frame loop (rtx.frames.FramePipeline: pipelined streams, interleaved 16-row
trace blocks, the strip exchange of the G-buffer rows, the strip-local denoise with its histogram
all-reduce and accumulation / history / RGBA8 row all-gathers) run by N ranks sharing one GPU over
gloo.  Every rank must end each run holding the single-rank frame bit for bit: RGBA8, the final
HDR (history buffer), the accumulation buffer, the exposure state, and the float4 HDR copy
(FramePipeline.frame(hdr=True), which a strip-local rank can only produce after the rows exchange).

BASELINE config 5 is 3840x2160, 4 spp, split over 8 GPUs: test_eight_ranks_4k runs exactly that
layout (34 denoise blocks of 64 rows over 8 ranks, 5-tile G-buffer halos, 8-way interleaved
trace blocks) on one GPU."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render(rank, world, port, out_dir, size, frames, tag, hdr):
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.dist import strip_config
    from rtx.frames import FramePipeline

    W, H = size
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = rtx.write_config(os.path.join(out_dir, "%sc%d_%d.toml" % (tag, rank, world)), W, H, spp=4,
                           extra=strip_config(world, rank))
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    fp = FramePipeline(rt, dev, pipelined=True, world=world, rank=rank, backend="gloo")
    if world > 1:
        i = rt.info()
        assert (i.denoiseRowBegin, i.denoiseRowEnd) == (fp.denoise.a, fp.denoise.b)
    cam0 = rt.camera
    for f in range(1, frames + 1):
        c = rt.camera
        c.yaw = cam0.yaw + 0.02 * f  # a moving camera: the temporal passes reproject
        rt.camera = c
        fp.frame(f, hdr=hdr)
        print("%s rank %d/%d frame %d enqueued" % (tag, rank, world, f), flush=True)
    fp.finish()
    out = dict(rgba=rt.download("RGBA8", np.uint8).copy(), hist=rt.get_buffer("HISTORY_COLOR").copy(),
               acc=rt.get_buffer("ACCUMULATION").copy(), expo=rt.download("EXPOSURE", np.uint8).copy())
    if hdr:
        out["hdr"] = rt.download("HDR", np.uint8).copy()
    rt.cleanup()
    np.savez(os.path.join(out_dir, "%sr%d_of%d.npz" % (tag, rank, world)), **out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    print("%s rank %d/%d done" % (tag, rank, world), flush=True)


def run(tmp_path, world, size, frames, tag, hdr):
    import torch.multiprocessing as mp

    mp.start_processes(render, args=(1, 0, str(tmp_path), size, frames, tag, hdr), nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(world, free_port(), str(tmp_path), size, frames, tag, hdr), nprocs=world,
                       start_method="spawn")
    ref = np.load(tmp_path / ("%sr0_of1.npz" % tag))
    keys = ("rgba", "hist", "acc", "expo") + (("hdr",) if hdr else ())
    for r in range(world):
        got = np.load(tmp_path / ("%sr%d_of%d.npz" % (tag, r, world)))
        for k in keys:
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)
    sys.stdout.flush()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_hdr_output_after_strip_denoise(tmp_path, world):
    """FramePipeline.frame(hdr=True) on strip-local ranks: the float4 HDR copy is taken after the rows
    exchange, so it holds the whole frame (the advisor's round-2 finding: it used to be copied
    before the exchange, stale outside the strip)."""
    run(tmp_path, world, (256, 200), 3, "h", True)


def test_eight_ranks_4k(tmp_path):
    """BASELINE config 5's split: 3840x2160, 4 spp, 8 ranks (gloo, one GPU), three pipelined frames
    of a moving camera, against one rank."""
    run(tmp_path, 8, (3840, 2160), 3, "k8", False)
