"""The C-ABI multi-GPU split (include/rtx_dist.h: rtd_attach + the renderer's three hook stages) driving
the reference-style entry points: each rank just calls rt_draw_device / rt_draw, and the renderer asks
the hook for the G-buffer rows, the histogram and the denoise rows.  Two and three ranks share one GPU
(gloo through the host stands in for RCCL, which cannot run two ranks on one GPU); every rank's RGBA8
target and HDR output must equal a single-rank render bit for bit, for synchronous draws, pipelined
(RT_DRAW_ASYNC) draws and host-buffer rt_draw with an HDR copy — the advisor's round-2 finding that a
strip-local rank's draw target and HDR copy held one strip plus stale rows."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 256, 200, 3


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render(rank, world, port, out_dir, mode):
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.cdist import GlooHipComm, Strips
    from rtx.dist import strip_config

    torch.cuda.set_device(0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = rtx.write_config(os.path.join(out_dir, "%s%d_%d.toml" % (mode, rank, world)), W, H, spp=2,
                           extra=strip_config(world, rank))
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    strips = None
    if world > 1:
        strips = Strips(W, H, world, rank, GlooHipComm())
        strips.attach(rt)
    target = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    rgba = np.zeros((H, W, 4), np.uint8)
    hdr = np.zeros((H, W, 4), np.float32)
    cam0 = rt.camera
    for f in range(1, FRAMES + 1):
        c = rt.camera
        c.yaw = cam0.yaw + 0.02 * f
        rt.camera = c
        if mode == "draw":
            rt.draw(rgba, hdr)
        else:
            rt.draw_device(target.data_ptr(), 0, asynchronous=(mode == "async"))
    rt.sync()
    torch.cuda.synchronize()
    out = dict(rgba=(rgba.copy() if mode == "draw" else target.cpu().numpy()),
               dl=rt.download("RGBA8", np.uint8).copy(), hist=rt.get_buffer("HISTORY_COLOR").copy(),
               expo=rt.download("EXPOSURE", np.uint8).copy())
    if mode == "draw":
        out["hdr"] = hdr.copy()
    rt.cleanup()
    if strips is not None:
        strips.destroy()
    np.savez(os.path.join(out_dir, "%s_r%d_of%d.npz" % (mode, rank, world)), **out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    print("%s rank %d/%d done" % (mode, rank, world), flush=True)


@pytest.mark.parametrize("mode,world", [("sync", 2), ("async", 2), ("draw", 2), ("async", 3)])
def test_draw_entry_points_multirank(tmp_path, mode, world):
    import torch.multiprocessing as mp

    mp.start_processes(render, args=(1, 0, str(tmp_path), mode), nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(world, free_port(), str(tmp_path), mode), nprocs=world, start_method="spawn")
    ref = np.load(tmp_path / ("%s_r0_of1.npz" % mode))
    assert ref["rgba"].any()
    for r in range(world):
        got = np.load(tmp_path / ("%s_r%d_of%d.npz" % (mode, r, world)))
        for k in ref.files:
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)
