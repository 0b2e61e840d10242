"""The multi-GPU frame path (rtx/dist.py: interleaved row blocks + G-buffer all-gather, frame
pipelining with three bound G-buffer sets) run by two ranks sharing one GPU over gloo, which
moves the same device tensors RCCL would.  Every rank's final RGBA8 image and HDR colour must
equal a single-rank render of the same frames, bit for bit."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 256, 144, 4


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render(rank, world, port, out_dir, pipelined, gather_stream, strip_denoise=False, size=(W, H), frames=FRAMES,
           tag="", exchange=False):
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.dist import StripDenoise, StripGather, gbuffer_rows, strip_config

    W, H = size

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = rtx.write_config(os.path.join(out_dir, "c%d.toml" % rank), W, H, spp=2, extra=strip_config(world, rank))
    rt = rtx.RayTracer(W, H, cfg).init()
    rt.set_delta_time(16.667)
    rt.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    if pipelined:
        post = torch.cuda.Stream(dev)
        rt.set_post_stream(post.cuda_stream)
    sets = rtx.GBUFFER_SETS if pipelined else 1
    sg = StripGather(W, H, world, rank, dev, rt, sets=sets) if world > 1 else None
    gs = torch.cuda.Stream(dev) if (gather_stream and sg is not None) else None
    if gs is not None:
        rt.set_gather_stream(gs.cuda_stream)
    sd = StripDenoise(W, H, world, rank, dev, rt) if (strip_denoise and world > 1) else None
    need = None
    if sd is not None:
        i = rt.info()
        assert (i.denoiseRowBegin, i.denoiseRowEnd) == (sd.a, sd.b)
        assert (i.gbufferRowBegin, i.gbufferRowEnd) == gbuffer_rows(H, world, rank)
        if exchange:  # only the G-buffer rows each rank's strip-local denoise reads
            need = [gbuffer_rows(H, world, r) for r in range(world)]
    cam0 = rt.camera
    for f in range(1, frames + 1):
        c = rt.camera
        c.yaw = cam0.yaw + 0.02 * f
        rt.camera = c
        rt.build_bvh()
        rt.path_trace(f)
        if sg is not None:
            rt.sync()  # gloo reads the tensors on the host side: the strip must be complete
            move = sg.gather if need is None else (lambda: sg.exchange(need))
            if gs is not None:  # gathers on their own stream; the denoise waits for it
                gs.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(gs):
                    move()
            else:
                move()
        rt.denoise_post(f)
    rgba = rt.download("RGBA8", np.uint8).copy()
    hdr = rt.get_buffer("HISTORY_COLOR").copy()  # TemporalFilter2's output: the frame's final HDR
    acc = rt.get_buffer("ACCUMULATION").copy()
    expo = rt.download("EXPOSURE", np.uint8).copy()
    rt.cleanup()
    np.savez(os.path.join(out_dir, "%sr%d_of%d.npz" % (tag, rank, world)), rgba=rgba, hdr=hdr, acc=acc, expo=expo)
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined,gather_stream", [(True, False), (False, False), (True, True), (False, True)])
def test_two_ranks_one_gpu_match_single_rank(tmp_path, pipelined, gather_stream):
    """The renderer runs on torch's default stream (the null stream, handle 0) like the gathers:
    serial frames exercise exactly that ordering.  gather_stream: the gathers run on a stream of
    their own (rt_set_gather_stream), as bench.py does over RCCL."""
    import torch.multiprocessing as mp

    mp.start_processes(render, args=(1, 0, str(tmp_path), pipelined, gather_stream), nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(2, free_port(), str(tmp_path), pipelined, gather_stream), nprocs=2,
                       start_method="spawn")
    ref = np.load(tmp_path / "r0_of1.npz")
    for r in range(2):
        got = np.load(tmp_path / ("r%d_of2.npz" % r))
        for k in ("rgba", "hdr", "acc", "expo"):
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)


@pytest.mark.parametrize("pipelined,gather_stream", [(True, True), (False, False)])
def test_two_ranks_strip_local_denoise(tmp_path, pipelined, gather_stream):
    """Each rank denoises only its own 64-row-block strip (rt_set_collective_hook + rtx.dist.StripDenoise:
    histogram all-reduce, accumulation / history / RGBA8 row all-gathers); after 4 frames of a moving
    camera both ranks hold the single-rank frame bit for bit."""
    import torch.multiprocessing as mp

    mp.start_processes(render, args=(1, 0, str(tmp_path), pipelined, gather_stream), nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(2, free_port(), str(tmp_path), pipelined, gather_stream, True), nprocs=2,
                       start_method="spawn")
    ref = np.load(tmp_path / "r0_of1.npz")
    for r in range(2):
        got = np.load(tmp_path / ("r%d_of2.npz" % r))
        for k in ("rgba", "hdr", "acc", "expo"):
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)


def test_two_ranks_4k_strip_local_denoise(tmp_path):
    """Config 5's frame (3840x2160) split over two ranks (gloo on one GPU), strip-local denoise and
    the strip exchange of the G-buffers, two pipelined frames, against a single-rank render."""
    import torch.multiprocessing as mp

    args = (True, True, True, (3840, 2160), 2, "k", True)  # with the strip exchange
    mp.start_processes(render, args=(1, 0, str(tmp_path)) + args, nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(2, free_port(), str(tmp_path)) + args, nprocs=2, start_method="spawn")
    ref = np.load(tmp_path / "kr0_of1.npz")
    for r in range(2):
        got = np.load(tmp_path / ("kr%d_of2.npz" % r))
        for k in ("rgba", "hdr", "acc", "expo"):
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)


@pytest.mark.parametrize("pipelined", [True, False])
def test_two_ranks_strip_exchange(tmp_path, pipelined):
    """The strip exchange instead of the all-gather (StripGather.exchange: each rank receives only
    the G-buffer rows its strip-local denoise reads, gbuffer_rows): at 256x512 the two ranks need
    rows [0, 336) and [176, 512); after 4 frames of a moving camera both hold the single-rank frame."""
    import torch.multiprocessing as mp

    args = (pipelined, True, True, (256, 512), FRAMES, "x", True)
    mp.start_processes(render, args=(1, 0, str(tmp_path)) + args, nprocs=1, start_method="spawn")
    mp.start_processes(render, args=(2, free_port(), str(tmp_path)) + args, nprocs=2, start_method="spawn")
    ref = np.load(tmp_path / "xr0_of1.npz")
    for r in range(2):
        got = np.load(tmp_path / ("xr%d_of2.npz" % r))
        for k in ("rgba", "hdr", "acc", "expo"):
            assert np.array_equal(got[k], ref[k]), "rank %d %s" % (r, k)
