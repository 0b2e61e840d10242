#!/usr/bin/env python3
"""Stress the two-ranks-on-one-GPU gloo frame path (tests/test_gpu_multirank.py) for races:
per-frame RGBA8 + HDR of both ranks vs a single rank, over several repetitions."""
import os
import socket
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-ray-tracing_amd")]

W, H, FRAMES = 256, 144, 4


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render(rank, world, port, out_dir, pipelined):
    import torch
    import torch.distributed as dist

    import rtx
    from rtx.dist import StripGather, strip_config

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
    sg = StripGather(W, H, world, rank, dev, rt, sets=rtx.GBUFFER_SETS if pipelined else 1) if world > 1 else None
    cam0 = rt.camera
    imgs, gbufs = [], []
    for f in range(1, FRAMES + 1):
        c = rt.camera
        c.yaw = cam0.yaw + 0.02 * f
        rt.camera = c
        rt.build_bvh()
        rt.path_trace(f)
        if sg is not None:
            rt.sync()
            sg.gather()
        rt.denoise_post(f)
    imgs.append(rt.download("RGBA8", np.uint8).copy())  # final frame only, as the test does
    gbufs.append(rt.get_buffer("RENDER_COLOR").view(np.uint8).reshape(-1).copy())
    rt.cleanup()
    np.savez(os.path.join(out_dir, "r%d_of%d.npz" % (rank, world)), img=np.stack(imgs), gb=np.stack(gbufs))
    if world > 1:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    pipelined = (sys.argv[2] if len(sys.argv) > 2 else "pipe") == "pipe"
    d = tempfile.mkdtemp()
    mp.start_processes(render, args=(1, 0, d, pipelined), nprocs=1, start_method="spawn")
    ref = np.load(os.path.join(d, "r0_of1.npz"))
    for rep in range(reps):
        mp.start_processes(render, args=(2, free_port(), d, pipelined), nprocs=2, start_method="spawn")
        for r in range(2):
            got = np.load(os.path.join(d, "r%d_of2.npz" % r))
            a, b = got["img"][0], ref["img"][0]
            diff = np.nonzero(np.any(a.reshape(H, W, 4) != b.reshape(H, W, 4), axis=2))
            rows = sorted(set(diff[0].tolist()))
            print(rep, "rank", r, "final img", "ok" if not rows else "BAD rows %s..%s (%d px)" % (rows[0], rows[-1], len(diff[0])),
                  "hdr", "ok" if np.array_equal(got["gb"][0], ref["gb"][0]) else "BAD", flush=True)


if __name__ == "__main__":
    main()
