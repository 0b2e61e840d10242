"""The per-frame loop of RayTracer::draw (kernel.cu:259-398) as bench.py runs it.

bench.py times exactly this object's ``frame`` calls and the parity tests run the same object
(tests/test_gpu_bench_path.py), so the measured path is the tested path:

* the renderer's stages go to a high-priority torch stream (the trace chain is the critical
  path) and, pipelined, the denoise/post chain of frame f to a low-priority second stream
  (rt_set_post_stream) beside the trace kernels of frame f+1;
* with N ranks (rtx/dist.py) every rank path traces its interleaved row blocks, the G-buffers
  are all-gathered (RCCL on its own stream when the backend is nccl, after a host sync with
  gloo), and each rank denoises its own contiguous rows of the assembled frame (StripDenoise:
  the histogram all-reduce and the accumulation / history / RGBA8 row all-gathers the renderer
  asks for through its collective hook; strip_denoise=False denoises the whole frame on every rank).
"""
from __future__ import annotations


class FramePipeline:
    def __init__(self, rt, device, pipelined: bool = True, world: int = 1, rank: int = 0, backend: str = "nccl",
                 strip_denoise: bool = True):
        import torch

        import rtx
        from rtx.dist import StripDenoise, StripGather

        self.rt, self.device, self.pipelined = rt, device, pipelined
        self.world, self.rank = world, rank
        if pipelined:  # the trace chain outranks the denoise stream
            lo, hi = torch.cuda.Stream.priority_range()
            self.main = torch.cuda.Stream(device, priority=hi)
            self.post = torch.cuda.Stream(device, priority=lo)
            torch.cuda.set_stream(self.main)
        else:
            self.main, self.post = torch.cuda.current_stream(device), None
        rt.set_stream(torch.cuda.current_stream(device).cuda_stream)  # collectives order with the renderer
        if pipelined:
            rt.set_post_stream(self.post.cuda_stream)
        self.gather = (StripGather(rt.info().renderWidth, rt.info().renderHeight, world, rank, device, rt,
                                   sets=rtx.GBUFFER_SETS if pipelined else 1) if world > 1 else None)
        # RCCL gathers on a stream of their own: the next frame's path trace does not wait for the
        # collective, only the frame's own denoise does (rt_set_gather_stream)
        self.gs = torch.cuda.Stream(device) if (self.gather is not None and backend == "nccl") else None
        if self.gs is not None:
            rt.set_gather_stream(self.gs.cuda_stream)
        info = rt.info()
        self.denoise = (StripDenoise(info.renderWidth, info.renderHeight, world, rank, device, rt)
                        if (world > 1 and strip_denoise) else None)

    def frame(self, f: int, hdr: bool = False):
        """LBVH rebuild, path trace, (gather,) denoise + post of frame f, enqueued asynchronously."""
        import torch

        rt = self.rt
        rt.build_bvh()
        rt.path_trace(f)
        if self.gather is not None:
            if self.gs is not None:
                self.gs.wait_stream(torch.cuda.current_stream(self.device))  # this frame's path trace
                with torch.cuda.stream(self.gs):
                    self.gather.gather()
            else:
                rt.sync()  # gloo copies through the host: the strip must be complete
                self.gather.gather()
        rt.denoise_post(f, hdr)

    def finish(self):
        """Issue the last frame's deferred denoise/post and wait for every renderer stream."""
        self.rt.sync()
