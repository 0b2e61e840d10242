"""The per-frame loop of RayTracer::draw (kernel.cu:259-398) as bench.py runs it.

bench.py times exactly this object's ``frame`` calls and the parity tests run the same object
(tests/test_gpu_bench_path.py), so the measured path is the tested path:

* the renderer's stages go to a high-priority torch stream (the trace chain is the critical
  path) and, pipelined, the denoise/post chain of frame f to a low-priority second stream
  (rt_set_post_stream) beside the trace kernels of frame f+1;
* with N ranks (rtx/dist.py) every rank path traces its interleaved row blocks, the G-buffer
  rows each rank's denoise reads are exchanged (RCCL on its own stream when the backend is nccl,
  after a host sync with gloo: an all-to-all of the strip-plus-halo rows, or the all-gather when
  every rank denoises the whole frame), and each rank denoises its own contiguous rows (StripDenoise:
  the histogram all-reduce and the accumulation / history / RGBA8 row all-gathers the renderer
  asks for through its collective hook; strip_denoise=False denoises the whole frame on every rank).
"""
from __future__ import annotations


class FramePipeline:
    PRIORITIES = ("lo", "hi", "0")

    def __init__(self, rt, device, pipelined: bool = True, world: int = 1, rank: int = 0, backend: str = "nccl",
                 strip_denoise: bool = True, main_priority: str = "hi", post_priority: str = "lo"):
        """main_priority / post_priority: the torch stream priorities of the renderer's stream and the
        denoise/post stream ("hi", "lo" or "0", the normal priority); by default the trace chain
        outranks the denoise stream (A/B of other choices: DESIGN.md §7)."""
        import torch

        import rtx
        from rtx.dist import StripDenoise, StripGather, gbuffer_rows

        self.rt, self.device, self.pipelined = rt, device, pipelined
        self.world, self.rank = world, rank
        for p in (main_priority, post_priority):
            if p not in self.PRIORITIES:
                raise ValueError("stream priority must be one of %s, not %r" % (self.PRIORITIES, p))
        if pipelined:
            lo, hi = torch.cuda.Stream.priority_range()
            pick = {"lo": lo, "hi": hi, "0": 0}
            self.main = torch.cuda.Stream(device, priority=pick[main_priority])
            self.post = torch.cuda.Stream(device, priority=pick[post_priority])
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
        # with the strip-local denoise each rank receives only the G-buffer rows it reads
        self.need = ([gbuffer_rows(info.renderHeight, world, r) for r in range(world)]
                     if self.denoise is not None else None)

    def frame(self, f: int, hdr: bool = False):
        """LBVH rebuild, path trace, (gather,) denoise + post of frame f, enqueued asynchronously."""
        import torch

        rt = self.rt
        rt.build_bvh()
        rt.path_trace(f)
        if self.gather is not None:
            move = self.gather.gather
            if self.need is not None:  # strip-local denoise this frame: only the rows it reads
                i = rt.info()
                # decided by the renderer's flag, the same on every rank (a rank's G-buffer rows can
                # span the whole frame while its peers' do not: all ranks must enter one collective)
                if i.stripLocalDenoise:
                    if (i.gbufferRowBegin, i.gbufferRowEnd) != self.need[self.rank]:
                        raise RuntimeError("renderer and host disagree on the strip's G-buffer rows")
                    move = lambda: self.gather.exchange(self.need)  # noqa: E731
            if self.gs is not None:
                self.gs.wait_stream(torch.cuda.current_stream(self.device))  # this frame's path trace
                with torch.cuda.stream(self.gs):
                    move()
            else:
                rt.sync()  # gloo copies through the host: the strip must be complete
                move()
        rt.denoise_post(f, hdr)

    def finish(self):
        """Issue the last frame's deferred denoise/post and wait for every renderer stream."""
        self.rt.sync()
