"""Screen-strip multi-GPU split over torch.distributed.

One process per GPU.  Every rank rebuilds the (small) BVH itself and path traces the rows
[y0, y0 + rows) of the frame into caller-owned G-buffers; an all-gather (RCCL over xGMI on
the "nccl" backend, gloo in the CPU tests) then assembles the full-frame G-buffers on every
rank, where the denoiser and post chain run on the whole image.  That keeps the temporal
passes' reprojection (motion vectors can point anywhere on screen) and the wide à-trous
footprints exact: each rank's result is bit-identical to a single-GPU frame.

The G-buffers are flat uint8 torch tensors of ``world * rows_per_rank * W * bpp`` bytes (the
tail beyond H rows is scratch) bound into the renderer with ``rt_bind_buffer``, so the
all-gather works in place: rank r's strip is exactly chunk r of each tensor.
"""
from __future__ import annotations

import math

# path-trace G-buffers (pathtrace.cuh:123-127) and their bytes per pixel
GBUFFERS = (("RENDER_COLOR", 8), ("NORMAL", 8), ("ALBEDO", 8), ("DEPTH", 2), ("MOTION", 4))


def strip_rows(height: int, world: int, rank: int) -> tuple[int, int, int]:
    """(y0, rows, rows_per_rank) of rank's horizontal strip; strips are ceil(H / world) rows."""
    per = math.ceil(height / world)
    y0 = rank * per
    rows = max(0, min(per, height - y0))
    if rows < 1:
        raise ValueError("height %d too small for %d strips" % (height, world))
    return y0, rows, per


class StripGather:
    """Full-frame G-buffer tensors for one rank plus the in-place all-gather of the strips.

    With ``sets=rtx.GBUFFER_SETS`` (frame pipelining, ``RayTracer.set_post_stream``) every G-buffer
    set of the renderer is bound and ``gather`` assembles the set the last path trace wrote."""

    def __init__(self, width: int, height: int, world: int, rank: int, device, rt=None, sets: int = 1):
        import torch

        self.W, self.H, self.world, self.rank = width, height, world, rank
        self.rt = rt
        self.y0, self.rows, self.per = strip_rows(height, world, rank)
        self.sets = []
        for k in range(sets):
            tensors = {}
            for name, bpp in GBUFFERS:
                t = torch.zeros(world * self.per * width * bpp, dtype=torch.uint8, device=device)
                tensors[name] = t
                if rt is not None:
                    rt.bind_buffer(name, t.data_ptr(), t.numel(), gbuffer_set=k)
            self.sets.append(tensors)
        self.tensors = self.sets[0]

    def chunk(self, name: str, gbuffer_set: int = 0):
        t = self.sets[gbuffer_set][name]
        n = t.numel() // self.world
        return t[self.rank * n:(self.rank + 1) * n]

    def gather(self, group=None, gbuffer_set: int | None = None):
        """All-gather every rank's strip into every rank's full-frame tensors (in place)."""
        import torch.distributed as dist

        if gbuffer_set is None:
            gbuffer_set = self.rt.info().gbufferSet if (self.rt is not None and len(self.sets) > 1) else 0
        nccl = dist.get_backend(group) == "nccl"
        for name, _ in GBUFFERS:
            t = self.sets[gbuffer_set][name]
            n = t.numel() // self.world
            mine = t[self.rank * n:(self.rank + 1) * n]
            if nccl:
                dist.all_gather_into_tensor(t, mine, group=group)
            else:
                outs = [t[r * n:(r + 1) * n] for r in range(self.world)]
                dist.all_gather(outs, mine.clone(), group=group)

    def bytes_per_frame(self) -> int:
        """Bytes each rank receives per frame."""
        return sum(t.numel() for t in self.tensors.values()) * (self.world - 1) // self.world
