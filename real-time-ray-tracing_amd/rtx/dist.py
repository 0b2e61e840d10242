"""Multi-GPU frame split over torch.distributed.

One process per GPU.  Every rank rebuilds the (small) BVH itself and path traces its share of
the frame's rows into caller-owned G-buffers; an all-gather (RCCL over xGMI on the "nccl"
backend, gloo in the CPU tests) then assembles the full-frame G-buffers on every rank, where the
denoiser and post chain run on the whole image.  That keeps the temporal passes' reprojection
(motion vectors can point anywhere on screen) and the wide à-trous footprints exact: each
rank's result is bit-identical to a single-GPU frame.

Rows are dealt in blocks of ROW_BLOCK (= kRowBlock in the renderer) round-robin over the ranks
(config keys stripCount / stripIndex): the expensive rows — geometry, as opposed to sky — sit in
one band of the image (the top ~27 % in the default view), and contiguous strips would hand
nearly all of them to one or two ranks.  Block b of the frame belongs to rank b mod N.

The gather packs this rank's blocks of every G-buffer into one staging buffer, runs ONE
all_gather_into_tensor, and scatters the ranks' blocks back into the natural row order.
"""
from __future__ import annotations

import math

# path-trace G-buffers (pathtrace.cuh:123-127) and their bytes per pixel
GBUFFERS = (("RENDER_COLOR", 8), ("NORMAL", 8), ("ALBEDO", 8), ("DEPTH", 2), ("MOTION", 4))
ROW_BLOCK = 16  # kRowBlock (bvh_kernels.h)


def strip_rows(height: int, world: int, rank: int) -> tuple[int, int, int]:
    """(y0, rows, rows_per_rank) of rank's contiguous strip (config stripY0 / stripRows): strips
    are ceil(H / world) rows.  The multi-GPU bench uses interleaved blocks (strip_blocks)."""
    per = math.ceil(height / world)
    y0 = rank * per
    rows = max(0, min(per, height - y0))
    if rows < 1:
        raise ValueError("height %d too small for %d strips" % (height, world))
    return y0, rows, per


def strip_blocks(height: int, world: int, rank: int) -> list[tuple[int, int]]:
    """(y0, rows) of every row block rank owns with interleaved strips (row_of in the renderer)."""
    out = []
    b = rank
    while b * ROW_BLOCK < height:
        y0 = b * ROW_BLOCK
        out.append((y0, min(ROW_BLOCK, height - y0)))
        b += world
    if not out:
        raise ValueError("height %d too small for %d interleaved strips" % (height, world))
    return out


def strip_config(world: int, rank: int) -> str:
    """[render] keys of rank's interleaved strip, for rtx.write_config(extra=...)."""
    return "stripCount = %d\nstripIndex = %d\n" % (world, rank) if world > 1 else ""


class StripGather:
    """Full-frame G-buffer tensors for one rank plus the all-gather of the ranks' row blocks.

    With ``sets=rtx.GBUFFER_SETS`` (frame pipelining, ``RayTracer.set_post_stream``) every G-buffer
    set of the renderer is bound and ``gather`` assembles the set the last path trace wrote."""

    def __init__(self, width: int, height: int, world: int, rank: int, device, rt=None, sets: int = 1):
        import torch

        self.W, self.H, self.world, self.rank = width, height, world, rank
        self.rt = rt
        blocks = math.ceil(height / ROW_BLOCK)
        self.rounds = math.ceil(blocks / world)          # block b = round * world + rank
        rows = self.rounds * world * ROW_BLOCK           # padded: rows >= H are scratch
        self.blk = {name: ROW_BLOCK * width * bpp for name, bpp in GBUFFERS}
        self.off, o = {}, 0
        for name, _ in GBUFFERS:
            self.off[name] = o
            o += self.rounds * self.blk[name]
        self.stage_bytes = o
        self.stage_in = torch.zeros(o, dtype=torch.uint8, device=device)
        self.stage_out = torch.zeros(world * o, dtype=torch.uint8, device=device)
        self.sets = []
        for k in range(sets):
            tensors = {}
            for name, bpp in GBUFFERS:
                t = torch.zeros(rows * width * bpp, dtype=torch.uint8, device=device)
                tensors[name] = t
                if rt is not None:
                    rt.bind_buffer(name, t.data_ptr(), t.numel(), gbuffer_set=k)
            self.sets.append(tensors)
        self.tensors = self.sets[0]

    def blocks(self, name: str, gbuffer_set: int = 0):
        """View [rounds, world, block bytes] of a G-buffer: [:, r] are rank r's row blocks."""
        return self.sets[gbuffer_set][name].view(self.rounds, self.world, self.blk[name])

    def mine(self, name: str, gbuffer_set: int = 0):
        return self.blocks(name, gbuffer_set)[:, self.rank]

    def gather(self, group=None, gbuffer_set: int | None = None):
        """Every rank's row blocks into every rank's full-frame tensors (one collective)."""
        import torch.distributed as dist

        if gbuffer_set is None:
            gbuffer_set = self.rt.info().gbufferSet if (self.rt is not None and len(self.sets) > 1) else 0
        for name, _ in GBUFFERS:
            o, n = self.off[name], self.rounds * self.blk[name]
            self.stage_in[o:o + n].view(self.rounds, self.blk[name]).copy_(self.mine(name, gbuffer_set))
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(self.stage_out, self.stage_in, group=group)
        else:
            outs = list(self.stage_out.view(self.world, self.stage_bytes).unbind(0))
            dist.all_gather(outs, self.stage_in, group=group)
        every = self.stage_out.view(self.world, self.stage_bytes)
        for name, _ in GBUFFERS:
            o, n = self.off[name], self.rounds * self.blk[name]
            src = every[:, o:o + n].view(self.world, self.rounds, self.blk[name]).permute(1, 0, 2)
            self.blocks(name, gbuffer_set).copy_(src)

    def bytes_per_frame(self) -> int:
        """Bytes each rank receives per frame."""
        return self.stage_bytes * (self.world - 1)
