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
all_gather_into_tensor, and scatters the ranks' blocks back into the natural row order.  With the
strip-local denoise (StripDenoise) a rank reads the G-buffers only in its strip plus the denoise's
halo (gbuffer_rows), so StripGather.exchange replaces the all-gather by one all-to-all that sends
each rank only the blocks inside its rows: at 1080p on 8 GPUs a rank receives ~0.25 instead of
0.875 of the frame's 62 MB of G-buffers.
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
        """Bytes each rank receives per frame (the full all-gather)."""
        return self.stage_bytes * (self.world - 1)

    # ---- strip exchange: with a strip-local denoise (StripDenoise) rank r reads the G-buffers only
    # in rows need[r] = gbuffer_rows(H, N, r) (its strip plus the denoise's halo), so instead of the
    # all-gather every rank sends each other rank just its row blocks inside that rank's rows.
    def _rounds_in(self, rows: tuple[int, int], owner: int) -> tuple[int, int]:
        """[j0, j1): the rounds j whose block b = j * world + owner intersects rows [lo, hi)."""
        lo, hi = rows
        j0 = 0
        while j0 < self.rounds and ((j0 * self.world + owner) + 1) * ROW_BLOCK <= lo:
            j0 += 1
        j1 = j0
        while j1 < self.rounds and (j1 * self.world + owner) * ROW_BLOCK < hi:
            j1 += 1
        return j0, j1

    def _plan(self, need):
        """Send / receive (rounds range, bytes) per peer for the row ranges need[r] of every rank."""
        blk_all = sum(self.blk.values())
        send, recv = [], []
        for r in range(self.world):
            js = self._rounds_in(need[r], self.rank) if r != self.rank else (0, 0)
            jr = self._rounds_in(need[self.rank], r) if r != self.rank else (0, 0)
            send.append((js, (js[1] - js[0]) * blk_all))
            recv.append((jr, (jr[1] - jr[0]) * blk_all))
        return send, recv

    def exchange(self, need, group=None, gbuffer_set: int | None = None):
        """Each rank's row blocks to the ranks whose rows need[r] = (lo, hi) they fall in (one
        all-to-all); rows outside need[self.rank] are left as they are."""
        import torch
        import torch.distributed as dist

        if gbuffer_set is None:
            gbuffer_set = self.rt.info().gbufferSet if (self.rt is not None and len(self.sets) > 1) else 0
        send, recv = self._plan(need)
        key = tuple(need)
        if getattr(self, "_xkey", None) != key:  # staging sized for this plan
            dev = self.stage_in.device
            self._xsend = torch.zeros(max(1, sum(n for _, n in send)), dtype=torch.uint8, device=dev)
            self._xrecv = torch.zeros(max(1, sum(n for _, n in recv)), dtype=torch.uint8, device=dev)
            self._xkey = key
        o = 0
        for (j0, j1), n in send:  # per peer: every G-buffer's blocks of rounds [j0, j1)
            for name, _ in GBUFFERS:
                m = (j1 - j0) * self.blk[name]
                if m:
                    self._xsend[o:o + m].view(j1 - j0, self.blk[name]).copy_(self.mine(name, gbuffer_set)[j0:j1])
                o += m
        ins, outs = [n for _, n in send], [n for _, n in recv]
        sbuf, rbuf = self._xsend[:sum(ins)], self._xrecv[:sum(outs)]
        if dist.get_backend(group) == "nccl":
            dist.all_to_all_single(rbuf, sbuf, output_split_sizes=outs, input_split_sizes=ins, group=group)
        else:  # gloo: all-to-all on host tensors
            rh = torch.empty(rbuf.numel(), dtype=torch.uint8)
            dist.all_to_all_single(rh, sbuf.cpu(), output_split_sizes=outs, input_split_sizes=ins, group=group)
            rbuf.copy_(rh)
        o = 0
        for q, ((j0, j1), n) in enumerate(recv):
            for name, _ in GBUFFERS:
                m = (j1 - j0) * self.blk[name]
                if m:
                    self.blocks(name, gbuffer_set)[j0:j1, q].copy_(rbuf[o:o + m].view(j1 - j0, self.blk[name]))
                o += m

    def exchange_bytes_per_frame(self, need) -> int:
        """Bytes this rank receives per frame with the strip exchange."""
        return sum(n for _, n in self._plan(need)[1])


DENOISE_BLOCK = 64  # kDenoiseBlock (bvh_kernels.h): one texel row of the 1/64 DownScale4 level


def denoise_rows(height: int, world: int, rank: int) -> tuple[int, int]:
    """[a, b) rows rank denoises in the strip-local denoise (denoise_rows in the renderer): the
    frame's 64-row blocks split into `world` contiguous runs as evenly as whole blocks allow."""
    nb = math.ceil(height / DENOISE_BLOCK)
    if nb < world:
        raise ValueError("height %d has fewer 64-row blocks than %d ranks" % (height, world))
    b0, b1 = rank * nb // world, (rank + 1) * nb // world
    return b0 * DENOISE_BLOCK, min(b1 * DENOISE_BLOCK, height)


GBUF_HALO_TILES = 5  # kGbufHaloTiles (bvh_kernels.h)


def gbuffer_rows(height: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) G-buffer rows rank's strip-local denoise reads (gbuffer_rows in the renderer): its
    denoise rows widened by GBUF_HALO_TILES 16-row tiles on each side."""
    a, b = denoise_rows(height, world, rank)
    t0, t1 = a // 16, (b + 15) // 16
    return max(0, (t0 - GBUF_HALO_TILES) * 16), min(height, (t1 + GBUF_HALO_TILES) * 16)


class StripDenoise:
    """The strip-local denoise's exchanges (rt_set_collective_hook).

    Every rank denoises only its contiguous rows (plus the halo its passes read, inside the
    renderer) instead of the whole frame.  Per frame the renderer asks for two collectives, enqueued
    on the stream the denoise runs on:
      * HOOK_HISTOGRAM: all-reduce (sum) of the 64-bin luminance histogram — each rank counted the
        Histogram2 texels of its own rows — before AutoExposure reads it;
      * HOOK_ROWS: all-gather of every rank's rows of the accumulation buffer, of the history
        buffer TemporalFilter2 just wrote (the frame's final HDR) and of the RGBA8 output, which the
        next frame's temporal passes read at reprojected positions anywhere on screen.
    The four buffers are caller-owned tensors bound into the renderer, so the collectives move
    them in place; the rows travel in one staging buffer per rank (padded to the largest strip):
    20 B per pixel of the strip.  On a separate process group, so these collectives never
    interleave with the G-buffer gathers of StripGather on one communicator."""

    def __init__(self, width: int, height: int, world: int, rank: int, device, rt=None, group=None):
        import torch
        import torch.distributed as dist

        self.W, self.H, self.world, self.rank, self.device = width, height, world, rank, device
        self.rows = [denoise_rows(height, world, r) for r in range(world)]
        self.a, self.b = self.rows[rank]
        self.max_rows = max(b - a for a, b in self.rows)
        P = width * height
        u8 = dict(dtype=torch.uint8, device=device)
        self.accum = torch.zeros(P * 8, **u8)
        self.history = [torch.zeros(P * 8, **u8), torch.zeros(P * 8, **u8)]
        self.rgba = torch.zeros(P * 4, **u8)
        self.histogram = torch.zeros(64, dtype=torch.int32, device=device)
        self.row_bytes = width * (8 + 8 + 4)
        self.send = torch.zeros(self.max_rows * self.row_bytes, **u8)
        self.recv = torch.zeros(world * self.max_rows * self.row_bytes, **u8)
        self.group = group if group is not None else (dist.new_group(list(range(world))) if world > 1 else None)
        self.rt = rt
        if rt is not None:
            rt.bind_buffer("ACCUMULATION", self.accum.data_ptr(), self.accum.numel())
            rt.bind_buffer("HISTORY_COLOR", self.history[0].data_ptr(), self.history[0].numel(), gbuffer_set=0)
            rt.bind_buffer("HISTORY_COLOR", self.history[1].data_ptr(), self.history[1].numel(), gbuffer_set=1)
            rt.bind_buffer("HISTOGRAM", self.histogram.data_ptr(), 256)
            rt.bind_buffer("RGBA8", self.rgba.data_ptr(), self.rgba.numel())
            rt.set_collective_hook(self.hook)

    def bytes_per_frame(self) -> int:
        """Bytes each rank receives per frame for the rows exchange."""
        return (self.world - 1) * self.max_rows * self.row_bytes

    def _views(self, history_set: int):
        W, H = self.W, self.H
        return (self.accum.view(H, W * 8), self.history[history_set].view(H, W * 8), self.rgba.view(H, W * 4))

    def exchange_histogram(self):
        import torch.distributed as dist

        dist.all_reduce(self.histogram, group=self.group)

    def exchange_rows(self, history_set: int):
        import torch.distributed as dist

        acc, his, rgb = self._views(history_set)
        W, n = self.W, self.b - self.a
        s = self.send.view(self.max_rows, self.row_bytes)
        s[:n, :W * 8].copy_(acc[self.a:self.b])
        s[:n, W * 8:W * 16].copy_(his[self.a:self.b])
        s[:n, W * 16:].copy_(rgb[self.a:self.b])
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        else:
            dist.all_gather(list(self.recv.view(self.world, -1).unbind(0)), self.send, group=self.group)
        every = self.recv.view(self.world, self.max_rows, self.row_bytes)
        for r, (a, b) in enumerate(self.rows):
            if r == self.rank:
                continue
            m = b - a
            acc[a:b].copy_(every[r, :m, :W * 8])
            his[a:b].copy_(every[r, :m, W * 8:W * 16])
            rgb[a:b].copy_(every[r, :m, W * 16:])

    def hook(self, stage: int, stream: int, x):
        """rt_set_collective_hook callback: enqueue the exchange on the renderer's stream."""
        import torch

        s = torch.cuda.ExternalStream(stream, device=self.device) if stream else torch.cuda.default_stream(self.device)
        with torch.cuda.stream(s):
            if stage == 0:
                self.exchange_histogram()
            else:
                assert (x.rowBegin, x.rowEnd) == (self.a, self.b), "renderer and host disagree on the strip"
                self.exchange_rows(int(x.historySet))
