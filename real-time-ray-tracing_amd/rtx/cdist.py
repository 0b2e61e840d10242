"""ctypes mirror of include/rtx_dist.h (librtx.so's rtd_* functions): the multi-GPU screen split as
C-ABI code over a pluggable communicator — what a non-Python host links instead of rtx/dist.py.

Two communicators for the tests:
* ThreadComm: every rank a thread of one process, host memory (the CPU tests);
* GlooHipComm: one process per rank over torch.distributed (gloo), device buffers moved through
  the host with the HIP runtime torch already loaded (the GPU tests; a real node plugs RCCL in,
  INTEGRATION.md §3)."""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import BUF, HOOK_GBUFFERS, HOOK_HISTOGRAM, HOOK_ROWS, load_library  # noqa: F401

SZ = C.c_size_t
ALL_GATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, SZ, C.c_void_p)
ALL_REDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, SZ, C.c_void_p)
ALL_TO_ALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(SZ), C.POINTER(SZ), C.c_void_p,
                             C.POINTER(SZ), C.POINTER(SZ), C.c_void_p)
COPY2D_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, SZ, C.c_void_p, SZ, SZ, SZ, C.c_void_p)
ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, SZ)
RELEASE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)


class RtdComm(C.Structure):
    _fields_ = [("arg", C.c_void_p), ("all_gather", ALL_GATHER_FN), ("all_reduce_sum_i32", ALL_REDUCE_FN),
                ("all_to_allv", ALL_TO_ALLV_FN), ("copy2d", COPY2D_FN), ("alloc", ALLOC_FN), ("release", RELEASE_FN)]


class RtdGbuffers(C.Structure):
    _fields_ = [("color", C.c_void_p), ("normal", C.c_void_p), ("albedo", C.c_void_p), ("depth", C.c_void_p),
                ("motion", C.c_void_p)]


DIST_SIGNATURES = {
    "rtd_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(RtdComm), C.POINTER(C.c_void_p)]),
    "rtd_destroy": (None, [C.c_void_p]),
    "rtd_last_error": (C.c_char_p, [C.c_void_p]),
    "rtd_denoise_rows": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rtd_gbuffer_rows": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rtd_gbuffer_bytes": (SZ, [C.c_void_p, C.c_int]),
    "rtd_recv_bytes": (SZ, [C.c_void_p, C.c_int, C.c_int]),
    "rtd_exchange_gbuffers": (C.c_int, [C.c_void_p, C.POINTER(RtdGbuffers), C.c_int, C.c_void_p]),
    "rtd_exchange_histogram": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtd_exchange_rows": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rtd_attach": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rtd_hook": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
}
GB_NAMES = ("RENDER_COLOR", "NORMAL", "ALBEDO", "DEPTH", "MOTION")

_bound = False


def lib():
    global _bound
    L = load_library()
    if not _bound:
        for name, (res, args) in DIST_SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _bound = True
    return L


def _arr(p, n):
    return [int(p[i]) for i in range(n)]


class Strips:
    """One rank's rtd_strips.  comm: an object with all_gather(send, recv, nbytes, stream),
    all_reduce_sum_i32(ptr, count, stream), all_to_allv(send, sb, so, recv, rb, ro, stream) and
    optionally copy2d / alloc / release (None: the library's HIP defaults)."""

    def __init__(self, width, height, world, rank, comm):
        self.L = lib()
        self.world, self.rank, self.comm = world, rank, comm

        def guard(fn):
            def w(*a):
                try:
                    r = fn(*a)
                    return 0 if r is None else r
                except Exception:
                    import traceback
                    traceback.print_exc()
                    return 1
            return w

        c = RtdComm()
        self._keep = []
        c.all_gather = ALL_GATHER_FN(guard(lambda arg, s, r, n, st: comm.all_gather(s, r, n, st)))
        c.all_reduce_sum_i32 = ALL_REDUCE_FN(guard(lambda arg, b, n, st: comm.all_reduce_sum_i32(b, n, st)))
        c.all_to_allv = ALL_TO_ALLV_FN(guard(lambda arg, s, sb, so, r, rb, ro, st: comm.all_to_allv(
            s, _arr(sb, world), _arr(so, world), r, _arr(rb, world), _arr(ro, world), st)))
        if getattr(comm, "copy2d", None) is not None:
            c.copy2d = COPY2D_FN(guard(lambda arg, d, dp, s, sp, w, h, st: comm.copy2d(d, dp, s, sp, w, h, st)))
        if getattr(comm, "alloc", None) is not None:
            c.alloc = ALLOC_FN(lambda arg, n: comm.alloc(n))
            c.release = RELEASE_FN(lambda arg, p: comm.release(p))
        self._c = c
        h = C.c_void_p()
        rc = self.L.rtd_create(width, height, world, rank, C.byref(c), C.byref(h))
        if rc != 0:
            raise RuntimeError("rtd_create failed (%d)" % rc)
        self.h = h

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError("%s failed (%d): %s" % (what, rc, self.L.rtd_last_error(self.h).decode()))

    def denoise_rows(self, r):
        a, b = C.c_int32(), C.c_int32()
        self._check(self.L.rtd_denoise_rows(self.h, r, C.byref(a), C.byref(b)), "rtd_denoise_rows")
        return a.value, b.value

    def gbuffer_rows(self, r):
        a, b = C.c_int32(), C.c_int32()
        self._check(self.L.rtd_gbuffer_rows(self.h, r, C.byref(a), C.byref(b)), "rtd_gbuffer_rows")
        return a.value, b.value

    def gbuffer_bytes(self, name):
        return int(self.L.rtd_gbuffer_bytes(self.h, BUF[name]))

    def recv_bytes(self, stage, strip_local=True):
        return int(self.L.rtd_recv_bytes(self.h, stage, 1 if strip_local else 0))

    def exchange_gbuffers(self, ptrs, strip_local=True, stream=None):
        g = RtdGbuffers(*[ptrs[n] for n in GB_NAMES])
        self._check(self.L.rtd_exchange_gbuffers(self.h, C.byref(g), 1 if strip_local else 0, stream),
                    "rtd_exchange_gbuffers")

    def exchange_histogram(self, ptr, stream=None):
        self._check(self.L.rtd_exchange_histogram(self.h, ptr, stream), "rtd_exchange_histogram")

    def exchange_rows(self, accum, history, rgba, stream=None):
        self._check(self.L.rtd_exchange_rows(self.h, accum, history, rgba, stream), "rtd_exchange_rows")

    def attach(self, rt):
        self._check(self.L.rtd_attach(self.h, rt.h), "rtd_attach")
        self.rt = rt

    def destroy(self):
        if self.h:
            self.L.rtd_destroy(self.h)
            self.h = None


class ThreadComm:
    """world ranks as threads of one process over host memory: ThreadComm(world).rank(r) is rank r's
    communicator (a barrier-synchronised exchange through shared slots)."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.mem = {}
        self.lock = threading.Lock()

    def rank(self, r):
        return _ThreadRank(self, r)


class _ThreadRank:
    def __init__(self, hub, r):
        self.hub, self.r = hub, r

    def _swap(self, item):
        h = self.hub
        h.bar.wait()
        h.slots[self.r] = item
        h.bar.wait()
        got = list(h.slots)
        h.bar.wait()
        return got

    def all_gather(self, send, recv, n, stream):
        got = self._swap(C.string_at(send, n))
        for q, b in enumerate(got):
            C.memmove(recv + q * n, b, n)

    def all_reduce_sum_i32(self, buf, count, stream):
        mine = np.frombuffer(C.string_at(buf, 4 * count), np.int32).copy()
        got = self._swap(mine)
        tot = np.sum(np.stack(got), axis=0, dtype=np.int64).astype(np.int32)
        C.memmove(buf, tot.tobytes(), 4 * count)

    def all_to_allv(self, send, sb, so, recv, rb, ro, stream):
        out = {q: C.string_at(send + so[q], sb[q]) for q in range(self.hub.world) if sb[q]}
        got = self._swap(out)
        for q in range(self.hub.world):
            if rb[q]:
                b = got[q][self.r]
                assert len(b) == rb[q], (self.r, q, len(b), rb[q])
                C.memmove(recv + ro[q], b, rb[q])

    def copy2d(self, dst, dpitch, src, spitch, width, height, stream):
        for y in range(height):
            C.memmove(dst + y * dpitch, src + y * spitch, width)

    def alloc(self, n):
        b = C.create_string_buffer(max(16, n))
        with self.hub.lock:
            self.hub.mem[C.addressof(b)] = b
        return C.addressof(b)

    def release(self, p):
        with self.hub.lock:
            self.hub.mem.pop(p, None)


class GlooHipComm:
    """One process per rank over torch.distributed (gloo); the library's device buffers move through
    the host with hipMemcpy of the HIP runtime torch loaded (the stream is drained first).  A test
    stand-in for RCCL, which cannot run two ranks on one GPU."""

    def __init__(self, group=None):
        import os

        import torch.distributed as dist

        self.dist, self.group = dist, group
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
        if path is None or not os.path.exists(path):
            raise RuntimeError("libamdhip64 not loaded")
        self.hip = C.CDLL(path)
        self.hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.hip.hipStreamSynchronize.argtypes = [C.c_void_p]

    def _sync(self, stream):
        if self.hip.hipStreamSynchronize(stream) != 0:
            raise RuntimeError("hipStreamSynchronize failed")

    def _d2h(self, p, n):
        a = np.empty(n, np.uint8)
        if n and self.hip.hipMemcpy(a.ctypes.data, p, n, 2) != 0:  # hipMemcpyDeviceToHost
            raise RuntimeError("hipMemcpy D2H failed")
        return a

    def _h2d(self, p, a):
        if a.size and self.hip.hipMemcpy(p, a.ctypes.data, a.size, 1) != 0:  # hipMemcpyHostToDevice
            raise RuntimeError("hipMemcpy H2D failed")

    def all_gather(self, send, recv, n, stream):
        import torch

        self._sync(stream)
        t = torch.from_numpy(self._d2h(send, n))
        outs = [torch.empty(n, dtype=torch.uint8) for _ in range(self.dist.get_world_size(self.group))]
        self.dist.all_gather(outs, t, group=self.group)
        self._h2d(recv, torch.cat(outs).numpy())

    def all_reduce_sum_i32(self, buf, count, stream):
        import torch

        self._sync(stream)
        t = torch.from_numpy(self._d2h(buf, 4 * count).view(np.int32).copy())
        self.dist.all_reduce(t, group=self.group)
        self._h2d(buf, t.numpy().view(np.uint8))

    def all_to_allv(self, send, sb, so, recv, rb, ro, stream):
        import torch

        self._sync(stream)
        world = self.dist.get_world_size(self.group)
        s = torch.from_numpy(np.concatenate([self._d2h(send + so[q], sb[q]) for q in range(world)]))
        r = torch.empty(sum(rb), dtype=torch.uint8)
        self.dist.all_to_all_single(r, s, output_split_sizes=list(rb), input_split_sizes=list(sb), group=self.group)
        rn = r.numpy()
        o = 0
        for q in range(world):
            self._h2d(recv + ro[q], np.ascontiguousarray(rn[o:o + rb[q]]))
            o += rb[q]
