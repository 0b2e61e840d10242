"""The RCCL code paths on the one GPU a test box has.  RCCL refuses two ranks on one device ("Duplicate
GPU detected", tools/rccl_probe.py), so the multi-rank tests move the same bytes over gloo; here the
RCCL branches themselves run at world size 1 on a real communicator: rtx/dist.py's
all_gather_into_tensor / all_to_all_single / all_reduce calls (backend "nccl", the one bench.py uses on
a node) and lib/librtx_rccl.so's rtd_comm (ncclAllGather, ncclAllReduce, grouped send/recv)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def dist_worker(rank, port, out_dir):
    import torch
    import torch.distributed as dist

    from rtx.dist import StripDenoise, StripGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    W, H = 64, 80
    sg = StripGather(W, H, 1, 0, dev)
    for name, t in sg.tensors.items():
        t.copy_(torch.arange(t.numel(), device=dev, dtype=torch.int64).remainder(251).to(torch.uint8))
    before = {k: v.clone() for k, v in sg.tensors.items()}
    sg.gather()  # all_gather_into_tensor over RCCL
    sg.exchange([(0, H)])  # all_to_all_single with split sizes (nothing to move at world 1)
    sd = StripDenoise(W, H, 1, 0, dev, group=dist.group.WORLD)
    sd.histogram.copy_(torch.arange(64, dtype=torch.int32, device=dev))
    sd.exchange_histogram()  # all_reduce
    sd.accum.fill_(7)
    sd.exchange_rows(0)  # all_gather_into_tensor of the strip rows
    torch.cuda.synchronize()
    ok = all(torch.equal(before[k], sg.tensors[k]) for k in before)
    ok = ok and torch.equal(sd.histogram.cpu(), torch.arange(64, dtype=torch.int32)) and int(sd.accum.min()) == 7
    np.save(os.path.join(out_dir, "dist_ok.npy"), np.array([ok]))
    dist.destroy_process_group()


def test_dist_py_nccl_branches_world1(tmp_path):
    import torch.multiprocessing as mp

    mp.start_processes(dist_worker, args=(free_port(), str(tmp_path)), nprocs=1, start_method="spawn")
    assert bool(np.load(tmp_path / "dist_ok.npy")[0])


def test_librtx_rccl_comm_world1(rtx):
    import torch

    from rtx.cdist import RtdComm

    lib = C.CDLL(os.path.join(ROOT, "real-time-ray-tracing_amd", "lib", "librtx_rccl.so"))
    torch.cuda.set_device(0)
    uid = C.create_string_buffer(128)
    assert lib.rtd_rccl_get_unique_id(uid) == 0
    comm = C.c_void_p()
    assert lib.rtd_rccl_comm_init(1, 0, uid, C.byref(comm)) == 0
    rc = RtdComm()
    assert lib.rtd_comm_rccl(comm, C.byref(rc)) == 0
    s = torch.cuda.current_stream().cuda_stream
    a = torch.arange(256, dtype=torch.uint8, device="cuda")
    b = torch.zeros(256, dtype=torch.uint8, device="cuda")
    assert rc.all_gather(rc.arg, a.data_ptr(), b.data_ptr(), 256, s) == 0
    h = torch.arange(64, dtype=torch.int32, device="cuda")
    assert rc.all_reduce_sum_i32(rc.arg, C.cast(h.data_ptr(), C.c_void_p), 64, s) == 0
    zero = (C.c_size_t * 1)(0)
    assert rc.all_to_allv(rc.arg, a.data_ptr(), zero, zero, b.data_ptr(), zero, zero, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(h.cpu(), torch.arange(64, dtype=torch.int32))
    lib.rtd_rccl_comm_destroy(comm)
