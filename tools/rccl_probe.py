#!/usr/bin/env python3
"""Can two RCCL ranks share one GPU here?  2 processes on cuda:0, backend nccl: all_gather_into_tensor,
all_to_all_single with split sizes, all_reduce (the calls rtx/dist.py makes).  Prints per-rank results."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def rank_main(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((4,), rank + 1, dtype=torch.uint8, device=dev)
    out = torch.empty(4 * world, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, x)
    s = torch.arange(world * 2, dtype=torch.uint8, device=dev) + 10 * rank
    r = torch.empty(world * 2, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(r, s, output_split_sizes=[2] * world, input_split_sizes=[2] * world)
    h = torch.full((64,), rank + 1, dtype=torch.int32, device=dev)
    dist.all_reduce(h)
    torch.cuda.synchronize()
    print("rank %d: gather %s a2a %s reduce %d" % (rank, out.tolist(), r.tolist(), int(h[0])), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.start_processes(rank_main, args=(world, 29611), nprocs=world, start_method="spawn")
