"""Probe: can two processes hold RCCL ranks on the same GPU through the C-ABI communicator?
usage: python tools/rccl_two_rank_probe.py   (spawns 2 ranks; gloo rendezvous on 127.0.0.1)"""
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from topology_aware_learning_amd.comm import shared_halo_comm

    dev = torch.device("cuda", 0)
    comm = shared_halo_comm(world, rank, dev)
    x = torch.full((1024,), float(rank + 1), device=dev)
    y = torch.zeros(1024, device=dev)
    peer = 1 - rank
    sends = [None] * world
    recvs = [None] * world
    sends[peer], recvs[peer] = x, y
    comm.exchange(sends, recvs)
    torch.cuda.synchronize()
    print(f"rank {rank}: received {y[0].item()} (expected {peer + 1})", flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2, 29533), nprocs=2)
