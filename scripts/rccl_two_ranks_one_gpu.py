"""Probe: can two RCCL ranks share one GPU on this pool? Spawns 2 processes on device 0, nccl backend, one
all-reduce. Usage: python scripts/rccl_two_ranks_one_gpu.py (prints one line per rank, exit code 0 when both agree)."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _rank(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce -> {t.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(2, port), nprocs=2, join=True)
    sys.exit(0)
