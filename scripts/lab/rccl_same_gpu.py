"""Probe: can two RCCL ranks share one GPU on the box? (world 2, both on cuda:0)"""
import os
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29533"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    t = torch.full((1 << 20,), rank + 1, dtype=torch.int32, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print("rank", rank, "sum", int(t[0]), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2,), nprocs=2)
