"""Probe: which gloo collectives accept cuda tensors (2 ranks sharing cuda:0)?"""
import os
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = "29541"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.full((1024,), rank + 1, dtype=torch.int32, device="cuda")
    res = {}
    for name, fn in [
        ("all_reduce", lambda: dist.all_reduce(t.clone())),
        ("reduce", lambda: dist.reduce(t.clone(), dst=0)),
        ("all_gather_list", lambda: dist.all_gather([torch.empty_like(t) for _ in range(world)], t)),
        ("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(torch.empty(world * 1024, dtype=torch.int32, device="cuda"), t)),
        ("gather", lambda: dist.gather(t, [torch.empty_like(t) for _ in range(world)] if rank == 0 else None, dst=0)),
        ("broadcast", lambda: dist.broadcast(t.clone(), src=0)),
    ]:
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = "FAIL " + str(e).splitlines()[0][:80]
    if rank == 0:
        for k, v in res.items():
            print(k, v, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(run, args=(2,), nprocs=2)
