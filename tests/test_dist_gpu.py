"""The sharded pipeline (sheep_amd.dist) with the real HIP kernels: 2 and 3 ranks sharing cuda:0
over gloo (RCCL refuses two ranks on one device; gloo carries device tensors).  Everything but
the collective library is the multi-GPU product path: DeviceOps, the degree all-reduce, the
pst sum-reduce, the parent gather and the P-way forest merge on rank 0."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, scale, seed, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sheep_amd import device
        from sheep_amd.dist import DeviceOps, build_tree_sharded, shard_bounds

        device.init(0)
        m = 16 << scale
        lo, hi = shard_bounds(m, rank, world)
        uv = device.rmat(scale, 16, seed, lo, hi)
        seq, parent, pst, n = build_tree_sharded(uv, 1 << scale, DeviceOps())
        torch.cuda.synchronize()
        if rank == 0:
            q.put((seq[:n].cpu().numpy().view(np.uint32).copy(),
                   parent[:n].cpu().numpy().view(np.uint32).copy(),
                   pst[:n].cpu().numpy().view(np.uint32).copy()))
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,scale", [(2, 14), (3, 13)])
def test_sharded_device_pipeline_equals_serial(oracle, world, scale):
    seed = 60 + world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_worker, args=(world, _port(), scale, seed, q), nprocs=world,
                            join=False, start_method="spawn")
    # read before joining: rank 0 cannot exit while its result still sits in the queue's pipe
    seq, parent, pst = q.get(timeout=150)
    while not pc.join(timeout=60):
        pass
    uv = oracle.rmat(scale, 16, seed)
    oseq = oracle.degree_sequence(uv)
    p, s = oracle.build_tree(uv, oseq)
    assert np.array_equal(seq, oseq)
    assert np.array_equal(parent, p) and np.array_equal(pst, s)
