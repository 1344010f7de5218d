"""The lockstep multi-GPU tree build (sheep_ls_*, sheep_amd.dist.build_tree_lockstep) with the
real HIP kernels: P shards held in one process on cuda:0 (sheep_amd.dist.lockstep_local, the
all-gathers as device copies) and 2 ranks sharing cuda:0 over gloo (the product orchestration).
Every case is bit-exact against the CPU checker's serial graph2tree (seq, parent, pst)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _u32(t, n):
    return t[:n].cpu().numpy().view(np.uint32)


def _expect(oracle, uv, mode=0):
    oseq = oracle.degree_sequence(uv, mode) if mode else oracle.degree_sequence(uv)
    p, s = oracle.build_tree(uv, oseq)
    return oseq, p, s


def _run_local(uv_np, P, n_ids, mode=0):
    import torch

    from sheep_amd import device
    from sheep_amd.dist import lockstep_local, shard_bounds

    device.init(0)
    m = uv_np.shape[0]
    full = torch.from_numpy(uv_np.astype(np.uint32).view(np.int32)).to("cuda").view(torch.uint32)
    shards = []
    for r in range(P):
        lo, hi = shard_bounds(m, r, P)
        shards.append(full[lo:hi].contiguous())
    seq, parent, pst, n = lockstep_local(shards, n_ids, mode)
    torch.cuda.synchronize()
    return _u32(seq, n), _u32(parent, n), _u32(pst, n)


@pytest.mark.parametrize("scale,P", [(12, 1), (13, 2), (14, 3), (15, 5), (19, 2)])
def test_lockstep_local_rmat(oracle, scale, P):
    uv = oracle.rmat(scale, 16, 70 + scale)
    seq, parent, pst = _run_local(uv, P, 1 << scale)
    oseq, p, s = _expect(oracle, uv)
    assert np.array_equal(seq, oseq)
    assert np.array_equal(parent, p)
    assert np.array_equal(pst, s)


def test_lockstep_local_file_mode_powerlaw(oracle):
    uv = oracle.powerlaw(50000, 400000, 2.2, 20.0, 9)
    seq, parent, pst = _run_local(uv, 4, 50000, mode=1)
    oseq, p, s = _expect(oracle, uv, mode=1)
    assert np.array_equal(seq, oseq)
    assert np.array_equal(parent, p) and np.array_equal(pst, s)


@pytest.mark.parametrize("P", [3, 4, 12])
def test_lockstep_local_known_answer_and_empty_shards(oracle, P):
    # P = 12 > 10 records: two shards hold no record at all
    ka = np.array([[0, 1], [1, 0], [2, 2], [1, 2], [3, 4], [4, 1], [6, 5], [5, 6], [5, 6],
                   [2, 4]], np.uint32)
    seq, parent, pst = _run_local(ka, P, 7)
    assert seq.tolist() == [3, 0, 2, 4, 5, 6, 1]
    assert parent.tolist() == [3, 6, 3, 6, 5, 0xFFFFFFFF, 0xFFFFFFFF]
    assert pst.tolist() == [1, 2, 2, 1, 3, 0, 0]


def _worker(rank, world, port, scale, seed, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sheep_amd import device
        from sheep_amd.dist import DeviceOps, build_tree_lockstep, shard_bounds

        device.init(0)
        m = 16 << scale
        lo, hi = shard_bounds(m, rank, world)
        uv = device.rmat(scale, 16, seed, lo, hi)
        seq, parent, pst, n = build_tree_lockstep(uv, 1 << scale, DeviceOps())
        torch.cuda.synchronize()
        q.put((rank, _u32(seq, n).copy(), _u32(parent, n).copy(),
               _u32(pst, n).copy() if pst is not None else None))
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_lockstep_two_ranks_gloo_same_device(oracle):
    world, scale, seed = 2, 14, 81
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_worker, args=(world, _port(), scale, seed, q), nprocs=world,
                            join=False, start_method="spawn")
    got = dict((r, (a, b, c)) for r, a, b, c in (q.get(timeout=150) for _ in range(world)))
    while not pc.join(timeout=60):
        pass
    uv = oracle.rmat(scale, 16, seed)
    oseq, p, s = _expect(oracle, uv)
    for r in range(world):  # every rank holds the whole tree
        assert np.array_equal(got[r][0], oseq)
        assert np.array_equal(got[r][1], p)
    assert np.array_equal(got[0][2], s)
