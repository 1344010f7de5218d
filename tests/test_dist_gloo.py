"""The sharded pipeline (sheep_amd.dist) on CPU with gloo: world_size 2, 3 and 4, edge shards
as graph2tree -l i/P, degree all-reduce, partial trees, pst sum-reduce + parent gather to
rank 0 and one P-way forest merge.
The per-rank kernels are the CPU checker here (test-only backend); the orchestration and the
collectives are the product code."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class CheckerOps:
    """Test-only stand-in for the HIP kernels: the CPU checker on torch CPU tensors."""

    def __init__(self, O):
        self.O = O
        self.seq = None

    def degree(self, uv, n_ids, mode):
        deg = torch.from_numpy(self.O.degree(uv.numpy(), mode, n_ids).astype(np.uint32))
        return deg, torch.zeros_like(deg)

    def sequence(self, deg):
        self.seq = self.O.sequence(deg.numpy().astype(np.uint32))
        rmap = np.full(deg.numel(), 0xFFFFFFFF, np.uint32)
        rmap[self.seq] = np.arange(len(self.seq), dtype=np.uint32)
        return torch.from_numpy(self.seq.copy()), torch.from_numpy(rmap), len(self.seq)

    def build_tree(self, uv, rmap, seq, n_seq, deg_local, selfc, mode):
        p, s = self.O.build_tree(uv.numpy(), self.seq)
        return torch.from_numpy(p.copy()), torch.from_numpy(s.copy())

    def merge_forests(self, stack, n):
        z = np.zeros(n, np.uint32)
        p = stack[0].numpy().copy()
        for r in range(1, stack.shape[0]):
            p, _ = self.O.merge(p, z, stack[r].numpy().copy(), z)
        return torch.from_numpy(np.ascontiguousarray(p))

    def now(self):
        import time

        return time.perf_counter()

    def lockstep(self, uv, rmap, seq, n_seq, deg):
        return CheckerLockstep(self.O, uv.numpy(), rmap.numpy(), self.seq, n_seq)

    def merge_into(self, pa, sa, pb, sb, n):
        p, s = self.O.merge(pa.numpy(), sa.numpy(), pb.numpy(), sb.numpy())
        pa.copy_(torch.from_numpy(p))
        sa.copy_(torch.from_numpy(s))


class CheckerLockstep:
    """Test-only stand-in for one rank's sheep_ls_* session: four rank bins as the buckets,
    every record of the bucket kept (no union-find), the tree built by the checker from the
    pairs gathered from all ranks.  Exercises the orchestration and its collectives."""

    def __init__(self, O, uv, rmap, seq, n_seq):
        self.O, self.uv, self.seq, self.n = O, uv, seq, n_seq
        x, y = rmap[uv[:, 0]].astype(np.uint64), rmap[uv[:, 1]].astype(np.uint64)
        keep = uv[:, 0] != uv[:, 1]
        lo, hi = np.minimum(x, y)[keep], np.maximum(x, y)[keep]
        self.bounds = [n_seq * i // 4 for i in range(4)] + [n_seq]
        self.items = [((hi << np.uint64(32)) | lo)[(hi >= self.bounds[k]) & (hi < self.bounds[k + 1])]
                      .view(np.int64) for k in range(4)]
        self.bin_counts = np.array([len(i) for i in self.items] + [int((~keep).sum())], np.int64)
        self.pairs = []

    def plan(self, global_counts):
        assert len(global_counts) == 5
        return 4, 1

    def map(self, k, send, count=None):
        n = len(self.items[k])
        send[1:1 + n] = torch.from_numpy(self.items[k])
        self.n_kept = n
        if count is None:
            return n
        count.fill_(n)

    def pack(self, k, send, cap):
        send[0] = 0
        send[1 + self.n_kept:1 + cap] = -1

    def apply(self, k, recv, P, cap):
        for r in range(P):
            blk = recv[r * (1 + cap) + 1:(r + 1) * (1 + cap)].numpy().view(np.uint64)
            self.pairs.append(blk[blk != np.uint64(2 ** 64 - 1)])

    def finish(self, seq, deg_local, selfc, mode):
        it = np.concatenate(self.pairs) if self.pairs else np.zeros(0, np.uint64)
        hi, lo = (it >> np.uint64(32)).astype(np.int64), (it & np.uint64(0xFFFFFFFF)).astype(np.int64)
        uv = np.stack([self.seq[lo], self.seq[hi]], axis=1).astype(np.uint32)
        parent, _ = self.O.build_tree(uv, self.seq)
        _, pst = self.O.build_tree(self.uv, self.seq)
        return torch.from_numpy(parent.copy()), torch.from_numpy(pst.copy())

    def free(self):
        pass


def _worker(rank, world, port, scale, result_q, lockstep=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from sheep_amd.dist import build_tree_lockstep, build_tree_sharded, shard_bounds

        m = 16 << scale
        lo, hi = shard_bounds(m, rank, world)
        uv = torch.from_numpy(O.rmat(scale, 16, 3, lo, hi).astype(np.uint32))
        build = build_tree_lockstep if lockstep else build_tree_sharded
        seq, parent, pst, n = build(uv, 1 << scale, CheckerOps(O))
        if rank == 0:
            result_q.put((seq.numpy().copy(), parent.numpy().copy(), pst.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,lockstep", [(2, False), (3, False), (4, False), (2, True),
                                            (3, True)])
def test_sharded_equals_serial(oracle, world, lockstep):
    scale = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_worker, args=(world, _free_port(), scale, q, lockstep), nprocs=world,
                            join=False, start_method="spawn")
    # read before joining: rank 0 cannot exit while its result still sits in the queue's pipe
    seq, parent, pst = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    uv = oracle.rmat(scale, 16, 3)
    oseq = oracle.degree_sequence(uv)
    p, s = oracle.build_tree(uv, oseq)
    assert np.array_equal(seq, oseq)
    assert np.array_equal(parent, p) and np.array_equal(pst, s)


def test_shard_bounds_cover():
    from sheep_amd.dist import shard_bounds

    for m in (0, 1, 7, 1000):
        for P in (1, 2, 3, 8):
            b = [shard_bounds(m, r, P) for r in range(P)]
            assert b[0][0] == 0 and b[-1][1] == m
            assert all(b[i][1] == b[i + 1][0] for i in range(P - 1))
