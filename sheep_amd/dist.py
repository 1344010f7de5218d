"""Edge-sharded multi-GPU tree construction: one process per GPU, torch.distributed over RCCL.

This is the MI355X replacement of graph2tree -i -r (graph2tree.cpp:134-200):
  1. every rank holds a contiguous shard of the edge records (graph_wrapper.h:48-49, -l i/P);
  2. per-rank degrees are summed with ONE all-reduce over xGMI (mpiSequence's MPI_Allreduce,
     sequence.h:78) and every rank derives the identical seq/rank map on its own GPU;
  3. every rank builds its partial elimination tree (jtree.cpp:112-145 on its shard);
  4. partial trees are combined by a log2(P) pairwise reduce to rank 0 (mpi_merge's
     MPI_Reduce with the merge op, jnode.cpp:213-250; scripts/reduce-worker.sh's pairing):
     at step s, rank r with r % 2s == s sends (parent, pst) to r - s, which merges in place.
The merge is exact and associative, so the result equals the serial tree for any P.

The kernel operations are injected (``ops``) so the same orchestration runs on the GPU
(``sheep_amd.device``) and, in the CPU gloo tests, on a test-only backend.
"""
import torch
import torch.distributed as dist


def _i32(t):
    return t.view(torch.int32)


def shard_bounds(m, rank, world):
    """Contiguous record range of a rank: [m*r/P, m*(r+1)/P) (the -l part/num_parts split)."""
    return m * rank // world, m * (rank + 1) // world


def build_tree_sharded(uv_shard, n_ids, ops, mode=0, group=None, timings=None):
    """Returns (seq, parent, pst, n_seq) on rank 0 and (seq, None, None, n_seq) elsewhere."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    deg_local, selfc = ops.degree(uv_shard, n_ids, mode)
    deg = deg_local.clone() if world > 1 else deg_local
    if world > 1:
        dist.all_reduce(_i32(deg), op=dist.ReduceOp.SUM, group=group)
    seq, rmap, n_seq = ops.sequence(deg)
    # pst of the partial tree comes from this shard's own degrees (pre-all-reduce)
    parent, pst = ops.build_tree(uv_shard, rmap, seq, n_seq, deg_local, selfc, mode)
    step = 1
    while step < world:
        if rank % (2 * step) == 0:
            src = rank + step
            if src < world:
                pb = torch.empty_like(parent)
                sb = torch.empty_like(pst)
                dist.recv(_i32(pb), src=src, group=group)
                dist.recv(_i32(sb), src=src, group=group)
                ops.merge_into(parent, pst, pb, sb, n_seq)
        elif rank % (2 * step) == step:
            dist.send(_i32(parent), dst=rank - step, group=group)
            dist.send(_i32(pst), dst=rank - step, group=group)
            return seq, None, None, n_seq
        step *= 2
    return seq, parent, pst, n_seq


class DeviceOps:
    """The HIP kernels behind the C-ABI, on torch's current stream."""

    def __init__(self):
        from . import device

        self.d = device

    def degree(self, uv, n_ids, mode):
        return self.d.degree_ex(uv, n_ids, mode)

    def sequence(self, deg):
        return self.d.sequence(deg)

    def build_tree(self, uv, rmap, seq, n_seq, deg_local, selfc, mode):
        return self.d.build_tree_deg(uv, rmap, seq, n_seq, deg_local, selfc, mode)

    def merge_into(self, pa, sa, pb, sb, n):
        self.d.merge_into(pa, sa, pb, sb, n)
