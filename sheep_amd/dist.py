"""Edge-sharded multi-GPU tree construction: one process per GPU, torch.distributed over RCCL.

This is the MI355X replacement of graph2tree -i -r (graph2tree.cpp:134-200):
  1. every rank holds a contiguous shard of the edge records (graph_wrapper.h:48-49, -l i/P);
  2. per-rank degrees are summed with ONE all-reduce over xGMI (mpiSequence's MPI_Allreduce,
     sequence.h:78) and every rank derives the identical seq/rank map on its own GPU;
  3. every rank builds its partial elimination tree (jtree.cpp:112-145 on its shard);
  4. the partial trees are reduced to rank 0 (mpi_merge's MPI_Reduce with the merge op,
     jnode.cpp:213-250): pst_weight with ONE sum-reduce (the merge adds them, jnode.cpp:
     174-201), the parent arrays with one gather, after which rank 0 builds the elimination
     tree of the union of all P forests in a single pass (sheep_merge_forests_dev).  Pairwise
     merging (the reference's reduce tree, and scripts/reduce-worker.sh) would put log2(P)
     dependent merges on the critical path; the merge is exact and associative, so one
     P-way merge gives the same tree.
The result equals the serial tree for any P.

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
    if world == 1:
        return seq, parent, pst, n_seq
    if timings is not None:
        timings["partial_tree"] = ops.now()
    dist.reduce(_i32(pst), dst=0, op=dist.ReduceOp.SUM, group=group)
    mine = parent[:n_seq].contiguous()
    if rank == 0:
        stack = torch.empty((world, n_seq), dtype=parent.dtype, device=parent.device)
        dist.gather(_i32(mine), gather_list=[_i32(stack[r]) for r in range(world)], dst=0,
                    group=group)
        if timings is not None:
            timings["gather"] = ops.now()
        parent = ops.merge_forests(stack, n_seq)
        return seq, parent, pst, n_seq
    dist.gather(_i32(mine), dst=0, group=group)
    return seq, None, None, n_seq


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
        out = self.d.build_tree_deg(uv, rmap, seq, n_seq, deg_local, selfc, mode)
        from . import capi

        self.build_timings = capi.last_timings()  # this rank's partial tree, for the bench
        return out

    def merge_into(self, pa, sa, pb, sb, n):
        self.d.merge_into(pa, sa, pb, sb, n)

    def merge_forests(self, stack, n):
        return self.d.merge_forests(stack, n)

    def now(self):
        import time

        torch.cuda.synchronize()
        return time.perf_counter()
