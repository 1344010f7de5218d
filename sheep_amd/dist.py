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


def _all_gather(recv, send, group):
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        n = send.numel()
        dist.all_gather([recv[r * n:(r + 1) * n] for r in range(recv.numel() // n)], send,
                        group=group)


def _lockstep_loop(ls, nbk, slots, m_local, world, dev, group):
    """Bucket by bucket: map, MAX of the kept counts, pack, all-gather, apply."""
    send = torch.empty(slots + max(m_local, 1), dtype=torch.int64, device=dev)
    recv = torch.empty(0, dtype=torch.int64, device=dev)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    for k in range(nbk):
        if world > 1:  # one host round trip per bucket: the MAX of the kept counts
            ls.map(k, send, cnt)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
            cap = int(cnt.item())
        else:
            cap = ls.map(k, send)
        width = slots + cap
        if send.numel() < width:  # another rank kept more pairs than this one has records
            grown = torch.empty(width, dtype=torch.int64, device=dev)
            grown[:send.numel()].copy_(send)
            send = grown
        ls.pack(k, send, cap)
        if recv.numel() < world * width:
            recv = torch.empty(world * width, dtype=torch.int64, device=dev)
        if world > 1:
            _all_gather(recv[:world * width], send[:width], group)
        else:
            recv[:width].copy_(send[:width])
        ls.apply(k, recv, world, cap)


def _lockstep_loop_pipelined(ls, nbk, slots, m_local, world, dev, group):
    """The same loop with bucket k+1 mapped and exchanged on a side stream while bucket k is
    applied on the current one (the session double-buffers by bucket parity): the map and the
    collectives hide behind the apply, which is the serial part."""
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    send = [torch.empty(slots + max(m_local, 1), dtype=torch.int64, device=dev)]
    recv = [torch.empty(0, dtype=torch.int64, device=dev) for _ in range(2)]
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    applied = [torch.cuda.Event(), torch.cuda.Event()]
    exchanged = [torch.cuda.Event(), torch.cuda.Event()]
    caps = {}

    def produce(k):  # on the side stream; the host waits only for the count's MAX
        with torch.cuda.stream(side):
            ls.map(k, send[0], cnt)
            dist.all_reduce(cnt, op=dist.ReduceOp.MAX, group=group)
            cap = int(cnt.item())
            width = slots + cap
            if send[0].numel() < width:
                grown = torch.empty(width, dtype=torch.int64, device=dev)
                grown[:send[0].numel()].copy_(send[0])
                send[0] = grown
            ls.pack(k, send[0], cap)
            r = recv[k & 1]
            if r.numel() < world * width:
                r = recv[k & 1] = torch.empty(world * width, dtype=torch.int64, device=dev)
            _all_gather(r[:world * width], send[0][:width], group)
            exchanged[k & 1].record(side)
        caps[k] = cap

    side.wait_stream(main)
    produce(0)
    for k in range(nbk):
        main.wait_event(exchanged[k & 1])
        ls.apply(k, recv[k & 1], world, caps.pop(k))
        applied[k & 1].record(main)
        if k + 1 < nbk:
            if k >= 1:  # bucket k+1 reuses the parity buffers of bucket k-1
                side.wait_event(applied[(k + 1) & 1])
            produce(k + 1)
    main.wait_stream(side)


def build_tree_lockstep(uv_shard, n_ids, ops, mode=0, group=None, timings=None, split=True):
    """graph2tree -i -r without partial trees (the default for P > 1).

    Steps 1-2 as build_tree_sharded.  Then every rank bins ITS records by hi (bins from the
    global degrees) and the ranks walk the kb rank buckets together: each maps its own records
    of the bucket against its replica of the union-find, the kept pairs and giant marks of all
    ranks are all-gathered over RCCL, and every rank applies all of them, so the replicas stay
    identical and every rank ends with the whole elimination tree.  pst_weight is the sum of
    the ranks' own pst (one sum-reduce to rank 0, as mpi_merge's merge adds them).
    split (P > 1, when the session supports it): every rank applies the union-find part of
    every bucket but the zipper of its own buckets only (k mod P); the disjoint forests are
    summed at the end.
    Returns (seq, parent, pst, n_seq) on rank 0 and (seq, parent, None, n_seq) elsewhere."""
    import numpy as np

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = uv_shard.device
    deg_local, selfc = ops.degree(uv_shard, n_ids, mode)
    deg = deg_local.clone() if world > 1 else deg_local
    if world > 1:
        dist.all_reduce(_i32(deg), op=dist.ReduceOp.SUM, group=group)
    seq, rmap, n_seq = ops.sequence(deg)
    ls = ops.lockstep(uv_shard, rmap, seq, n_seq, deg)
    try:
        counts = torch.from_numpy(np.ascontiguousarray(ls.bin_counts)).to(dev)
        if world > 1:
            dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        nbk, slots = ls.plan(counts.cpu().numpy())
        split = world > 1 and split and hasattr(ls, "split")
        if split:  # bucket k's zipper on rank k mod P only (sheep_ls_split)
            ls.split(rank, world)
        if timings is not None:
            timings["binned"] = ops.now()
        if dist.is_initialized() and dev.type == "cuda":
            _lockstep_loop_pipelined(ls, nbk, slots, uv_shard.shape[0], world, dev, group)
        else:
            _lockstep_loop(ls, nbk, slots, uv_shard.shape[0], world, dev, group)
        parent, pst = ls.finish(seq, deg_local, selfc, mode)
    finally:
        ls.free()
    if split:  # the ranks' forests are disjoint: sum parent + 1 (INVALID + 1 = 0)
        p = _i32(parent[:n_seq])
        p.add_(1)
        dist.all_reduce(p, op=dist.ReduceOp.SUM, group=group)
        p.sub_(1)
    if timings is not None:
        timings["tree"] = ops.now()
    if world > 1:
        dist.reduce(_i32(pst), dst=0, op=dist.ReduceOp.SUM, group=group)
    return seq, parent, (pst if rank == 0 else None), n_seq


def lockstep_local(shards, n_ids, mode=0, stats=None, split=True):
    """The lockstep build of build_tree_lockstep for P shards held by ONE process on one
    device (the all-gathers become device copies): the one-GPU rehearsal of the P-rank path.
    stats (dict, optional) receives per-rank kernel times {"kb_map": [...], "kb_apply": [...]}.
    Returns (seq, parent, pst, n_seq)."""
    import numpy as np

    from . import capi, device

    P = len(shards)
    dev = shards[0].device
    parts = [device.degree_ex(uv, n_ids, mode) for uv in shards]
    deg = parts[0][0].clone()
    for d, _ in parts[1:]:
        deg.view(torch.int32).add_(d.view(torch.int32))
    seq, rmap, n_seq = device.sequence(deg)
    sess = [device.Lockstep(uv, rmap, seq, n_seq, deg) for uv in shards]
    try:
        g = np.sum([s.bin_counts for s in sess], axis=0)
        plans = [s.plan(g) for s in sess]
        nbk, slots = plans[0]
        split = split and P > 1
        if split:
            for r, s in enumerate(sess):
                s.split(r, P)
        sends = [torch.empty(slots + max(uv.shape[0], 1), dtype=torch.int64, device=dev)
                 for uv in shards]
        for k in range(nbk):
            ns = [s.map(k, sends[r]) for r, s in enumerate(sess)]
            cap = max(ns)
            if stats is not None:
                stats["kept"] = stats.get("kept", 0) + sum(ns)
                stats["gathered"] = stats.get("gathered", 0) + P * cap
            for r, s in enumerate(sess):
                if sends[r].numel() < slots + cap:
                    grown = torch.empty(slots + cap, dtype=torch.int64, device=dev)
                    grown[:sends[r].numel()].copy_(sends[r])
                    sends[r] = grown
                s.pack(k, sends[r], cap)
            recv = torch.cat([x[:slots + cap] for x in sends])
            for s in sess:
                s.apply(k, recv, P, cap)
        pst = None
        parent = None
        for r, s in enumerate(sess):
            p, w = s.finish(seq, parts[r][0], parts[r][1], mode)
            if stats is not None:
                for name, ms in capi.last_timings():
                    stats.setdefault(name, []).append(ms)
            if split:  # disjoint forests: sum parent + 1 (INVALID + 1 = 0)
                p.view(torch.int32).add_(1)
            if parent is None:
                parent, pst = p, w
            else:
                if split:
                    parent.view(torch.int32).add_(p.view(torch.int32))
                elif not torch.equal(parent[:n_seq], p[:n_seq]):
                    raise RuntimeError("lockstep replicas diverged at rank %d" % r)
                pst.view(torch.int32).add_(w.view(torch.int32))
        if split:
            parent.view(torch.int32).sub_(1)
    finally:
        for s in sess:
            s.free()
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
        out = self.d.build_tree_deg(uv, rmap, seq, n_seq, deg_local, selfc, mode)
        from . import capi

        self.build_timings = capi.last_timings()  # this rank's partial tree, for the bench
        return out

    def lockstep(self, uv, rmap, seq, n_seq, deg):
        return self.d.Lockstep(uv, rmap, seq, n_seq, deg)

    def merge_into(self, pa, sa, pb, sb, n):
        self.d.merge_into(pa, sa, pb, sb, n)

    def merge_forests(self, stack, n):
        return self.d.merge_forests(stack, n)

    def now(self):
        import time

        torch.cuda.synchronize()
        return time.perf_counter()
