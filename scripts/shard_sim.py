#!/usr/bin/env python3
"""Lab: the P-rank edge-sharded pipeline (sheep_amd/dist.py) simulated on ONE GPU.

Each rank's work runs back to back on cuda:0 and is timed on its own, so the critical path
of a real P-GPU run can be estimated: max over ranks of (degree), the degree all-reduce
(not simulated: a sum on one GPU), the sequence, max over ranks of (partial tree), then
the P-way forest merge on rank 0 (gather and pst reduce not simulated).
The merged tree is checked against the single-GPU tree.

    python scripts/shard_sim.py [--scale 26] [--ranks 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sheep_amd import capi, device  # noqa: E402
from sheep_amd.dist import shard_bounds  # noqa: E402


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = fn()
    e.record()
    torch.cuda.synchronize()
    return out, s.elapsed_time(e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--seed", type=int, default=26)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    device.init(0)
    m, n_ids = 16 << a.scale, 1 << a.scale
    P = a.ranks
    shards = []
    for r in range(P):
        lo, hi = shard_bounds(m, r, P)
        shards.append(device.rmat(a.scale, 16, a.seed, lo, hi))
    torch.cuda.synchronize()
    res = {}
    for rep in range(a.reps):
        t_deg, degs = [], []
        for sh in shards:
            (d, sc), t = timed(lambda: device.degree_ex(sh, n_ids))
            degs.append((d, sc))
            t_deg.append(t)
        deg = degs[0][0].view(torch.int32).clone()
        for d, _ in degs[1:]:
            deg += d.view(torch.int32)
        deg = deg.view(torch.uint32)
        (seq, rank, n_seq), t_seq = timed(lambda: device.sequence(deg))
        trees, t_build = [], []
        for sh, (d, sc) in zip(shards, degs):
            tr, t = timed(lambda: device.build_tree_deg(sh, rank, seq, n_seq, d, sc))
            phases = {k: round(v, 3) for k, v in capi.last_timings()}
            trees.append(tr)
            t_build.append(t)
        pst = trees[0][1].view(torch.int32).clone()
        for _, s_ in trees[1:]:
            pst += s_.view(torch.int32)
        stack = torch.stack([p[:n_seq] for p, _ in trees])
        merged, t_merge = timed(lambda: device.merge_forests(stack, n_seq))
        merge_phases = {k: round(v, 3) for k, v in capi.last_timings()}
        rounds = [t_merge]
        nonroot = [int((p[:n_seq].view(torch.int32) != -1).sum()) for p, _ in trees[:1]]
        res = {"P": P, "scale": a.scale, "n_seq": n_seq,
               "degree_ms": [round(x, 3) for x in t_deg], "sequence_ms": round(t_seq, 3),
               "build_ms": [round(x, 3) for x in t_build], "merge_round_ms": [round(x, 3) for x in rounds],
               "critical_ms_no_comm": round(max(t_deg) + t_seq + max(t_build) + sum(rounds), 3),
               "rank0_tree_edges": nonroot[0], "last_build_phases": phases,
               "merge_phases": merge_phases}
    # check against the single-GPU tree
    uv = device.rmat(a.scale, 16, a.seed)
    s1, p1, w1, n1 = device.graph2tree(uv, n_ids)
    p0, w0 = merged, pst.view(torch.uint32)
    res["bit_exact_vs_single"] = bool(n1 == n_seq and torch.equal(p1[:n1].view(torch.int32), p0[:n1].view(torch.int32))
                                      and torch.equal(w1[:n1].view(torch.int32), w0[:n1].view(torch.int32)))
    (_, t1) = timed(lambda: device.graph2tree(uv, n_ids))
    res["single_gpu_ms"] = round(t1, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
