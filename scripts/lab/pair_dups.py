#!/usr/bin/env python3
"""Lab: how many of the split lockstep's kept pairs (b, root) are repeats, per rank and over all
ranks?  Runs the one-GPU lockstep rehearsal (sheep_amd.dist.lockstep_local's loop, split) at
P ranks and counts distinct pairs per bucket with torch.unique.  One JSON line.

    python scripts/lab/pair_dups.py [--scale 26] [--P 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--P", type=int, default=8)
    args = ap.parse_args()
    from sheep_amd import device
    from sheep_amd.dist import shard_bounds

    device.init(0)
    torch.cuda.set_device(0)
    n_ids, m, P = 1 << args.scale, 16 << args.scale, args.P
    uv = device.rmat(args.scale, 16, args.scale)
    shards = [uv[slice(*shard_bounds(m, r, P))] for r in range(P)]
    parts = [device.degree_ex(x, n_ids, 0) for x in shards]
    deg = parts[0][0].clone()
    for d, _ in parts[1:]:
        deg.view(torch.int32).add_(d.view(torch.int32))
    seq, rmap, n_seq = device.sequence(deg)
    sess = [device.Lockstep(x, rmap, seq, n_seq, deg) for x in shards]
    tot = {"kept": 0, "distinct_rank": 0, "distinct_all": 0, "distinct_g_all": 0}
    per_bucket = []
    try:
        g = np.sum([s.bin_counts for s in sess], axis=0)
        nbk, slots = [s.plan(g) for s in sess][0]
        for r, s in enumerate(sess):
            s.split(r, P)
        sends = [torch.empty(slots + max(x.shape[0], 1), dtype=torch.int64, device=uv.device)
                 for x in shards]
        for k in range(nbk):
            ns = [s.map(k, sends[r]) for r, s in enumerate(sess)]
            cap = max(ns)
            pairs = [sends[r][slots:slots + ns[r]].clone() for r in range(P)]
            dr = sum(int(torch.unique(p).numel()) for p in pairs)
            allp = torch.cat(pairs)
            da = int(torch.unique(allp).numel())
            dg = int(torch.unique(allp & 0xFFFFFFFF).numel())
            tot["kept"] += sum(ns)
            tot["distinct_rank"] += dr
            tot["distinct_all"] += da
            tot["distinct_g_all"] += dg
            per_bucket.append([k, sum(ns), dr, da, dg])
            for r, s in enumerate(sess):
                if sends[r].numel() < slots + cap:
                    grown = torch.empty(slots + cap, dtype=torch.int64, device=uv.device)
                    grown[:sends[r].numel()].copy_(sends[r])
                    sends[r] = grown
                s.pack(k, sends[r], cap)
            recv = torch.cat([x[:slots + cap] for x in sends])
            for s in sess:
                s.apply(k, recv, P, cap)
        for r, s in enumerate(sess):
            s.finish(seq, parts[r][0], parts[r][1], 0)
    finally:
        for s in sess:
            s.free()
    print(json.dumps({"P": P, "scale": args.scale, **tot, "buckets": per_bucket}))


if __name__ == "__main__":
    main()
