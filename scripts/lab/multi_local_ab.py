#!/usr/bin/env python3
"""Lab: wall time of the P-rank driver run as P threads on one GPU (sheep_graph2tree_multi_local)
under option settings, e.g. the sharded sequence and the split apply on / off.  The ranks share
the GPU, so the wall time is the ranks' summed work, not one rank's latency.  One JSON line per
setting.

    python scripts/lab/multi_local_ab.py [--scale 26] [--P 8] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from sheep_amd import capi, device
    from sheep_amd.dist import shard_bounds

    device.init(0)
    torch.cuda.set_device(0)
    n_ids, m = 1 << args.scale, 16 << args.scale
    uv = device.rmat(args.scale, 16, args.scale)
    shards = [uv[slice(*shard_bounds(m, r, args.P))].contiguous() for r in range(args.P)]
    del uv
    ref = None
    for opts in [{"ls_seq": 0, "ls_split": 0}, {"ls_seq": 1, "ls_split": 0},
                 {"ls_seq": 0, "ls_split": 1}, {"ls_seq": 1, "ls_split": 1}]:
        for k, v in opts.items():
            capi.set_option(k, v)
        best = None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = device.graph2tree_multi_local(shards, n_ids)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        n = out[3]
        got = tuple(x[:n].cpu() for x in out[:3])
        if ref is None:
            ref = got
        same = all(torch.equal(a, b) for a, b in zip(ref, got))
        print(json.dumps({"P": args.P, "scale": args.scale, **opts, "wall_ms": round(1e3 * best, 2),
                          "same_as_first": same}), flush=True)
        del out


if __name__ == "__main__":
    main()
