#!/usr/bin/env python3
"""Tree-insert variant lab: times every SHEEP_TREE_VARIANT on one R-MAT graph, checks that all
variants give the identical tree, and prints the step/CAS counters of an instrumented run."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sheep_amd import capi, device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=24)
ap.add_argument("--variants", default="zip:12,kb:128,kb:512,kb:2048")
ap.add_argument("--reps", type=int, default=2)
args = ap.parse_args()
device.init(0)
S = args.scale
uv = device.rmat(S, 16, S)
deg = device.degree(uv, 1 << S)
seq, rank, n_seq = device.sequence(deg)
torch.cuda.synchronize()
print("scale", S, "records", uv.shape[0], "n_seq", n_seq, flush=True)
ref = None
for v in args.variants.split(","):
    algo, knob = v.split(":")
    os.environ["SHEEP_TREE_ALGO"] = algo
    os.environ["SHEEP_TREE_VARIANT" if algo == "zip" else "SHEEP_KB_BUCKETS"] = knob
    os.environ["SHEEP_TREE_STATS"] = "0"
    best = 1e9
    for _ in range(args.reps):
        t0 = time.perf_counter()
        parent, pst = device.build_tree(uv, rank, n_seq)
        torch.cuda.synchronize()
        ph = dict(capi.last_timings())
        best = min(best, ph["tree_insert"])
    same = None
    if ref is None:
        ref = (parent.clone(), pst.clone())
    else:
        same = bool(torch.equal(parent, ref[0]) and torch.equal(pst, ref[1]))
    os.environ["SHEEP_TREE_STATS"] = os.environ.get("LAB_STATS", "1")
    device.build_tree(uv, rank, n_seq)
    torch.cuda.synchronize()
    print("variant %s tree_insert %.2f ms  other %s  same=%s" % (
        v, best, {k: round(x, 2) for k, x in ph.items() if k != "tree_insert"}, same), flush=True)
