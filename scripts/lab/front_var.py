#!/usr/bin/env python3
"""Lab: run-to-run variation of the front half (degree pass beside the first partition pass):
per repetition of graph2tree on RMAT-26, the degree / part_first / sequence / partition phases.
One JSON line per process.

    python scripts/lab/front_var.py [--scale 26] [--reps 6]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


COLS = ("degree_sample", "front_fused", "degree_hist", "degree", "part_first", "sequence",
        "partition", "edge_pass", "tree_insert")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    from sheep_amd import capi, device

    device.init(0)
    uv, n_ids = device.rmat(a.scale, 16, a.scale), 1 << a.scale
    torch.cuda.synchronize()
    rows = []
    for _ in range(a.reps + 1):
        device.graph2tree(uv, n_ids)
        torch.cuda.synchronize()
        t = dict(capi.last_timings())
        rows.append([round(t.get(k, 0), 2) for k in COLS])
    print(json.dumps({"hwq": os.environ.get("GPU_MAX_HW_QUEUES"), "cols": " ".join(COLS), "reps": rows[1:]}), flush=True)


if __name__ == "__main__":
    main()
