#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer boundary.

graph2tree's serial call sequence through the C-ABI with HOST buffers, as the reference's
lib/ binds it (sequence.h degreeSequence -> sheep_degree_seq, JTree -> sheep_build_tree): the
edge records live in pageable host memory (a numpy array, as LLAMA's graph lives in RAM), each
call uploads them, and seq / parent / pst come back to the host.  This is never bench.py's
`value` (that one starts with the records resident in HBM); it is the rate a CLI user sees.

    python scripts/host_boundary_bench.py [--scale 26] [--steps 3]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=26)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()

    from sheep_amd import api, device

    torch.cuda.set_device(0)
    device.init(0)
    n_ids = 1 << args.scale
    uv_d = device.rmat(args.scale, args.edgefactor, args.seed)
    torch.cuda.synchronize()
    uv = uv_d.cpu().numpy()  # pageable host copy; the device copy is freed before timing
    del uv_d
    torch.cuda.empty_cache()
    m = uv.shape[0]

    seq = api.degree_sequence(uv, n_ids=n_ids)  # warm-up: scratch allocation, code objects
    api.build_tree(uv, seq)
    t_sort, t_map = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        seq = api.degree_sequence(uv, n_ids=n_ids)
        t1 = time.perf_counter()
        tree = api.build_tree(uv, seq)
        t2 = time.perf_counter()
        t_sort.append(t1 - t0)
        t_map.append(t2 - t1)
    sort_s, map_s = float(np.median(t_sort)), float(np.median(t_map))
    print(json.dumps({
        "what": "host-pointer boundary, PCIe-inclusive (sheep_degree_seq + sheep_build_tree "
                "from pageable host records; two uploads of 8 B/record, seq/parent/pst back)",
        "workload": "rmat%d_ef%d" % (args.scale, args.edgefactor), "records": m,
        "n_seq": int(seq.size), "sorted_s": sort_s, "mapped_s": map_s,
        "edges_per_s": m / (sort_s + map_s), "steps": args.steps,
        "roots": int((tree.parent == 0xFFFFFFFF).sum()),
    }), flush=True)


if __name__ == "__main__":
    main()
