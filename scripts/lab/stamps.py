#!/usr/bin/env python3
"""Per-phase clock split of the stamped kernels (scripts/lab/stamp_build.py) over graph2tree
steps: for each kernel, the shader clocks thread 0 of each block spent between consecutive
barriers, summed over blocks, as fractions of the kernel's total.  Run on the GPU box with the
lab library in place of sheep_amd/libsheep_amd.so.

    python scripts/lab/stamps.py [--scale 26] [--steps 3] [--names k_front_fused k_edge_bin k_part]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--workload", default="rmat")
    ap.add_argument("--names", nargs="+", default=["k_front_fused", "k_edge_bin", "k_part"])
    ap.add_argument("--raw", action="store_true", help="print the first 16 counters as they are")
    args = ap.parse_args()
    import torch

    from sheep_amd import capi, device

    device.init(0)
    if args.workload == "rmat":
        n_ids = 1 << args.scale
        uv = device.rmat(args.scale, 16, args.scale)
    else:
        n_ids, m, g, i0, seed = device.POWERLAW[args.workload]
        uv = device.powerlaw(n_ids, m, g, i0, seed)
    L = capi.lib()
    buf = (ctypes.c_ulonglong * 256)()
    device.graph2tree(uv, n_ids)
    torch.cuda.synchronize()
    L.sheep_lab_stamps(buf, 256)  # clears
    for _ in range(args.steps):
        device.graph2tree(uv, n_ids)
    torch.cuda.synchronize()
    phases = dict(capi.last_timings())
    L.sheep_lab_stamps(buf, 256)
    out = {"workload": args.workload, "scale": args.scale, "steps": args.steps,
           "phases_ms": {k: round(v, 3) for k, v in phases.items() if not k.endswith("#")}}
    if args.raw:
        out["raw"] = [int(buf[i]) for i in range(16)]
        # (the refresh-count lab build: (B0, giant-member misses) per bucket in slots 16 ..)
        per = sorted((int(buf[16 + 2 * i]), int(buf[17 + 2 * i])) for i in range(113)
                     if buf[17 + 2 * i])
        if per:
            out["per_bucket"] = per
    for kid, name in enumerate([] if args.raw else args.names):
        v = [int(buf[16 * kid + i]) for i in range(16)]
        tot = sum(v)
        if tot:
            out[name] = {"clocks_G": round(tot / 1e9, 3),
                         "frac": [round(x / tot, 3) for x in v if x]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
