#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE in separate runs,
as MI355X_MICROARCH.md prescribes) -> profiles/pmc_traffic.json[key].

    python scripts/pmc_summary.py KEY FETCH_DIR WRITE_DIR [--steps S]

FETCH_SIZE / WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE counts 1/2 of a wide (16 B/lane)
coalesced streaming read; the other access widths of this path (8-B streams, 4-B random
gathers) are uncalibrated, so hbm_bytes_per_launch is the raw sum and the x2 column is given
beside it."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d, counter):
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return tot, n


def main():
    key, fdir, wdir = sys.argv[1:4]
    fet, nf = load(fdir, "FETCH_SIZE")
    wr, nw = load(wdir, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fet) | set(wr)):
        launches = max(nf.get(k, 0), nw.get(k, 0))
        f = fet.get(k, 0.0) / max(nf.get(k, 1), 1)
        w = wr.get(k, 0.0) / max(nw.get(k, 1), 1)
        out[k] = {"launches": launches, "FETCH_SIZE_KB_per_launch": f,
                  "WRITE_SIZE_KB_per_launch": w, "hbm_bytes_per_launch": (f + w) * 1024,
                  "hbm_bytes_per_launch_fetch_x2": (2 * f + w) * 1024}
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    tab = json.load(open(path)) if os.path.exists(path) else {}
    tab[key] = out
    json.dump(tab, open(path, "w"), indent=1, sort_keys=True)
    print("wrote %d kernels under %s" % (len(out), key))


if __name__ == "__main__":
    main()
