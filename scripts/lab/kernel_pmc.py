#!/usr/bin/env python3
"""Sum one counter per kernel (name prefix match) over a rocprofv3 --pmc output directory.
    python scripts/lab/kernel_pmc.py DIR COUNTER [kernel-prefix ...]"""
import collections
import csv
import glob
import os
import re
import sys

d, counter = sys.argv[1], sys.argv[2]
pref = sys.argv[3:] or ["k_front_fused", "k_part", "k_edge_bin", "k_degb_hist16s"]
tot = collections.defaultdict(float)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sheep::", "")
        for p in pref:
            if k.startswith(p):
                tot[p] += float(r["Counter_Value"])
for p in pref:
    print("%-16s %s %.3f GB" % (p, counter, tot[p] * 1024 / 1e9))
