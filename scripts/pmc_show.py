#!/usr/bin/env python3
"""Print per-kernel PMC sums of rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE in GB, as the
counters report them: FETCH_SIZE is raw, not doubled; others as counted).

    python scripts/pmc_show.py gpurun_out/pmc_fh [REGEX]"""
import collections
import csv
import glob
import re
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sheep::", "")
        if len(sys.argv) > 2 and not re.search(sys.argv[2], k):
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print("%-34s %s" % (k[:34], "  ".join("%s=%s" % (c, ("%.2fGB" % (x * 1024 / 1e9)) if "SIZE" in c
                                                    else "%.3g" % x) for c, x in sorted(v.items()))))
