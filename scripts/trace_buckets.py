#!/usr/bin/env python3
"""Per-bucket kernel time (us) of the kb tree build from a rocprofv3 --kernel-trace csv:
the last tree build in the trace (from the last launch that ends the grouping by hi:
k_edge_bin, k_bin_scatter or k_kb_bounds)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows)
       if any(k in r["Kernel_Name"] for k in ("k_kb_bounds", "k_edge_bin", "k_bin_scatter"))]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
last = rows[idx[which]:idx[which + 1]] if which != -1 else rows[idx[-1]:]
per = collections.defaultdict(lambda: collections.defaultdict(float))
tot = collections.defaultdict(float)
b = -1
t0 = int(last[0]["Start_Timestamp"])
t_end = t0
for r in last:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sheep::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "kb_map" in n or ("kb_union" in n and b >= 0 and "kb_union" in per[b]):
        b += 1
    if "kb_" not in n:
        continue
    if b < 0:
        b = 0
    per[b][n] += d
    tot[n] += d
    t_end = max(t_end, int(r["End_Timestamp"]))
for k in sorted(per):
    print(k, {n: round(v) for n, v in per[k].items()})
print("totals us", {n: round(v) for n, v in tot.items()}, "span us", (t_end - t0) / 1e3,
      "buckets", len(per))
