#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats csv compactly: name, calls, avg/max/total ms per step."""
import csv
import sys

steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"].split("(")[0].replace("void ", "").replace("sheep::", "")
    print("%-32s calls %5s  avg %8.3f ms  max %8.3f ms  total/step %8.3f ms  %5s%%" % (
        n[:32], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["MaxNs"]) / 1e6,
        float(r["TotalDurationNs"]) / 1e6 / steps, r["Percentage"][:5]))
