"""Per-launch durations of one kernel from a rocprofv3 kernel_trace csv, in dispatch order:
    python scripts/trace_map.py TRACE.csv k_kb_map [skip_launches]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[skip:]]
print("launches", len(d), "total_us %.1f" % sum(d))
print(" ".join("%.0f" % x for x in d))
