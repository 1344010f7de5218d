"""Sum rocprofv3 --pmc counter_collection.csv rows of one kernel: per-counter totals and per
launch means.   python scripts/pmc_kernel.py COUNTERS.csv KERNEL_SUBSTRING"""
import collections
import csv
import sys

tot = collections.defaultdict(float)
disp = set()
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] not in r["Kernel_Name"]:
        continue
    disp.add(r["Dispatch_Id"])
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(len(disp), 1)
print("dispatches", len(disp))
for k, v in sorted(tot.items()):
    print("%-28s total %.4g  per-launch %.4g" % (k, v, v / n))
