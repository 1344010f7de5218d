"""Summary of scripts/pmc_front.sh output (one CSV per pass): per kernel, HBM bytes per launch
(FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE doubled for gfx950's wide-read undercount,
MI355X_MICROARCH.md), L2 hit rate, the
share of wave cycles waiting / issue-stalled / active, and instruction counts per launch.
  python scripts/pmc_table.py gpurun_out/pmc_front"""
import collections
import csv
import glob
import os
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "p_counter_collection.csv"))):
    pas = os.path.basename(os.path.dirname(path))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sheep::", "")[:34]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((pas, r["Dispatch_Id"]))
for k, d in tot.items():
    n = len([x for x in disp[k] if x[0] == "p1"]) or 1
    wc = d["SQ_WAVE_CYCLES"] or 1
    hit = d["TCC_HIT_sum"] / max(1, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    print("== %s launches %d" % (k, n))
    print("  per launch: FETCH x2 %.1f MB  WRITE %.1f MB  L2 hit %.2f" %
          (2 * d["FETCH_SIZE"] / n / 1e3, d["WRITE_SIZE"] / n / 1e3, hit))
    print("  wave cycles: wait %.2f issue-stall %.2f active %.2f | lds %.2f lds-stall %.2f valu %.2f" %
          tuple(d[c] / wc for c in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                    "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU"]))
    print("  insts per launch: lds %.3g (bank conflicts %.3g) vmem rd %.3g wr %.3g valu %.3g salu %.3g; waves %.3g" %
          tuple(d[c] / n for c in ["SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD",
                                   "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"]))
