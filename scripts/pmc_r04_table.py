#!/usr/bin/env python3
"""Per-kernel counter table from scripts/pmc_r04.sh passes (one CSV per pass) plus the kernel
trace stats of the same command: per step, the kernel's time, HBM bytes (FETCH_SIZE x2 for
gfx950's wide-read undercount and raw, WRITE_SIZE), L2 hit rate, L2 atomics, LDS instructions
and bank-conflict cycles, and wave occupancy.

    python scripts/pmc_r04_table.py PMC_DIR STATS_CSV [--steps S] [--json OUT]

PMC_DIR holds <pass>/**/run_counter_collection.csv (pass = fetch, write, tcc, lds, wave);
STATS_CSV is rocprofv3's run_kernel_stats.csv of a run with STATS_STEPS steps (+ warmups,
given by --stats-steps)."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def kname(s):
    s = re.sub(r"\(.*", "", s).replace("void ", "").replace("sheep::", "")
    return s.strip()


def short(k):
    base, _, targ = k.partition("<")
    return base + ("<" + targ.split(",")[0].rstrip(">") + ">" if targ else "")


def load_pass(d):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(kname(r["Kernel_Name"]))
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("stats")
    ap.add_argument("--steps", type=int, default=1, help="graph2tree steps in each pmc pass")
    ap.add_argument("--stats-steps", type=int, default=5, help="steps (incl. warmup) of the stats run")
    ap.add_argument("--json")
    a = ap.parse_args()
    passes = {}
    for p in sorted(os.listdir(a.pmc)):
        if os.path.isdir(os.path.join(a.pmc, p)):
            passes[p] = load_pass(os.path.join(a.pmc, p))
    ms = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for r in csv.DictReader(open(a.stats)):
        k = short(kname(r["Name"]))
        ms[k] += float(r["TotalDurationNs"]) / 1e6 / a.stats_steps
        calls[k] += int(r["Calls"])
    rows = {}
    for k in sorted(ms, key=lambda k: -ms[k]):
        if ms[k] < 0.05 or k.startswith("k_rmat"):
            continue
        c = collections.defaultdict(float)
        for p, (tot, n) in passes.items():
            for cn, v in tot.get(k, {}).items():
                c[cn] = v / a.steps
        hit = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        rows[k] = {
            "ms_per_step": round(ms[k], 3), "launches_per_step": calls[k] / a.stats_steps,
            "fetch_GB_raw": round(c["FETCH_SIZE"] * 1024 / 1e9, 3),
            "fetch_GB_x2": round(2 * c["FETCH_SIZE"] * 1024 / 1e9, 3),
            "write_GB": round(c["WRITE_SIZE"] * 1024 / 1e9, 3),
            "l2_hit": round(hit, 3) if c["TCC_HIT_sum"] + c["TCC_MISS_sum"] else None,
            "l2_req_G": round((c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) / 1e9, 3),
            "l2_atomic_G": round(c["TCC_ATOMIC_sum"] / 1e9, 4) if "TCC_ATOMIC_sum" in c else None,
            "lds_inst_M": round(c["SQ_INSTS_LDS"] / 1e6, 2),
            "lds_conflict_frac": round(c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_LDS_IDX_ACTIVE"]), 3)
            if c["SQ_LDS_IDX_ACTIVE"] else None,
            "wait_frac": round(c["SQ_WAIT_ANY"] / wc, 3) if c["SQ_WAVE_CYCLES"] else None,
            "lds_wait_frac": round(c["SQ_WAIT_INST_LDS"] / wc, 3) if c["SQ_WAVE_CYCLES"] else None,
            "vmem_rd_M": round(c["SQ_INSTS_VMEM_RD"] / 1e6, 2),
            "vmem_wr_M": round(c["SQ_INSTS_VMEM_WR"] / 1e6, 2),
        }
        r = rows[k]
        r["hbm_GB_s_raw"] = round((r["fetch_GB_raw"] + r["write_GB"]) / (ms[k] * 1e-3), 1)
    hdr = ("kernel", "ms", "fetch x2 GB", "write GB", "L2 hit", "L2 req G", "L2 atom G",
           "LDS inst M", "LDS confl", "wait", "lds wait")
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    for k, r in rows.items():
        vals = [k, r["ms_per_step"], r["fetch_GB_x2"], r["write_GB"], r["l2_hit"], r["l2_req_G"],
                r["l2_atomic_G"], r["lds_inst_M"], r["lds_conflict_frac"], r["wait_frac"],
                r["lds_wait_frac"]]
        print("| " + " | ".join("-" if v is None else str(v) for v in vals) + " |")
    tot_f = sum(r["fetch_GB_raw"] for r in rows.values())
    tot_w = sum(r["write_GB"] for r in rows.values())
    print("\nper step: FETCH raw %.1f GB (x2 %.1f), WRITE %.1f GB, raw total %.1f GB"
          % (tot_f, 2 * tot_f, tot_w, tot_f + tot_w))
    if a.json:
        json.dump({"kernels": rows, "fetch_GB_raw": tot_f, "write_GB": tot_w}, open(a.json, "w"),
                  indent=1)


if __name__ == "__main__":
    main()
