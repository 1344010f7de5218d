"""Per-bucket kernel times of the kb loop from a rocprofv3 --kernel-trace database (rocpd
sqlite): one graph2tree_dev call (the STEP-th, counted by k_degb_count), one line per bucket
apply (grouped at each k_kb_refresh), and the totals.

  python scripts/kb_buckets.py gpurun_out/prof/run_results.db [--step 2] [--quiet]
"""
import argparse
import collections
import re
import sqlite3

APPLY = ["k_kb_refresh", "k_kb_spine", "k_kb_zip", "k_kb_union", "k_kb_label"]
OTHER = ["k_kb_map", "k_gb_rebase"]


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("sheep::", "")
    return re.sub(r"<.*", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = [(short(n), s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    starts = [i for i, r in enumerate(rows) if r[0] == "k_degb_count"] + [len(rows)]
    step = rows[starts[a.step]:starts[a.step + 1]]
    buckets, cur = [], None
    for n, s, e in step:
        if n == "k_kb_refresh":
            cur = collections.Counter()
            buckets.append(cur)
        if cur is not None and n in APPLY:
            cur[n] += (e - s) / 1e3
    tot = collections.Counter()
    for n, s, e in step:
        if n in APPLY + OTHER:
            tot[n] += (e - s) / 1e3
    if not a.quiet:
        print("bucket " + " ".join("%8s" % n[5:] for n in APPLY) + "   (us)")
        for i, b in enumerate(buckets):
            print("%6d " % i + " ".join("%8.0f" % b.get(n, 0) for n in APPLY))
    print("totals (ms):", {k: round(v / 1e3, 2) for k, v in tot.most_common()})
    ap_k = [(s, e) for n, s, e in step if n in APPLY]
    if ap_k:
        print("apply span (ms): %.2f, apply kernel sum %.2f" %
              ((ap_k[-1][1] - ap_k[0][0]) / 1e6, sum(tot[n] for n in APPLY) / 1e3))


if __name__ == "__main__":
    main()
