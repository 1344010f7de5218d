"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite, the default output
of ROCm 7): calls, average and max duration, and total per step, a step being one call of the
kernel named by --per (default k_degb_count: one per graph2tree_dev).

  python scripts/kstats_db.py gpurun_out/prof/run_results.db [--per k_degb_count] [--top 40]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", default="k_degb_count")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for name, dur in c.execute("select name, duration from kernels"):
        short = re.sub(r"\(.*", "", name).replace("void ", "").replace("sheep::", "")
        g = agg[short]
        g[0] += 1
        g[1] += dur
        g[2] = max(g[2], dur)
    steps = max(1, sum(v[0] for k, v in agg.items() if k == a.per))
    total = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]
    for k, (n, t, mx) in rows:
        print(f"{k[:40]:40s} calls {n:5d}  avg {t / n / 1e6:8.3f} ms  max {mx / 1e6:8.3f} ms  "
              f"total/step {t / steps / 1e6:8.3f} ms  {100 * t / total:5.2f}%")


if __name__ == "__main__":
    main()
