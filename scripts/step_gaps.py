"""Device idle time inside the last graph2tree step of a rocprofv3 --kernel-trace CSV: the step
runs from the last launch of its first kernel (default k_front_sample) to the end of the trace.
Prints the step's span, the time some kernel was running (union over streams), and every gap
of at least --min-us with the kernels either side, so host round trips show up as named gaps.
  python scripts/step_gaps.py gpurun_out/gaps/r22/run_kernel_trace.csv [--first k_front_sample]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first", default="k_front_sample")
    ap.add_argument("--min-us", type=float, default=10.0)
    ap.add_argument("--prev", action="store_true",
                    help="the step before the last one, up to the last step's first kernel: its "
                         "gaps then include the host time between two calls")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    if not starts:
        raise SystemExit(f"no {a.first} in the trace")
    rows = rows[starts[-2]:starts[-1] + 1] if a.prev and len(starts) > 1 else rows[starts[-1]:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48])
          for r in rows]
    t0 = iv[0][0]
    busy = 0
    gaps = []
    cur_s, cur_e, last = iv[0]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            if (s - cur_e) / 1e3 >= a.min_us:
                gaps.append(((cur_e - t0) / 1e3, (s - cur_e) / 1e3, last, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            last = n
    busy += cur_e - cur_s
    span = (cur_e - t0) / 1e3
    print(f"kernels {len(iv)}  span {span:.1f} us  busy {busy / 1e3:.1f} us  idle {span - busy / 1e3:.1f} us")
    print(f"gaps >= {a.min_us} us: {len(gaps)}, {sum(g[1] for g in gaps):.1f} us")
    for at, g, before, after in gaps:
        print(f"  at {at:8.1f} us  {g:7.1f} us  after {before}  before {after}")


if __name__ == "__main__":
    main()
