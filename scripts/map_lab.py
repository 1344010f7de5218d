"""kb map lab: RMAT-26 (or --scale) graph2tree under option sets; kb_map / tree phase times and,
with --stats, the map's find count (SHEEP_TREE_STATS=1 totals on stderr)."""
import argparse
import json
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

from sheep_amd import capi, device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--lib", default=None, help="a lab build of libsheep_amd.so")
ap.add_argument("--workload", default="rmat", choices=["rmat", "lj", "twitter"])
ap.add_argument("sets", nargs="*", default=["{}"])
a = ap.parse_args()
if a.lib:
    capi.lib_path = a.lib
device.init(0)
if a.workload == "rmat":
    uv, n_ids = device.rmat(a.scale, 16, a.scale), 1 << a.scale
else:
    n_ids, m, gamma, i0, seed = device.POWERLAW[a.workload]
    uv = device.powerlaw(n_ids, m, gamma, i0, seed)
torch.cuda.synchronize()
for js in a.sets:
    opts = json.loads(js)
    old = {k: capi.set_option(k, v) for k, v in opts.items()}
    res = []
    for _ in range(a.reps + 1):
        device.graph2tree(uv, n_ids)
        torch.cuda.synchronize()
        res.append(dict(capi.last_timings()))
    t = res[1:]
    avg = {k: round(sum(r.get(k, 0) for r in t) / len(t), 3) for k in t[0]}
    print(json.dumps({"lib": a.lib, "workload": a.workload, "opts": opts, "t": avg}), flush=True)
    for k, v in old.items():
        capi.set_option(k, v)
