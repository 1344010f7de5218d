#!/bin/bash
# GPU parity suite, kb kernel stats (rocprof) of the default options, then map_lab phase times
# on RMAT-26, RMAT-22 and the LJ shape for the option sets given as JSON args.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log &&
bash scripts/lab/prof_tree_opts.sh '{}' &&
timeout -k 10 300 python scripts/map_lab.py --scale 26 --reps 3 "$@" > gpurun_out/kc26.log 2>&1 &&
timeout -k 10 200 python scripts/map_lab.py --scale 22 --reps 5 "$@" > gpurun_out/kc22.log 2>&1 &&
timeout -k 10 200 python scripts/map_lab.py --workload lj --reps 5 "$@" > gpurun_out/kclj.log 2>&1 &&
python - <<'PY'
import json
for f in ("kc26", "kc22", "kclj"):
    for l in open("gpurun_out/%s.log" % f):
        if l.startswith("{"):
            d = json.loads(l); t = d["t"]
            print(f, d["opts"], "tree", t["tree_insert"], "map", t["kb_map"], "total", round(sum(v for k, v in t.items() if k not in ("kb_map", "kb_map#", "kb_loop_host")), 3))
PY
