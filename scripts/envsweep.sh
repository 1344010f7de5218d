#!/bin/bash
# RMAT-26 bench under a list of environment settings: ENVS="A=1,B=2 A=3 ..." (comma = several vars)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for e in $ENVS; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/es_$i.log 2>&1 || exit 1
  echo "$e $(grep '^{' gpurun_out/es_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]["phases_ms"]; print(round(d["ms_per_step"],2), r["tree_insert"], r.get("kb_map"))')"
done
