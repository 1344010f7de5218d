#!/bin/bash
# rocprof kernel stats of the front half (degree .. bin scatter) under lab builds given as args
# (scripts/lab/libsheep_NAME.so), first partition pass not overlapped; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/front
export TMPDIR=/tmp
OPTS=${OPTS:-'{"part_overlap": 0}'}
for v in "$@"; do
  rm -rf "gpurun_out/front/$v"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/front/$v" -o run -- \
    python scripts/map_lab.py --scale ${SCALE:-26} --reps 3 --lib "scripts/lab/libsheep_$v.so" "$OPTS" \
    > "gpurun_out/front/$v.log" 2>&1 || { echo "FAIL $v"; exit 1; }
  echo "== $v"; grep '^{' "gpurun_out/front/$v.log" | cut -c1-300
  python scripts/kstats.py "gpurun_out/front/$v/run_kernel_stats.csv" 4 | grep -vE "kb_|k_rmat|k_iota|fill|copy" | head -24
done
