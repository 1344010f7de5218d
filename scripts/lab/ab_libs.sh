#!/bin/bash
# map_lab phase times of lab builds (scripts/lab/libsheep_NAME.so) given as args; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
OPTS=${OPTS:-'{}'}
for v in "$@"; do
  timeout -k 10 200 python scripts/map_lab.py --scale ${SCALE:-26} --workload ${WL:-rmat} --reps ${REPS:-3} --lib "scripts/lab/libsheep_$v.so" "$OPTS" \
    > "gpurun_out/ab/$v.log" 2>&1 || { echo "FAIL $v"; exit 1; }
  grep '^{' "gpurun_out/ab/$v.log" | cut -c1-400
done
