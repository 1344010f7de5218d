#!/bin/bash
# kb bucket-count sweep of the one-GPU loop at RMAT-26 (SHEEP_KB_BUCKETS = K_e, SHEEP_KB_RANKB = K_r)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
KS=${KS:-"48,48 64,64 80,80 64,32 96,64"}
for k in $KS; do
  k=${k/,/ }
  set -- $k
  SHEEP_KB_BUCKETS=$1 SHEEP_KB_RANKB=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ks_$1_$2.log 2>&1 || exit 1
  echo "$1 $2 $(grep '^{' gpurun_out/ks_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["roofline"]["phases_ms"]["tree_insert"], d["roofline"]["launches_per_step"])')"
done
