#!/bin/bash
# Per-bucket kernel times of one RMAT-26 (or $WL) tree build: rocprofv3 kernel trace of map_lab.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- \
  python scripts/map_lab.py --scale ${SCALE:-26} --workload ${WL:-rmat} --reps 1 > gpurun_out/trace.log 2>&1 &&
python scripts/trace_buckets.py gpurun_out/trace/run_kernel_trace.csv > gpurun_out/trace_buckets.txt && tail -3 gpurun_out/trace_buckets.txt
