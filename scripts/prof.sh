#!/bin/bash
# rocprofv3 kernel stats of a short RMAT bench run -> gpurun_out/prof/run_kernel_stats.csv
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --scale ${SCALE:-26} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
