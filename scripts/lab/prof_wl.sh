#!/bin/bash
# rocprof kernel trace of a short bench run of one workload: WL=lj|twitter|rmat [SCALE=..]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_$WL
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WL -o run -- python bench.py --workload ${WL:-rmat} --scale ${SCALE:-26} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/prof_$WL.log 2>&1
