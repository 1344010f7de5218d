#!/bin/bash
# Refresh the round's evidence: default bench line (with both CPU baselines), LJ/twitter lines,
# rocprofv3 kernel stats of the headline run, FETCH_SIZE / WRITE_SIZE passes (separate runs).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && echo "bench ok" &&
timeout -k 10 300 python bench.py --workload lj --no-cpu-baseline > gpurun_out/bench_lj.log 2>&1 && echo "lj ok" &&
timeout -k 10 400 python bench.py --workload twitter --no-cpu-baseline > gpurun_out/bench_tw.log 2>&1 && echo "tw ok" &&
rm -rf gpurun_out/prof && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && echo "prof ok" &&
rm -rf gpurun_out/pmc/fetch && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/fetch.log 2>&1 && echo "fetch ok" &&
rm -rf gpurun_out/pmc/write && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/write.log 2>&1 && echo "write ok"
