#!/bin/bash
# Extra evidence beside refresh_profiles.sh: RMAT-22 checked against the CPU checker, the smoke
# test, and the one-rank RCCL run of the multi-GPU driver.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --scale 22 --check --no-cpu-baseline > gpurun_out/bench_r22check.log 2>&1 && echo "r22 check ok" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --lockstep-1 --no-cpu-baseline > gpurun_out/ls1.log 2>&1 && echo "ls1 ok" &&
timeout -k 10 400 python scripts/lockstep_sim.py --P 2 8 > gpurun_out/lsim.log 2>&1 && echo "lsim ok" && grep '^{' gpurun_out/lsim.log | cut -c1-300
