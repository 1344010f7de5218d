#!/bin/bash
# GPU parity suite, then the direct hi-binning A/B on RMAT-26 / LJ / twitter shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python scripts/map_lab.py --scale 26 --reps 3 '{}' '{"bin_direct": 0}' '{}' > gpurun_out/ab_rmat26.log 2>&1 && cat gpurun_out/ab_rmat26.log | grep '^{' | cut -c1-420 &&
timeout -k 10 300 python scripts/map_lab.py --workload twitter --reps 2 '{}' '{"bin_direct": 0}' > gpurun_out/ab_tw.log 2>&1 && cat gpurun_out/ab_tw.log | grep '^{' | cut -c1-420 &&
timeout -k 10 300 python scripts/map_lab.py --workload lj --reps 5 '{}' '{"bin_direct": 0}' > gpurun_out/ab_lj.log 2>&1 && cat gpurun_out/ab_lj.log | grep '^{' | cut -c1-420
