#!/bin/bash
# GPU parity suite, then map_lab A/B of option sets ($@, JSON) on RMAT-26 and the LJ shape.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python scripts/map_lab.py --scale 26 --reps 3 "$@" > gpurun_out/ab_knob26.log 2>&1 &&
timeout -k 10 300 python scripts/map_lab.py --workload lj --reps 5 "$@" > gpurun_out/ab_knoblj.log 2>&1 &&
grep -h '^{' gpurun_out/ab_knob26.log gpurun_out/ab_knoblj.log | cut -c1-420
