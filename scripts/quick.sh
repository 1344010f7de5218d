#!/bin/bash
# Quick GPU iteration: parity tests, then the RMAT-26 bench (no CPU baseline); stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 400 python bench.py --scale 22 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/bench22.log 2>&1 && echo "bench22 ok" &&
timeout -k 10 600 python bench.py --scale ${SCALE:-26} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench26.log 2>&1 && echo "bench26 ok"
