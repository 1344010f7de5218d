#!/bin/bash
# Everything a round's end needs in one GPU call: the GPU suite, smoke, then scripts/evidence.sh
# (bench lines, kernel stats, PMC passes) into gpurun_out/ev.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo suite_fail; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; tail gpurun_out/smoke.log; exit 1; }
echo smoke_ok
OUT=gpurun_out/ev bash scripts/evidence.sh
