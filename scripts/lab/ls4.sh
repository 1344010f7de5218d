# lockstep loop at N = 1 over a one-rank RCCL group vs the single-GPU path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lockstep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ls_test.log 2>&1 && echo "ls tests ok" &&
timeout -k 10 300 python bench.py --lockstep-1 --scale 22 --steps 2 --warmup 1 --no-cpu-baseline --check > gpurun_out/ls1_check.log 2>&1 && echo "check ok" &&
timeout -k 10 300 python bench.py --lockstep-1 --scale 26 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ls1_26.log 2>&1 && echo "ls1 ok"
