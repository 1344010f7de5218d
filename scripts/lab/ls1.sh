set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lockstep_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ls_test.log 2>&1 && echo "ls tests ok" &&
timeout -k 10 300 python scripts/lockstep_sim.py --scale 22 --P 2 4 8 > gpurun_out/ls_sim22.log 2>&1 && echo "sim22 ok" &&
timeout -k 10 400 python scripts/lockstep_sim.py --scale 26 --P 2 4 8 > gpurun_out/ls_sim26.log 2>&1 && echo "sim26 ok"
