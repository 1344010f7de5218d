set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lockstep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ls_test.log 2>&1 && echo "ls tests ok" &&
timeout -k 10 300 python bench.py --lockstep-1 --scale 26 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ls1_26.log 2>&1 && echo "ls1 ok" &&
timeout -k 10 300 python scripts/lockstep_sim.py --scale 26 --P 8 --reps 2 > gpurun_out/ls_sim26.log 2>&1 && echo "sim ok" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --backend gloo --same-device --check --scale 22 --steps 1 --warmup 1 > gpurun_out/ls_bench4.log 2>&1 && echo "bench4 ok"
