#!/bin/bash
# N > 1 rehearsals on one GPU: the lockstep loop over a one-rank RCCL group (checked), and the
# N = 2 bench path with both ranks on cuda:0 over gloo (checked; timings meaningless).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --lockstep-1 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/ls1.log 2>&1 && echo "lockstep-1 ok" &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 1 --warmup 1 --scale 24 --backend gloo --same-device --check --no-cpu-baseline > gpurun_out/gloo2.log 2>&1 && echo "gloo2 ok"
