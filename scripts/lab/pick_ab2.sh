#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 python scripts/map_lab.py --scale 26 --reps 2 '{}' '{"kb_pick": 0}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 44, "kb_rankb": 44}' '{"kb_buckets": 36, "kb_rankb": 36}' '{"kb_buckets": 32, "kb_rankb": 32}' > gpurun_out/pk26.log 2>&1 &&
timeout -k 10 400 python scripts/map_lab.py --workload twitter --reps 2 '{}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 32, "kb_rankb": 32}' > gpurun_out/pktw.log 2>&1 &&
timeout -k 10 300 python scripts/map_lab.py --workload lj --reps 4 '{}' '{"kb_pick": 0}' > gpurun_out/pklj.log 2>&1 &&
timeout -k 10 300 python scripts/map_lab.py --scale 22 --reps 4 '{}' '{"kb_pick": 0}' > gpurun_out/pk22.log 2>&1 &&
grep -h '^{' gpurun_out/pk26.log gpurun_out/pktw.log gpurun_out/pklj.log gpurun_out/pk22.log | cut -c1-400
