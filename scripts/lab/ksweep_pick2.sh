#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/map_lab.py --scale 26 --reps 3 '{}' '{"kb_buckets": 36, "kb_rankb": 36}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 44, "kb_rankb": 44}' '{"kb_buckets": 40, "kb_rankb": 48}' > gpurun_out/ks26b.log 2>&1 &&
timeout -k 10 400 python scripts/map_lab.py --workload twitter --reps 2 '{}' '{"kb_buckets": 36, "kb_rankb": 36}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 44, "kb_rankb": 44}' '{"kb_buckets": 40, "kb_rankb": 48}' > gpurun_out/kstwb.log 2>&1 &&
timeout -k 10 400 python scripts/map_lab.py --scale 25 --reps 3 '{}' '{"kb_buckets": 40, "kb_rankb": 40}' > gpurun_out/ks25b.log 2>&1 &&
grep -h '^{' gpurun_out/ks26b.log gpurun_out/kstwb.log gpurun_out/ks25b.log | cut -c1-400
