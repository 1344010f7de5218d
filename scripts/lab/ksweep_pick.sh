#!/bin/bash
# kb bucket-count sweep with the device-picked anchor (RMAT-26, twitter shape, LJ shape).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python scripts/map_lab.py --scale 26 --reps 2 '{}' '{"kb_buckets": 32, "kb_rankb": 32}' '{"kb_buckets": 40, "kb_rankb": 40}' '{"kb_buckets": 40, "kb_rankb": 16}' '{"kb_buckets": 48, "kb_rankb": 16}' '{"kb_buckets": 56, "kb_rankb": 24}' > gpurun_out/ks26.log 2>&1 &&
timeout -k 10 400 python scripts/map_lab.py --workload twitter --reps 2 '{}' '{"kb_buckets": 32, "kb_rankb": 32}' '{"kb_buckets": 40, "kb_rankb": 16}' '{"kb_buckets": 48, "kb_rankb": 16}' '{"kb_buckets": 56, "kb_rankb": 24}' > gpurun_out/kstw.log 2>&1 &&
timeout -k 10 300 python scripts/map_lab.py --workload lj --reps 4 '{}' '{"kb_buckets": 8, "kb_rankb": 4}' '{"kb_buckets": 12, "kb_rankb": 4}' '{"kb_buckets": 6, "kb_rankb": 6}' > gpurun_out/kslj.log 2>&1 &&
grep -h '^{' gpurun_out/ks26.log gpurun_out/kstw.log gpurun_out/kslj.log | cut -c1-400
