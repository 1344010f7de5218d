#!/bin/bash
# rocprof kernel stats of a short RMAT-26 bench under each env setting "NAME=V[,NAME=V]" given as args
set -o pipefail
mkdir -p gpurun_out/envp
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1)); rm -rf gpurun_out/envp/p$i
  ( IFS=','; for kv in $spec; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/envp/p$i -o run -- python bench.py --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline > gpurun_out/envp/b$i.log 2>&1 ) || exit 1
  echo "== $spec"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/envp/b$i.log; python scripts/kstats.py gpurun_out/envp/p$i/run_kernel_stats.csv | grep -E "kb_"
done
