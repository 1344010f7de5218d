#!/bin/bash
# rocprof kernel stats of the kb loop kernels under option sets given as JSON args ($1, $2, ...);
# stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/treeopts
export TMPDIR=/tmp
i=0
for o in "$@"; do
  i=$((i + 1))
  rm -rf "gpurun_out/treeopts/$i"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/treeopts/$i" -o run -- \
    python scripts/map_lab.py --scale ${SCALE:-26} --workload ${WL:-rmat} --reps 3 "$o" \
    > "gpurun_out/treeopts/$i.log" 2>&1 || { echo "FAIL $o"; exit 1; }
  echo "== $o"; grep '^{' "gpurun_out/treeopts/$i.log" | cut -c1-300
  python scripts/kstats.py "gpurun_out/treeopts/$i/run_kernel_stats.csv" 4 | grep -E "kb_" | head -12
done
