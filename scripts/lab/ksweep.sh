#!/bin/bash
# kb bucket-count sweep: ms/step and tree phase per K_e:K_r and workload
#   WLS="lj rmat" KS="8:8 64:64" SCALE=26 bash scripts/lab/ksweep.sh
set -o pipefail
mkdir -p gpurun_out/ksweep
for wl in ${WLS:-lj rmat}; do
  for kk in ${KS:-8:8 16:8 32:8 32:16 64:16 64:64}; do
    ke=${kk%%:*}; kr=${kk#*:}
    f=gpurun_out/ksweep/${wl}_${ke}_${kr}.log
    SHEEP_KB_BUCKETS=$ke SHEEP_KB_RANKB=$kr timeout -k 10 300 python bench.py --workload $wl --scale ${SCALE:-26} --steps 3 --warmup 1 --no-cpu-baseline > $f 2>&1 || exit 1
    echo "$wl ${SCALE:-26} $ke $kr $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), d['roofline']['phases_ms']['tree_insert'])")"
  done
done
