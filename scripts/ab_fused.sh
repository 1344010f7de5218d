#!/bin/bash
# A/B of the first partition pass: beside the degree pass (SHEEP_PART_OVERLAP=2) against fused
# into the degree scatter (3), on the four GPU configs; one bench line each under $OUT.
set -o pipefail
OUT=${OUT:-gpurun_out/ab_fused}
mkdir -p "$OUT"
for ov in 2 3; do
  for w in "rmat --scale 26" "twitter" "lj" "rmat --scale 22 --seed 22"; do
    tag=$(echo "$w" | tr -d ' -')
    SHEEP_PART_OVERLAP=$ov timeout -k 10 200 python bench.py --no-cpu-baseline --workload $w \
      > "$OUT/ov${ov}_${tag}.json" 2>> "$OUT/err.log" || exit $?
  done
  echo "ov $ov done"
done
