mkdir -p gpurun_out
for spec in "64 64" "32 32" "16 16" "16 64" "64 16"; do set -- $spec
  SHEEP_KB_BUCKETS=$1 SHEEP_KB_RANKB=$2 timeout -k 10 300 python scripts/shard_sim.py --scale 26 --ranks 8 --reps 2 > gpurun_out/simk_$1_$2.log 2>&1 || exit 1
done
