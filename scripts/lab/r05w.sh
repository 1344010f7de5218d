# Rank-cut count sweep on small configs (K_e = 8): RMAT-22 seeds 22 / 5 / 9, LJ shape, RMAT-23.
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
for a in "--scale 22 --seed 22" "--scale 22 --seed 5" "--scale 22 --seed 9" "--workload lj" "--scale 23 --seed 23"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - "SHEEP_KB_RANKB=10 SHEEP_KB_BUCKETS=8" "SHEEP_KB_RANKB=12 SHEEP_KB_BUCKETS=8" "SHEEP_KB_RANKB=16 SHEEP_KB_BUCKETS=8" "SHEEP_KB_RANKB=12 SHEEP_KB_BUCKETS=6" || exit 1
done
