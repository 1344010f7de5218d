# Small-config knob sweep at HEAD: the unpipelined kb loop and bucket counts (RMAT-22 seed 22,
# LJ shape, RMAT-23/24 as controls), two runs each.
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
for a in "--scale 22 --seed 22" "--workload lj" "--scale 23 --seed 23" "--scale 24 --seed 24"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_KB_PIPE=0 "SHEEP_KB_RANKB=6 SHEEP_KB_BUCKETS=6" "SHEEP_KB_RANKB=12 SHEEP_KB_BUCKETS=8" - SHEEP_KB_PIPE=0 || exit 1
done
