# (round 6) Added with its results in commit 731ab19: SHEEP_LAB 2048 (12 rank cuts for dense graphs) was built in the gitignored csrc_lab copy; adopted as kb_counts' dense rule (sheep_capi.cpp). The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: SHEEP_LAB=2048 = 12 rank cuts + 8 edge cuts for dense graphs (mean degree >= 40) below
# 2^29 records (R-MAT 21-24; LJ's mean degree 28 keeps the default).  Across seeds and scales.
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
for a in "--scale 22 --seed 22" "--scale 22 --seed 5" "--scale 22 --seed 9" "--scale 22 --seed 1" "--scale 22 --seed 2" "--scale 21 --seed 21" "--scale 23 --seed 23" "--scale 23 --seed 7" "--scale 24 --seed 24" "--scale 24 --seed 3" "--workload lj"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_LAB=2048 - SHEEP_LAB=2048 || exit 1
done
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --no-cpu-baseline --check --steps 3 --warmup 1" SHEEP_LAB=2048 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 23 --seed 23 --no-cpu-baseline --check --steps 2 --warmup 1" SHEEP_LAB=2048 || exit 1
