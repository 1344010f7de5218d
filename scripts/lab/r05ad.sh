# (round 6) Added with its results in commit 288eb22: SHEEP_LAB 128 / 256 (birth-window weights) were built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: the birth window (fresh anchors) and the sweep plan weigh a directly binned bucket by
# SHEEP_LAB=128 its estimated records, SHEEP_LAB=256 its exact records (the bins' fill, read
# back with the overflow words) instead of its capacity (which adds 5 % + 8192 slots per bin).
# Hypothesis: the capacity closes the window a bucket early where the bins are many and thin
# (LJ at 12 rank cuts: the bucket after the birth mapped stale, its zipper 2.5 ms).
export TMPDIR=/tmp
O=gpurun_out/r05ad; mkdir -p $O
for a in "--scale 22 --seed 22" "--scale 22 --seed 5" "--scale 22 --seed 9" "--workload lj" "--scale 23 --seed 23" "--scale 24 --seed 24"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_LAB=128 SHEEP_LAB=256 "SHEEP_LAB=256 SHEEP_KB_RANKB=12" || exit 1
done
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=128 SHEEP_LAB=256 - SHEEP_LAB=256 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 26 --seed 5 --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=256 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=256 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --no-cpu-baseline --check --steps 3 --warmup 1" SHEEP_LAB=256 "SHEEP_LAB=256 SHEEP_KB_RANKB=12" || exit 1
