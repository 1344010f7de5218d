# (round 6) Added with its results in commit 0bc0256: SHEEP_LAB 128 (estimate-weighted birth window) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B on top of the dense rank cuts: SHEEP_LAB=128 = the birth window and sweeps weigh a binned
# bucket by its estimated records (no capacity slack).
export TMPDIR=/tmp
O=gpurun_out/r05aj; mkdir -p $O
for a in "--scale 22 --seed 22" "--scale 22 --seed 5" "--scale 22 --seed 9" "--workload lj" "--scale 23 --seed 23" "--scale 24 --seed 24" "--scale 24 --seed 3"; do
  OUT=$O bash scripts/ab_env.sh "$a --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_LAB=128 - SHEEP_LAB=128 || exit 1
done
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=128 - SHEEP_LAB=128 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 26 --seed 5 --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=128 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=128 || exit 1
