# (round 6) Added with its results in commit 173f10d: the sweep placements (SHEEP_LAB_SWEEP*) were built in the gitignored csrc_lab copy; beside-the-map variants dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 "SHEEP_LAB_SWEEP=3 SHEEP_LAB_SWEEP_SEQ=1" SHEEP_LAB_SWEEP=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 26 --seed 5 --steps 6 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=2 SHEEP_LAB_SWEEP=3 || exit 1
