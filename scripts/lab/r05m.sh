# (round 6) Added with its results in commit 67647ab: the sparse-word sweep skip (SHEEP_LAB_SWEEP_MINPOP) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP_MINPOP=1 SHEEP_LAB_SWEEP_MINPOP=8 SHEEP_LAB_SWEEP_MINPOP=24 - || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP_MINPOP=1 SHEEP_LAB_SWEEP_MINPOP=8 SHEEP_LAB_SWEEP_MINPOP=24 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP_MINPOP=1 SHEEP_LAB_SWEEP_MINPOP=8 SHEEP_LAB_SWEEP_MINPOP=24 || exit 1
