# (round 6) Added with its results in commit 173f10d: the sweep alpha values (SHEEP_LAB_SWEEP) were built in the gitignored csrc_lab copy; alpha 2 adopted (SWEEP_ALPHA, sheep_capi.cpp). The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 SHEEP_LAB_SWEEP=60 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 24 --seed 24 --steps 10 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
