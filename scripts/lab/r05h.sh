export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
OUT=$O bash scripts/ab_env.sh "--steps 8 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 SHEEP_LAB_SWEEP=60 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --steps 20 --warmup 3 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 24 --seed 24 --steps 10 --warmup 2 --no-cpu-baseline" - SHEEP_LAB_SWEEP=15 SHEEP_LAB_SWEEP=25 SHEEP_LAB_SWEEP=40 || exit 1
