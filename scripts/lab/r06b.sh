# Round 6: the fused front pass's tile groups (SHEEP_FF_GROUPS, default 8: each group of tiles
# writes its own subregion of every region, read back through the second pass's tile map).
# The GPU suite at the default, then bench lines alternating 8 / 1, then WRITE_SIZE and
# FETCH_SIZE of one RMAT-26 step at 8 and at 1 (one --pmc pass each).
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_FF_GROUPS=1 - SHEEP_FF_GROUPS=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_FF_GROUPS=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_FF_GROUPS=1 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_FF_GROUPS=1 || exit 1
for G in 8 1; do
  OUT=$O/pmc_g$G PASSES="write fetch" SHEEP_FF_GROUPS=$G bash scripts/pmc_r04.sh || exit 1
done
