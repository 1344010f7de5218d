# The GPU suite with the kb loop's state initialised behind the edge pass readback (new), then
# A/B bench lines against HEAD (base).
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 2 || exit 1
