# The dense-cut range widened to 1.5 x 2^25 .. 1.5 x 2^27 records: parity subset, RMAT-22 /
# RMAT-23 checked, LJ unchanged.
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --no-cpu-baseline --check --steps 10 --warmup 3" - || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 23 --seed 23 --no-cpu-baseline --check --steps 4 --warmup 2" - || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - || exit 1
