export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fullsize_tree or rmat or power" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_lib.sh "--steps 8 --warmup 2 --no-cpu-baseline" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --steps 5 --warmup 2 --no-cpu-baseline" 1 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --check --steps 20 --warmup 3 --no-cpu-baseline" 1 || exit 1
