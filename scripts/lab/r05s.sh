# (round 6) Added with its results in commit e40dfd7: SHEEP_LAB 4 (split histogram buckets through partial counts) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# GPU suite on the readback merge (fused pass: error / overflow words with the degree stats;
# the sequence's radix tail sized from the stats); the suite again with SHEEP_LAB=4 (split
# histogram buckets through partial counts + k_degb_combine instead of global atomics); then
# A/B bench lines: base = HEAD 5b56007 + event pool, new = this build, with and without bit 4.
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
SHEEP_LAB=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lab4.log 2>&1 || { tail -30 $O/pytest_lab4.log; exit 1; }
tail -2 $O/pytest_lab4.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=4 - SHEEP_LAB=4 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=4 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --no-cpu-baseline --check --steps 20 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
