# Round 6: k_kb_spine's searches for the next / previous marked word as wave ballots (new)
# against HEAD 476fcbf (base: one thread per word walking up to 64 words each way).  The GPU suite
# on new, then bench lines alternating (RMAT-22 checked), then the evidence set at new.
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 1 || exit 1
