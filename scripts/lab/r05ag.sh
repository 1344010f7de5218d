# (round 6) Added with its results in commit e825ef2: SHEEP_LAB 1024 (deferred kept-pair writes in k_kb_map) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: SHEEP_LAB=1024 = k_kb_map writes chunk j's kept pairs during chunk j + 1 (no wave waits
# for the chunk's reservation, a returning atomic on one counter shared by every block).
# Hypothesis: the reservation's round trip is exposed once per chunk (all waves wait at the
# barrier behind wave 0); the map's time per bucket should drop, most in the hub buckets.
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
SHEEP_LAB=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lab1024.log 2>&1 || { tail -30 $O/pytest_lab1024.log; exit 1; }
tail -2 $O/pytest_lab1024.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=1024 - SHEEP_LAB=1024 - SHEEP_LAB=1024 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=1024 - SHEEP_LAB=1024 || exit 1
OUT=$O bash scripts/ab_env.sh "--scale 22 --seed 22 --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_LAB=1024 - SHEEP_LAB=1024 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" - SHEEP_LAB=1024 || exit 1
