# (round 6) Added with its results in commit 7217ac4: SHEEP_LAB 512 (tile-relative write-out bases) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: SHEEP_LAB=512 = tile-relative write-out bases in the fused pass (y: base + slot while the
# slot is below the run's end; x: base + slot) and the edge pass (base + slot): one LDS table
# read fewer per written record.
export TMPDIR=/tmp
O=gpurun_out/r05af; mkdir -p $O
SHEEP_LAB=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lab512.log 2>&1 || { tail -30 $O/pytest_lab512.log; exit 1; }
tail -2 $O/pytest_lab512.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=512 - SHEEP_LAB=512 - SHEEP_LAB=512 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=512 || exit 1
