# (round 6) Added with its results in commit b73dd66: SHEEP_LAB 64 (second partition pass as 1024 x 8) was built in the gitignored csrc_lab copy; dropped. The SHEEP_LAB knob is gone, so
# re-running this script now compares identical code.
# A/B: SHEEP_LAB=64 = the second partition pass as 1024 threads x 8 records (32 waves per CU,
# 60 VGPRs) instead of 512 x 16 (16 waves, 104 VGPRs); same 8192-record tiles and LDS.
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
SHEEP_LAB=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lab64.log 2>&1 || { tail -30 $O/pytest_lab64.log; exit 1; }
tail -2 $O/pytest_lab64.log
OUT=$O bash scripts/ab_env.sh "--no-cpu-baseline --steps 10 --warmup 3" - SHEEP_LAB=64 - SHEEP_LAB=64 || exit 1
OUT=$O bash scripts/ab_env.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" - SHEEP_LAB=64 || exit 1
