# Round 6: refresh-linked pairs written as (union-find root, b) so that k_kb_union needs no
# parent load and starts its find at a root (new), against HEAD 7edd1ea where they were
# (KB_LINKED, g') (base = sheep_amd/libsheep_amd_base.so).  The GPU suite on new, then bench
# lines alternating; RMAT-22 checked.
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc = 0 ] || exit 1
OUT=$O bash scripts/ab_lib.sh "--no-cpu-baseline --steps 10 --warmup 3" 3 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload twitter --no-cpu-baseline --steps 6 --warmup 2" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--workload lj --no-cpu-baseline --steps 20 --warmup 3" 2 || exit 1
OUT=$O bash scripts/ab_lib.sh "--scale 22 --seed 22 --check --no-cpu-baseline --steps 20 --warmup 3" 1 || exit 1
