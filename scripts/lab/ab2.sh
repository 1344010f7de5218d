# A/B: finer buckets in the percolation window (SHEEP_KB_TRANS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/ab_check24.log 2>&1 && echo "check24 ok" &&
for cfg in 0 4 8 2; do SHEEP_KB_TRANS=$cfg timeout -k 10 300 python bench.py --scale 26 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab2_t$cfg.log 2>&1 || exit 1; echo "T=$cfg ok"; done &&
for cfg in 0 4; do SHEEP_KB_TRANS=$cfg timeout -k 10 300 python bench.py --workload lj --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab2_lj_t$cfg.log 2>&1 || exit 1; SHEEP_KB_TRANS=$cfg timeout -k 10 300 python bench.py --workload twitter --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab2_tw_t$cfg.log 2>&1 || exit 1; echo "pl T=$cfg ok"; done &&
SHEEP_KB_TRANS=4 timeout -k 10 300 python scripts/lockstep_sim.py --scale 26 --P 8 --reps 2 > gpurun_out/ab2_sim.log 2>&1 && echo "sim ok"
