set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_check.sh &&
timeout -k 10 300 python bench.py --workload lj --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_lj.log 2>&1 && echo "lj ok" &&
timeout -k 10 300 python bench.py --workload twitter --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tw.log 2>&1 && echo "tw ok"
