set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log &&
bash scripts/lab/prof_tree_opts.sh '{}' &&
timeout -k 10 200 python scripts/map_lab.py --scale 22 --reps 5 '{}' '{}' > gpurun_out/zl22.log 2>&1 &&
timeout -k 10 200 python scripts/map_lab.py --workload lj --reps 5 '{}' '{}' > gpurun_out/zllj.log 2>&1 &&
grep -h '^{' gpurun_out/zl22.log gpurun_out/zllj.log | cut -c1-330
