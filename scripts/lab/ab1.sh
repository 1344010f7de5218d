# A/B: giant fold (default on) and read-only map finds; parity tests first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --scale 24 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/ab_check24.log 2>&1 && echo "check24 ok" &&
for cfg in "SHEEP_KB_FOLD=0" "SHEEP_KB_FOLD=1" "SHEEP_KB_MAPFIND=ro" ; do env $cfg timeout -k 10 300 python bench.py --scale 26 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$cfg.log 2>&1 || exit 1; echo "$cfg ok"; done &&
for cfg in "SHEEP_KB_FOLD=0" "SHEEP_KB_FOLD=1"; do env $cfg timeout -k 10 300 python scripts/lockstep_sim.py --scale 26 --P 8 --reps 2 > gpurun_out/ab_sim_$cfg.log 2>&1 || exit 1; echo "sim $cfg ok"; done
