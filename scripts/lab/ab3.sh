# A/B: non-temporal record loads in the kb map
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --scale 22 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/ab3_check.log 2>&1 && echo "check ok" &&
SHEEP_KB_NT=1 timeout -k 10 300 python bench.py --scale 22 --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/ab3_check_nt.log 2>&1 && echo "check nt ok" &&
for cfg in 0 1 0 1; do SHEEP_KB_NT=$cfg timeout -k 10 300 python bench.py --scale 26 --steps 5 --warmup 2 --no-cpu-baseline >> gpurun_out/ab3_nt$cfg.log 2>&1 || exit 1; echo "NT=$cfg ok"; done
