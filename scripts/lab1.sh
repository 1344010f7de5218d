set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lab/sort_lab.py 26 > gpurun_out/sort_lab.log 2>&1
