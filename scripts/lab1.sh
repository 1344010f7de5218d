set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/lab/gather_lab.py 26 > gpurun_out/gather_lab.log 2>&1
