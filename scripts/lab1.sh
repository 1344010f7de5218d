set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export LAB_STATS=1
SCALE=26 timeout -k 10 300 bash scripts/lab_env.sh "SHEEP_KB_MAPMODE=0:kb:64" "SHEEP_KB_MAPMODE=1:kb:64" > gpurun_out/lab_mm.log 2>&1
