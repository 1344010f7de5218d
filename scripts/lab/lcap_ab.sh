set -o pipefail
bash scripts/lab/ab_libs.sh base lcap2048 base lcap2048 &&
OPTS='{"kb_gsum": 0}' bash scripts/lab/ab_libs.sh base lcap2048 &&
SCALE=22 REPS=5 bash scripts/lab/ab_libs.sh base lcap2048 &&
SCALE=22 REPS=5 OPTS='{"kb_gsum": 0}' bash scripts/lab/ab_libs.sh base lcap2048
