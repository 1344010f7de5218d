#!/bin/bash
# A/B of environment settings (SHEEP_* options) on bench.py lines, one process per setting:
#   OUT=gpurun_out/ab  bash scripts/ab_env.sh "<bench args>" "<env A>" "<env B>" ...
# ("-" = no extra environment).  One JSON line per run in $OUT/ab.jsonl, tagged with its env.
set -o pipefail
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
ARGS=$1
shift
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  line=$(env $E timeout -k 10 240 python bench.py $ARGS 2>> "$OUT/ab.err") || { echo "run failed: $E"; exit 1; }
  python - "$E" "$ARGS" "$line" >> "$OUT/ab.jsonl" <<'EOF'
import json, sys
r = json.loads(sys.argv[3])
ph = (r.get("roofline") or {}).get("phases_ms", {})
print(json.dumps({"env": sys.argv[1], "args": sys.argv[2], "ms": round(r["ms_per_step"], 3),
                  "phases": ph, "check": r.get("check")}))
EOF
  echo "done: $E"
done
