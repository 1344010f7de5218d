#!/bin/bash
# Runs tree_lab once per environment setting given as args "NAME=VAL[,NAME=VAL]:variants"
SCALE=${SCALE:-24}
for spec in "$@"; do
  envs=${spec%%:*}; variants=${spec#*:}
  echo "== $envs"
  ( IFS=','; for kv in $envs; do export "$kv"; done
    timeout -k 10 200 python scripts/tree_lab.py --scale $SCALE --reps 1 --variants $variants 2>&1 | grep -v amdgpu.ids ) || exit 1
done
