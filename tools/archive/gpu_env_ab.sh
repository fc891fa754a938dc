#!/bin/bash
# A/B of a runtime switch: VAR=name VALUES="0 1" over several workloads (default library),
# interleaved twice.
cd "$(dirname "$0")/.." || exit 1
VAR=${VAR:-BDPT_BLOCK_MAJOR}
CFGS=${CFGS:-"CBspheres 480 360 128 5 2;scenes/CBlucy_standin.dae 1920 1080 128 5 1;CBgems 480 360 64 5 2"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for a in "${CFG_LIST[@]}"; do
  for r in 1 2; do
    for v in ${VALUES:-0 1}; do
      echo "== $VAR=$v round $r | $a"
      env "$VAR=$v" timeout -k 10 300 python3 tools/prof_render.py $a || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
