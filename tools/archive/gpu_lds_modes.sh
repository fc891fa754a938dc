#!/bin/bash
# One workload under every forced LDS mode (BDPT_LDS_MODE), default library.
cd "$(dirname "$0")/.." || exit 1
ARGS=${ARGS:-"CBgems 480 360 64 5 2"}
for m in ${MODES:-0 1 2}; do
  echo "== LDS mode $m"
  BDPT_LDS_MODE=$m timeout -k 10 300 python3 tools/prof_render.py $ARGS || { echo "STOP rc=$?"; exit 1; }
done
