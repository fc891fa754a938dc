#!/bin/bash
# Treelet-size sensitivity of LDS mode 2: the same workload with the LDS treelet capped.
cd "$(dirname "$0")/.." || exit 1
ARGS=${ARGS:-"scenes/CBlucy_standin.dae 1920 1080 16 5 2"}
for n in ${NTOPS:-1000000 256 64 16}; do
  echo "== ntop cap $n"
  BDPT_NTOP_MAX=$n timeout -k 10 300 python3 tools/prof_render.py $ARGS || { echo "STOP rc=$?"; exit 1; }
done
