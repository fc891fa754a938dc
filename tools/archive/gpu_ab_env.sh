#!/bin/bash
# A/B of runtime switches (environment variables read at bdpt_create) on one device:
# ENVS="A=1 B=2;A=0" (';' between variants), interleaved rounds, one process per run.
# STATS=1 adds one counting launch per variant (tools/prof_render.py BDPT_STATS=1).
cd "$(dirname "$0")/.." || exit 1
ARGS=${ARGS:-"scenes/CBlucy_standin.dae 1920 1080 16 5 2"}
IFS=';' read -ra VARS <<< "${ENVS:-X=0}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in "${VARS[@]}"; do
    echo "== [$e] round $r"
    env $e timeout -k 10 300 python3 tools/prof_render.py $ARGS || { echo "STOP rc=$?"; exit 1; }
  done
done
if [ -n "$STATS" ]; then
  for e in "${VARS[@]}"; do
    echo "== [$e] stats"
    env $e BDPT_STATS=1 timeout -k 10 300 python3 tools/prof_render.py ${STATS_ARGS:-$ARGS} || { echo "STOP rc=$?"; exit 1; }
  done
fi
