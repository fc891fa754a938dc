#!/bin/bash
# samples-per-lane sweep (bdpt_params.samples_per_lane via BDPT_SPL) of the megakernel.
cd "$(dirname "$0")/.." || exit 1
CFGS=${CFGS:-"CBspheres 480 360 128 5 2;scenes/CBlucy_standin.dae 1920 1080 128 5 1"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for a in "${CFG_LIST[@]}"; do
  for spl in ${SPLS:-0 2 4 8 16 32}; do
    echo "== spl $spl | $a"
    BDPT_SPL=$spl timeout -k 10 300 python3 tools/prof_render.py $a || { echo "STOP rc=$?"; exit 1; }
  done
done
