#!/bin/bash
# Phase split (s_memtime, BDPT_PHASE_PROF build build_var_ph.so) of several workloads.
cd "$(dirname "$0")/.." || exit 1
CFGS=${CFGS:-"CBspheres 480 360 64 5 1;scenes/CBlucy_standin.dae 1920 1080 8 5 1;CBgems 480 360 32 5 1"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for a in "${CFG_LIST[@]}"; do
  echo "== $a"
  BDPT_LIB=$PWD/build_var_ph.so BDPT_PHASES=1 timeout -k 10 300 python3 -X faulthandler tools/prof_render.py $a || { echo "STOP rc=$?"; exit 1; }
done
