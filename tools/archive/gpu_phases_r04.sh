#!/bin/bash
# Phase split (BDPT_PHASE_PROF build build_var_ph.so) of the north star and the C5 shape, round 4.
cd "$(dirname "$0")/.." || exit 1
for a in "scenes/CBlucy_standin.dae 1920 1080 8 5 1" "C5"; do
  if [ "$a" = C5 ]; then export BDPT_ENV=synth:1024x512 BDPT_RR=1; a="scenes/CBlucy_standin.dae 1920 1080 8 8 1"; fi
  echo "== $a ${BDPT_ENV:-} ${BDPT_RR:+rr}"
  BDPT_LIB=$PWD/build_var_ph.so BDPT_PHASES=1 timeout -k 10 300 python3 tools/prof_render.py $a 2>&1 | grep -v "^W2026" || exit 1
done
