#!/bin/bash
# Interleaved A/B timing of library variants (build_var_*.so) on one device, one process per run.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out
mkdir -p $OUT
ARGS=${ARGS:-"CBspheres 480 360 128 5 2"}
for r in 1 2; do
  for lib in build_var_*.so; do
    echo "== $lib round $r"
    BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_render.py $ARGS || { echo "STOP rc=$?"; exit 1; }
  done
done
