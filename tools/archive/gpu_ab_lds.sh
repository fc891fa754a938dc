#!/bin/bash
# A/B of block size (build_var_b*.so) x LDS staging mode (LDS_MODES, BDPT_LDS_MODE) on three scenes.
cd "$(dirname "$0")/.." || exit 1
for sc in "CBspheres 480 360 128 5 2" "CBgems 480 360 64 5 2" "CBempty 480 360 128 5 2"; do
  for lib in build_var_*.so; do
    for lm in ${LDS_MODES:-0 1 2}; do
      echo "== $sc $lib lds=$lm"
      BDPT_LDS_MODE=$lm BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_render.py $sc || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
