#!/bin/bash
# A/B of library builds on the GPU box: LIBS="a.so b.so" CFGS=("scene W H spp M launches" ...)
# PIPES="1 2". Each line: config, library, pipeline, Msamples/s (tools/prof_render.py).
cd "$(dirname "$0")/.." || exit 1
LIBS=${LIBS:-bidirectional-pathtracing_amd/libbdpt_amd.so}
PIPES=${PIPES:-1}
CFGS=${CFGS:-"CBspheres 480 360 128 5 2;scenes/CBlucy_standin.dae 1920 1080 8 5 2;CBgems 480 360 64 5 2"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for cfg in "${CFG_LIST[@]}"; do
  for lib in $LIBS; do
    for pipe in $PIPES; do
      echo "== $cfg | $lib | pipeline $pipe"
      BDPT_LIB=$PWD/$lib BDPT_PIPELINE=$pipe timeout -k 10 300 python3 tools/prof_render.py $cfg || { echo STOP; exit 1; }
    done
  done
done
