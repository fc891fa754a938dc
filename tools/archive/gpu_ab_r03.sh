#!/bin/bash
# Interleaved A/B of library builds on one GPU box (tools/prof_render.py, one process per run).
#   LIBS="build_var_a.so build_var_b.so" ROUNDS=2 tools/gpu_ab_r03.sh
# CFGS: ';'-separated "scene W H spp M launches"; a leading "c5:" adds C5's synthetic sky + roulette.
cd "$(dirname "$0")/.." || exit 1
LIBS=${LIBS:-bidirectional-pathtracing_amd/libbdpt_amd.so}
ROUNDS=${ROUNDS:-2}
CFGS=${CFGS:-"scenes/CBlucy_standin.dae 1920 1080 8 5 2;scenes/CBlucy_standin.dae 800 600 32 5 2;CBgems 960 540 32 7 2;CBspheres 480 360 64 5 2;c5:scenes/CBlucy_standin.dae 1920 1080 8 8 2"}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "${CFG_LIST[@]}"; do
    for lib in $LIBS; do
      envs=""
      c=$cfg
      if [[ $cfg == c5:* ]]; then envs="BDPT_ENV=synth:1024x512 BDPT_RR=1"; c=${cfg#c5:}; fi
      echo "== r$r | $cfg | $lib"
      env $envs BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_render.py $c || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
