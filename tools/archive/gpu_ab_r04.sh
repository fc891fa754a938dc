#!/bin/bash
# Round-4 A/B on one GPU box: parity screen of every library (tools/check_variant.py), then ROUNDS
# interleaved rounds of tools/prof_render.py over CFGS for every library.
#   LIBS="build_var_a.so build_var_b.so" ROUNDS=3 [SPLS="0 8"] tools/gpu_ab_r04.sh
# CFGS: ';'-separated "scene W H spp M launches"; a leading "c5:" adds C5's synthetic sky + roulette.
cd "$(dirname "$0")/.." || exit 1
LIBS=${LIBS:-bidirectional-pathtracing_amd/libbdpt_amd.so}
ROUNDS=${ROUNDS:-3}
SPLS=${SPLS:-0}
CFGS=${CFGS:-"scenes/CBlucy_standin.dae 1920 1080 8 5 2;c5:scenes/CBlucy_standin.dae 1920 1080 8 8 2;CBgems 960 540 32 7 2;CBspheres 480 360 64 5 2"}
for lib in $LIBS; do
  echo "== parity $lib"
  BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/check_variant.py || { echo "STOP parity rc=$?"; exit 1; }
done
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "${CFG_LIST[@]}"; do
    for spl in $SPLS; do
      for lib in $LIBS; do
        envs="BDPT_SPL=$spl"
        c=$cfg
        if [[ $cfg == c5:* ]]; then envs="$envs BDPT_ENV=synth:1024x512 BDPT_RR=1"; c=${cfg#c5:}; fi
        echo "== r$r | $cfg | spl $spl | $lib"
        env $envs BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_render.py $c || { echo "STOP rc=$?"; exit 1; }
      done
    done
  done
done
