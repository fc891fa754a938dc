#!/bin/bash
# Timing-only A/B (no parity screen: for variants that drop work on purpose to bound its cost).
#   LIBS="a.so b.so" ROUNDS=3 CFGS="scene W H spp M launches;..." tools/gpu_ab_timing.sh
cd "$(dirname "$0")/.." || exit 1
ROUNDS=${ROUNDS:-3}
IFS=';' read -ra CFG_LIST <<< "$CFGS"
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "${CFG_LIST[@]}"; do
    for lib in $LIBS; do
      envs="BDPT_SPL=0"; c=$cfg
      if [[ $cfg == c5:* ]]; then envs="$envs BDPT_ENV=synth:1024x512 BDPT_RR=1"; c=${cfg#c5:}; fi
      echo "== r$r | $cfg | $lib"
      env $envs BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/prof_render.py $c || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
