#!/bin/bash
# Two-library A/B on the mesh workloads: LIBS="build_var_a.so build_var_b.so" (default: the
# quantized-node pair q0 / q1) on the north-star stand-in, CBbunny, the C5 shape (stand-in +
# synthetic sky + roulette, m8) and CBgems (LDS-resident BVH2), two interleaved rounds.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
LIBS=${LIBS:-"build_var_q0.so build_var_q1.so"}
for r in 1 2; do
  LIBS="$LIBS" CFGS="scenes/CBlucy_standin.dae 1920 1080 32 5 2;scenes/CBbunny.dae 800 600 64 5 2;CBgems 480 360 64 5 2" \
    bash tools/ab_libs.sh || exit 1
  BDPT_ENV=synth:1024x512 BDPT_RR=1 LIBS="$LIBS" CFGS="scenes/CBlucy_standin.dae 1920 1080 16 8 2" bash tools/ab_libs.sh || exit 1
done
