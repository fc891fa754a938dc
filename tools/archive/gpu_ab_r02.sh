#!/bin/bash
# Round-2 A/B session: every build_var_*.so on the three A/B scenes (two interleaved rounds),
# then the GPU test suite on the default library.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
LIBS=$(ls build_var_*.so | tr '\n' ' ')
CFGS=${CFGS:-"scenes/CBlucy_standin.dae 1920 1080 32 5 2;CBspheres 480 360 128 5 2;CBgems 480 360 64 5 2"}
for r in 1 2; do
  LIBS="$LIBS" CFGS="$CFGS" bash tools/ab_libs.sh 2>&1 | grep -v amdgpu.ids || exit 1
done
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_pytest.log; exit $rc
fi
