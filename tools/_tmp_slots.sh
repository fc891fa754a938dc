cd "$(dirname "$0")/.." || exit 1
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q 2>&1 | tail -2
for cfg in "CBspheres 480 360 128 5 2" "scenes/CBlucy_standin.dae 1920 1080 8 5 2" "CBgems 480 360 64 5 2"; do
  for lib in build_var_a.so build_var_b.so; do
  for pipe in 1 2; do
  echo "== $cfg $lib $pipe"
  BDPT_LIB=$PWD/$lib BDPT_WF_SLOTS=4194304 BDPT_PIPELINE=$pipe timeout -k 10 300 python3 tools/prof_render.py $cfg || { echo STOP; exit 1; }
  done
  done
done
