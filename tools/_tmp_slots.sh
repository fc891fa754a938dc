cd "$(dirname "$0")/.." || exit 1
for cfg in "CBspheres 480 360 128 5 2" "scenes/CBlucy_standin.dae 1920 1080 8 5 2" "CBgems 480 360 64 5 2"; do
  for lib in build_var_w3.so build_var_w4.so build_var_w5.so; do
  echo "== $cfg $lib"
  BDPT_LIB=$PWD/$lib BDPT_PIPELINE=1 timeout -k 10 300 python3 tools/prof_render.py $cfg || { echo STOP; exit 1; }
  done
done
