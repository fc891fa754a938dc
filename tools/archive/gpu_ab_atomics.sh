mkdir -p gpurun_out
for lib in build_var_lane.so build_var_lsplat.so build_var_leye.so; do echo "== parity $lib"; BDPT_LIB=$PWD/$lib timeout -k 10 300 python3 tools/check_variant.py || { echo "STOP parity"; exit 1; }; done > gpurun_out/ab_at_parity.log 2>&1
cat gpurun_out/ab_at_parity.log | grep -v "^W2026"
LIBS="build_var_base.so build_var_lane.so build_var_lsplat.so build_var_leye.so build_var_nosplat.so build_var_noeye.so" ROUNDS=3 CFGS="scenes/CBlucy_standin.dae 1920 1080 8 5 2;CBgems 960 540 32 7 2" timeout -k 10 600 bash tools/gpu_ab_timing.sh > gpurun_out/ab_atomics.log 2>&1
grep -E "^==|Msamples" gpurun_out/ab_atomics.log | paste - - | sed 's/ | spl 0//' | cut -c1-160
