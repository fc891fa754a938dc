mkdir -p gpurun_out/r04r
timeout -k 10 300 python -u -m pytest -v --timeout 200 tests/test_cli.py tests/test_integration.py -m gpu > gpurun_out/r04r/t_cli_int.log 2>&1
tail -3 gpurun_out/r04r/t_cli_int.log
(timeout -k 10 600 oracle/_ref/ref_driver_amd -A -t 8 -s 128 -m 5 -r 1920 1080 -f gpurun_out/r04r/loop_a.png scenes/CBlucy_standin.dae | tr "\r" "\n" | grep -v "Rendering\.\.\. [0-9]*%$" | tail -4; timeout -k 10 300 bidirectional-pathtracing_amd/pathtracer -s 128 -m 5 -r 1920 1080 -f gpurun_out/r04r/cli.png --no-stats scenes/CBlucy_standin.dae 2>&1 | tail -2; python3 tools/cmp_png.py gpurun_out/r04r/loop_a.png gpurun_out/r04r/cli.png) > gpurun_out/r04r/loop_A128.log 2>&1
rm -f gpurun_out/r04r/*.png
cat gpurun_out/r04r/loop_A128.log
LIBS="build_var_base.so build_var_early.so build_var_earlyc.so build_var_earlya.so" ROUNDS=3 CFGS="scenes/CBlucy_standin.dae 1920 1080 8 5 2;c5:scenes/CBlucy_standin.dae 1920 1080 8 8 2" timeout -k 10 900 tools/gpu_ab_r04.sh > gpurun_out/r04r/ab_early.log 2>&1
grep -E "==|Msamples|ms" gpurun_out/r04r/ab_early.log | tail -40
