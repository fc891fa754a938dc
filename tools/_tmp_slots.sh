cd "$(dirname "$0")/.." || exit 1
timeout -k 10 600 python3 bench.py --scene scenes/CBlucy_standin.dae --width 1920 --height 1080 --spp 128 --steps 2 --warmup 1 > gpurun_out/bench_lucy1080.log 2>&1 || exit 1
tail -1 gpurun_out/bench_lucy1080.log
timeout -k 10 600 python3 bench.py --scene scenes/CBlucy_standin.dae --width 800 --height 600 --spp 128 --steps 3 --warmup 1 > gpurun_out/bench_lucy800.log 2>&1 || exit 1
tail -1 gpurun_out/bench_lucy800.log
timeout -k 10 600 python3 bench.py --scene scenes/CBgems.dae --width 1920 --height 1080 --spp 256 --max-depth 7 --steps 1 --warmup 1 --no-parity > gpurun_out/bench_gems1080.log 2>&1 || exit 1
tail -1 gpurun_out/bench_gems1080.log
