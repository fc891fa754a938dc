#!/usr/bin/env python3
"""Minimal profiling target (no torch): renders one C2 frame (CBspheres 480x360, m=5) with N
launches of `spp` samples through the C-ABI. Used under rocprofv3 (kernel trace / PMC passes)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bidirectional-pathtracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import bdpt_amd as B  # noqa: E402
from _util import golden_scene  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "CBspheres"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (480, 360)
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 128
M = int(sys.argv[5]) if len(sys.argv) > 5 else 5
launches = int(sys.argv[6]) if len(sys.argv) > 6 else 2
if os.environ.get("BDPT_LIB"):   # a variant build replaces the default library (loaded once)
    B._lib = B.load_library(os.environ["BDPT_LIB"])
sc = B.load_dae(scene, W, H) if scene.endswith(".dae") else golden_scene(scene, W, H)
if os.environ.get("BDPT_ENV"):   # synth:WxH: the synthetic sky of tools/envmap.py (C5's stand-in map)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from envmap import synth_envmap
    ew, eh = (int(v) for v in os.environ["BDPT_ENV"].split(":")[1].split("x"))
    sc.set_envmap(synth_envmap(ew, eh))
pt = B.BidirectionalPathTracer(sc, W, H, spp * launches, M, seed=5489, samples_per_lane=int(os.environ.get("BDPT_SPL", "0")),
                               collect_stats=os.environ.get("BDPT_STATS") == "1",
                               russian_roulette=os.environ.get("BDPT_RR") == "1")
if os.environ.get("BDPT_WARM", "1") == "1":   # code-object load + first-launch setup, untimed
    pt.raytrace_tiles([], 0, 1)
    pt.sync()
    pt.clear()
t0 = time.perf_counter()
for k in range(launches):
    pt.raytrace_tiles([], k * spp, spp)
pt.sync()
dt = time.perf_counter() - t0
print(f"{scene} {W}x{H} s{spp}x{launches} m{M}: {dt*1e3:.1f} ms, "
      f"{W*H*spp*launches/dt/1e6:.1f} Msamples/s ")
if os.environ.get("BDPT_PHASES"):
    import ctypes as C
    arr = (C.c_uint64 * 16)()
    pt.lib.bdpt_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    pt.lib.bdpt_debug_counters(pt.ctx, arr)
    tot = arr[0] + arr[1] + arr[2]
    print("phase cycles (wave-summed): prepare %.3g (%.1f%%)  conn-gen %.3g (%.1f%%)  flush %.3g (%.1f%%)" % (
        arr[0], 100 * arr[0] / tot, arr[1], 100 * arr[1] / tot, arr[2], 100 * arr[2] / tot))
    print("  of prepare: walk closest-hit traversal %.1f%% (wave-summed, divergent lanes counted once)" % (
        100 * arr[3] / max(1, arr[0])))
    print("  of prepare: light vertex L[1] %.1f%%, hit -> next ray (shading, vertex, sample_f) %.1f%%" % (
        100 * arr[8] / max(1, arr[0]), 100 * arr[9] / max(1, arr[0])))
    print("  walk iterations: %.4g wave-level x 64 lanes, %.4g lane-level -> %.1f%% of the lane slots; "
          "connection cells %.4g x 64, (i, j) pairs %.4g -> %.1f%%" % (
              arr[4], arr[5], 100 * arr[5] / max(1, 64 * arr[4]), arr[6], arr[7],
              100 * arr[7] / max(1, 64 * arr[6])))
    lane = (C.c_uint64 * 16)()
    pt.lib.bdpt_debug_lane_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    pt.lib.bdpt_debug_lane_counters(pt.ctx, lane)
    names = ["closest-hit node steps", "closest-hit prim tests", "any-hit node steps", "any-hit prim tests",
             "walk shading (hit -> next ray)", "walk iterations", "connection evaluations (make_conn)",
             "connection-ray flushes (rays)"]
    print("  lane use per phase: wave-level iterations, mean active lanes of 64, share of all wave-iterations")
    tw = sum(lane[2 * k] for k in range(8) if k != 5)
    for k, nm in enumerate(names):
        w_, l_ = lane[2 * k], lane[2 * k + 1]
        print(f"    {nm:38s} {w_:14d}  {l_ / max(1, w_):6.2f} / 64 = {100 * l_ / max(1, 64 * w_):5.1f}%"
              + ("" if k == 5 else f"   {100 * w_ / max(1, tw):5.1f}% of iterations"))
if os.environ.get("BDPT_STATS") == "1":
    st = pt.stats()
    n = max(1, st.samples)
    print("per sample: " + ", ".join(f"{f} {getattr(st, f) / n:.2f}" for f, _ in st._fields_))
pt.close()
