#!/usr/bin/env python3
"""Parity screen of an A/B library build (BDPT_LIB=build_var_x.so) before timing it: renders small
frames of the north-star, C4 and C5 shapes and prints the per-pixel RMSE against oracle mode 2
(test infrastructure; the tests proper run on the default library). Exit 1 if any exceeds 1e-4."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "bidirectional-pathtracing_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import bdpt_amd as B  # noqa: E402
from _util import MODE_C32, golden_scene, oracle_render  # noqa: E402

if os.environ.get("BDPT_LIB"):
    B._lib = B.load_library(os.environ["BDPT_LIB"])
from bench import STANDIN, ensure_standin  # noqa: E402
from envmap import synth_envmap  # noqa: E402

ensure_standin(os.path.join(REPO, STANDIN))
bad = 0
for name, W, H, S, M, env, rr, spl in [("standin", 192, 108, 3, 5, False, False, 0),
                                       ("standin", 192, 108, 5, 8, True, True, 0),
                                       ("standin", 160, 90, 9, 8, True, True, 8),
                                       ("CBgems", 128, 96, 3, 7, False, False, 0),
                                       ("CBspheres", 96, 72, 5, 5, False, False, 4)]:
    sc = B.load_dae(os.path.join(REPO, STANDIN), W, H) if name == "standin" else golden_scene(name, W, H)
    if env:
        sc.set_envmap(synth_envmap(256, 128))
    pt = B.BidirectionalPathTracer(sc, W, H, S, M, seed=5489, russian_roulette=rr, samples_per_lane=spl)
    try:
        pt.raytrace_tiles()
    except B.BDPTError as e:   # a BDPT_ONLY_MAXV variant build has one depth class only
        if "variant build" not in str(e):
            raise
        print(f"{name} m{M}: skipped ({e})", flush=True)
        pt.close()
        continue
    g = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    ref = oracle_render(sc, W, H, S, M, MODE_C32, rr=rr)[0]
    rmse = float(np.sqrt(np.mean((g - ref) ** 2)))
    ok = rmse < 1e-4 and np.isfinite(g).all()
    bad += not ok
    print(f"{name} {W}x{H} s{S} m{M} env={env} rr={rr} spl={spl}: rmse {rmse:.3e} {'ok' if ok else 'FAIL'}", flush=True)
sys.exit(1 if bad else 0)
