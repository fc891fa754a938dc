#!/usr/bin/env python3
"""CPU diagnostics (no GPU): the distribution of node steps per closest-hit query of the device
traversal (bdpt_core.h compiled for the host with -DBDPT_STEP_HIST, one lane, the same tree and
visit order as the GPU), and its expected maximum over the 48 lanes that walk in a wave — the
wave-level iteration count of the node loop. Used to screen tree-building
changes before a GPU run; results are checked bit-exact against oracle mode 2 at the same time.

  python3 tools/step_hist.py [env KEY=VAL ...]     e.g. BDPT_COLLAPSE=sah
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bidirectional-pathtracing_amd"), os.path.join(REPO, "tests")]
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import bdpt_amd as B  # noqa: E402
from _util import MODE_C32, golden_scene, oracle_render  # noqa: E402

CS = os.path.join(REPO, "bidirectional-pathtracing_amd", "csrc")
LIB = "/tmp/libcore_stephist.so"
subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-DBDPT_STEP_HIST",
                "-I" + os.path.join(REPO, "include"), "-I" + CS, "-o", LIB,
                os.path.join(REPO, "tests", "native", "core_cpu.cpp"), os.path.join(CS, "bdpt_scene.cpp")], check=True)
lib = C.CDLL(LIB)
for name, W, H, spp, M, lm in [("standin", 192, 108, 2, 5, 2), ("CBbunny", 160, 120, 2, 5, 2),
                               ("CBgems", 192, 108, 2, 7, 0)]:
    if name == "standin":
        sc = B.load_dae(os.path.join(REPO, "scenes", "CBlucy_standin.dae"), W, H)
    elif name == "CBbunny":
        sc = B.load_dae(os.path.join(REPO, "scenes", "CBbunny.dae"), W, H)
    else:
        sc = golden_scene(name, W, H)
    eye, light, st = np.zeros((H, W, 3)), np.zeros((H, W, 3)), np.zeros(8)
    pd = C.POINTER(C.c_double)
    d = sc.desc()
    rc = lib.core_cpu_render(C.byref(d), W, H, spp, M, C.c_uint64(5489), 0, spp, None, 0, eye.ctypes.data_as(pd),
                             light.ctypes.data_as(pd), st.ctypes.data_as(pd), lm, 0)
    assert rc == 0
    hh = (C.c_ulonglong * 1024)()
    lib.core_cpu_step_hist(hh)
    hh = np.array(hh, dtype=np.float64)
    h, ha, ho, hm = hh[:256], hh[256:512], hh[512:768], hh[768:]
    n, k = h.sum(), np.arange(256)
    cdf = np.cumsum(h) / n
    emax = float(np.sum(1 - cdf[:255] ** 48))
    cdfa = np.cumsum(ha) / max(1, ha.sum())
    emaxa = float(np.sum(1 - cdfa[:255] ** 64))
    ref = oracle_render(sc, W, H, spp, M, MODE_C32, seed=5489, threads=8)
    exact = np.array_equal(eye, ref[1]) and np.array_equal(light, ref[2])
    print(f"{name} LM{lm}: steps/query mean {(h * k).sum() / n:.3f} p90 {int(np.searchsorted(cdf, .9))} "
          f"p99 {int(np.searchsorted(cdf, .99))} E[max of 48] {emax:.2f}; prim tests/query "
          f"{(st[4] + st[5]) / max(1, st[1] + st[2]):.3f}; any-hit steps/query mean "
          f"{(ha * k).sum() / max(1, ha.sum()):.3f} E[max of 64] {emaxa:.2f}; bit-exact vs mode 2: {exact}", flush=True)
    cdfo = np.cumsum(ho) / max(1, ho.sum())
    print(f"  given the final hit distance: mean {(ho * k).sum() / max(1, ho.sum()):.3f} p99 "
          f"{int(np.searchsorted(cdfo, .99))} E[max of 48] {float(np.sum(1 - cdfo[:255] ** 48)):.2f}; queries that "
          f"hit nothing: {hm.sum() / max(1, n):.3%} of all, their mean {(hm * k).sum() / max(1, hm.sum()):.2f}", flush=True)
