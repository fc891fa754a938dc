#!/usr/bin/env python3
"""Probe (GPU box): the north star's connection rays traced by a kernel of their own
(tools/anyhit_probe.hip) at 4 / 8 waves per SIMD, tree in HBM (LM 0) or treelet in LDS (LM 2), in
three orders — as the CPU build generated them (pixel by pixel), shuffled (what a flush sees), and
binned by direction octant + origin Morton code (what a coherence pass would give). The rays are
the any-hit queries of a CPU-build render of the stand-in (BDPT_STEP_HIST diagnostics lib), tiled
to a few million. Prints Grays/s per case.

  python3 tools/anyhit_probe.py [npix]     (npix random pixels of the 1920x1080 north-star frame, 1 spp)
"""
import ctypes as C
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "bidirectional-pathtracing_amd")]
import bdpt_amd as B  # noqa: E402

CS = os.path.join(REPO, "bidirectional-pathtracing_amd", "csrc")
DUMP = os.path.join(REPO, "tools", "bin", "libcore_dump.so")
PROBE = os.path.join(REPO, "tools", "bin", "libanyhit_probe.so")


def build():
    if not os.path.exists(DUMP):
        subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-DBDPT_STEP_HIST",
                        "-I" + os.path.join(REPO, "include"), "-I" + CS, "-o", DUMP,
                        os.path.join(REPO, "tests", "native", "core_cpu.cpp"), os.path.join(CS, "bdpt_scene.cpp")],
                       check=True)
    if not os.path.exists(PROBE):
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fno-slp-vectorize",
                        "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(REPO, "include"), "-I" + CS,
                        os.path.join(REPO, "tools", "anyhit_probe.hip"), os.path.join(CS, "bdpt_scene.cpp"),
                        "-o", PROBE], check=True)


def morton10(v):
    v = v.astype(np.uint64) & 0x3FF
    v = (v | (v << 16)) & 0x30000FF
    v = (v | (v << 8)) & 0x300F00F
    v = (v | (v << 4)) & 0x30C30C3
    v = (v | (v << 2)) & 0x9249249
    return v


def main():
    W, H, spp = 1920, 1080, 1
    npix = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    build()
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBlucy_standin.dae"), W, H)
    lib = C.CDLL(DUMP)
    pd = C.POINTER(C.c_double)
    eye, light, st = np.zeros((H, W, 3)), np.zeros((H, W, 3)), np.zeros(8)
    d = sc.desc()
    lib.core_cpu_ray_dump(1)
    t0 = time.time()
    pix = np.random.default_rng(3).choice(W * H, npix, replace=False)
    pix = np.ascontiguousarray(np.stack([pix % W, pix // W], 1).astype(np.int32))
    assert lib.core_cpu_render(C.byref(d), W, H, spp, 5, C.c_uint64(5489), 0, spp,
                               pix.ctypes.data_as(C.POINTER(C.c_int)), npix, eye.ctypes.data_as(pd),
                               light.ctypes.data_as(pd), st.ctypes.data_as(pd), 2, 0) == 0
    lib.core_cpu_ray_dump_get.restype = C.c_longlong
    n = lib.core_cpu_ray_dump_get(None, C.c_longlong(0))
    rays = np.empty((n, 8), np.float32)
    lib.core_cpu_ray_dump_get(rays.ctypes.data_as(C.POINTER(C.c_float)), C.c_longlong(n))
    lib.core_cpu_ray_dump(0)
    print(f"{n} any-hit rays from {npix} pixels of {W}x{H} s{spp} m5 ({n / (npix * spp):.2f} per sample), "
          f"CPU {time.time() - t0:.1f} s",
          flush=True)
    reps = max(1, (4 << 20) // n)
    base = np.tile(rays, (reps, 1))
    rng = np.random.default_rng(1)
    lo, hi = rays[:, :3].min(0), rays[:, :3].max(0)
    q = ((base[:, :3] - lo) / np.maximum(hi - lo, 1e-6) * 1023).astype(np.int64).clip(0, 1023)
    key = ((((base[:, 3] < 0).astype(np.uint64) << 2) | ((base[:, 4] < 0).astype(np.uint64) << 1)
            | (base[:, 5] < 0).astype(np.uint64)) << 30) | morton10(q[:, 0]) | (morton10(q[:, 1]) << 1) \
        | (morton10(q[:, 2]) << 2)
    orders = {"generated": base, "shuffled": base[rng.permutation(len(base))],
              "binned": base[np.argsort(key, kind="stable")]}
    pr = C.CDLL(PROBE)
    pr.probe_any.argtypes = [C.POINTER(B.SceneDesc), C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int, C.c_int,
                             C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    ref = None
    for lm in (0, 2):
        for wpe in (4, 8):
            for name, rr in orders.items():
                rr = np.ascontiguousarray(rr)
                ms, occ, ntop = C.c_float(), C.c_int(), C.c_int()
                occl = pr.probe_any(C.byref(d), rr.ctypes.data_as(C.POINTER(C.c_float)), len(rr), lm, wpe, 5,
                                    C.byref(ms), C.byref(occ), C.byref(ntop))
                assert occl >= 0
                if ref is None:
                    ref = occl
                assert occl == ref, (occl, ref)   # every order and kernel: the same occluded count
                print(f"LM {lm} waves/SIMD {occ.value} (asked {wpe}) treelet {ntop.value:4d} {name:9s}: "
                      f"{ms.value:7.3f} ms for {len(rr)} rays = {len(rr) / ms.value / 1e6:6.2f} Grays/s, "
                      f"{occl / len(rr):.3f} occluded", flush=True)


if __name__ == "__main__":
    main()
