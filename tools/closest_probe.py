#!/usr/bin/env python3
"""Probe (GPU box): the north star's walk queries (closest hit) traced by a kernel of their own
(tools/closest_probe.hip) with the product's trace_closest and with trace_closest_coop (lane
donation), tree in HBM (LM 0) or treelet in LDS (LM 2), in the order the CPU build generated them
(pixel by pixel) and shuffled. The two traversals must return the same (t, key) for every ray.
Prints Grays/s per case and the node visits (the coop form visits more: helpers prune with the
owner's distance at donation time).

  python3 tools/closest_probe.py [npix]     (npix random pixels of the 1920x1080 frame, 1 spp)
  (the CPU dump runs here or on the box; built libraries go to tools/bin/)
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
DUMP = os.path.join(REPO, "tools", "bin", "libcore_dump_closest.so")
PROBE = os.path.join(REPO, "tools", "bin", "libclosest_probe.so")
PROBE_PH = os.path.join(REPO, "tools", "bin", "libclosest_probe_ph.so")   # + lane-use profile
RAYS = os.path.join(REPO, "tools", "bin", "closest_rays.npy")
RAYS_ANY = os.path.join(REPO, "tools", "bin", "anyhit_rays.npy")


def build(probe=True):
    os.makedirs(os.path.dirname(DUMP), exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-DBDPT_STEP_HIST",
                    "-I" + os.path.join(REPO, "include"), "-I" + CS, "-o", DUMP,
                    os.path.join(REPO, "tests", "native", "core_cpu.cpp"), os.path.join(CS, "bdpt_scene.cpp")],
                   check=True)
    if probe:
        for out, extra in ((PROBE, []), (PROBE_PH, ["-DBDPT_PHASE_PROF"])):
            subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fno-slp-vectorize",
                            "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(REPO, "include"), "-I" + CS,
                            os.path.join(REPO, "tools", "closest_probe.hip"), os.path.join(CS, "bdpt_scene.cpp"),
                            "-o", out] + extra + [a for a in sys.argv if a.startswith("-D")], check=True)


def dump(sc, W, H, npix, kind=2):
    lib = C.CDLL(DUMP)
    pd = C.POINTER(C.c_double)
    eye, light, st = np.zeros((H, W, 3)), np.zeros((H, W, 3)), np.zeros(8)
    d = sc.desc()
    lib.core_cpu_ray_dump(kind)
    pix = np.random.default_rng(3).choice(W * H, npix, replace=False)
    pix = np.ascontiguousarray(np.stack([pix % W, pix // W], 1).astype(np.int32))
    assert lib.core_cpu_render(C.byref(d), W, H, 1, 5, C.c_uint64(5489), 0, 1,
                               pix.ctypes.data_as(C.POINTER(C.c_int)), npix, eye.ctypes.data_as(pd),
                               light.ctypes.data_as(pd), st.ctypes.data_as(pd), 2, 0) == 0
    lib.core_cpu_ray_dump_get.restype = C.c_longlong
    n = lib.core_cpu_ray_dump_get(None, C.c_longlong(0))
    rays = np.empty((n, 8), np.float32)
    lib.core_cpu_ray_dump_get(rays.ctypes.data_as(C.POINTER(C.c_float)), C.c_longlong(n))
    lib.core_cpu_ray_dump(0)
    return rays


def main():
    W, H = 1920, 1080
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    npix = int(args[0]) if args else 60000
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBlucy_standin.dae"), W, H)
    if "--dump-only" in sys.argv:   # the CPU part (this container): rays -> tools/bin/closest_rays.npy
        build(probe=False)
        t0 = time.time()
        for kind, path in ((2, RAYS), (1, RAYS_ANY)):
            rays = dump(sc, W, H, npix, kind)
            np.save(path, rays)
            print(f"{len(rays)} {'closest' if kind == 2 else 'any'}-hit rays from {npix} pixels "
                  f"({len(rays) / npix:.2f} per sample), CPU {time.time() - t0:.1f} s -> {path}", flush=True)
        return
    if "--build-only" in sys.argv:
        build()
        return
    ph = "--phases" in sys.argv
    pr = C.CDLL(PROBE_PH if ph else PROBE)
    pr.probe_closest.argtypes = [C.POINTER(B.SceneDesc), C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                 C.POINTER(C.c_ulonglong)]
    pr.probe_cfg_name.restype = C.c_char_p
    d = sc.desc()
    cfgs = [int(x) for x in os.environ.get("PROBE_CFGS", "0,1,2,3,4,5,6").split(",")]
    for any_hit, lm in ((0, 2), (1, 2)):
        rays = np.load(RAYS_ANY if any_hit else RAYS)
        reps = max(1, (4 << 20) // len(rays))
        base = np.tile(rays, (reps, 1))
        rng = np.random.default_rng(1)
        orders = {"generated": base, "shuffled": base[rng.permutation(len(base))]}
        for name, rr in orders.items():
            rr = np.ascontiguousarray(rr)
            outs = []
            for coop in cfgs:
                ms, ntop, nodes9 = C.c_float(), C.c_int(), (C.c_ulonglong * 9)()
                out = np.empty((len(rr), 2), np.int32)
                rc = pr.probe_closest(C.byref(d), rr.ctypes.data_as(C.POINTER(C.c_float)), len(rr), lm, coop, any_hit, 5,
                                      C.byref(ms), C.byref(ntop), out.ctypes.data_as(C.POINTER(C.c_int)),
                                      nodes9)
                assert rc == 0
                nodes = nodes9[0]
                outs.append(out)
                lp = list(nodes9)[1:]
                k = 2 if any_hit else 0   # LP_ANODE / LP_CNODE, then the primitive tests
                prof = (f"; node loop {lp[2 * k] / len(rr) * 64:.2f} wave-iterations per 64 rays at "
                        f"{lp[2 * k + 1] / max(1, 64 * lp[2 * k]):.1%} lane use, prim tests "
                        f"{lp[2 * k + 2] / len(rr) * 64:.2f} at {lp[2 * k + 3] / max(1, 64 * lp[2 * k + 2]):.1%}") if ph else ""
                print(f"{'any    ' if any_hit else 'closest'} LM {lm} treelet {ntop.value:4d} {name:9s} "
                      f"{pr.probe_cfg_name(coop).decode():11s}: "
                      f"{ms.value:7.3f} ms for {len(rr)} rays = {len(rr) / ms.value / 1e6:6.2f} Grays/s, "
                      f"{nodes / len(rr) / 4:.2f} node steps/ray, hits {np.mean(out[:, 1] >= 0):.3f}{prof}", flush=True)
            for k in range(1, len(outs)):
                same = np.array_equal(outs[0], outs[k])
                if not same:
                    print(f"  config {cfgs[k]}: {np.sum(np.any(outs[0] != outs[k], axis=1))} rays differ", flush=True)
                    sys.exit(1)
            print("  identical (t bits, key) for every ray in every configuration", flush=True)


if __name__ == "__main__":
    main()
