"""The reference's unidirectional PathTracer (pathtracer.cpp:47-340), CPU.

  * oracle mode 0 (fp64, the reference's four TU-static RNG engines, -t 1 tile order) is bit-exact
    against the reference's own PathTracer (oracle/_ref/ref_driver -U; fixtures from
    tools/make_pt_golden.py): sampleBuffer and sampleCountBuffer (adaptive sampling), with
    MicrofacetBSDF, delta BSDFs, roulette (-m 0), hemisphere sampling (-H, -l 2), the thin lens
    (-b, -d), the environment light, ambient (InfiniteHemisphereLight) and directional lights;
  * the device code (bdpt_core.h pt_pixel, compiled for the CPU) is bit-exact against oracle
    mode 2 (fp32 device semantics, counter RNG) on the same configurations.
The GPU kernel is checked against mode 2 in tests/test_gpu_parity.py.
"""
import ctypes as C
import os

import numpy as np
import pytest

import bdpt_amd as B
from _util import MODE_C32, MODE_REF, REPO, oracle_pt_render

PT = os.path.join(REPO, "tests", "golden", "pt")
NAMES = ["lambertian", "delta", "microfacet", "roulette", "hemisphere", "env_lens", "adaptive",
         "bunny_microfacet", "ambient", "ambient_microfacet_env", "directional_ambient", "directional",
         "batch_rounding"]


def _load(name):
    g = np.load(os.path.join(PT, name + ".npz"))
    W, H = int(g["W"]), int(g["H"])
    sc = B.load_dae(os.path.join(REPO, "scenes", str(g["scene"]) + ".dae"), W, H)
    if bool(g["env"]):
        sc.set_envmap(B.load_exr(os.path.join(REPO, "tests", "golden", "env", "sky_32x16_zip_half.exr")))
    kw = dict(ns_area_light=int(g["nal"]), batch=int(g["batch"]), tol=float(g["tol"]),
              hemisphere=bool(g["hemi"]), lens_radius=float(g["lens"]), focal_distance=float(g["focal"]))
    return sc, g, W, H, int(g["spp"]), int(g["max_depth"]), kw


@pytest.mark.parametrize("name", NAMES)
def test_oracle_mode0_bit_exact_vs_reference_pathtracer(name):
    sc, g, W, H, spp, M, kw = _load(name)
    img, cnt, _ = oracle_pt_render(sc, W, H, spp, M, MODE_REF, threads=1, **kw)
    assert np.array_equal(cnt, g["counts"])
    assert np.array_equal(img, g["image"]), np.abs(img - g["image"]).max()


def test_batch_rounded_sample_counts():
    """ns_aa 4 below samplesPerBatch 32: the reference runs one whole batch and records
    num_samples = 32 for every pixel (pathtracer.cpp:301-337) — the reference's own counts
    (fixture batch_rounding, ref_driver -U) and oracle mode 0 agree on it, and so does mode 2 (the
    device semantics); tests/test_gpu_reduce.py asserts the same value for the GPU's reduced counts."""
    sc, g, W, H, spp, M, kw = _load("batch_rounding")
    assert spp == 4 and kw["batch"] == 32
    assert (g["counts"] == 32).all()
    for mode in (MODE_REF, MODE_C32):
        _, cnt, _ = oracle_pt_render(sc, W, H, spp, M, mode, threads=4, **kw)
        assert (cnt == 32).all()


_core = None


def core():
    global _core
    if _core is None:
        import sys
        sys.path.insert(0, REPO)
        import __graft_entry__ as ge
        ge.build_core_cpu()
        lib = C.CDLL(ge.CORE_CPU_SO)
        P = C.POINTER(C.c_double)
        lib.core_cpu_pt_render.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_uint64, C.c_int, C.c_int, C.c_float, C.c_int, C.c_double,
                                           C.c_double, P, C.POINTER(C.c_int)]
        _core = lib
    return _core


def core_pt_render(sc, W, H, spp, M, seed, ns_area_light, batch, tol, hemisphere, lens_radius, focal_distance):
    img = np.zeros((H, W, 3))
    cnt = np.zeros((H, W), np.int32)
    d = sc.desc()
    rc = core().core_cpu_pt_render(C.byref(d), W, H, spp, M, seed, ns_area_light, batch, tol, 1 if hemisphere else 0,
                                   lens_radius, focal_distance, img.ctypes.data_as(C.POINTER(C.c_double)),
                                   cnt.ctypes.data_as(C.POINTER(C.c_int)))
    assert rc == 0
    return img, cnt


@pytest.mark.parametrize("name", NAMES)
def test_device_pathtracer_bit_exact_vs_oracle_mode2(name):
    sc, g, W, H, spp, M, kw = _load(name)
    W, H = W // 2, H // 2
    sc = B.retarget_camera(sc, W, H) if "screenDist" in sc.camera else B.load_dae(
        os.path.join(REPO, "scenes", str(g["scene"]) + ".dae"), W, H)
    if bool(g["env"]):
        sc.set_envmap(B.load_exr(os.path.join(REPO, "tests", "golden", "env", "sky_32x16_zip_half.exr")))
    img, cnt = core_pt_render(sc, W, H, spp, M, 77, kw["ns_area_light"], kw["batch"], kw["tol"], kw["hemisphere"],
                              kw["lens_radius"], kw["focal_distance"])
    oimg, ocnt, _ = oracle_pt_render(sc, W, H, spp, M, MODE_C32, seed=77, threads=1, **kw)
    assert np.isfinite(img).all()
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(img, oimg), np.abs(img - oimg).max()


def test_pathtracer_rejects_invalid_settings():
    """Argument checks happen in bdpt_create before any device call."""
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 16, 12, 4, 3
    p.integrator = B.INTEGRATOR_PT
    p.ns_area_light = -1
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), 16, 12)
    ctx = C.c_void_p()
    assert B.load_library().bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == B.BDPT_E_INVALID
