"""Test helpers: load the oracle (test infrastructure) and golden fixtures."""
import ctypes as C
import json
import os
import subprocess

import numpy as np

import bdpt_amd as B

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")

MODE_REF, MODE_C64, MODE_C32 = 0, 1, 2


def build_oracle(force=False):
    src = os.path.join(REPO, "oracle", "bdpt_oracle.cpp")
    if force or not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared",
                        "-I" + os.path.join(REPO, "include"), "-o", ORACLE_SO, src, "-lpthread"],
                       check=True)
    return ORACLE_SO


_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        lib = C.CDLL(build_oracle())
        P = C.POINTER(C.c_double)
        lib.oracle_render.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int, P, P, P, P]
        lib.oracle_render_ex.argtypes = lib.oracle_render.argtypes + [C.c_int]
        lib.oracle_pt_render.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_float, C.c_int,
                                         C.c_double, C.c_double, C.c_int, P, C.POINTER(C.c_int), P]
        lib.oracle_env_tables.argtypes = [C.POINTER(B.SceneDesc), P, P, P]
        lib.oracle_env_sample.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, P, P, P, P]
        lib.oracle_env_lookup.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, P, P, P]
        lib.oracle_bvh_info.argtypes = [C.POINTER(B.SceneDesc), C.POINTER(C.c_int),
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.oracle_trace_rays.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.POINTER(C.c_float),
                                          C.c_int, C.c_int, C.POINTER(C.c_float),
                                          C.POINTER(C.c_int)]
        lib.oracle_philox.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_uint32)]
        lib.oracle_philox.restype = None
        lib.oracle_cos_sin_2pi.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        lib.oracle_cos_sin_2pi.restype = None
        lib.oracle_mt_first.argtypes = [C.c_int, P]
        lib.oracle_mt_first.restype = C.c_double
        lib.oracle_set_hit_frame_ref.argtypes = [C.c_int]
        lib.oracle_set_hit_frame_ref.restype = None
        _oracle = lib
    return _oracle


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def oracle_render(scene, W, H, spp, max_depth, mode, seed=5489, s0=0, count=None, threads=None,
                  rr=False):
    """Returns (sample, eye, light, stats) as float64 arrays (H, W, 3); row 0 = bottom."""
    lib = oracle()
    if count is None:
        count = spp - s0
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    eye = np.zeros((H, W, 3))
    light = np.zeros((H, W, 3))
    samp = np.zeros((H, W, 3))
    st = np.zeros(8)
    d = scene.desc()
    rc = lib.oracle_render_ex(C.byref(d), W, H, spp, max_depth, mode, seed, s0, count, threads,
                              _p(eye), _p(light), _p(samp), _p(st), 1 if rr else 0)
    if rc != 0:
        raise RuntimeError(f"oracle_render rc={rc}")
    if mode != MODE_REF:
        samp = eye + light
    return samp, eye, light, st


def oracle_pt_render(scene, W, H, spp, max_depth, mode, seed=5489, ns_area_light=1, batch=32, tol=0.05,
                     hemisphere=False, lens_radius=0.0, focal_distance=4.7, threads=None):
    """The oracle's unidirectional PathTracer (pathtracer.cpp): (image (H, W, 3) = sampleBuffer,
    counts (H, W) = sampleCountBuffer, stats)."""
    lib = oracle()
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    img = np.zeros((H, W, 3))
    cnt = np.zeros((H, W), dtype=np.int32)
    st = np.zeros(8)
    d = scene.desc()
    rc = lib.oracle_pt_render(C.byref(d), W, H, spp, max_depth, mode, seed, ns_area_light, batch, tol,
                              1 if hemisphere else 0, lens_radius, focal_distance, threads, _p(img),
                              cnt.ctypes.data_as(C.POINTER(C.c_int)), _p(st))
    if rc != 0:
        raise RuntimeError(f"oracle_pt_render rc={rc}")
    return img, cnt, st


_ndev = None


def device_count() -> int:
    """Visible GPUs (torch.cuda.device_count(), which counts without initialising HIP on this
    image); 0 in the CPU container. The >= 2-device tests skip below 2."""
    global _ndev
    if _ndev is None:
        try:
            import torch
            _ndev = int(torch.cuda.device_count())
        except Exception:
            _ndev = 0
    return _ndev


def golden_scene(name, width=None, height=None):
    sc = B.scene_from_json(os.path.join(GOLD, "scenes", name + ".json"))
    if width is not None:
        sc = B.retarget_camera(sc, width, height)
    return sc


def golden_index():
    with open(os.path.join(GOLD, "hdr", "index.json")) as f:
        return json.load(f)
