"""C-ABI boundary checks that need no GPU: libbdpt_amd.so loads and exports every function
include/bdpt/bdpt.h declares; argument and scene validation happen before any device call."""
import ctypes as C
import os
import re
import subprocess

import pytest

import bdpt_amd as B
from _util import REPO, golden_scene

HEADER = os.path.join(REPO, "include", "bdpt", "bdpt.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(bdpt_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_function():
    names = declared_functions()
    assert len(names) >= 18
    lib = B.load_library()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", B.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (bdpt_\w+)", out))
    assert set(names) <= exported, sorted(set(names) - exported)


def test_abi_version():
    assert B.load_library().bdpt_abi_version() == 9   # v2: envmap + RR; v3: integrator; v4: LDS stats; v5: camera settings; v6: env-table stats; v7: camera lens settings; v8: frame rectangles; v9: RCCL frame reduce


def test_frame_reduce_loads_rccl_and_validates_arguments():
    """bdpt_reduce_*: the product loads RCCL itself (dlopen librccl.so.1, no GPU needed for
    ncclGetVersion), and rejects bad arguments before touching a device."""
    lib = B.load_library()
    v = lib.bdpt_reduce_rccl_version()
    assert v >= 20000, lib.bdpt_last_error()   # NCCL_VERSION_CODE of RCCL 2.x
    h = C.c_void_p()
    assert lib.bdpt_reduce_create(None, 1, C.byref(h)) == B.BDPT_E_INVALID
    arr = (C.c_void_p * 1)(None)
    assert lib.bdpt_reduce_create(arr, 0, C.byref(h)) == B.BDPT_E_INVALID
    assert lib.bdpt_reduce_create(arr, 1, C.byref(h)) == B.BDPT_E_INVALID and not h.value
    assert lib.bdpt_reduce_frames(None, 0) == B.BDPT_E_INVALID
    assert lib.bdpt_reduce_ranks(None) == B.BDPT_E_INVALID
    lib.bdpt_reduce_destroy(None)


def test_null_arguments_rejected():
    lib = B.load_library()
    assert lib.bdpt_create(None, None, None) == -1
    assert b"null" in lib.bdpt_last_error()


def test_unsupported_material_rejected_before_device():
    sc = golden_scene("CBspheres", 32, 24)
    sc.mats[0].type = 5   # BDPT_MAT_MICROFACET: its sample_pdf asserts under BDPT (advanced_bsdf.cpp:144-148)
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 32, 24, 1, 5
    ctx = C.c_void_p()
    lib = B.load_library()
    assert lib.bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == -2
    assert not ctx.value


def test_ambient_light_rejected_under_bdpt_only():
    """An ambient light (GLScene::AmbientLight -> InfiniteHemisphereLight) only implements sample_L
    (light.cpp:62-98): the BDPT integrator rejects it before touching a device; the PathTracer
    accepts it (bdpt_create then fails only for want of a device here)."""
    sc = B.load_dae(os.path.join(REPO, "scenes", "bunny.dae"), 32, 24)
    assert [l.type for l in sc.lights] == [B.LIGHT_HEMISPHERE]
    lib = B.load_library()
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 32, 24, 1, 5
    ctx = C.c_void_p()
    assert lib.bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == B.BDPT_E_UNSUPPORTED
    assert b"InfiniteHemisphereLight" in lib.bdpt_last_error()
    p.integrator = B.INTEGRATOR_PT
    assert lib.bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) != B.BDPT_E_UNSUPPORTED
    sc = B.load_dae(os.path.join(REPO, "scenes", "teapot.dae"), 32, 24)   # DirectionalLight
    assert [l.type for l in sc.lights] == [B.LIGHT_DIRECTIONAL]
    p.integrator = B.INTEGRATOR_BDPT
    assert lib.bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == B.BDPT_E_UNSUPPORTED


def test_material_id_range_rejected_before_device():
    """The path store keeps a vertex's material id in 16 signed bits (bdpt_core.h VtxS): a scene
    with 32,768 materials is rejected with BDPT_E_UNSUPPORTED instead of wrapping on the device;
    32,767 passes the scene checks (and then needs a device)."""
    sc = golden_scene("CBspheres", 32, 24)
    lib = B.load_library()
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 32, 24, 1, 5
    ctx = C.c_void_p()
    for n, unsupported in ((32768, True), (32767, False)):
        mats = [sc.mats[i] for i in range(sc.nmat)] + [sc.mats[0]] * (n - sc.nmat)
        big = B.Scene(sc.prim_type, sc.prim_geom, sc.prim_mat.copy(), mats,
                      [sc.lights[i] for i in range(sc.nlight)], sc.camera)
        big.prim_mat[0] = n - 1   # the last material is used
        rc = lib.bdpt_create(C.byref(big.desc()), C.byref(p), C.byref(ctx))
        assert (rc == B.BDPT_E_UNSUPPORTED) == unsupported, (n, rc, lib.bdpt_last_error())
        if unsupported:
            assert b"32767" in lib.bdpt_last_error()
        if ctx.value:
            lib.bdpt_destroy(ctx)
            ctx = C.c_void_p()


def test_bad_frame_size_rejected():
    sc = golden_scene("CBspheres", 32, 24)
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 0, 24, 1, 5
    ctx = C.c_void_p()
    assert B.load_library().bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == -1


def test_dae_missing_file():
    with pytest.raises(Exception):
        B.load_dae(os.path.join(REPO, "scenes", "no_such_scene.dae"))


def test_depth_limits_rejected_before_device():
    """The kernels hold a subpath in a fixed array: m <= 126 is instantiated (the reference's vectors
    have no cap, bidirection.cpp:84-86); m = 127 is rejected cleanly with the reason, as is a
    PathTracer depth past its 21 recorded vertices. m = 126 passes the checks (then needs a device)."""
    sc = golden_scene("CBspheres", 32, 24)
    lib = B.load_library()
    p = B.Params()
    p.width, p.height, p.spp = 32, 24, 1
    ctx = C.c_void_p()
    for m, pt, unsupported in ((127, False, True), (126, False, False), (63, False, False), (22, True, True),
                               (21, True, False)):
        p.max_depth = m
        p.integrator = B.INTEGRATOR_PT if pt else B.INTEGRATOR_BDPT
        rc = lib.bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx))
        assert (rc == B.BDPT_E_UNSUPPORTED) == unsupported, (m, pt, rc, lib.bdpt_last_error())
        if unsupported:
            assert b"max_depth" in lib.bdpt_last_error()
        if ctx.value:
            lib.bdpt_destroy(ctx)
            ctx = C.c_void_p()
