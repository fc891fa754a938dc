"""Environment light and Russian roulette (semantics: DESIGN.md §9), CPU.

Pinned against the reference itself (fixtures from tools/make_env_golden.py, which runs the
reference's own code built by oracle/ref.mk):
  * the OpenEXR reader (bdpt_exr_load) vs the reference's load_exr + tinyexr: bit-exact maps;
  * the oracle's fp64 environment math vs EnvironmentLight::init / sample_L / sample_dir
    (environment_light.cpp): bit-exact tables, samples and lookups (mode 1), and the fp32 device
    forms (mode 2) within fp32 tolerance;
  * BDPT with the environment light (which the reference cannot run: sample_Le & co. assert,
    environment_light.cpp:182-208) vs the reference's unidirectional PathTracer with the same map
    on a diffuse-only scene: converged image means agree (statistical, tolerance below).
Russian roulette has no reference run either; it is checked for unbiasedness (RR on vs off).
Device-code parity for both features: tests/test_core_cpu.py (bit-exact) and test_gpu_parity.py.
"""
import ctypes as C
import os

import numpy as np
import pytest

import bdpt_amd as B
from _util import MODE_C32, MODE_C64, REPO, golden_scene, oracle, oracle_render

ENV = os.path.join(REPO, "tests", "golden", "env")
MAPS = ["sky_32x16_zip_half", "sky_24x12_none_float", "sky_24x12_zips_half"]


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _scene_with(name):
    sc = golden_scene("CBspheres_lambertian", 32, 24)
    sc.set_envmap(B.load_exr(os.path.join(ENV, name + ".exr")))
    return sc


@pytest.mark.parametrize("name", MAPS)
def test_exr_reader_matches_reference_load_exr(name):
    g = np.load(os.path.join(ENV, name + ".npz"))
    img = B.load_exr(os.path.join(ENV, name + ".exr"))
    assert img.shape == g["rgb"].shape
    assert np.array_equal(img.astype(np.float64), g["rgb"])


@pytest.mark.parametrize("comp,pix", [("rle", "half"), ("rle", "float"), ("zip", "float"), ("none", "half")])
def test_exr_reader_roundtrip(tmp_path, comp, pix):
    """Layouts the reference's tinyexr build does not read (RLE) or that no fixture covers."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from envmap import synth_envmap, write_exr
    src = synth_envmap(40, 20, seed=3)
    p = str(tmp_path / "m.exr")
    write_exr(p, src, comp, pix)
    want = src.astype(np.float16).astype(np.float32) if pix == "half" else src
    assert np.array_equal(B.load_exr(p), want)


def test_exr_reader_errors(tmp_path):
    p = tmp_path / "bad.exr"
    p.write_bytes(b"not an exr file at all")
    with pytest.raises(B.BDPTError):
        B.load_exr(str(p))
    with pytest.raises(B.BDPTError):
        B.load_exr(str(tmp_path / "missing.exr"))


@pytest.mark.parametrize("name", MAPS)
def test_env_tables_match_reference(name):
    g = np.load(os.path.join(ENV, name + ".npz"))
    h, w = g["rgb"].shape[:2]
    m, c, p = np.zeros(h), np.zeros(w * h), np.zeros(w * h)
    sc = _scene_with(name)
    d = sc.desc()
    assert oracle().oracle_env_tables(C.byref(d), _p(m), _p(c), _p(p)) == 0
    assert np.array_equal(m, g["marginal_y"])
    assert np.array_equal(c, g["conds_y"])
    assert np.array_equal(p, g["pdf_envmap"])


def _ref_uniforms(n):
    """The uniforms of the reference's first n sample_L calls in a fresh process: the grid sample
    draws (y, x) from sampler.cpp's engine, the texel jitter (x, y) from environment_light.cpp's;
    both engines start default-seeded, so both read the same mt19937 sequence U0, U1, ..."""
    U = np.zeros(2 * n)
    oracle().oracle_mt_first(2 * n, _p(U))
    u = np.zeros((n, 4))
    u[:, 0], u[:, 1] = U[1::2], U[0::2]   # grid (x, y): y is drawn first
    u[:, 2], u[:, 3] = U[0::2], U[1::2]   # jitter x, then y
    return np.ascontiguousarray(u.reshape(-1))


@pytest.mark.parametrize("name", MAPS)
def test_env_sample_L_matches_reference(name):
    g = np.load(os.path.join(ENV, name + ".npz"))
    n = g["sample_pdf"].shape[0]
    u = _ref_uniforms(n)
    sc = _scene_with(name)
    d = sc.desc()
    for mode in (MODE_C64, MODE_C32):
        wi, pdf, rad = np.zeros(3 * n), np.zeros(n), np.zeros(3 * n)
        assert oracle().oracle_env_sample(C.byref(d), mode, n, _p(u), _p(wi), _p(pdf), _p(rad)) == 0
        wi, rad = wi.reshape(-1, 3), rad.reshape(-1, 3)
        if mode == MODE_C64:   # the reference's fp64 libm expressions: bit-exact
            assert np.array_equal(wi, g["sample_wi"])
            assert np.array_equal(pdf, g["sample_pdf"])
            assert np.array_equal(rad, g["sample_L"])
        else:                  # the device's fp32 semantics
            assert np.abs(wi - g["sample_wi"]).max() < 1e-6
            assert np.abs(pdf / g["sample_pdf"] - 1).max() < 1e-5
            assert np.abs(rad - g["sample_L"]).max() < 1e-4 * max(1.0, np.abs(g["sample_L"]).max())


@pytest.mark.parametrize("name", MAPS)
def test_env_sample_dir_matches_reference(name):
    g = np.load(os.path.join(ENV, name + ".npz"))
    dirs = g["dirs"]
    n = dirs.shape[0]
    sc = _scene_with(name)
    d = sc.desc()
    rad, pdf = np.zeros(3 * n), np.zeros(n)
    flat = np.ascontiguousarray(dirs.reshape(-1))
    assert oracle().oracle_env_lookup(C.byref(d), MODE_C64, n, _p(flat), _p(rad), _p(pdf)) == 0
    assert np.array_equal(rad.reshape(-1, 3), g["sample_dir"])
    # device semantics (unit directions): fp32 polynomial atan2 / acos, same texels
    unit = np.ascontiguousarray((dirs / np.linalg.norm(dirs, axis=1, keepdims=True)).reshape(-1))
    rad2, pdf2 = np.zeros(3 * n), np.zeros(n)
    assert oracle().oracle_env_lookup(C.byref(d), MODE_C32, n, _p(unit), _p(rad2), _p(pdf2)) == 0
    assert np.abs(rad2.reshape(-1, 3) - g["sample_dir"]).max() < 1e-3 * np.abs(g["sample_dir"]).max()


def _envonly_scene():
    g = np.load(os.path.join(ENV, "envonly_pt.npz"))
    W, H = int(g["W"]), int(g["H"])
    sc = B.load_dae(os.path.join(ENV, "CBspheres_envonly.dae"), W, H)
    assert sc.nlight == 0
    sc.set_envmap(B.load_exr(os.path.join(ENV, "sky_32x16_zip_half.exr")))
    return sc, g


@pytest.mark.parametrize("rr", [False, True])
def test_env_bdpt_converges_to_reference_pathtracer(rr):
    """BDPT lit only by the environment (all strategies incl. escaped eye rays, light subpaths
    from the emission disk, fresh env samples) vs the reference's own unidirectional PathTracer
    (next-event estimation through sample_L + sample_dir on escape) with the same map and depth.
    Measured: the image means agree within 0.3%, 4x4-block means within 4% (noise of the sun
    lobe). Tolerances: 1.5% on the mean, 10% per block."""
    sc, g = _envonly_scene()
    W, H, depth = int(g["W"]), int(g["H"]), int(g["depth"])
    ref = g["image"]
    samp = oracle_render(sc, W, H, 256, depth, MODE_C64, seed=7, rr=rr)[0]
    assert np.isfinite(samp).all()
    m, mr = samp.mean(axis=(0, 1)), ref.mean(axis=(0, 1))
    assert np.abs(m / mr - 1).max() < 0.015, (m, mr)
    blk = lambda a: a.reshape(4, H // 4, 4, W // 4, 3).mean(axis=(1, 3))
    assert np.abs(blk(samp) / blk(ref) - 1).max() < 0.10


def test_russian_roulette_unbiased():
    """RR on vs off (same scene, depth and samples): image means agree within noise."""
    sc = golden_scene("CBspheres_lambertian", 48, 36)
    a = oracle_render(sc, 48, 36, 128, 10, MODE_C64, seed=11, rr=False)[0]
    b = oracle_render(sc, 48, 36, 128, 10, MODE_C64, seed=11, rr=True)[0]
    assert np.isfinite(b).all()
    ma, mb = a.mean(axis=(0, 1)), b.mean(axis=(0, 1))
    assert np.abs(mb / ma - 1).max() < 0.02, (ma, mb)


def test_retired_wavefront_pipeline_rejected():
    """pipeline 2 (the wavefront pipeline, retired in round 5) is rejected before any device call."""
    sc = _scene_with("sky_32x16_zip_half")
    p = B.Params()
    p.width, p.height, p.spp, p.max_depth = 32, 24, 1, 5
    p.pipeline = B.PIPELINE_WAVEFRONT
    ctx = C.c_void_p()
    assert B.load_library().bdpt_create(C.byref(sc.desc()), C.byref(p), C.byref(ctx)) == B.BDPT_E_UNSUPPORTED
    assert not ctx.value
