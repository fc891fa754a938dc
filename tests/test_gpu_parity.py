"""GPU parity: the HIP path (libbdpt_amd.so through the C-ABI) against the oracle's COUNTER32 mode
(oracle/bdpt_oracle.cpp, fp32 device semantics) at the same seed.

Tolerance (north star): per-pixel RMSE < 1e-4 over the fp64 sample buffer (eye + light images).
Sample paths are computed with identical fp32 operations on both sides; the only expected
difference is the order of fp32 atomic additions of the light-image splats and of the per-lane
eye sums, ~1e-7 relative.
"""
import ctypes as C
import os

import numpy as np
import pytest

import bdpt_amd as B
from _util import MODE_C32, REPO, golden_scene, oracle, oracle_render

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4
PIPES = [pytest.param(B.PIPELINE_MEGAKERNEL, id="mega")]   # the wavefront pipeline was retired in round 5


def _gpu_render(sc, W, H, S, M, seed=5489, tiles=(), ranges=None, spl=0, stats=False,
                pipeline=B.PIPELINE_AUTO, rr=False):
    pt = B.BidirectionalPathTracer(sc, W, H, S, M, seed=seed, samples_per_lane=spl,
                                   collect_stats=stats, pipeline=pipeline, russian_roulette=rr)
    try:
        if ranges is None:
            ranges = [(0, S)]
        for a, b in ranges:
            pt.raytrace_tiles(list(tiles), a, b - a)
        out = {k: pt.read_frame(v).astype(np.float64)
               for k, v in (("sample", B.FRAME_SAMPLE), ("eye", B.FRAME_EYE),
                            ("light", B.FRAME_LIGHT))}
        out["stats"] = pt.stats()
        return out
    finally:
        pt.close()


def _rmse(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.mark.parametrize("pipe", PIPES)
@pytest.mark.parametrize("name,W,H,S,M", [
    ("CBspheres_lambertian", 160, 120, 4, 5),
    ("CBspheres", 160, 120, 4, 5),
    ("CBgems", 160, 120, 2, 7),
    ("CBempty", 96, 72, 4, 5),
    ("CBspheres_refract", 96, 72, 2, 5),
    ("CBspheres", 96, 72, 2, 1),
    ("CBspheres", 96, 72, 1, 12),
    ("CBspheres", 96, 72, 2, 20),    # the m <= 32 kernel (the reference has no depth cap)
    ("CBgems", 64, 48, 1, 32),
    ("CBspheres", 64, 48, 1, 62),    # the m <= 62 kernel
    ("CBspheres", 48, 36, 1, 100),   # the m <= 126 kernel (128-bit delta masks)
])
def test_parity_vs_oracle(name, W, H, S, M, pipe):
    sc = golden_scene(name, W, H)
    g = _gpu_render(sc, W, H, S, M, pipeline=pipe)
    samp, eye, light, st = oracle_render(sc, W, H, S, M, MODE_C32)
    assert np.isfinite(g["sample"]).all()
    r = _rmse(g["sample"], samp)
    re = _rmse(g["eye"], eye)
    rl = _rmse(g["light"], light)
    print(f"{name} {W}x{H} s{S} m{M}: rmse sample {r:.3e} eye {re:.3e} light {rl:.3e} "
          f"mean gpu {g['sample'].mean():.6f} oracle {samp.mean():.6f}")
    assert r < RMSE_TOL and re < RMSE_TOL and rl < RMSE_TOL


@pytest.mark.parametrize("lds", [None, 0])
@pytest.mark.parametrize("name,M", [("CBbunny", 5), ("CBcoil", 5), ("CBcoil", 8)])
def test_mesh_scene_parity_vs_oracle(name, M, lds, monkeypatch):
    """The reference's mesh scenes that the BDPT integrator renders (scenes/*.dae loaded by the
    product's loader) against oracle mode 2: the default LDS mode (treelet) and the tree in HBM."""
    if lds is not None:
        monkeypatch.setenv("BDPT_LDS_MODE", str(lds))
    W, H, S = 96, 72, 2
    sc = B.load_dae(os.path.join(REPO, "scenes", name + ".dae"), W, H)
    g = _gpu_render(sc, W, H, S, M)
    samp, eye, light, st = oracle_render(sc, W, H, S, M, MODE_C32)
    r, re, rl = _rmse(g["sample"], samp), _rmse(g["eye"], eye), _rmse(g["light"], light)
    print(f"{name} {W}x{H} s{S} m{M} lds {lds}: rmse sample {r:.3e} eye {re:.3e} light {rl:.3e}")
    assert samp.mean() > 0
    assert r < RMSE_TOL and re < RMSE_TOL and rl < RMSE_TOL


@pytest.mark.parametrize("pipe", PIPES)
def test_parity_c2_full_frame(pipe):
    """Config C2's frame (CBspheres 480x360, m=5) at 4 spp: full-size FOV (splats land anywhere)."""
    sc = golden_scene("CBspheres", 480, 360)
    g = _gpu_render(sc, 480, 360, 4, 5, pipeline=pipe)
    samp = oracle_render(sc, 480, 360, 4, 5, MODE_C32)[0]
    assert _rmse(g["sample"], samp) < RMSE_TOL


@pytest.mark.parametrize("pipe", PIPES)
def test_tiles_and_sample_ranges_compose(pipe):
    """raytrace_tile over 32x32 tiles (raytraced_renderer.cpp:297-301) and split sample ranges give
    the same image as one full-frame launch (sample keys are global: (pixel, sample))."""
    W, H, S, M = 100, 70, 4, 5
    sc = golden_scene("CBspheres", W, H)
    full = _gpu_render(sc, W, H, S, M, pipeline=pipe)
    tiles = [(x, y, 32, 32) for y in range(0, H, 32) for x in range(0, W, 32)]
    tiled = _gpu_render(sc, W, H, S, M, tiles=tiles, ranges=[(0, 1), (1, 3), (3, 4)], spl=1,
                        pipeline=pipe)
    assert _rmse(full["sample"], tiled["sample"]) < 1e-6


@pytest.mark.parametrize("pipe", PIPES)
def test_stats_counters_match_oracle(pipe):
    """In-kernel counters (roofline bytes) against the oracle's counts of the same traversal work:
    the device skips zero-contribution connection rays, the rest of a zero-throughput walk
    (megakernel, bdpt_core.h prepare_sample) and culls boxes, so its closest-hit queries, hits,
    shadow rays and node visits are <= the oracle's (which walks on, as the reference does)."""
    W, H, S, M = 64, 48, 2, 5
    sc = golden_scene("CBspheres", W, H)
    g = _gpu_render(sc, W, H, S, M, stats=True, pipeline=pipe)
    st = g["stats"]
    o = oracle_render(sc, W, H, S, M, MODE_C32)[3]
    assert st.samples == W * H * S
    assert 0.9 * int(o[1]) <= st.closest_rays <= int(o[1])
    assert 0.9 * int(o[6]) <= st.hits <= int(o[6])
    assert 0 < st.shadow_rays <= int(o[2])
    assert 0 < st.tri_tests + st.sph_tests
    # the megakernel runs this 14-primitive scene with the flat leaf list (no node fetches)
    assert st.node_visits > 0 or pipe == B.PIPELINE_MEGAKERNEL


def test_trace_rays_matches_oracle():
    sc = golden_scene("CBgems", 160, 120)
    rng = np.random.default_rng(7)
    n = 20000
    o = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    o[:, 1] = rng.uniform(0.05, 1.4, n)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.full((n, 1), 1e-5, np.float32),
                           np.full((n, 1), np.inf, np.float32)], axis=1).astype(np.float32)
    pt = B.BidirectionalPathTracer(sc, 160, 120, 1, 5)
    try:
        t, prim = pt.trace_rays(rays, any_hit=False)
        ta, _ = pt.trace_rays(rays, any_hit=True)
    finally:
        pt.close()
    ot = np.empty(n, np.float32)
    op = np.empty(n, np.int32)
    d_ = sc.desc()
    oracle().oracle_trace_rays(C.byref(d_), 2, rays.ctypes.data_as(C.POINTER(C.c_float)), n, 0,
                               ot.ctypes.data_as(C.POINTER(C.c_float)),
                               op.ctypes.data_as(C.POINTER(C.c_int)))
    assert np.array_equal(prim, op)
    assert np.array_equal(t[op >= 0], ot[op >= 0])
    assert np.array_equal(np.isfinite(ta), op >= 0)


@pytest.mark.parametrize("name", ["CBbunny", "CBgems"])
def test_trace_rays_zero_direction_components_match_oracle(name):
    """Rays with exact 0 / -0 direction components (axis-aligned, in coordinate planes) through the
    device traversal: the same closest hits as the oracle's mode-2 tracer, any-hit agreeing. The
    traversal before round 5's safe_inv culled boxes such rays run through inside a slab
    (tests/test_core_cpu.py has the CPU-build and brute-force checks)."""
    from test_core_cpu import zero_component_rays, zero_ray_scene
    sc, lo, hi = zero_ray_scene(name)
    n = 3000
    rays = zero_component_rays(n, 11, lo, hi)
    pt = B.BidirectionalPathTracer(sc, 32, 24, 1, 5)
    try:
        t, prim = pt.trace_rays(rays, any_hit=False)
        ta, _ = pt.trace_rays(rays, any_hit=True)
    finally:
        pt.close()
    ot = np.empty(n, np.float32)
    op = np.empty(n, np.int32)
    d_ = sc.desc()
    oracle().oracle_trace_rays(C.byref(d_), 2, rays.ctypes.data_as(C.POINTER(C.c_float)), n, 0,
                               ot.ctypes.data_as(C.POINTER(C.c_float)),
                               op.ctypes.data_as(C.POINTER(C.c_int)))
    assert (op >= 0).sum() > n // 2
    assert np.array_equal(prim, op)
    assert np.array_equal(t[op >= 0], ot[op >= 0])
    assert np.array_equal(np.isfinite(ta), op >= 0)


def test_unsupported_material_rejected():
    sc = golden_scene("CBspheres", 32, 24)
    sc.mats[0].type = B.MAT_MICROFACET
    with pytest.raises(B.BDPTError):
        B.BidirectionalPathTracer(sc, 32, 24, 1, 5)


# --- environment light + Russian roulette: the EXT kernels -----------------------
def _with_env(sc, w=64, h=32):
    import os
    import sys
    from _util import REPO
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from envmap import synth_envmap
    sc.set_envmap(synth_envmap(w, h))
    return sc


@pytest.mark.parametrize("lds", ["0", "1", "2", "3"])
@pytest.mark.parametrize("name,W,H,S,M,rr,env", [
    ("CBspheres_lambertian", 128, 96, 4, 5, False, True),
    ("CBspheres", 128, 96, 4, 8, True, True),
    ("CBgems", 128, 96, 2, 7, True, False),
    ("CBempty", 96, 72, 4, 5, True, True),
])
def test_parity_env_rr_vs_oracle(name, W, H, S, M, rr, env, lds, monkeypatch):
    """EXT megakernel (every LDS mode: scene in HBM, whole scene in LDS, BFS treelet, flat leaf
    list) vs mode 2."""
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    sc = golden_scene(name, W, H)
    if env:
        _with_env(sc)
    g = _gpu_render(sc, W, H, S, M, rr=rr)
    samp, eye, light, st = oracle_render(sc, W, H, S, M, MODE_C32, rr=rr)
    assert np.isfinite(g["sample"]).all()
    r = _rmse(g["sample"], samp)
    print(f"EXT {name} {W}x{H} s{S} m{M} rr={rr} env={env} lds={lds}: rmse {r:.3e} "
          f"mean gpu {g['sample'].mean():.6f} oracle {samp.mean():.6f}")
    assert r < RMSE_TOL and _rmse(g["eye"], eye) < RMSE_TOL and _rmse(g["light"], light) < RMSE_TOL


def test_parity_env_only_scene():
    """The environment as the only light (no area light in the scene)."""
    import os
    from _util import REPO
    env = os.path.join(REPO, "tests", "golden", "env")
    sc = B.load_dae(os.path.join(env, "CBspheres_envonly.dae"), 96, 72)
    sc.set_envmap(B.load_exr(os.path.join(env, "sky_32x16_zip_half.exr")))
    g = _gpu_render(sc, 96, 72, 4, 12, rr=True)
    samp = oracle_render(sc, 96, 72, 4, 12, MODE_C32, rr=True)[0]
    assert _rmse(g["sample"], samp) < RMSE_TOL


# --- the unidirectional PathTracer: k_pt vs oracle mode 2 ----------------
@pytest.mark.parametrize("lds", ["0", "1", "2", "3"])
@pytest.mark.parametrize("scene,W,H,S,M,kw", [
    ("CBspheres_lambertian", 96, 72, 8, 5, dict(samples_per_batch=4, max_tolerance=0.05)),
    ("CBspheres", 96, 72, 8, 5, dict(samples_per_batch=4, max_tolerance=0.05)),
    ("CBspheres_microfacet_al_ag", 96, 72, 4, 5, dict(samples_per_batch=4, max_tolerance=0.05)),
    ("CBspheres", 64, 48, 4, 0, dict(samples_per_batch=4, max_tolerance=0.05)),
    ("CBspheres_lambertian", 64, 48, 4, 4, dict(samples_per_batch=4, max_tolerance=0.05, ns_area_light=2,
                                                direct_hemisphere_sample=True)),
    ("CBgems", 64, 48, 4, 6, dict(samples_per_batch=2, max_tolerance=0.1, lens_radius=0.05, focal_distance=4.0)),
    # an ambient light (InfiniteHemisphereLight) on a 28k-triangle mesh, diffuse and microfacet
    ("bunny", 64, 48, 4, 4, dict(samples_per_batch=2, max_tolerance=0.05, ns_area_light=2)),
    ("bunny_microfacet_cu", 64, 48, 2, 3, dict(samples_per_batch=2, max_tolerance=0.05)),
    # DirectionalLight (+ ambient on banana)
    ("banana", 64, 48, 2, 3, dict(samples_per_batch=2, max_tolerance=0.05, ns_area_light=2)),
    ("teapot", 64, 48, 4, 4, dict(samples_per_batch=4, max_tolerance=0.05)),
])
def test_pathtracer_parity_vs_oracle(scene, W, H, S, M, kw, lds, monkeypatch):
    import os
    from _util import REPO, oracle_pt_render
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    sc = B.load_dae(os.path.join(REPO, "scenes", scene + ".dae"), W, H)
    pt = B.PathTracer(sc, W, H, S, M, seed=31, **kw)
    try:
        pt.raytrace_tiles()
        img = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
        cnt = pt.read_sample_counts()
    finally:
        pt.close()
    o_img, o_cnt, _ = oracle_pt_render(sc, W, H, S, M, MODE_C32, seed=31, ns_area_light=kw.get("ns_area_light", 1),
                                       batch=kw["samples_per_batch"], tol=kw["max_tolerance"],
                                       hemisphere=kw.get("direct_hemisphere_sample", False),
                                       lens_radius=kw.get("lens_radius", 0.0),
                                       focal_distance=kw.get("focal_distance", 4.7))
    r = _rmse(img, o_img)
    mism = float(np.mean(cnt != o_cnt))
    print(f"PT {scene} {W}x{H} s{S} m{M} lds={lds}: rmse {r:.3e} count mismatch {mism:.4f} "
          f"mean gpu {img.mean():.6f} oracle {o_img.mean():.6f}")
    assert np.isfinite(img).all()
    # the GPU's fp32 erf/exp/log differ from glibc's by ulps (microfacet): rare adaptive-stop or
    # roulette flips are allowed; per-pixel RMSE stays within the north-star tolerance
    assert mism <= 0.01 and r < RMSE_TOL


def test_pathtracer_env_and_tiles():
    """The environment light under the PathTracer, rendered as two tiles (whole pixels)."""
    import os
    from _util import REPO, oracle_pt_render
    W, H, S, M = 64, 48, 4, 4
    sc = _with_env(B.load_dae(os.path.join(REPO, "scenes", "CBspheres_lambertian.dae"), W, H))
    pt = B.PathTracer(sc, W, H, S, M, seed=3, samples_per_batch=4)
    try:
        pt.raytrace_tiles([(0, 0, 64, 20), (0, 20, 64, 28)])
        img = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
        with pytest.raises(B.BDPTError):
            pt.raytrace_tiles([], 1, 2)   # partial sample ranges are rejected
    finally:
        pt.close()
    o_img = oracle_pt_render(sc, W, H, S, M, MODE_C32, seed=3, batch=4)[0]
    assert _rmse(img, o_img) < RMSE_TOL


@pytest.mark.parametrize("lds", ["0", "1", "2", "3"])
def test_lds_modes_agree_c2(lds, monkeypatch):
    """Every traversal mode of k_bdpt_sample on C2's scene (the bench default runs LM 3, the flat
    leaf list, for scenes of <= 24 primitives) vs the oracle."""
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    W, H, S, M = 160, 120, 4, 5
    sc = golden_scene("CBspheres", W, H)
    g = _gpu_render(sc, W, H, S, M)
    samp = oracle_render(sc, W, H, S, M, MODE_C32)[0]
    assert _rmse(g["sample"], samp) < RMSE_TOL


# --- the north-star kernel path: the CBlucy stand-in (114,304 triangles) ---------------------------
# The device BVH4 (73k nodes) does not fit in LDS: the default LDS mode 2 stages its first 1024
# BFS nodes (the treelet every ray starts in) and reads the rest from HBM; these cases cover that
# hand-off, deep stacks and the C3 / north-star / C5 frame sizes (BASELINE configs).
def _standin(W, H):
    import os
    import sys
    from _util import REPO
    sys.path.insert(0, REPO)
    from bench import STANDIN, ensure_standin
    path = os.path.join(REPO, STANDIN)
    ensure_standin(path)
    return B.load_dae(path, W, H)


def _check_frames(g, ref, label):
    samp, eye, light = ref[0], ref[1], ref[2]
    assert np.isfinite(g["sample"]).all()
    r, re_, rl = _rmse(g["sample"], samp), _rmse(g["eye"], eye), _rmse(g["light"], light)
    print(f"{label}: rmse sample {r:.3e} eye {re_:.3e} light {rl:.3e} mean gpu {g['sample'].mean():.6f} "
          f"oracle {samp.mean():.6f}")
    assert r < RMSE_TOL and re_ < RMSE_TOL and rl < RMSE_TOL


def test_standin_c3_frame_default_mode():
    """C3's frame (800x600, m=5) at 2 spp through the default path: LDS mode 2 (treelet in LDS,
    BVH4 below it in HBM); the stats show both kinds of node fetch."""
    W, H, S, M = 800, 600, 2, 5
    sc = _standin(W, H)
    g = _gpu_render(sc, W, H, S, M, stats=True)
    st = g["stats"]
    assert st.lds_mode == 2
    assert 0 < st.lds_node_visits < st.node_visits
    _check_frames(g, oracle_render(sc, W, H, S, M, MODE_C32), "stand-in 800x600 s2 m5")


def test_standin_northstar_frame_and_tiles():
    """The north-star frame (1920x1080, m=5, FOV quirk at 1080p) at 1 spp, full frame vs the
    oracle; then a subset of 32x32 tiles (raytrace_tile): their eye image equals the full render's
    on those pixels (a pixel's eye value depends on its own samples only)."""
    W, H, S, M = 1920, 1080, 1, 5
    sc = _standin(W, H)
    ref = oracle_render(sc, W, H, S, M, MODE_C32)
    g = _gpu_render(sc, W, H, S, M)
    _check_frames(g, ref, "stand-in 1920x1080 s1 m5")
    tiles = [(x, y, 32, 32) for y in range(0, H, 32) for x in range(0, W, 32) if (x // 32 + 3 * (y // 32)) % 7 == 0]
    gt = _gpu_render(sc, W, H, S, M, tiles=tiles)
    mask = np.zeros((H, W), bool)
    for x, y, w, h in tiles:
        mask[y:y + h, x:x + w] = True
    assert _rmse(gt["eye"][mask], ref[1][mask]) < RMSE_TOL
    assert np.all(gt["eye"][~mask] == 0)


@pytest.mark.parametrize("lds,ntop", [("0", None), ("2", None), ("2", "64"), ("2", "1")])
def test_standin_lds_modes(lds, ntop, monkeypatch):
    """Scene wholly in HBM (LM 0) and treelets of 1024 / 64 / 1 nodes (BDPT_NTOP_MAX) in front of
    the HBM part: the hand-off depth changes, the image does not."""
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    if ntop:
        monkeypatch.setenv("BDPT_NTOP_MAX", ntop)
    W, H, S, M = 320, 240, 2, 5
    sc = _standin(W, H)
    g = _gpu_render(sc, W, H, S, M, stats=True)
    assert g["stats"].lds_mode == int(lds)
    _check_frames(g, oracle_render(sc, W, H, S, M, MODE_C32), f"stand-in LM {lds} ntop {ntop}")


@pytest.mark.parametrize("lds", ["0", "2"])
def test_standin_c5_shaped(lds, monkeypatch):
    """C5's shape at a small frame: the stand-in + an environment light + Russian roulette at m=8
    (EXT kernel) with the mesh BVH from HBM / the treelet."""
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    W, H, S, M = 384, 216, 2, 8
    sc = _with_env(_standin(W, H), 256, 128)
    g = _gpu_render(sc, W, H, S, M, rr=True)
    _check_frames(g, oracle_render(sc, W, H, S, M, MODE_C32, rr=True), f"stand-in + env + RR m8 LM {lds}")


@pytest.mark.parametrize("env", [{"BDPT_BVH": "ref"}, {"BDPT_SAH_LEAF": "1"},
                                 {"BDPT_SAH_BINS": "4", "BDPT_SAH_CT": "4"}], ids=["ref_tree", "leaf1", "bins4"])
@pytest.mark.parametrize("scene", ["standin", "CBgems"])
def test_device_tree_knobs(scene, env, monkeypatch):
    """The device traversing the reference's own midpoint tree (BDPT_BVH=ref, bvh.cpp:51-129) or
    other SAH trees (BDPT_SAH_LEAF / _CT / _BINS) renders the same image: the tree's shape decides
    no result. The stand-in runs the treelet + HBM kernel (LM 2), CBgems the
    whole-scene-in-LDS one (LM 1)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    W, H, S, M = (256, 144, 2, 5) if scene == "standin" else (160, 120, 2, 7)
    sc = _standin(W, H) if scene == "standin" else golden_scene("CBgems", W, H)
    _check_frames(_gpu_render(sc, W, H, S, M), oracle_render(sc, W, H, S, M, MODE_C32), f"{scene} {env}")


@pytest.mark.parametrize("env", [{"BDPT_XCD_GROUPS": "1"}, {"BDPT_BLOCK_MAJOR": "0"},
                                 {"BDPT_XCD_GROUPS": "1", "BDPT_BLOCK_MAJOR": "0"}])
def test_ticket_orders(env, monkeypatch):
    """The work-item orders kept as A/B switches (XCD-grouped tickets with their per-group counters
    and exhaustion hand-over; chunk-major order) render the same image."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    W, H, S, M = 200, 150, 5, 5      # 5 spp: a ragged last chunk of the 2-sample work items
    sc = _standin(W, H)
    _check_frames(_gpu_render(sc, W, H, S, M), oracle_render(sc, W, H, S, M, MODE_C32), f"tickets {env}")


def test_concurrent_tile_callers():
    """The reference's caller model: N host threads drive raytrace_tile (and raytrace_pixel) on
    one PathTracer (raytraced_renderer.cpp:325-327,610-615). The ctx serialises the calls; the image
    equals one full-frame render."""
    import threading
    W, H, S, M = 160, 120, 2, 5
    sc = golden_scene("CBgems", W, H)
    full = _gpu_render(sc, W, H, S, M)
    pt = B.BidirectionalPathTracer(sc, W, H, S, M)
    try:
        tiles = [(x, y, 32, 32) for y in range(0, H, 32) for x in range(0, W, 32)]
        todo = list(tiles)
        lock = threading.Lock()
        errs = []

        def worker():
            try:
                while True:
                    with lock:
                        if not todo:
                            return
                        t = todo.pop()
                    pt.raytrace_tile(*t)
            except Exception as e:   # pragma: no cover - reported below
                errs.append(e)
        th = [threading.Thread(target=worker) for _ in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs
        got = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    finally:
        pt.close()
    assert _rmse(got, full["sample"]) < 1e-6
    # 1x1 tiles (raytrace_pixel) back to back: the staging ring never waits for the GPU
    pt = B.BidirectionalPathTracer(sc, W, H, S, M)
    try:
        for x in range(8):
            pt.raytrace_pixel(40 + x, 60)
        eye = pt.read_frame(B.FRAME_EYE).astype(np.float64)
    finally:
        pt.close()
    assert _rmse(eye[60, 40:48], full["eye"][60, 40:48]) < RMSE_TOL
    assert np.count_nonzero(eye.sum(axis=2)) <= 8


def test_env_table_read_counters():
    """bdpt_stats v6: the environment-table reads the bench adds to the algorithmic bytes are
    counted in scenes with an environment light (a direction sampled for some light vertices and
    for the fresh light sample of (i, 1) connections; radiance lookups for escaped eye rays, with a
    pdf lookup for each that carries a contribution) and are zero without one."""
    W, H, S, M = 96, 72, 2, 8
    sc = golden_scene("CBspheres_lambertian", W, H)
    st0 = _gpu_render(sc, W, H, S, M, stats=True)["stats"]
    assert (st0.env_samples, st0.env_lookups, st0.env_pdf_lookups) == (0, 0, 0)
    st = _gpu_render(_with_env(sc), W, H, S, M, stats=True, rr=True)["stats"]
    assert st.samples == W * H * S
    assert st.env_samples > 0 and st.env_lookups > 0
    assert 0 < st.env_pdf_lookups <= st.env_lookups


def test_c4_full_frame():
    """Config C4's frame: CBgems 1920x1080, m=7 (the FOV quirk at 1080p, camera.cpp:83-89; splats
    landing anywhere, bidirection.cpp:457-466; the scene whole in LDS, LM 1) at 1 spp vs the
    oracle: sample, eye and light images each within the RMSE tolerance."""
    W, H, S, M = 1920, 1080, 1, 7
    sc = golden_scene("CBgems", W, H)
    g = _gpu_render(sc, W, H, S, M, stats=True)
    assert g["stats"].samples == W * H * S
    _check_frames(g, oracle_render(sc, W, H, S, M, MODE_C32), "C4 CBgems 1920x1080 s1 m7")


def test_c5_full_frame():
    """Config C5's frame: the Lucy stand-in + the synthetic 1024x512 sky the bench uses (DESIGN.md
    §9) at 1920x1080, m=8, Russian roulette on (the EXT kernel, compact pair lists) at 1 spp."""
    W, H, S, M = 1920, 1080, 1, 8
    sc = _with_env(_standin(W, H), 1024, 512)
    g = _gpu_render(sc, W, H, S, M, rr=True, stats=True)
    assert g["stats"].samples == W * H * S
    _check_frames(g, oracle_render(sc, W, H, S, M, MODE_C32, rr=True), "C5 stand-in + env 1920x1080 s1 m8 RR")


# Speculative traversal (bdpt_core.h spec_trav) descends with the ray's t before a postponed leaf
# shrinks it, and an any-hit query may finish on a leaf after extra descent: the device visits a
# superset of what one lane alone visits. Measured on the stand-in at 256x144 s1 m5 (LM 0 and 2):
# node visits 1.0071x, triangle tests 1.0017x the replay's (profiles/r03_pytest_gpu.log).
SPEC_EXCESS = 1.03


@pytest.mark.parametrize("lds", ["2", "0"])
def test_standin_counters_match_cpu_replay(lds, monkeypatch):
    """The roofline's counters (N_node, N_tri per ray, counted in-kernel) against a
    CPU replay of the same BVH4 traversal: bdpt_core.h compiled for the host (tests/native/core_cpu,
    one lane, so no speculation) renders the same samples. Query and hit counts are equal (also to
    the oracle's closest-hit queries and hits); node visits and triangle tests are at least the
    replay's and at most SPEC_EXCESS times it. (The oracle walks zero-throughput subpaths on to the
    depth cap, as the reference does; the device ends them: its counts are <= the oracle's.)"""
    from test_core_cpu import core_render
    monkeypatch.setenv("BDPT_LDS_MODE", lds)
    W, H, S, M = 256, 144, 1, 5
    sc = _standin(W, H)
    st = _gpu_render(sc, W, H, S, M, stats=True)["stats"]
    assert st.lds_mode == int(lds)
    _, _, cs = core_render(sc, W, H, S, M, seed=5489, lds_mode=0)
    o = oracle_render(sc, W, H, S, M, MODE_C32)[3]
    assert st.samples == W * H * S
    assert st.closest_rays == int(cs[1]) <= int(o[1])
    assert st.hits == int(cs[6]) <= int(o[6])
    assert st.shadow_rays == int(cs[2])
    nodes, tris = int(cs[3]), int(cs[4])
    print(f"LM {lds}: nodes gpu {st.node_visits} replay {nodes} ({st.node_visits / nodes:.4f}); "
          f"tris gpu {st.tri_tests} replay {tris} ({st.tri_tests / tris:.4f})")
    assert nodes <= st.node_visits <= SPEC_EXCESS * nodes
    assert tris <= st.tri_tests <= SPEC_EXCESS * tris
