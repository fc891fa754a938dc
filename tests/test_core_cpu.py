"""CPU checks of the device pipeline (bdpt_core.h + bdpt_scene.cpp compiled with g++ into the
test-only tests/native/libcorecpu.so) against the oracle's mode 2 (fp32 device semantics):
bit-exact per-pixel eye and light images, and the product BVH's primitive order vs the
reference's own BVH (dumped by oracle/_ref/ref_driver into tests/golden/scenes/*.json)."""
import ctypes as C
import os

import numpy as np
import pytest

import bdpt_amd as B
from _util import MODE_C32, REPO, golden_scene, oracle_render

_core = None


def core():
    global _core
    if _core is None:
        import sys
        sys.path.insert(0, REPO)
        import __graft_entry__ as g
        g.build_core_cpu()
        lib = C.CDLL(g.CORE_CPU_SO)
        P = C.POINTER(C.c_double)
        lib.core_cpu_render.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int,
                                        P, P, P, C.c_int, C.c_int]
        lib.core_cpu_scene_info.argtypes = [C.POINTER(B.SceneDesc), C.POINTER(C.c_int),
                                            C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _core = lib
    return _core


def core_render(scene, W, H, spp, M, seed=5489, s0=0, count=None, lds_mode=0, rr=False):
    lib = core()
    count = spp - s0 if count is None else count
    eye = np.zeros((H, W, 3))
    light = np.zeros((H, W, 3))
    st = np.zeros(8)
    d = scene.desc()
    pd = C.POINTER(C.c_double)
    rc = lib.core_cpu_render(C.byref(d), W, H, spp, M, seed, s0, count, None, 0,
                             eye.ctypes.data_as(pd), light.ctypes.data_as(pd), st.ctypes.data_as(pd), lds_mode,
                             1 if rr else 0)
    assert rc == 0
    return eye, light, st


CASES = [("CBspheres", 32, 24, 2, 5), ("CBspheres_lambertian", 32, 24, 2, 5), ("CBgems", 32, 24, 1, 7),
         ("CBempty", 32, 24, 2, 5), ("CBspheres_refract", 24, 18, 2, 5), ("CBspheres", 24, 18, 1, 8),
         ("CBspheres", 24, 18, 3, 1),
         # the m <= 32 and m <= 62 kernels (64-bit delta masks): mirror / glass chains run long here
         ("CBspheres", 24, 18, 2, 20), ("CBgems", 24, 18, 1, 32),
         # the m <= 62 kernel
         ("CBspheres", 24, 18, 1, 62),
         # the m <= 126 kernel (128-bit delta masks)
         ("CBspheres", 16, 12, 1, 100)]


@pytest.mark.parametrize("lds_mode", [0, 1, 3])
@pytest.mark.parametrize("name,W,H,spp,M", CASES)
def test_device_pipeline_bit_exact_vs_oracle_mode2(name, W, H, spp, M, lds_mode):
    """lds_mode 0 traverses the 4-wide tree (HBM kernels), 1 the binary one (scene in LDS), 3 the
    flat leaf list (tiny scenes)."""
    sc = golden_scene(name, W, H)
    eye, light, st = core_render(sc, W, H, spp, M, seed=1234, lds_mode=lds_mode)
    _, oeye, olight, ost = oracle_render(sc, W, H, spp, M, MODE_C32, seed=1234, threads=1)
    assert np.isfinite(eye).all() and np.isfinite(light).all()
    assert np.array_equal(eye, oeye), f"eye max diff {np.abs(eye - oeye).max()}"
    assert np.array_equal(light, olight), f"light max diff {np.abs(light - olight).max()}"


EXT_CASES = [("CBspheres_lambertian", 32, 24, 2, 5, False, True), ("CBspheres", 32, 24, 2, 5, False, True),
             ("CBempty", 32, 24, 2, 5, False, True), ("CBspheres", 32, 24, 2, 8, True, False),
             ("CBgems", 32, 24, 1, 7, True, True), ("CBspheres_lambertian", 24, 18, 2, 8, True, True),
             ("CBspheres", 24, 18, 2, 24, True, True), ("CBspheres", 24, 18, 1, 50, True, True),
             # non-power-of-two map: the guide tables' cells (powers of two) straddle CDF entries
             ("CBspheres_lambertian", 24, 18, 4, 5, False, (37, 19))]


@pytest.mark.parametrize("lds_mode", [0, 1])
@pytest.mark.parametrize("name,W,H,spp,M,rr,env", EXT_CASES)
def test_device_pipeline_bit_exact_env_rr(name, W, H, spp, M, rr, env, lds_mode):
    """The EXT kernels' code (environment light, Russian roulette) vs mode 2."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from envmap import synth_envmap
    sc = golden_scene(name, W, H)
    if env:
        sc.set_envmap(synth_envmap(*(env if isinstance(env, tuple) else (32, 16))))
    eye, light, st = core_render(sc, W, H, spp, M, seed=99, lds_mode=lds_mode, rr=rr)
    _, oeye, olight, ost = oracle_render(sc, W, H, spp, M, MODE_C32, seed=99, threads=1, rr=rr)
    assert np.isfinite(eye).all() and np.isfinite(light).all()
    assert np.array_equal(eye, oeye), f"eye max diff {np.abs(eye - oeye).max()}"
    assert np.array_equal(light, olight), f"light max diff {np.abs(light - olight).max()}"


@pytest.mark.parametrize("name", ["CBspheres", "CBgems", "CBempty", "CBspheres_refract"])
def test_product_bvh_matches_reference_bvh(name):
    import json
    with open(os.path.join(REPO, "tests", "golden", "scenes", name + ".json")) as f:
        js = json.load(f)
    sc = golden_scene(name)
    n = sc.desc().nprim
    depth, ref_nodes = C.c_int(), C.c_int()
    order = (C.c_int * n)()
    assert core().core_cpu_scene_info(C.byref(sc.desc()), C.byref(depth), C.byref(ref_nodes), order) == 0
    bvh = js["bvh"]
    assert depth.value == bvh["depth"]
    assert ref_nodes.value == bvh["nodes"]
    assert list(order) == list(bvh["dfs_prim_order"])


@pytest.mark.parametrize("name,n,nsph", [("CBspheres", 14, 2), ("CBspheres_lambertian", 14, 2), ("CBempty", 12, 0)])
def test_flat_list_is_one_run_of_primitives(name, n, nsph):
    """LDS mode 3 walks the flat leaf list as primitives 0..n-1 with the next record prefetched; that
    needs the device tree's leaves to hold the primitives as one consecutive run (flat_prims), which
    the builder guarantees — checked here on the Cornell-box scenes the flat mode serves."""
    lib = core()
    lib.core_cpu_flat_prims.restype = C.c_int
    mask = C.c_uint32(0)
    sc = golden_scene(name, 32, 24)
    assert lib.core_cpu_flat_prims(C.byref(sc.desc()), C.byref(mask)) == n
    assert bin(mask.value).count("1") == nsph


@pytest.mark.parametrize("lds_mode", [0, 2])
@pytest.mark.parametrize("scene,W,H,spp,M", [("scenes/CBbunny.dae", 64, 48, 2, 5),
                                             ("scenes/CBlucy_standin.dae", 48, 36, 2, 5)])
def test_device_pipeline_bit_exact_mesh_trees(scene, W, H, spp, M, lds_mode):
    """The 4-wide tree of a mesh scene (thousands of nodes; bvh.cpp:161-188 closest-hit semantics
    over a deep tree) vs mode 2: every padded child box must contain its primitives, or a hit goes
    missing and the images differ. lds_mode 2 runs the north star's kernel path: the BFS treelet
    read through the LDS node fetch (the same array on the CPU), the rest through the global one."""
    path = os.path.join(REPO, scene)
    if not os.path.exists(path):
        pytest.skip(f"{scene} not generated (tools/gen_standin.py, __graft_entry__.build)")
    sc = B.load_dae(path, W, H)
    eye, light, st = core_render(sc, W, H, spp, M, seed=77, lds_mode=lds_mode)
    _, oeye, olight, ost = oracle_render(sc, W, H, spp, M, MODE_C32, seed=77, threads=1)
    assert np.isfinite(eye).all() and np.isfinite(light).all()
    assert np.array_equal(eye, oeye), f"eye max diff {np.abs(eye - oeye).max()}"
    assert np.array_equal(light, olight), f"light max diff {np.abs(light - olight).max()}"


def test_triangle_early_outs_exact(tmp_path):
    """tri_test with its division-free early-outs (a quotient certainly < 0 or > 1) decides, and
    rounds t / b1 / b2, exactly as the plain three-division Möller–Trumbore predicate
    (triangle.cpp:57-95) on 1M random and near-boundary cases (tests/native/tri_exact.cpp)."""
    import subprocess
    exe = str(tmp_path / "tri_exact")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I" + os.path.join(REPO, "include"),
                    "-I" + os.path.join(REPO, "bidirectional-pathtracing_amd", "csrc"), "-o", exe,
                    os.path.join(REPO, "tests", "native", "tri_exact.cpp")], check=True)
    out = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout


@pytest.mark.parametrize("env", [{"BDPT_BVH": "ref"}, {"BDPT_SAH_LEAF": "1"}, {"BDPT_SAH_LEAF": "2", "BDPT_SAH_CT": "0.25"},
                                 {"BDPT_SAH_BINS": "4", "BDPT_SAH_CT": "4"}], ids=["ref", "leaf1", "leaf2_ct", "bins4"])
@pytest.mark.parametrize("scene,W,H,spp,M", [("scenes/CBgems.dae", 32, 24, 1, 7), ("scenes/CBbunny.dae", 40, 30, 1, 5)])
def test_device_tree_knobs_bit_exact(scene, W, H, spp, M, env, monkeypatch):
    """The device tree's shape changes no result (closest hits by t, equal-t ties by the reference
    tree's leaf order): BDPT_BVH=ref builds the device tree from the reference's own
    midpoint tree (bvh.cpp:51-129) instead of the binned SAH; BDPT_SAH_LEAF / _CT / _BINS change
    the SAH tree's leaf size, termination cost and bin count. Each is bit-exact vs mode 2."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = B.load_dae(os.path.join(REPO, scene), W, H)
    for lm in (0, 1):
        eye, light, _ = core_render(sc, W, H, spp, M, seed=5, lds_mode=lm)
        _, oeye, olight, _ = oracle_render(sc, W, H, spp, M, MODE_C32, seed=5, threads=1)
        assert np.array_equal(eye, oeye) and np.array_equal(light, olight), (env, lm)


def test_device_tree_knobs_change_the_tree(monkeypatch):
    """...and they do select another tree: BDPT_BVH=ref has the reference tree's depth and node
    count (19 / 18,565 for CBbunny, tests/golden/scenes/facts.json), the default SAH tree others,
    and a SAH leaf size of 1 more nodes than the default's."""
    import json
    with open(os.path.join(REPO, "tests", "golden", "scenes", "facts.json")) as f:
        facts = json.load(f)["CBbunny"]
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBbunny.dae"), 32, 24)
    lib = core()
    lib.core_cpu_dev_tree.restype = C.c_int

    def tree(**env):
        for k in ("BDPT_BVH", "BDPT_SAH_LEAF"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        depth, nodes = C.c_int(), C.c_int()
        assert lib.core_cpu_dev_tree(C.byref(sc.desc()), C.byref(depth), C.byref(nodes)) == 0
        return depth.value, nodes.value

    assert tree(BDPT_BVH="ref") == (facts["bvh_depth"], facts["bvh_nodes"])
    sah = tree()
    assert sah != (facts["bvh_depth"], facts["bvh_nodes"])
    assert tree(BDPT_SAH_LEAF="1")[1] > sah[1]


@pytest.mark.parametrize("lds_mode", [0, 1, 2])
@pytest.mark.parametrize("name", ["CBbunny", "CBspheres"])
def test_traversal_with_zero_direction_components_matches_brute_force(name, lds_mode):
    """Rays whose direction has exact 0 / -0 components (axis-aligned, in a coordinate plane) find the
    same closest hit (primitive and t) through the 4-wide (lds_mode 0, 2) and binary (1) trees as a
    loop over every primitive with the same tests and tie rule. Such a component made the slab
    test's inverse infinite: inf - inf plane distances, and a box the ray runs through inside one of
    its slabs was culled — the round-5 traversal before the fix missed 1,006 of these 1,195 hits
    on CBbunny. bdpt_core.h safe_inv replaces a zero component by +-2^-100."""
    lib = core()
    lib.core_cpu_trace_check.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.c_int, C.c_uint64,
                                         C.POINTER(C.c_int)]
    if name == "CBbunny":
        sc = B.load_dae(os.path.join(REPO, "scenes", "CBbunny.dae"), 32, 24)
    else:
        sc = golden_scene(name, 32, 24)
    hits = C.c_int()
    bad = lib.core_cpu_trace_check(C.byref(sc.desc()), lds_mode, 1400 if name == "CBbunny" else 7000, 12345,
                                   C.byref(hits))
    assert bad == 0
    assert hits.value > 500


def zero_component_rays(n, seed, lo, hi):
    """n rays (o, d, tmin, tmax) from origins uniform in [lo, hi] whose directions have exact 0 / -0
    components: one axis zeroed, two axes zeroed (axis-aligned), and none, in turn."""
    rng = np.random.default_rng(seed)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    k = np.arange(n)
    sign = np.where(k % 16 >= 8, np.float32(-0.0), np.float32(0.0))
    for a in range(3):
        d[k % 7 == a, a] = sign[k % 7 == a]
        two = k % 7 == 3 + a
        d[two, (a + 1) % 3] = 0.0
        d[two, (a + 2) % 3] = sign[two]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d, np.full((n, 1), 1e-5, np.float32), np.full((n, 1), np.inf, np.float32)],
                          axis=1).astype(np.float32)


def zero_ray_scene(name):
    if name == "CBbunny":
        return B.load_dae(os.path.join(REPO, "scenes", "CBbunny.dae"), 32, 24), (-0.9, 0.05, -0.9), (0.9, 1.4, 0.9)
    return golden_scene(name, 32, 24), (-0.9, 0.05, -0.9), (0.9, 1.4, 0.9)


@pytest.mark.parametrize("lds_mode", [0, 1, 2])
@pytest.mark.parametrize("name", ["CBbunny", "CBgems"])
def test_zero_component_rays_match_oracle(name, lds_mode):
    """The same rays through bdpt_trace_rays' traversal (CPU build) and the oracle's mode-2 tracer
    (the reference's BVH and BBox::intersect, fp32): identical closest-hit primitives and t, and
    any-hit agrees with them (the GPU side: tests/test_gpu_parity.py)."""
    from _util import oracle
    sc, lo, hi = zero_ray_scene(name)
    n = 3000
    rays = zero_component_rays(n, 11, lo, hi)
    lib = core()
    lib.core_cpu_trace_rays.argtypes = [C.POINTER(B.SceneDesc), C.c_int, C.POINTER(C.c_float), C.c_int, C.c_int,
                                        C.POINTER(C.c_float), C.POINTER(C.c_int)]
    d_ = sc.desc()
    PF, PI = C.POINTER(C.c_float), C.POINTER(C.c_int)
    t, p, ta, pa, ot, op = (np.empty(n, np.float32), np.empty(n, np.int32), np.empty(n, np.float32),
                            np.empty(n, np.int32), np.empty(n, np.float32), np.empty(n, np.int32))
    assert lib.core_cpu_trace_rays(C.byref(d_), lds_mode, rays.ctypes.data_as(PF), n, 0, t.ctypes.data_as(PF),
                                   p.ctypes.data_as(PI)) == 0
    assert lib.core_cpu_trace_rays(C.byref(d_), lds_mode, rays.ctypes.data_as(PF), n, 1, ta.ctypes.data_as(PF),
                                   pa.ctypes.data_as(PI)) == 0
    oracle().oracle_trace_rays(C.byref(d_), 2, rays.ctypes.data_as(PF), n, 0, ot.ctypes.data_as(PF),
                               op.ctypes.data_as(PI))
    assert (op >= 0).sum() > n // 2
    assert np.array_equal(p, op)
    assert np.array_equal(t[op >= 0], ot[op >= 0])
    assert np.array_equal(pa >= 0, op >= 0)


@pytest.mark.parametrize("lds_mode", [0, 2])
@pytest.mark.parametrize("name,M", [("CBbunny", 5), ("CBcoil", 5), ("CBcoil", 8), ("CBlucy_standin", 5)])
def test_mesh_scenes_bit_exact_vs_oracle_mode2(name, M, lds_mode):
    """The reference's mesh scenes under BDPT (scenes/*.dae through the product's loader): the CPU
    build of the device pipeline is bit-exact against oracle mode 2 with the 4-wide tree in HBM (0)
    and with its treelet read through the LDS path (2)."""
    W, H, spp = 40, 30, 2
    sc = B.load_dae(os.path.join(REPO, "scenes", name + ".dae"), W, H)
    eye, light, _ = core_render(sc, W, H, spp, M, lds_mode=lds_mode)
    _, oeye, olight, _ = oracle_render(sc, W, H, spp, M, MODE_C32, threads=8)
    assert oeye.mean() + olight.mean() > 0
    assert np.array_equal(eye, oeye) and np.array_equal(light, olight)
