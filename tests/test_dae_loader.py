"""Host COLLADA loader (bdpt_dae_load, dae_loader.cpp) against the reference's own loader: the scene
dumps in tests/golden/scenes/*.json were written by oracle/_ref/ref_driver (ColladaParser +
Application::load of the reference) from the same .dae files; every camera, light, material,
sphere and triangle (positions and the halfedge-mesh vertex normals) must match bit for bit.
CPU only (no device call)."""
import hashlib
import json
import os

import numpy as np
import pytest

import bdpt_amd as B
from _util import GOLD, REPO

SCENES = os.path.join(REPO, "scenes")


@pytest.mark.parametrize("name", ["CBspheres", "CBspheres_lambertian", "CBspheres_refract", "CBgems",
                                  "CBempty", "CBspheres_microfacet_al_ag"])
def test_loader_bit_exact_vs_reference_loader(name, tmp_path):
    out = tmp_path / f"{name}.json"
    with open(os.path.join(GOLD, "scenes", name + ".json")) as f:
        ref = json.load(f)
    cam = ref["camera"]
    B.load_dae(os.path.join(SCENES, name + ".dae"), cam["screenW"], cam["screenH"], dump_json=str(out))
    with open(out) as f:
        got = json.load(f)
    for k in ("lights", "materials", "prim_order", "spheres", "triangles"):
        assert got[k] == ref[k], k
    for k, v in cam.items():
        assert got["camera"][k] == v, k


@pytest.mark.parametrize("name", ["banana", "teapot"])
def test_loader_directional_scenes_vs_reference_loader(name, tmp_path):
    """dae/keenan/banana.dae (ambient + directional) and dae/meshedit/teapot.dae (directional): the
    reference dump's lights / materials / camera verbatim, the geometry by sha256 (fixtures from
    tools/make_pt_golden.py)."""
    with open(os.path.join(GOLD, "scenes", name + ".compact.json")) as f:
        ref = json.load(f)
    cam = ref["camera"]
    out = tmp_path / f"{name}.json"
    B.load_dae(os.path.join(SCENES, name + ".dae"), cam["screenW"], cam["screenH"], dump_json=str(out))
    with open(out) as f:
        got = json.load(f)
    assert got["lights"] == ref["lights"] and got["materials"] == ref["materials"]
    for k in ("prim_order", "spheres", "triangles"):
        assert hashlib.sha256(json.dumps(got[k], sort_keys=True).encode()).hexdigest() == ref[k + "_sha256"], k
    for k, v in cam.items():
        assert got["camera"][k] == v, k


def test_loader_scene_feeds_renderer_like_json():
    """load_dae and scene_from_json(reference dump) give identical scene descriptors."""
    a = B.load_dae(os.path.join(SCENES, "CBgems.dae"), 480, 360)
    b = B.scene_from_json(os.path.join(GOLD, "scenes", "CBgems.json"))
    assert np.array_equal(a.prim_type, b.prim_type)
    assert np.array_equal(a.prim_geom, b.prim_geom)
    assert np.array_equal(a.prim_mat, b.prim_mat)
    da, db = a.desc(), b.desc()
    assert list(da.camera.c2w) == list(db.camera.c2w) and list(da.camera.w2c) == list(db.camera.w2c)
    assert da.camera.hfov_deg == db.camera.hfov_deg and da.camera.vfov_deg == db.camera.vfov_deg


def test_bunny_facts_and_standin():
    """CBbunny against the reference loader's facts (tests/golden/scenes/facts.json) and the CBlucy
    stand-in (tools/gen_standin.py) against SURVEY.md §8d: 114,316 primitives, 73,023 reference
    BVH nodes, depth 23."""
    import ctypes as C
    from test_core_cpu import core
    with open(os.path.join(GOLD, "scenes", "facts.json")) as f:
        facts = json.load(f)["CBbunny"]
    for name, nprim, nodes, depth in (("CBbunny", facts["nprim"], facts["bvh_nodes"], facts["bvh_depth"]),
                                      ("CBlucy_standin", 114316, 73023, 23)):
        path = os.path.join(SCENES, name + ".dae")
        if name == "CBlucy_standin" and not os.path.exists(path):
            import sys
            sys.path.insert(0, REPO)
            import __graft_entry__ as g
            g.build_scenes()
        sc = B.load_dae(path, 800, 600)
        assert sc.nprim == nprim
        d, n = C.c_int(), C.c_int()
        order = (C.c_int * sc.nprim)()
        assert core().core_cpu_scene_info(C.byref(sc.desc()), C.byref(d), C.byref(n), order) == 0
        assert (n.value, d.value) == (nodes, depth)
    cam = facts["camera"]
    sc = B.load_dae(os.path.join(SCENES, "CBbunny.dae"), 800, 600)
    assert list(sc.camera["pos"]) == cam["pos"]
