#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs oracle/_ref/ref_driver (the reference's own hot-path sources compiled by oracle/ref.mk;
this container only — /root/reference does not exist on the GPU box) at -t 1, where the
reference is bit-deterministic, and stores:
  tests/golden/scenes/<scene>.json   the static scene the reference integrator saw
                                     (primitives in scene order, BSDFs, lights, camera, BVH facts)
  tests/golden/hdr/index.json        per render config: sha256 of the fp64 sample/eye/light
                                     buffers, their means, rays traced, prim tests
  tests/golden/hdr/<cfg>.npz         full fp64 buffers for the small configs
Usage: python3 tools/make_golden.py   (needs `make -f oracle/ref.mk` first)
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
GOLD = os.path.join(REPO, "tests", "golden")

SCENES = ["CBspheres_lambertian", "CBspheres", "CBgems", "CBempty", "CBspheres_refract"]
# (scene, W, H, spp, max_depth, keep_full_buffers)
RENDERS = [
    ("CBspheres_lambertian", 64, 48, 2, 5, True),
    ("CBspheres", 64, 48, 2, 5, True),
    ("CBgems", 64, 48, 2, 7, True),
    ("CBempty", 64, 48, 2, 5, True),
    ("CBspheres", 160, 120, 1, 5, False),
    ("CBspheres_lambertian", 480, 360, 1, 5, False),
    # BASELINE.json configs[0] itself: CBspheres_lambertian 480x360 -s 4 -m 5 at -t 1
    ("CBspheres_lambertian", 480, 360, 4, 5, False),
    ("CBspheres", 480, 360, 1, 5, False),
    ("CBgems", 240, 180, 1, 7, False),
    ("CBspheres", 96, 72, 3, 1, False),
    ("CBspheres", 96, 72, 1, 8, False),
    ("CBbunny", 80, 60, 1, 5, False),
    # higher-spp renders for the per-pixel statistical bridge between the reference's own
    # mt19937 stream and the counter-RNG modes (tests/test_bridge.py)
    ("CBspheres", 64, 48, 64, 5, True),
    ("CBgems", 64, 48, 64, 7, True),
    ("CBbunny", 64, 48, 64, 5, True),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def run(scene, W, H, S, M, out_prefix, json_path=None, render=True):
    cmd = [DRIVER, "-t", "1", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f",
           out_prefix + ".png"]
    if render:
        cmd += ["-o", out_prefix]
    else:
        cmd += ["-n"]
    if json_path:
        cmd += ["-j", json_path]
    cmd.append(os.path.join(REF, "dae", "sky", scene + ".dae"))
    p = subprocess.run(cmd, capture_output=True, text=True, check=True)
    m = re.search(r"rays=(\d+) isects=(\d+)", p.stdout)
    return (int(m.group(1)), int(m.group(2))) if m else (None, None)


def main():
    only = sys.argv[1:]   # optional render keys: regenerate just those (index entries merged)
    if not os.path.exists(DRIVER):
        sys.exit("build oracle/_ref first: make -f oracle/ref.mk -j8")
    os.makedirs(os.path.join(GOLD, "scenes"), exist_ok=True)
    os.makedirs(os.path.join(GOLD, "hdr"), exist_ok=True)
    tmp = tempfile.mkdtemp()
    for s in ([] if only else SCENES):
        run(s, 480, 360, 1, 1, os.path.join(tmp, s), os.path.join(GOLD, "scenes", s + ".json"),
            render=False)
    # BVH facts of the large mesh (scene JSON too big to commit): dump to tmp, keep the stats.
    if not only:
        bunny_json = os.path.join(tmp, "CBbunny.json")
        run("CBbunny", 480, 360, 1, 1, os.path.join(tmp, "CBbunny"), bunny_json, render=False)
        with open(bunny_json) as f:
            bj = json.load(f)
        facts = {"CBbunny": {"nprim": len(bj["prim_order"]), "bvh_nodes": bj["bvh"]["nodes"],
                             "bvh_leaves": bj["bvh"]["leaves"], "bvh_depth": bj["bvh"]["depth"],
                             "camera": bj["camera"], "lights": bj["lights"],
                             "materials": bj["materials"],
                             "scene_sha256": hashlib.sha256(json.dumps(
                                 [bj["triangles"], bj["spheres"]]).encode()).hexdigest()}}
        with open(os.path.join(GOLD, "scenes", "facts.json"), "w") as f:
            json.dump(facts, f, indent=1)
    index = {}
    if only:
        with open(os.path.join(GOLD, "hdr", "index.json")) as f:
            index = json.load(f)
    for scene, W, H, S, M, keep in RENDERS:
        key = f"{scene}_{W}x{H}_s{S}_m{M}"
        if only and key not in only:
            continue
        pre = os.path.join(tmp, key)
        rays, isects = run(scene, W, H, S, M, pre)
        bufs = {n: np.load(f"{pre}_{n}.npy") for n in ("sample", "eye", "light")}
        index[key] = {
            "scene": scene, "W": W, "H": H, "spp": S, "max_depth": M, "rays": rays,
            "prim_tests": isects,
            "sha256": {n: sha(b) for n, b in bufs.items()},
            "mean": {n: [float(x) for x in b.reshape(-1, 3).mean(axis=0)] for n, b in bufs.items()},
            "full": keep,
        }
        if keep:
            np.savez_compressed(os.path.join(GOLD, "hdr", key + ".npz"), **bufs)
        print(key, rays, index[key]["mean"]["sample"], flush=True)
    with open(os.path.join(GOLD, "hdr", "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
