#!/usr/bin/env python3
"""Generates tests/golden/env/ from the reference itself (run in this container, where
/root/reference and oracle/_ref/ exist; the GPU box only reads the committed outputs).

  * sky_*.exr: synthetic environment maps written by tools/envmap.py (the reference's exr/*.exr
    are Git-LFS pointers), in the layouts load_exr accepts (ZIP / ZIPS / NONE; HALF / FLOAT);
  * <exr>.npz: what the reference's own code computes from them (oracle/_ref/ref_env_kat):
    tinyexr's decoded map (load_exr, main.cpp:40-77), EnvironmentLight::init's tables, the
    first N sample_L calls of a fresh process and sample_dir for fixed directions;
  * CBspheres_envonly.dae: scenes/CBspheres_lambertian.dae (the reference's scene) with the
    area light and its emissive quad removed — a diffuse-only scene lit by the environment;
  * envonly_pt.npz: the reference's unidirectional PathTracer (oracle/_ref/ref_driver -U) on it
    with the environment map: the converged image the BDPT environment light is checked against
    (tests/test_env.py; BDPT with an environment light is not runnable in the reference).

usage: python tools/make_env_golden.py
"""
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from envmap import synth_envmap, write_exr  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "env")
KAT = os.path.join(REPO, "oracle", "_ref", "ref_env_kat")
DRV = os.path.join(REPO, "oracle", "_ref", "ref_driver")

MAPS = [("sky_32x16_zip_half.exr", 32, 16, "zip", "half"),
        ("sky_24x12_none_float.exr", 24, 12, "none", "float"),
        ("sky_24x12_zips_half.exr", 24, 12, "zips", "half")]
N_SAMPLES = 4096   # sample_L calls per map: glibc sin vs sincos last-bit cases occur ~1 in 5000
PT = dict(W=64, H=48, spp=512, depth=12, threads=8)


def lookup_dirs():
    """Fibonacci-sphere directions plus the axes (poles included)."""
    k = np.arange(40) + 0.5
    y = 1 - 2 * k / 40
    r = np.sqrt(1 - y * y)
    ph = np.pi * (1 + 5 ** 0.5) * k
    d = np.stack([r * np.cos(ph), y, r * np.sin(ph)], -1)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], float)
    return np.concatenate([d, axes])


def envonly_dae(src, dst):
    s = open(src).read()
    for node in ("Area", "light"):
        s, n = re.subn(r'\s*<node id="%s" name="%s" type="NODE">.*?</node>' % (node, node), "", s, flags=re.S)
        assert n == 1, node
    open(dst, "w").write(s)


def main():
    os.makedirs(OUT, exist_ok=True)
    dirs = lookup_dirs()
    with tempfile.TemporaryDirectory() as tmp:
        dpath = os.path.join(tmp, "dirs.txt")
        np.savetxt(dpath, dirs, fmt="%.17g")
        for name, w, h, comp, pix in MAPS:
            exr = os.path.join(OUT, name)
            write_exr(exr, synth_envmap(w, h), comp, pix)
            js = os.path.join(tmp, "kat.json")
            subprocess.run([KAT, exr, str(N_SAMPLES), dpath, js], cwd=tmp, check=True,
                           stdout=subprocess.DEVNULL)
            k = json.load(open(js))
            np.savez_compressed(os.path.join(OUT, name.replace(".exr", ".npz")),
                                rgb=np.array(k["rgb"]).reshape(h, w, 3),
                                pdf_envmap=np.array(k["pdf_envmap"]), marginal_y=np.array(k["marginal_y"]),
                                conds_y=np.array(k["conds_y"]),
                                sample_wi=np.array(k["sample_wi"]).reshape(-1, 3),
                                sample_pdf=np.array(k["sample_pdf"]),
                                sample_L=np.array(k["sample_L"]).reshape(-1, 3),
                                dirs=np.array(k["dirs"]).reshape(-1, 3),
                                sample_dir=np.array(k["sample_dir"]).reshape(-1, 3))
            print("wrote", name, flush=True)
        dae = os.path.join(OUT, "CBspheres_envonly.dae")
        envonly_dae(os.path.join(REPO, "scenes", "CBspheres_lambertian.dae"), dae)
        pre = os.path.join(tmp, "pt")
        cmd = [DRV, "-U", "-e", os.path.join(OUT, MAPS[0][0]), "-a", "64", "0", "-s", str(PT["spp"]),
               "-m", str(PT["depth"]), "-t", str(PT["threads"]), "-r", str(PT["W"]), str(PT["H"]),
               "-o", pre, dae]
        subprocess.run(cmd, cwd=tmp, check=True, stdout=subprocess.DEVNULL)
        img = np.load(pre + "_sample.npy", allow_pickle=False)
        np.savez_compressed(os.path.join(OUT, "envonly_pt.npz"), image=img,
                            cmd=np.array(" ".join(os.path.basename(c) if os.path.isabs(c) else c for c in cmd)),
                            **{k: np.array(v) for k, v in PT.items()})
        print("wrote envonly_pt.npz mean", img.mean(axis=(0, 1)), flush=True)


if __name__ == "__main__":
    main()
