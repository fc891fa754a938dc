#!/usr/bin/env python3
"""Generates tests/golden/pt/ — the reference's own unidirectional PathTracer (pathtracer.cpp:47-340,
which the reference builds but never instantiates, raytraced_renderer.cpp:53) rendered by
oracle/_ref/ref_driver -U at -t 1 (bit-deterministic), for SURVEY.md §8 row f4:
  <cfg>.npz : sampleBuffer (fp64, row 0 = bottom), sampleCountBuffer (int32) and the settings;
  tests/golden/scenes/CBspheres_microfacet_al_ag.json : the reference loader's dump of the
    microfacet scene (MicrofacetBSDF eta / k / alpha);
  tests/golden/scenes/{banana,teapot}.compact.json : the loader dumps of the directional-light scenes
    (geometry as sha256 of its canonical JSON).
Run in this container (needs /root/reference and `make -f oracle/ref.mk`).
usage: python tools/make_pt_golden.py [config ...]   (default: every config)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(REPO, "oracle", "_ref", "ref_driver")
OUT = os.path.join(REPO, "tests", "golden", "pt")
SKY = os.path.join(REPO, "tests", "golden", "env", "sky_32x16_zip_half.exr")

# name: (scene, W, H, spp, max_depth, extra flags as (flag, value...) and the settings dict)
CONFIGS = {
    "lambertian": ("CBspheres_lambertian", 64, 48, 8, 5, dict(batch=4, tol=0.05)),
    "delta": ("CBspheres", 64, 48, 8, 5, dict(batch=4, tol=0.05)),
    "microfacet": ("CBspheres_microfacet_al_ag", 64, 48, 4, 5, dict(batch=4, tol=0.05)),
    "roulette": ("CBspheres", 48, 36, 4, 0, dict(batch=4, tol=0.05)),
    "hemisphere": ("CBspheres_lambertian", 48, 36, 4, 4, dict(batch=4, tol=0.05, nal=2, hemi=True)),
    "env_lens": ("CBspheres_lambertian", 48, 36, 4, 4, dict(batch=4, tol=0.05, env=True, lens=0.05, focal=4.0)),
    "adaptive": ("CBempty", 48, 36, 32, 5, dict(batch=8, tol=0.1)),
    "bunny_microfacet": ("CBbunny_microfacet_cu", 48, 36, 2, 4, dict(batch=2, tol=0.05)),
    # an ambient light (GLScene::AmbientLight -> InfiniteHemisphereLight, light.cpp:55-70)
    "ambient": ("bunny", 48, 36, 2, 3, dict(batch=2, tol=0.05, nal=2)),
    "ambient_microfacet_env": ("bunny_microfacet_cu", 48, 36, 2, 3, dict(batch=2, tol=0.05, env=True)),
    # DirectionalLight (light.cpp:11-23): dae/keenan/banana.dae (+ ambient), dae/meshedit/teapot.dae
    "directional_ambient": ("banana", 48, 36, 2, 3, dict(batch=2, tol=0.05, nal=2)),
    "directional": ("teapot", 48, 36, 4, 4, dict(batch=4, tol=0.05)),
    # ns_aa below samplesPerBatch: the reference still runs one whole batch, so every pixel records
    # num_samples = 32 (pathtracer.cpp:301-337); the rule the GPU reduce's count test asserts
    "batch_rounding": ("CBspheres", 48, 36, 4, 5, dict(batch=32, tol=0.0)),
}
# loader dumps too large to keep whole: lights, materials and camera verbatim, the geometry hashed
COMPACT_DUMPS = ["banana", "teapot"]


def compact_dump(js):
    out = {k: js[k] for k in ("lights", "materials", "camera")}
    for k in ("prim_order", "spheres", "triangles"):
        out[k + "_sha256"] = hashlib.sha256(json.dumps(js[k], sort_keys=True).encode()).hexdigest()
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        subprocess.run([DRV, "-n", "-r", "800", "600", "-j",
                        os.path.join(REPO, "tests", "golden", "scenes", "CBspheres_microfacet_al_ag.json"),
                        os.path.join(REPO, "scenes", "CBspheres_microfacet_al_ag.dae")], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL)
        for name in COMPACT_DUMPS:
            js = os.path.join(tmp, name + ".json")
            subprocess.run([DRV, "-n", "-r", "800", "600", "-j", js, os.path.join(REPO, "scenes", name + ".dae")],
                           cwd=tmp, check=True, stdout=subprocess.DEVNULL)
            with open(js) as f:
                dump = compact_dump(json.load(f))
            with open(os.path.join(REPO, "tests", "golden", "scenes", name + ".compact.json"), "w") as f:
                json.dump(dump, f, indent=1)
        for name, (scene, W, H, spp, M, st) in CONFIGS.items():
            if len(sys.argv) > 1 and name not in sys.argv[1:]:
                continue
            pre = os.path.join(tmp, name)
            cmd = [DRV, "-U", "-t", "1", "-s", str(spp), "-m", str(M), "-r", str(W), str(H),
                   "-a", str(st["batch"]), str(st["tol"]), "-l", str(st.get("nal", 1)), "-o", pre]
            if st.get("hemi"):
                cmd.append("-H")
            if st.get("env"):
                cmd += ["-e", SKY]
            if "lens" in st:
                cmd += ["-b", str(st["lens"]), "-d", str(st["focal"])]
            cmd.append(os.path.join(REPO, "scenes", scene + ".dae"))
            subprocess.run(cmd, cwd=tmp, check=True, stdout=subprocess.DEVNULL)
            img = np.load(pre + "_sample.npy", allow_pickle=False)
            cnt = np.fromfile(pre + "_count.bin", dtype=np.int32).reshape(H, W)
            np.savez_compressed(os.path.join(OUT, name + ".npz"), image=img, counts=cnt, scene=np.array(scene),
                                W=W, H=H, spp=spp, max_depth=M, batch=st["batch"], tol=np.float32(st["tol"]),
                                nal=st.get("nal", 1), hemi=bool(st.get("hemi", False)), env=bool(st.get("env", False)),
                                lens=st.get("lens", 0.0), focal=st.get("focal", 4.7))
            print(f"{name}: {scene} {W}x{H} s{spp} m{M} mean {img.mean():.6f} mean count {cnt.mean():.2f}", flush=True)


if __name__ == "__main__":
    sys.exit(main())
