#!/usr/bin/env python3
"""Reference PNG fixtures for the output stage: renders the small golden
configs with the reference's own binary (oracle/_ref/ref_driver, -t 1, deterministic) and keeps
its PNG + _rate.png next to the HDR buffers of the same run, checking those buffers are the ones
already committed (tests/golden/hdr/*.npz). THIS CONTAINER ONLY (needs /root/reference)."""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")
CFGS = [("CBspheres_lambertian", 64, 48, 2, 5), ("CBspheres", 64, 48, 2, 5), ("CBgems", 64, 48, 2, 7),
        ("CBempty", 64, 48, 2, 5)]
# the -p cell render (render_to_file's cell branch, raytraced_renderer.cpp:622-646): its PNG is the
# cell alone, its _rate.png the whole frame; 64 spp so the cell image can be compared statistically
CELLS = [("CBgems", 64, 48, 64, 5, (8, 4, 48, 24)),
         # a cell holding 32-aligned pixels ((32, 16), (32, 32)): the binding's set_cell case
         ("CBgems", 64, 48, 64, 5, (16, 12, 40, 28))]


def main():
    os.makedirs(os.path.join(GOLD, "png"), exist_ok=True)
    tmp = tempfile.mkdtemp()
    for scene, W, H, S, M in CFGS:
        key = f"{scene}_{W}x{H}_s{S}_m{M}"
        pre = os.path.join(tmp, key)
        subprocess.run([DRIVER, "-t", "1", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f",
                        pre + ".png", "-o", pre, os.path.join("/root/reference/dae/sky", scene + ".dae")],
                       check=True, capture_output=True)
        ref = np.load(os.path.join(GOLD, "hdr", key + ".npz"))["sample"]
        if not np.array_equal(np.load(pre + "_sample.npy"), ref):
            sys.exit(f"{key}: reference run differs from the committed HDR fixture")
        shutil.copy(pre + ".png", os.path.join(GOLD, "png", key + ".png"))
        shutil.copy(pre + "_rate.png", os.path.join(GOLD, "png", key + "_rate.png"))
        print(key, "ok")
    for scene, W, H, S, M, (x, y, dx, dy) in CELLS:
        key = f"{scene}_{W}x{H}_s{S}_m{M}_cell_{x}_{y}_{dx}_{dy}"
        pre = os.path.join(tmp, key)
        subprocess.run([DRIVER, "-t", "1", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-p", str(x), str(y),
                        str(dx), str(dy), "-f", pre + ".png", os.path.join("/root/reference/dae/sky", scene + ".dae")],
                       check=True, capture_output=True)
        shutil.copy(pre + ".png", os.path.join(GOLD, "png", key + ".png"))
        shutil.copy(pre + "_rate.png", os.path.join(GOLD, "png", key + "_rate.png"))
        print(key, "ok")


if __name__ == "__main__":
    main()
