"""Bridge between the parity links: the counter-RNG fp32 semantics (oracle mode 2,
which the GPU matches per pixel) against the reference itself. Per-sample values cannot match
(different random numbers), so the image means are compared within their noise: the reference's
own 1-spp means at 480x360 (tests/golden/hdr/index.json, dumped by the reference binary) against
mode-2 renders of the same configs, with the noise level estimated from independent 1-spp mode-2
frames. CPU only."""
import numpy as np
import pytest

from _util import MODE_C32, golden_index, golden_scene, oracle_render


@pytest.mark.parametrize("key", ["CBspheres_480x360_s1_m5", "CBspheres_lambertian_480x360_s1_m5"])
def test_counter_fp32_mode_matches_reference_means(key):
    ref = golden_index()[key]
    W, H, M = ref["W"], ref["H"], ref["max_depth"]
    sc = golden_scene(ref["scene"], W, H)
    K = 4
    means = []
    for s in range(K):   # K independent 1-spp frames (global sample indices s)
        img = oracle_render(sc, W, H, 1, M, MODE_C32, seed=5489, s0=s, count=1)[0]
        means.append(img.reshape(-1, 3).mean(axis=0))
    means = np.array(means)
    ours = means.mean(axis=0)
    sigma1 = means.std(axis=0, ddof=1)                  # noise of one 1-spp frame mean
    tol = 5 * np.sqrt(sigma1 ** 2 + sigma1 ** 2 / K) + 1e-4
    diff = np.abs(ours - np.array(ref["mean"]["sample"]))
    assert (diff < tol).all(), f"{key}: mode-2 mean {ours} vs reference {ref['mean']['sample']} (tol {tol})"
