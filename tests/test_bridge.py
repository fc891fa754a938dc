"""Bridge between the parity links: the counter-RNG fp32 semantics (oracle mode 2,
which the GPU matches per pixel) against the reference itself. Per-sample values cannot match
(different random numbers), so the comparison is statistical.

* Image means: the reference's own 1-spp means at 480x360 (tests/golden/hdr/index.json, dumped by
  the reference binary) against mode-2 renders of the same configs, within their noise.
* Per pixel: the reference's own 64-spp frames (tools/make_golden.py: oracle/_ref/ref_driver -t 1,
  64x48 s64 of CBspheres, CBgems and CBbunny) against 64-spp mode-2 frames. The deviation of each
  pixel, in units of its standard error, must have the same tail shares as the deviations between
  independent mode-2 frames (tests/_parity.py: the per-pixel values are heavy-tailed — caustic
  splats in the light image — so the null is mode 2 itself, not a Gaussian). CPU only; the GPU
  form is tests/test_gpu_parity.py::test_gpu_matches_reference_per_pixel."""
import os

import numpy as np
import pytest

from _parity import check_tails, null_calibrated_tails
from _util import GOLD, MODE_C32, REPO, golden_index, golden_scene, oracle_render

# (fixture key, scene, max_depth)
HI_SPP = [("CBspheres_64x48_s64_m5", "CBspheres", 5), ("CBgems_64x48_s64_m7", "CBgems", 7),
          ("CBbunny_64x48_s64_m5", "CBbunny", 5)]
N_VAR, N_NULL = 256, 6


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


def hi_spp_fixture(key):
    g = golden_index()[key]
    return g, np.load(os.path.join(GOLD, "hdr", key + ".npz"))["sample"]


@pytest.mark.parametrize("key,scene,M", HI_SPP)
def test_counter_fp32_mode_matches_reference_per_pixel(key, scene, M):
    import bdpt_amd as B
    g, ref = hi_spp_fixture(key)
    W, H, S = g["W"], g["H"], g["spp"]
    sc = B.load_dae(os.path.join(REPO, "scenes", scene + ".dae"), W, H)

    def frame(s0, n):   # mode 2, global samples [s0, s0 + n), weight 1/n
        return oracle_render(sc, W, H, n, M, MODE_C32, s0=s0, count=n)[0]

    A = frame(0, S)
    var1 = np.array([frame(S + k, 1) for k in range(N_VAR)]).var(0, ddof=1)
    nulls = [frame(S + N_VAR + S * k, S) for k in range(N_NULL)]
    r = null_calibrated_tails(ref, A, nulls, var1, S)
    print(key, "reference", np.round(r["ref_tails"], 4), round(r["ref_mean_z"], 3), "nulls",
          np.round(r["null_tails"].mean(0), 4), np.round(r["null_mean_z"], 3))
    check_tails(r, key)


@pytest.mark.gpu
@pytest.mark.parametrize("key,scene,M", HI_SPP)
def test_gpu_matches_reference_per_pixel(key, scene, M):
    """The same per-pixel bridge with the GPU in place of mode 2: libbdpt_amd.so's 64-spp frame
    against the reference binary's own (tools/make_golden.py), the null from independent GPU
    frames."""
    import bdpt_amd as B
    g, ref = hi_spp_fixture(key)
    W, H, S = g["W"], g["H"], g["spp"]
    sc = B.load_dae(os.path.join(REPO, "scenes", scene + ".dae"), W, H)

    def frames(s0, n, count):   # `count` frames of n samples each, from global sample s0 on
        pt = B.BidirectionalPathTracer(sc, W, H, n, M, seed=5489)
        out = []
        try:
            for k in range(count):
                pt.clear()
                pt.raytrace_tiles([], s0 + k * n, n)
                out.append(pt.read_frame(B.FRAME_SAMPLE).astype(np.float64))
        finally:
            pt.close()
        return out

    A = frames(0, S, 1)[0]
    var1 = np.array(frames(S, 1, N_VAR)).var(0, ddof=1)
    nulls = frames(S + N_VAR, S, N_NULL)
    r = null_calibrated_tails(ref, A, nulls, var1, S)
    print(key, "reference", np.round(r["ref_tails"], 4), round(r["ref_mean_z"], 3), "nulls",
          np.round(r["null_tails"].mean(0), 4), np.round(r["null_mean_z"], 3))
    check_tails(r, key)
