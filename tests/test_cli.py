"""The `pathtracer` CLI end to end on the GPU: .dae -> host loader -> libbdpt_amd.so -> PNG, against
the oracle's COUNTER32 render of the same scene (loaded from the reference loader's dump) pushed
through the same output stage. Tonemapped bytes may differ by one step where a pixel sits on a
quantisation boundary (GPU vs CPU differ by ~1e-7 relative from fp32 atomic ordering)."""
import os
import subprocess

import numpy as np
import pytest

from _util import MODE_C32, REPO, device_count, golden_scene, oracle_render
from test_output_stage import CLI, read_png

pytestmark = pytest.mark.gpu


def _check_report(stdout, samples):
    """The reference's end-of-render report on stdout (raytraced_renderer.cpp:679-682), in the same
    format: the regex bench.py uses on the reference binary must parse it, and the counters must be
    those of this render (every pixel-sample traces at least its camera ray)."""
    import re
    m = re.findall(r"Rendering\.\.\. 100%! \(([0-9.]+)s\)", stdout)
    assert m and float(m[-1]) > 0, stdout
    rays = int(re.search(r"\[PathTracer\] BVH traced (\d+) rays\.", stdout).group(1))
    assert rays >= samples
    mrays = float(re.search(r"\[PathTracer\] Average speed ([0-9.]+) million rays per second\.", stdout).group(1))
    # the time is printed to 0.1 ms (%.4f) and a small render takes a few ms: allow that rounding
    secs = float(m[-1])
    assert abs(mrays - rays / secs * 1e-6) <= mrays * (0.5e-4 / secs + 1e-3) + 1e-3
    tests = float(re.search(r"\[PathTracer\] Averaged ([0-9.]+) intersection tests per ray\.", stdout).group(1))
    assert tests > 0


def test_cli_renders_scene_like_oracle(tmp_path):
    W, H, S, M = 64, 48, 2, 5
    out = tmp_path / "cbs.png"
    r = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f", str(out),
                        os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Job completed" in r.stdout
    _check_report(r.stdout, W * H * S)
    ours = read_png(out)
    ref_hdr = oracle_render(golden_scene("CBspheres", W, H), W, H, S, M, MODE_C32)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    ref = read_png(tmp_path / "ref.png")
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size
    assert os.path.exists(tmp_path / "cbs_rate.png")


@pytest.mark.parametrize("cell", [(8, 4, 48, 24), (16, 12, 40, 28)])
def test_cli_cell_render(tmp_path, cell):
    """-p x y dx dy renders one cell (RaytracedRenderer::render_to_file's cell branch,
    raytraced_renderer.cpp:622-646): the PNG is the cell alone (dx x dy, as raytrace_cell copies it
    out of the frame buffer and save_image writes that buffer), the _rate.png the whole frame with
    the cell's pixels sampled. Against the reference binary's own cell render of the same scene
    (tests/golden/png/, tools/make_golden_png.py, -t 1, 64 spp): the rate image byte-equal; the cell
    image, rendered with other random numbers, correlated with the reference's (a vertically
    flipped cell decorrelates: measured 0.49 vs 0.20 with the CPU build of the device code) and of
    the same mean brightness."""
    W, H, S, M = 64, 48, 64, 5
    x0, y0, dx, dy = cell
    key = f"CBgems_{W}x{H}_s{S}_m{M}_cell_{x0}_{y0}_{dx}_{dy}"
    out = tmp_path / "cell.png"
    r = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-p", str(x0), str(y0), str(dx), str(dy),
                        "-f", str(out), "--no-stats", os.path.join(REPO, "scenes", "CBgems.dae")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ours = read_png(out)
    ref = read_png(os.path.join(REPO, "tests", "golden", "png", key + ".png"))
    assert ours.shape == ref.shape == (dy, dx, 4)
    assert np.array_equal(read_png(tmp_path / "cell_rate.png"),
                          read_png(os.path.join(REPO, "tests", "golden", "png", key + "_rate.png")))
    a, b = ours[..., :3].astype(float).ravel(), ref[..., :3].astype(float).ravel()
    corr = np.corrcoef(a, b)[0, 1]
    flipped = np.corrcoef(ours[::-1, :, :3].astype(float).ravel(), b)[0, 1]
    print(f"cell: corr {corr:.3f} (flipped {flipped:.3f}), means {a.mean():.2f} / {b.mean():.2f}")
    assert corr > 0.35 and corr > flipped + 0.15 and abs(a.mean() - b.mean()) < 2.0


def test_cli_environment_map_and_roulette(tmp_path):
    """-e map.exr (the reference's flag, load_exr) + --rr on the environment-only scene, against the
    oracle's COUNTER32 render of the same inputs through the same output stage."""
    import bdpt_amd as B
    env = os.path.join(REPO, "tests", "golden", "env")
    W, H, S, M = 64, 48, 2, 8
    out = tmp_path / "env.png"
    dae = os.path.join(env, "CBspheres_envonly.dae")
    exr = os.path.join(env, "sky_32x16_zip_half.exr")
    r = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-e", exr, "--rr", "-f",
                        str(out), dae], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ours = read_png(out)
    sc = B.load_dae(dae, W, H)
    sc.set_envmap(B.load_exr(exr))
    ref_hdr = oracle_render(sc, W, H, S, M, MODE_C32, rr=True)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    ref = read_png(tmp_path / "ref.png")
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size


@pytest.mark.parametrize("scene", ["CBspheres_microfacet_al_ag", "banana"])
def test_cli_pathtracer(tmp_path, scene):
    """--pt: the reference's unidirectional PathTracer with its -l / -a flags on scenes BDPT rejects
    (a microfacet scene; dae/keenan/banana.dae with its ambient and directional lights), against the
    oracle's mode 2 through the same output stage."""
    import bdpt_amd as B
    from _util import oracle_pt_render
    W, H, S, M = 48, 36, 4, 4
    out = tmp_path / "pt.png"
    dae = os.path.join(REPO, "scenes", scene + ".dae")
    r = subprocess.run([CLI, "--pt", "-s", str(S), "-m", str(M), "-l", "2", "-a", "2", "0", "-r", str(W), str(H),
                        "-f", str(out), dae], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ours = read_png(out)
    sc = B.load_dae(dae, W, H)
    ref_hdr = oracle_pt_render(sc, W, H, S, M, MODE_C32, ns_area_light=2, batch=2, tol=0.0)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    ref = read_png(tmp_path / "ref.png")
    d = np.abs(ours.astype(int) - ref.astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size
    assert os.path.exists(tmp_path / "pt_rate.png")   # sampleCountBuffer / ns_aa, as save_sampling_rate_image


@pytest.mark.parametrize("gpus,spp", [(2, 2), (3, 4)])
def test_cli_multi_gpu_split(tmp_path, gpus, spp):
    """-g N: the sample range split over N workers (one context and one host thread each) and the
    frames summed by the C-ABI's reduce (bdpt_reduce_frames: on-device sum of the contexts sharing a
    GPU, then the RCCL ncclReduce, inside the timed region). --devices puts every worker on device 0
    so a one-GPU box runs the N-worker path; the image must match one render of all samples (oracle
    mode 2). (-g 1, test_cli_renders_scene_like_oracle, makes no reducer: one context holds the
    whole frame, so a one-GPU render needs no RCCL.)"""
    W, H, M = 64, 48, 5
    out = tmp_path / "g.png"
    r = subprocess.run([CLI, "-s", str(spp), "-m", str(M), "-r", str(W), str(H), "-g", str(gpus), "--devices",
                        ",".join(["0"] * gpus), "-f", str(out), os.path.join(REPO, "scenes", "CBspheres.dae")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert f"{gpus} GPU(s)" in r.stderr
    ours = read_png(out)
    ref_hdr = oracle_render(golden_scene("CBspheres", W, H), W, H, spp, M, MODE_C32)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    d = np.abs(ours.astype(int) - read_png(tmp_path / "ref.png").astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size


@pytest.mark.skipif(device_count() < 2, reason="needs >= 2 visible GPUs (every box of this pool has one): "
                                               "-g 2 on distinct devices = a two-rank RCCL reduce over xGMI")
def test_cli_two_devices_default_placement(tmp_path):
    """-g 2 with the default placement (worker g on device g): two RCCL ranks, the cross-device
    ncclReduce of bdpt_reduce_frames into device 0's frames. Same image bar as the one-device split."""
    W, H, M, spp = 64, 48, 5, 4
    out = tmp_path / "g2.png"
    r = subprocess.run([CLI, "-s", str(spp), "-m", str(M), "-r", str(W), str(H), "-g", "2", "-f", str(out),
                        os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "2 GPU(s)" in r.stderr
    ref_hdr = oracle_render(golden_scene("CBspheres", W, H), W, H, spp, M, MODE_C32)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    d = np.abs(read_png(out).astype(int) - read_png(tmp_path / "ref.png").astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size
