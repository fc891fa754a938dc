"""The CLI's -c camera-settings file (main.cpp:120-121,177-178 -> Application::load_camera ->
Camera::load_settings, camera.cpp:172-186) through bdpt_camera_load_settings.

Pinned by tests/golden/cam/ (tools/make_cam_golden.py): the reference's own ref_driver loaded
CBspheres_orbit.txt after the -r 64 48 resize, dumped the camera it rendered with and rendered
64x48 s2 m5 at -t 1. The loader must reproduce that camera bit for bit — including the quirk that
load_settings leaves w2c at the placement's inverse — and the oracle's mode 0 must then reproduce the
reference's buffers bit for bit (the t = 1 splats exercise the stale w2c)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import bdpt_amd as B
from _util import MODE_C32, MODE_REF, REPO, oracle_render

CAM = os.path.join(REPO, "tests", "golden", "cam")
INDEX = json.load(open(os.path.join(CAM, "index.json")))
KEY = "CBspheres_orbit_64x48_s2_m5"


def _scene():
    g = INDEX[KEY]
    sc = B.load_dae(os.path.join(REPO, "scenes", g["scene"] + ".dae"), g["W"], g["H"])
    sc.load_camera(os.path.join(CAM, g["settings"]))
    return sc, g


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def test_loaded_camera_matches_reference():
    sc, _ = _scene()
    ref = json.load(open(os.path.join(CAM, "CBspheres_orbit.json")))["camera"]
    ours = sc.desc().camera
    assert list(ours.pos) == ref["pos"]
    assert [list(ours.c2w[3 * k:3 * k + 3]) for k in range(3)] == ref["c2w_cols"]
    assert [list(ours.w2c[3 * k:3 * k + 3]) for k in range(3)] == ref["w2c_cols"]   # stale, as the reference's
    assert (ours.hfov_deg, ours.vfov_deg, ours.nclip, ours.fclip) == (ref["hFov"], ref["vFov"], ref["nClip"],
                                                                      ref["fClip"])


def test_oracle_with_loaded_camera_bit_exact_vs_reference():
    sc, g = _scene()
    samp, eye, light, st = oracle_render(sc, g["W"], g["H"], g["spp"], g["max_depth"], MODE_REF)
    assert int(st[0]) == g["rays"] and int(st[4] + st[5]) == g["prim_tests"]
    assert np.count_nonzero(light) > 0          # the t = 1 splats went through the stale w2c
    for n, a in (("sample", samp), ("eye", eye), ("light", light)):
        assert _sha(a) == g["sha256"][n], n


def test_missing_settings_file_leaves_camera_unchanged(tmp_path):
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), 64, 48)
    before = dict(sc.camera)
    with pytest.raises(RuntimeError):
        sc.load_camera(str(tmp_path / "absent.txt"))
    assert sc.camera == before


@pytest.mark.parametrize("text,fclip", [("10 7.5 1.3333 0.2\n", "kept"), ("10 7.5 1.3333 0.2 x 1 2 3\n", 0.0)])
def test_short_settings_file_like_the_reference(tmp_path, text, fclip):
    """A truncated or malformed file, read with the reference's stream extractions: at end of file
    the remaining members keep their values; a token that does not parse zeroes that member (C++11
    num_get) and every later read fails, so pos / c2w keep theirs either way."""
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), 64, 48)
    before = dict(sc.camera)
    p = tmp_path / "short.txt"
    p.write_text(text)
    sc.load_camera(str(p))
    want = before["fClip"] if fclip == "kept" else fclip
    assert (sc.camera["hFov"], sc.camera["vFov"], sc.camera["nClip"], sc.camera["fClip"]) == (10.0, 7.5, 0.2, want)
    assert sc.camera["pos"] == before["pos"] and sc.camera["c2w_cols"] == before["c2w_cols"]


@pytest.mark.gpu
def test_gpu_render_with_loaded_camera():
    from test_gpu_parity import _check_frames, _gpu_render
    sc, g = _scene()
    W, H, S, M = g["W"], g["H"], g["spp"], g["max_depth"]
    _check_frames(_gpu_render(sc, W, H, S, M), oracle_render(sc, W, H, S, M, MODE_C32), "-c camera file")


@pytest.mark.gpu
def test_cli_camera_settings(tmp_path):
    from test_output_stage import CLI, read_png
    sc, g = _scene()
    W, H, S, M = g["W"], g["H"], g["spp"], g["max_depth"]
    out = tmp_path / "cam.png"
    r = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-c",
                        os.path.join(CAM, g["settings"]), "-f", str(out),
                        os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    ours = read_png(out)
    ref_hdr = oracle_render(sc, W, H, S, M, MODE_C32)[0]
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(ref_hdr, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    d = np.abs(ours.astype(int) - read_png(tmp_path / "ref.png").astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size


def _lens_file(tmp_path, focal, lens, short=False):
    """CBspheres_orbit.txt with its last line (focalDistance lensRadius) replaced, or dropped."""
    lines = open(os.path.join(CAM, INDEX[KEY]["settings"])).read().strip().split("\n")
    lines = lines[:-1] + ([] if short else [f"{focal} {lens}"])
    p = tmp_path / "lens.txt"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def test_settings_file_lens_replaces_config(tmp_path):
    """Camera::load_settings reads focalDistance and lensRadius last (camera.cpp:184) and so
    overwrites what set_camera took from -d / -b (raytraced_renderer.cpp:141-142); a file without
    that line leaves the config's values (the failed extraction of a double at EOF stores 0 only
    when characters were consumed; at EOF nothing is consumed and the members keep their values)."""
    g = INDEX[KEY]
    sc = B.load_dae(os.path.join(REPO, "scenes", g["scene"] + ".dae"), g["W"], g["H"])
    assert sc.load_camera(_lens_file(tmp_path, 3.25, 0.125), 4.7, 0.0) == (3.25, 0.125)
    sc = B.load_dae(os.path.join(REPO, "scenes", g["scene"] + ".dae"), g["W"], g["H"])
    fd, lr = sc.load_camera(_lens_file(tmp_path, 0, 0, short=True), 4.5, 0.25)
    # libstdc++ (GLIBCXX_3.4.30, checked with g++ 11.4 on `istringstream("1 2\n") >> x >> y >> a`):
    # the sentry fails at EOF before num_get runs, so a stays 4.5
    assert (fd, lr) == (4.5, 0.25)


@pytest.mark.gpu
def test_cli_pathtracer_uses_settings_file_lens(tmp_path):
    """pathtracer --pt -c file: the thin lens of the file (not -b / -d) renders the image, as in the
    reference (set_camera, then load_camera, then generate_ray_for_thin_lens, pathtracer.cpp:312)."""
    from test_output_stage import CLI, read_png
    from _util import oracle_pt_render
    g = INDEX[KEY]
    W, H, S, M = g["W"], g["H"], 4, 3
    path = _lens_file(tmp_path, 3.25, 0.125)
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres_lambertian.dae"), W, H)
    fd, lr = sc.load_camera(path, 1.0, 0.0)
    out = tmp_path / "pt.png"
    r = subprocess.run([CLI, "--pt", "-s", str(S), "-m", str(M), "-a", str(S), "0.0", "-b", "0", "-d", "1",
                        "-r", str(W), str(H), "-c", path, "-f", str(out),
                        os.path.join(REPO, "scenes", "CBspheres_lambertian.dae")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img, _, _ = oracle_pt_render(sc, W, H, S, M, MODE_C32, batch=S, tol=0.0, lens_radius=lr, focal_distance=fd)
    raw = tmp_path / "ref.f64"
    np.ascontiguousarray(img, dtype="<f8").tofile(raw)
    subprocess.run([CLI, "--tonemap", str(raw), str(W), str(H), str(tmp_path / "ref.png")], check=True)
    d = np.abs(read_png(out).astype(int) - read_png(tmp_path / "ref.png").astype(int))
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size
