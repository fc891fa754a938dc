"""The reference-side binding (integration/bidirection_amd.h) compiled against the
reference's own headers and objects: oracle/_ref/ref_driver_amd is ref_driver (the reference's
Application::load glue + RaytracedRenderer, built by oracle/ref.mk from /root/reference) with
BidirectionalPathTracerAMD swapped in for BidirectionalPathTracer (-G). It flattens the reference's
primitives, BSDFs, lights and camera into bdpt_scene_desc and renders through libbdpt_amd.so.

CPU: without a device, attach() must fail cleanly with BDPT_E_DEVICE (exit 23), after the whole
scene went through the flattening. GPU: its sampleBuffer must match the oracle's mode 2 render of the
same scene (the product loader's scene, bit-identical to the reference's per tests/test_dae_loader.py)
within the GPU parity tolerance. The binary is built in this container (the reference sources are
not on the GPU box); where it is absent the tests skip."""
import os
import subprocess

import numpy as np
import pytest

from _util import MODE_C32, REPO, oracle_render

AMD = os.path.join(REPO, "oracle", "_ref", "ref_driver_amd")
needs_bin = pytest.mark.skipif(not os.path.exists(AMD), reason="oracle/_ref/ref_driver_amd not built "
                                                               "(make -f oracle/ref.mk amd; needs /root/reference)")


def _run(tmp_path, scene, W, H, S, M):
    prefix = str(tmp_path / "amd")
    r = subprocess.run([AMD, "-G", "-t", "1", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-o", prefix,
                        os.path.join(REPO, "scenes", scene + ".dae")], capture_output=True, text=True, timeout=300,
                       cwd=tmp_path)
    return r, prefix + "_sample.npy"


@needs_bin
def test_binding_compiles_and_fails_cleanly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present: the GPU test covers the binding")
    r, _ = _run(tmp_path, "CBspheres", 64, 48, 2, 5)
    assert r.returncode == 23, r.stdout + r.stderr      # 20 - BDPT_E_DEVICE
    assert "no HIP device" in r.stderr


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("scene,M", [("CBspheres", 5), ("CBgems", 7)])
def test_binding_renders_like_the_oracle(tmp_path, scene, M):
    import bdpt_amd as B
    W, H, S = 64, 48, 2
    r, npy = _run(tmp_path, scene, W, H, S, M)
    assert r.returncode == 0, r.stdout + r.stderr
    ours = np.load(npy)                                  # (H, W, 3), row 0 = bottom
    sc = B.load_dae(os.path.join(REPO, "scenes", scene + ".dae"), W, H)
    ref = oracle_render(sc, W, H, S, M, MODE_C32)[0]
    rmse = float(np.sqrt(np.mean((ours - ref) ** 2)))
    assert rmse < 1e-4, rmse


def _run_loop(tmp_path, scene, W, H, S, M, threads=8):
    """-A: the binding behind the reference's own render loop (RaytracedRenderer::render_to_file with
    `threads` workers -> raytrace_tile -> raytrace_pixel -> write_to_framebuffer -> save_image), with
    the one-line swap of raytraced_renderer.cpp:53 done right after the renderer is constructed."""
    prefix = str(tmp_path / "loop")
    png = str(tmp_path / "loop.png")
    r = subprocess.run([AMD, "-A", "-t", str(threads), "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f", png,
                        "-o", prefix, os.path.join(REPO, "scenes", scene + ".dae")], capture_output=True, text=True,
                       timeout=300, cwd=tmp_path)
    return r, png, prefix


@needs_bin
def test_render_loop_binding_fails_cleanly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present: the GPU test covers the binding")
    r, _, _ = _run_loop(tmp_path, "CBspheres", 64, 48, 2, 5)
    assert r.returncode == 23, r.stdout + r.stderr
    assert "no HIP device" in r.stderr


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("scene,W,H,S,M", [("CBspheres", 200, 150, 2, 5), ("CBgems", 160, 100, 2, 7)])
def test_reference_render_loop_through_binding(tmp_path, scene, W, H, S, M):
    """The reference's unmodified render_to_file at -t 8 with BidirectionalPathTracerAMD in place:
    every 32x32 tile (raytraced_renderer.cpp:293-298) queued once, in at most one bdpt_render per
    tile (the binding batches the tiles queued while a launch runs), the PNG its own save_image
    writes equal to the product CLI's at the same seed (light-image splats are fp32 atomics in
    another order, so a byte may differ by one step where a value sits on a quantisation
    boundary), its sampleBuffer / eyeBuffer / lightBuffer within the parity tolerance of the
    oracle's mode 2, and its sampling-rate image all ns_aa (bidirection.cpp:539)."""
    import bdpt_amd as B
    from test_output_stage import CLI, read_png
    r, png, prefix = _run_loop(tmp_path, scene, W, H, S, M)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Rendering... 100%!" in r.stdout and "Job completed" in r.stdout
    ntiles = ((W + 31) // 32) * ((H + 31) // 32)
    launches = int(r.stdout.split("bdpt_render launches:")[1].split()[0])
    queued = int(r.stdout.split("bdpt_render launches:")[1].split()[2])
    assert queued == ntiles and 1 <= launches <= ntiles, (launches, queued, ntiles)
    sc = B.load_dae(os.path.join(REPO, "scenes", scene + ".dae"), W, H)
    samp, eye, light, _ = oracle_render(sc, W, H, S, M, MODE_C32)
    for name, ref in (("sample", samp), ("eye", eye), ("light", light)):
        ours = np.load(f"{prefix}_{name}.npy")
        rmse = float(np.sqrt(np.mean((ours - ref) ** 2)))
        assert rmse < 1e-4, (name, rmse)
    cli_png = tmp_path / "cli.png"
    rc = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f", str(cli_png), "--no-stats",
                         os.path.join(REPO, "scenes", scene + ".dae")], capture_output=True, text=True, timeout=300)
    assert rc.returncode == 0, rc.stderr
    a, b = read_png(png).astype(int), read_png(cli_png).astype(int)
    d = np.abs(a - b)
    print(f"{scene}: PNG bytes differing {np.count_nonzero(d)} of {d.size}, max {d.max()}")
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.001 * d.size
    rate_ref = read_png(tmp_path / "loop_rate.png")
    assert np.array_equal(rate_ref, read_png(tmp_path / "cli_rate.png"))


def _run_tile_loop(tmp_path, scene, W, H, S, M, threads=8):
    """-B: the reference's worker loop (raytrace_tile's raytrace_pixel calls over the 32x32 tile
    queue, `threads` workers) through the binding, without the per-tile whole-frame tonemap."""
    prefix = str(tmp_path / "tl")
    r = subprocess.run([AMD, "-B", "-t", str(threads), "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-o", prefix,
                        os.path.join(REPO, "scenes", scene + ".dae")], capture_output=True, text=True, timeout=300,
                       cwd=tmp_path)
    return r, prefix


@needs_bin
def test_tile_loop_fails_cleanly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present: the GPU test covers the binding")
    r, _ = _run_tile_loop(tmp_path, "CBspheres", 64, 48, 2, 5)
    assert r.returncode == 23, r.stdout + r.stderr
    assert "no HIP device" in r.stderr


@needs_bin
@pytest.mark.gpu
def test_tile_loop_batches_and_matches_oracle(tmp_path):
    """All tiles queued exactly once, fewer launches than tiles (batched), and the frame equal to
    oracle mode 2 within the GPU parity tolerance."""
    import bdpt_amd as B
    W, H, S, M = 320, 240, 2, 5
    r, prefix = _run_tile_loop(tmp_path, "CBspheres", W, H, S, M)
    assert r.returncode == 0, r.stdout + r.stderr
    print(r.stdout)
    line = r.stdout.split("binding tile loop:")[1]
    tiles = int(line.split(" tiles")[0].split(",")[-1])
    launches = int(line.split(" bdpt_render")[0].split(",")[-1])
    ntiles = ((W + 31) // 32) * ((H + 31) // 32)
    assert tiles == ntiles and 1 <= launches < ntiles, (tiles, launches, ntiles)
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    samp, eye, light, _ = oracle_render(sc, W, H, S, M, MODE_C32)
    for name, ref in (("sample", samp), ("eye", eye), ("light", light)):
        ours = np.load(f"{prefix}_{name}.npy")
        assert float(np.sqrt(np.mean((ours - ref) ** 2))) < 1e-4, name


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("threads,cell,hook", [(1, (8, 4, 48, 24), True), (1, (16, 12, 40, 28), True),
                                               (1, (8, 4, 48, 24), False)])
def test_reference_cell_render_through_binding(tmp_path, threads, cell, hook):
    """The reference's -p cell branch (render_to_file(x, y, dx, dy) -> raytrace_cell: 8x8 tiles at
    the cell's corner, raytraced_renderer.cpp:300-318, 622-646) with the binding in place.
    hook: the binding is told the cell (set_cell, the maintainer's line in render_to_file's cell
    branch) and renders it as one rectangle — also a cell holding 32-aligned pixels ((32, 16),
    (32, 32)), which the pixels alone would take for 32x32 tile corners. No hook (ref_driver -C):
    every pixel of a cell without 32-aligned pixels is queued alone, the lone pixels of a batch
    merge into rectangles, every batch refreshes the queued pixels' bounding box.
    The PNG (the cell alone) must equal the product CLI's -p render of the same cell and samples;
    the rate image the reference binary's own (the sampled pixels are exactly the cell's). One
    worker: with several, the reference's own unsynchronised whole-frame write_to_framebuffer calls
    (:619) race at the end."""
    from test_output_stage import CLI, read_png
    W, H, S, M = 64, 48, 64, 5
    x0, y0, dx, dy = cell
    png = str(tmp_path / "cell.png")
    r = subprocess.run([AMD, "-A"] + ([] if hook else ["-C"]) + ["-t", str(threads), "-s", str(S), "-m", str(M),
                        "-r", str(W), str(H), "-p", str(x0),
                        str(y0), str(dx), str(dy), "-f", png, os.path.join(REPO, "scenes", "CBgems.dae")],
                       capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Cell job completed" in r.stdout
    cli = tmp_path / "cli.png"
    rc = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-p", str(x0), str(y0), str(dx), str(dy),
                         "-f", str(cli), "--no-stats", os.path.join(REPO, "scenes", "CBgems.dae")],
                        capture_output=True, text=True, timeout=300)
    assert rc.returncode == 0, rc.stderr
    a, b = read_png(png).astype(int), read_png(cli).astype(int)
    assert a.shape == b.shape == (dy, dx, 4)
    d = np.abs(a - b)
    print(f"cell through the binding, -t {threads}: PNG bytes differing {np.count_nonzero(d)} of {d.size}, max {d.max()}")
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.002 * d.size
    key = f"CBgems_{W}x{H}_s{S}_m{M}_cell_{x0}_{y0}_{dx}_{dy}"
    assert np.array_equal(read_png(str(tmp_path / "cell_rate.png")),
                          read_png(os.path.join(REPO, "tests", "golden", "png", key + "_rate.png")))


def _two_ctx_env(devices):
    return dict(os.environ, BDPT_DEVICES=devices)


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["0,0", "0,1"])
def test_reference_render_loop_on_two_contexts(tmp_path, devices):
    """BDPT_DEVICES: the binding's contexts on the listed devices ("0,0": two contexts sharing the
    one GPU of this pool's boxes; "0,1": two GPUs, skipped below 2 devices). The reference's
    unmodified render_to_file at -t 8 hands tile batches to whichever context is free; finish()
    sums the contexts' frames with the RCCL reduce before save_image. The PNG must equal the
    product CLI's one-device render (fp32 splat order aside) and the buffers the oracle's mode 2."""
    from _util import device_count
    if devices == "0,1" and device_count() < 2:
        pytest.skip("needs >= 2 visible GPUs (this pool's boxes have one)")
    import bdpt_amd as B
    from test_output_stage import CLI, read_png
    W, H, S, M = 200, 150, 2, 5
    prefix = str(tmp_path / "loop")
    png = str(tmp_path / "loop.png")
    r = subprocess.run([AMD, "-A", "-t", "8", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f", png, "-o", prefix,
                        os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True, timeout=300,
                       cwd=tmp_path, env=_two_ctx_env(devices))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "2 device context(s)" in r.stdout, r.stdout
    ntiles = ((W + 31) // 32) * ((H + 31) // 32)
    queued = int(r.stdout.split("bdpt_render launches:")[1].split()[2])
    assert queued == ntiles
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    samp, eye, light, _ = oracle_render(sc, W, H, S, M, MODE_C32)
    for name, ref in (("sample", samp), ("eye", eye), ("light", light)):
        assert float(np.sqrt(np.mean((np.load(f"{prefix}_{name}.npy") - ref) ** 2))) < 1e-4, name
    cli_png = tmp_path / "cli.png"
    rc = subprocess.run([CLI, "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-f", str(cli_png), "--no-stats",
                         os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True, timeout=300)
    assert rc.returncode == 0, rc.stderr
    d = np.abs(read_png(png).astype(int) - read_png(cli_png).astype(int))
    print(f"two contexts ({devices}): PNG bytes differing {np.count_nonzero(d)} of {d.size}, max {d.max()}")
    assert d.max() <= 1 and np.count_nonzero(d) <= 0.001 * d.size


@needs_bin
@pytest.mark.gpu
def test_tile_loop_on_two_contexts(tmp_path):
    """The reference's worker loop through the binding with BDPT_DEVICES=0,0: batches on both
    contexts, the summed frame within the parity tolerance of oracle mode 2."""
    W, H, S, M = 320, 240, 2, 5
    prefix = str(tmp_path / "tl")
    r = subprocess.run([AMD, "-B", "-t", "8", "-s", str(S), "-m", str(M), "-r", str(W), str(H), "-o", prefix,
                        os.path.join(REPO, "scenes", "CBspheres.dae")], capture_output=True, text=True, timeout=300,
                       cwd=tmp_path, env=_two_ctx_env("0,0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "2 device context(s)" in r.stdout, r.stdout
    import bdpt_amd as B
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    samp, eye, light, _ = oracle_render(sc, W, H, S, M, MODE_C32)
    for name, ref in (("sample", samp), ("eye", eye), ("light", light)):
        assert float(np.sqrt(np.mean((np.load(f"{prefix}_{name}.npy") - ref) ** 2))) < 1e-4, name
