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
