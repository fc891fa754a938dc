"""The multi-GPU product path with more than one rank, on hardware: bench.py under torchrun, two
ranks sharing device 0 (--devices 0,0) over gloo — bdpt_amd.ShardedRender's sample-range split,
bdpt_copy_frame and the all-reduce of the device frame, the same code the RCCL runs take with the
backend string "nccl" (RCCL cannot put two ranks on one GPU). The reduced frame must equal one
single-rank render of the same samples, and per_rank must show both ranks' work."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import bdpt_amd as B
from _util import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_two_ranks_on_one_device_reduce_to_single_render(tmp_path, scaling):
    W, H, SPP, M, STEPS, WARM = 160, 120, 8, 5, 2, 1
    out = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--workload", "c2", "--width", str(W), "--height", str(H), "--spp", str(SPP),
           "--steps", str(STEPS), "--warmup", str(WARM), "--scaling", scaling, "--dist-backend", "gloo",
           "--devices", "0,0", "--dump-frame", str(out), "--no-cpu-baseline", "--no-parity"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, cwd=REPO, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line[k] for k in ("value", "n_gpus", "ms_per_step", "per_rank")}))
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    pr = line["per_rank"]
    assert pr["backend"] == "gloo" and pr["device"] == [0, 0] and len(pr["elapsed_s"]) == 2
    per_rank = SPP // 2 if scaling == "strong" else SPP
    assert pr["samples_per_step"] == [W * H * per_rank] * 2
    assert line["value"] > 0
    frame = np.load(out).astype(np.float64)
    # every rank's context accumulated its ranges of all WARM + STEPS steps: together, global
    # samples [0, (WARM + STEPS) * SPP) (strong) or [0, (WARM + STEPS) * 2 * SPP) (weak), with the
    # sample weight 1 / SPP (strong) or 1 / (2 SPP) (weak)
    ns = SPP if scaling == "strong" else 2 * SPP
    total = (WARM + STEPS) * ns
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.BidirectionalPathTracer(sc, W, H, ns, M, seed=5489)
    pt.raytrace_tiles([], 0, total)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    rmse = float(np.sqrt(np.mean((frame - single) ** 2)))
    print(f"reduced vs single-rank render: rmse {rmse:.3e}, mean {frame.mean():.6f} vs {single.mean():.6f}")
    assert rmse < 1e-6


@pytest.mark.timeout(600)
def test_rccl_world_size_one_all_reduce():
    """bench.py under torchrun at world size 1 with the default backend: the process group is
    RCCL ("nccl", init_process_group(device_id=...)), ShardedRender's all_reduce of the device
    frame runs on it (a one-rank RCCL collective on torch's stream after bdpt_copy_frame), and the
    frame equals a plain render of the same samples."""
    W, H, SPP, M, STEPS, WARM = 160, 120, 4, 5, 2, 1
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "frame.npy")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
               "--gpus", "1", "--workload", "c2", "--width", str(W), "--height", str(H), "--spp", str(SPP),
               "--steps", str(STEPS), "--warmup", str(WARM), "--dump-frame", out, "--no-cpu-baseline",
               "--no-parity"]
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, cwd=REPO, env=env)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        print(json.dumps({k: line[k] for k in ("value", "n_gpus", "per_rank")}))
        assert line["n_gpus"] == 1 and line["per_rank"]["backend"] == "nccl"
        assert "RCCL all-reduce" in line["config"]["workload"]
        frame = np.load(out).astype(np.float64)
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.BidirectionalPathTracer(sc, W, H, SPP, M, seed=5489)
    pt.raytrace_tiles([], 0, (WARM + STEPS) * SPP)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    rmse = float(np.sqrt(np.mean((frame - single) ** 2)))
    print(f"RCCL world-1 frame vs plain render: rmse {rmse:.3e}")
    assert rmse < 1e-6
