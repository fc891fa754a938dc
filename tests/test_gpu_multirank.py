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
from _util import REPO, device_count

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


def _bench_inprocess(tmp_path, gpus, devices, extra=(), W=160, H=120, SPP=8, STEPS=2, WARM=1):
    """bench.py --gpus N with no launcher: N contexts in one process, the C-ABI's RCCL reduce."""
    out = tmp_path / "frame.npy"
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--workload", "c2",
           "--width", str(W), "--height", str(H), "--spp", str(SPP), "--steps", str(STEPS), "--warmup", str(WARM),
           "--dump-frame", str(out), "--no-cpu-baseline", "--no-parity", *extra]
    if devices:
        cmd += ["--devices", devices]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, cwd=REPO, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps({k: line.get(k) for k in ("value", "n_gpus", "rccl_ranks", "ms_per_step", "per_rank")}))
    return line, np.load(out).astype(np.float64)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_inprocess_two_contexts_on_one_device(tmp_path, scaling):
    """bench.py --gpus 2 --devices 0,0 (no torchrun): two contexts on device 0, their sample ranges
    summed on the device and passed through a one-rank RCCL reduce; n_gpus 2, rccl_ranks 1, and the
    last step's reduced frame equal to one render of that step's samples."""
    W, H, SPP, M, STEPS, WARM = 160, 120, 8, 5, 2, 1
    line, frame = _bench_inprocess(tmp_path, 2, "0,0", ("--scaling", scaling), W, H, SPP, STEPS, WARM)
    assert line["n_gpus"] == 2 and line["rccl_ranks"] == 1 and line["scaling"] == scaling
    assert line["config"]["launch"] == "inprocess" and "bdpt_reduce_frames" in line["config"]["workload"]
    pr = line["per_rank"]
    assert pr["device"] == [0, 0] and len(pr["kernel_ms"]) == 2 and all(k > 0 for k in pr["kernel_ms"])
    per = SPP // 2 if scaling == "strong" else SPP
    assert pr["samples_per_step"] == [W * H * per] * 2
    last = WARM + STEPS - 1
    ns = SPP if scaling == "strong" else 2 * SPP
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.BidirectionalPathTracer(sc, W, H, ns, M, seed=5489)
    pt.raytrace_tiles([], last * ns, ns)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    rmse = float(np.sqrt(np.mean((frame - single) ** 2)))
    print(f"in-process reduce vs single render of step {last}: rmse {rmse:.3e}")
    assert rmse < 1e-6


@pytest.mark.timeout(600)
def test_bench_inprocess_pathtracer_row_bands(tmp_path):
    """The PathTracer through the same in-process path: row bands per context, frames and
    sampleCountBuffer reduced; the frame equals one whole-frame render bit for bit (disjoint bands)."""
    W, H, SPP, M = 96, 72, 4, 5
    line, frame = _bench_inprocess(tmp_path, 2, "0,0", ("--integrator", "pt"), W, H, SPP, 1, 1)
    assert line["n_gpus"] == 2 and line["rccl_ranks"] == 1
    # max_tolerance 0: every pixel runs whole batches of 32 (pathtracer.cpp:301-337)
    assert sum(line["per_rank"]["samples_per_step"]) == W * H * 32
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.PathTracer(sc, W, H, SPP, M, seed=5489, max_tolerance=0.0)
    pt.raytrace_tiles([], 0, SPP)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    assert np.array_equal(frame, single)


# --- >= 2 devices: these run by themselves on the first multi-GPU box (every box of this pool has
# one GPU, so they skip here with the reason) ----------------------------------------------------

two_gpus = pytest.mark.skipif(device_count() < 2, reason="needs >= 2 visible GPUs (this pool's boxes have one): "
                                                         "RCCL between distinct devices over xGMI")


@two_gpus
@pytest.mark.timeout(600)
def test_bench_inprocess_two_devices(tmp_path):
    """bench.py --gpus 2 on devices 0 and 1 (default placement): two RCCL ranks, the cross-device
    ncclReduce into device 0's frames; the frame equals the single render of the last step."""
    W, H, SPP, M, STEPS, WARM = 160, 120, 8, 5, 2, 1
    line, frame = _bench_inprocess(tmp_path, 2, None, (), W, H, SPP, STEPS, WARM)
    assert line["n_gpus"] == 2 and line["rccl_ranks"] == 2 and line["per_rank"]["device"] == [0, 1]
    last = WARM + STEPS - 1
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.BidirectionalPathTracer(sc, W, H, SPP, M, seed=5489)
    pt.raytrace_tiles([], last * SPP, SPP)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    assert float(np.sqrt(np.mean((frame - single) ** 2))) < 1e-6


@two_gpus
@pytest.mark.timeout(600)
def test_rccl_world_size_two_all_reduce(tmp_path):
    """ShardedRender under torchrun at world size 2 over RCCL ("nccl"): one rank per device, the
    all-reduce of the sample frame over xGMI; the frame equals one render of all the samples."""
    W, H, SPP, M, STEPS, WARM = 160, 120, 8, 5, 2, 1
    out = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--workload", "c2", "--width", str(W), "--height", str(H), "--spp", str(SPP),
           "--steps", str(STEPS), "--warmup", str(WARM), "--dump-frame", str(out), "--no-cpu-baseline",
           "--no-parity"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, cwd=REPO, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["per_rank"]["backend"] == "nccl" and line["per_rank"]["device"] == [0, 1]
    frame = np.load(out).astype(np.float64)
    sc = B.load_dae(os.path.join(REPO, "scenes", "CBspheres.dae"), W, H)
    pt = B.BidirectionalPathTracer(sc, W, H, SPP, M, seed=5489)
    pt.raytrace_tiles([], 0, (WARM + STEPS) * SPP)
    single = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    assert float(np.sqrt(np.mean((frame - single) ** 2))) < 1e-6
