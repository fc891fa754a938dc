"""The multi-GPU path on the CPU (gloo, world sizes 2 and 4): bdpt_amd.ShardedRender — the product's split
of every pixel's sample range across the ranks (rank_sample_range: strong = one fixed render split,
weak = a full spp per rank), the sample frame copied into a float32 tensor and ONE all-reduce of it
 — exactly as bench.py drives it over RCCL, with the renderer swapped for the
product's device code compiled for the CPU (bdpt_core.h + bdpt_scene.cpp in the test-only
tests/native/libcorecpu.so, bit-exact vs oracle mode 2 per tests/test_core_cpu.py). The reduced
frame must equal one render of all the ranks' samples up to summation order. The GPU form
(libbdpt_amd.so, two ranks on one device) is tests/test_gpu_multirank.py."""
import ctypes as C
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bdpt_amd as B
from _util import REPO, golden_scene

W, H, S, M = 24, 18, 2, 5
STEPS = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spp(world):
    """samples per pixel per step: one per rank at least under strong scaling"""
    return max(S, world)


def _total(world, scaling):
    """samples per pixel of the whole job (the ctx weight 1/ns_aa)"""
    return STEPS * _spp(world) if scaling == "strong" else STEPS * world * _spp(world)


class CoreCpuRenderer:
    """The two calls ShardedRender makes on a BidirectionalPathTracer, served by the device code
    compiled for the host: frames accumulate across renders like the device frames, and
    copy_frame writes the fp32 sample frame (eye + light) to the given address."""

    def __init__(self, scene, width, height, spp, max_depth):
        self.scene, self.W, self.H, self.spp, self.M = scene, width, height, spp, max_depth
        self.eye = np.zeros((height, width, 3))
        self.light = np.zeros((height, width, 3))

    def raytrace_tiles(self, tiles, spp_begin, spp_count):
        from test_core_cpu import core_render
        assert not tiles
        e, l, _ = core_render(self.scene, self.W, self.H, self.spp, self.M, s0=spp_begin, count=spp_count)
        self.eye += e
        self.light += l

    def copy_frame(self, which, ptr):
        assert which == B.FRAME_SAMPLE
        f = np.ascontiguousarray((self.eye + self.light).astype(np.float32))
        C.memmove(ptr, f.ctypes.data, f.nbytes)


def _worker(rank, world, port, out_path, scaling):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = golden_scene("CBspheres", W, H)
    frame = torch.zeros(H * W * 3, dtype=torch.float32)
    sh = B.ShardedRender(CoreCpuRenderer(sc, W, H, _total(world, scaling), M), frame, rank, world, _spp(world),
                         scaling, dist)
    for step in range(STEPS):
        sh.step(step)
    rows = sh.gather_floats([float(rank), float(W * H * sh.samples(0))], device="cpu")
    if rank == 0:
        np.save(out_path, frame.numpy().reshape(H, W, 3))
        np.save(out_path + ".rows.npy", np.array(rows))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_sharded_render_reduces_to_single_render(tmp_path, scaling, world):
    from test_core_cpu import core_render
    out = str(tmp_path / "reduced.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, scaling), nprocs=world, join=True)
    reduced = np.load(out)
    rows = np.load(out + ".rows.npy")
    assert rows[:, 0].tolist() == [float(r) for r in range(world)]   # every rank reported its row
    per_rank = _spp(world) // world if scaling == "strong" else _spp(world)
    assert rows[:, 1].tolist() == [W * H * per_rank] * world
    sc = golden_scene("CBspheres", W, H)
    tot = _total(world, scaling)
    eye, light, _ = core_render(sc, W, H, tot, M, s0=0, count=tot)
    single = (eye + light).astype(np.float32)
    assert np.abs(reduced - single).max() < 1e-5 * max(1.0, float(np.abs(single).max()))


@pytest.mark.parametrize("scaling", ["strong", "weak"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("spp", [1, 7, 128, 1024])
def test_sample_ranges_partition_the_job(world, spp, scaling):
    """Across steps and ranks the ranges are disjoint and cover [0, total) exactly (uneven strong
    splits included: 128 spp over 3 or 5 ranks, 1 spp over 8 ranks leaves ranks idle)."""
    seen = []
    for step in range(3):
        for r in range(world):
            b, n = B.rank_sample_range(step, r, world, spp, scaling)
            assert n >= 0
            seen += list(range(b, b + n))
            if scaling == "strong":
                assert spp // world <= n <= -(-spp // world)
    total = 3 * spp * (1 if scaling == "strong" else world)
    assert sorted(seen) == list(range(total))
