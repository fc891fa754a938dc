"""Multi-GPU sharding logic on the CPU (gloo, world size 2): each rank renders its global sample
range (bench.rank_sample_range, strong = one fixed render split across ranks, weak = a full spp per
rank) and the frames are sum-reduced to rank 0, as bench.py does over RCCL. The "renderer" here is
the oracle's COUNTER32 mode (test infrastructure) so the test runs without a GPU; the result must
equal one render of all ranks' samples up to summation order."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import MODE_C32, REPO, golden_scene, oracle_render

W, H, S, M = 24, 18, 2, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _total(world, scaling):
    """samples per pixel of the whole 2-step job (the ctx weight 1/ns_aa)"""
    return 2 * S if scaling == "strong" else 2 * world * S


def _worker(rank, world, port, out_path, scaling):
    sys.path.insert(0, REPO)
    from bench import rank_sample_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = golden_scene("CBspheres", W, H)
    frame = torch.zeros(H, W, 3, dtype=torch.float64)
    for step in range(2):
        base, n = rank_sample_range(step, rank, world, S, scaling)
        _, eye, light, _ = oracle_render(sc, W, H, _total(world, scaling), M, MODE_C32, s0=base, count=n,
                                         threads=1)
        frame += torch.from_numpy(eye + light)
    dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_sample_range_shards_reduce_to_single_render(tmp_path, scaling):
    world = 2
    out = str(tmp_path / "reduced.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, scaling), nprocs=world, join=True)
    reduced = np.load(out)
    sc = golden_scene("CBspheres", W, H)
    tot = _total(world, scaling)
    _, eye, light, _ = oracle_render(sc, W, H, tot, M, MODE_C32, s0=0, count=tot, threads=1)
    assert np.allclose(reduced, eye + light, rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("scaling", ["strong", "weak"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("spp", [1, 7, 128, 1024])
def test_sample_ranges_partition_the_job(world, spp, scaling):
    """Across steps and ranks the ranges are disjoint and cover [0, total) exactly (uneven strong
    splits included: 128 spp over 3 or 5 ranks, 1 spp over 8 ranks leaves ranks idle)."""
    sys.path.insert(0, REPO)
    from bench import rank_sample_range
    seen = []
    for step in range(3):
        for r in range(world):
            b, n = rank_sample_range(step, r, world, spp, scaling)
            assert n >= 0
            seen += list(range(b, b + n))
            if scaling == "strong":
                assert spp // world <= n <= -(-spp // world)
    total = 3 * spp * (1 if scaling == "strong" else world)
    assert sorted(seen) == list(range(total))
