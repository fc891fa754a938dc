"""Multi-GPU sharding logic on the CPU (gloo, world size 2): each rank renders its global sample
range (bench.rank_sample_range) and the frames are sum-reduced to rank 0, as bench.py does over
RCCL. The "renderer" here is the oracle's COUNTER32 mode (test infrastructure) so the test runs
without a GPU; the result must equal one render of all ranks' samples up to summation order."""
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


def _worker(rank, world, port, out_path):
    sys.path.insert(0, REPO)
    from bench import rank_sample_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = golden_scene("CBspheres", W, H)
    frame = torch.zeros(H, W, 3, dtype=torch.float64)
    for step in range(2):
        base, n = rank_sample_range(step, rank, world, S)
        _, eye, light, _ = oracle_render(sc, W, H, 2 * world * S, M, MODE_C32, s0=base, count=n, threads=1)
        frame += torch.from_numpy(eye + light)
    dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.destroy_process_group()


def test_sample_range_shards_reduce_to_single_render(tmp_path):
    world = 2
    out = str(tmp_path / "reduced.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    reduced = np.load(out)
    sc = golden_scene("CBspheres", W, H)
    _, eye, light, _ = oracle_render(sc, W, H, 2 * world * S, M, MODE_C32, s0=0, count=2 * world * S, threads=1)
    assert np.allclose(reduced, eye + light, rtol=1e-12, atol=1e-15)
