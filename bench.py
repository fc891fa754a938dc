#!/usr/bin/env python3
"""Benchmark of the BDPT hot path on MI355X (BASELINE.json metric: Msamples/s at m=5, plus
per-pixel RMSE vs the CPU path at a matched seed).

Workload (N=1): BASELINE.json configs[1] — dae/sky/CBspheres.dae (mirror + glass spheres),
480x360, 128 spp, -m 5, on one MI355X. One "step" = one full-frame render of 128 samples per
pixel (22.1 M pixel-samples) through the C-ABI (libbdpt_amd.so, k_bdpt_sample).
Multi-GPU (torchrun, one rank per GPU): weak scaling — rank r renders the global sample range
[r*128, (r+1)*128) of every pixel (sample keys are global, so the image is independent of the
rank count up to fp32 summation order) and the W*H*3 fp32 frames are summed over RCCL (xGMI)
onto rank 0 inside the timed region. value = all ranks' samples / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "bidirectional-pathtracing_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "Msamples/sec (spp×pixels/s) at m=5; per-pixel RMSE vs CPU at matched seed"
SCENE, W, H, SPP, M = "CBspheres", 480, 360, 128, 5
HBM_PEAK_GBPS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BYTES_NODE, BYTES_TRI, BYTES_SPH, BYTES_HIT = 32, 36, 16, 40


def rank_sample_range(step: int, rank: int, world: int, spp: int):
    """Global sample indices [begin, begin + spp) that `rank` renders in `step`: every step and
    rank owns a fresh range, so the N-GPU image equals a single render of N*spp samples (sample
    keys are global)."""
    return (step * world + rank) * spp, spp


def algorithmic_bytes(st) -> int:
    return (BYTES_NODE * st.node_visits + BYTES_TRI * st.tri_tests + BYTES_SPH * st.sph_tests
            + BYTES_HIT * st.hits)


def cpu_baseline(scene, name: str, threads: int, budget_s: float = 12.0, rr: bool = False) -> dict:
    """The oracle's fp64 reference-semantics path (mode COUNTER64: the reference's arithmetic,
    multi-threaded like the reference's -t N) timed on this host on a bounded sample of the same
    workload (full 480x360 frame, a few spp)."""
    from _util import MODE_C64, oracle_render
    done, t_tot, spp_run = 0, 0.0, 1
    s0 = 0
    while t_tot < budget_s * 0.8 and s0 < SPP:
        t0 = time.perf_counter()
        oracle_render(scene, W, H, SPP, M, MODE_C64, seed=5489, s0=s0, count=spp_run, threads=threads, rr=rr)
        dt = time.perf_counter() - t0
        t_tot += dt
        done += W * H * spp_run
        s0 += spp_run
        rate = W * H * spp_run / dt
        spp_run = max(1, min(SPP - s0, int((budget_s - t_tot) * rate / (W * H))))
    return {"value": done / t_tot / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{name} {W}x{H}, {done // (W * H)} spp of {SPP}, m={M}, oracle fp64 "
                      f"(reference arithmetic) with {threads} threads, {t_tot:.1f} s"}


REF_DRIVER = os.path.join(REPO, "oracle", "_ref", "ref_driver")


def cpu_baseline_reference(dae: str, name: str, threads: int, budget_s: float = 15.0):
    """The reference's own `-t N` CPU path: oracle/_ref/ref_driver (built by __graft_entry__.build()
    from the reference's sources: RaytracedRenderer + BidirectionalPathTracer, reference flags)
    rendering the same scene and resolution at a few spp. Render seconds are the reference's own
    "Rendering... 100%! (Xs)" report (tiles + its per-tile frame tonemap, excluding parse/BVH
    build). None when the binary is not present."""
    import re
    import subprocess
    import tempfile
    if not os.path.exists(REF_DRIVER) or not os.path.exists(dae):
        return None
    done, t_tot, spp_run, runs = 0, 0.0, 1, 0
    with tempfile.TemporaryDirectory() as td:
        while t_tot < budget_s * 0.6 and runs < 3:
            r = subprocess.run([REF_DRIVER, "-s", str(spp_run), "-t", str(threads), "-m", str(M), "-r", str(W),
                                str(H), "-f", os.path.join(td, "ref.png"), dae], capture_output=True,
                               text=True, timeout=600, cwd=td)
            m = re.findall(r"Rendering\.\.\. 100%! \(([0-9.]+)s\)", r.stdout)
            if r.returncode != 0 or not m:
                return None
            dt = float(m[-1])
            t_tot += dt
            done += W * H * spp_run
            runs += 1
            rate = W * H * spp_run / dt
            spp_run = max(1, int((budget_s - t_tot) * rate / (W * H)))
    return {"value": done / t_tot / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "reference",
            "sample": f"{name} {W}x{H}, {done // (W * H)} spp, m={M}: the reference's RaytracedRenderer + "
                      f"BidirectionalPathTracer (oracle/_ref/ref_driver, -O3 -mavx2) at -t {threads}, "
                      f"{t_tot:.1f} s of rendering"}


def parity_check(scene, seed: int, rr: bool = False) -> dict:
    """Per-pixel RMSE of the GPU sample buffer vs the oracle's COUNTER32 CPU path, same seed,
    same workload at 2 spp (the CPU side of the metric)."""
    import numpy as np
    import bdpt_amd as B
    from _util import MODE_C32, oracle_render
    S = 2
    pt = B.BidirectionalPathTracer(scene, W, H, S, M, seed=seed, russian_roulette=rr)
    pt.raytrace_tiles()
    g = pt.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    pt.close()
    ref = oracle_render(scene, W, H, S, M, MODE_C32, seed=seed,
                        threads=min(16, os.cpu_count() or 1), rr=rr)[0]
    return {"rmse": float(np.sqrt(np.mean((g - ref) ** 2))), "spp": S, "tolerance": 1e-4,
            "cpu": "oracle COUNTER32 (fp32 device semantics)"}


def main() -> int:
    global W, H, SPP, M
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--scene", default=SCENE,
                    help="golden scene name (tests/golden/scenes) or a .dae path, e.g. the north-star "
                         "stand-in scenes/CBlucy_standin.dae")
    ap.add_argument("--width", type=int, default=W)
    ap.add_argument("--height", type=int, default=H)
    ap.add_argument("--spp", type=int, default=SPP)
    ap.add_argument("--max-depth", type=int, default=M)
    ap.add_argument("--pipeline", type=int, default=0, help="0 auto, 1 megakernel, 2 wavefront")
    ap.add_argument("--envmap", default=None,
                    help="environment light (DESIGN.md §9): an .exr path, or synth:WxH for the "
                         "synthetic sky of tools/envmap.py (the reference's exr/*.exr are LFS pointers)")
    ap.add_argument("--rr", action="store_true", help="Russian roulette on both subpaths")
    ap.add_argument("--integrator", choices=["bdpt", "pt"], default="bdpt",
                    help="bdpt (the reference's BidirectionalPathTracer, the headline) or pt (its "
                         "unidirectional PathTracer, DESIGN.md §10; adaptive sampling off: every "
                         "pixel takes all spp; ranks split the frame into row bands)")
    args = ap.parse_args()
    W, H, SPP, M = args.width, args.height, args.spp, args.max_depth

    import numpy as np
    import torch
    import bdpt_amd as B
    from _util import golden_scene

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    scene = (B.load_dae(args.scene, W, H) if args.scene.endswith(".dae")
             else golden_scene(args.scene, W, H))
    env_desc = None
    if args.envmap:
        if args.envmap.startswith("synth:"):
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from envmap import synth_envmap
            ew, eh = (int(v) for v in args.envmap[6:].split("x"))
            scene.set_envmap(synth_envmap(ew, eh))
            env_desc = f"synthetic sky {ew}x{eh} (tools/envmap.py)"
        else:
            scene.set_envmap(B.load_exr(args.envmap))
            env_desc = os.path.basename(args.envmap)
    seed = 5489
    stream = torch.cuda.Stream(dev)          # a real stream: handle 0 would mean "ctx's own"
    torch.cuda.set_stream(stream)
    # weight 1/(world*SPP): the N-GPU image is an N*128-spp render
    use_pt = args.integrator == "pt"
    band = [(0, H * rank // world, W, H * (rank + 1) // world - H * rank // world)]
    if use_pt:   # whole pixels: each rank renders its row band with all SPP samples
        pt = B.PathTracer(scene, W, H, SPP, M, seed=seed, device=dev.index, max_tolerance=0.0)
    else:
        pt = B.BidirectionalPathTracer(scene, W, H, SPP * world, M, seed=seed, device=dev.index,
                                       pipeline=args.pipeline, russian_roulette=args.rr)
    pt.set_stream(stream.cuda_stream)
    frame = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)

    def render(k: int):
        if use_pt:
            pt.raytrace_tiles(band, 0, SPP)
        else:
            base, n = rank_sample_range(k, rank, world, SPP)   # fresh global sample range every step
            pt.raytrace_tiles([], base, n)

    def step(k: int):
        render(k)
        pt.copy_frame(B.FRAME_SAMPLE, frame.data_ptr())
        if dist is not None:
            dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        render(args.warmup + k)                     # k_bdpt_sample (k_pt): the dominant kernel
        ev[k][1].record(stream)
        pt.copy_frame(B.FRAME_SAMPLE, frame.data_ptr())
        if dist is not None:
            dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rank_samples = int(pt.read_sample_counts().astype(np.int64)[band[0][1]:band[0][1] + band[0][3]].sum()) \
        if use_pt else W * H * SPP
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pt.close()

    # algorithmic bytes of one launch: in-kernel counters on a separate, untimed launch of the
    # same workload (counting perturbs timing), SURVEY.md §8d.
    if use_pt:
        ps = B.PathTracer(scene, W, H, SPP, M, seed=seed, device=dev.index, max_tolerance=0.0,
                          collect_stats=True)
        ps.raytrace_tiles(band, 0, SPP)
    else:
        ps = B.BidirectionalPathTracer(scene, W, H, SPP * world, M, seed=seed, device=dev.index,
                                       collect_stats=True, pipeline=args.pipeline, russian_roulette=args.rr)
        ps.raytrace_tiles([], rank * SPP, SPP)
    st = ps.stats()
    ps.close()
    bytes_launch = algorithmic_bytes(st)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9

    if dist is not None and use_pt:
        t = torch.tensor([rank_samples], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        samples_total = float(t.item()) * args.steps
    else:
        samples_total = (rank_samples if use_pt else W * H * SPP * world) * args.steps
    value = samples_total / elapsed / 1e6
    traffic = None
    default_workload = ((args.scene, W, H, SPP, M) == (SCENE, 480, 360, 128, 5) and not args.envmap
                        and not args.rr and not use_pt)
    tpath = os.path.join(REPO, "profiles", "traffic_r01.json")   # PMC pass of this workload
    if default_workload and os.path.exists(tpath):
        with open(tpath) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return 0
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: fixed-seed renders (Philox counter RNG) of the reference's scene "
                f"{os.path.basename(args.scene)} as the reference loads it",
        "config": {"workload": f"{os.path.basename(args.scene)} {W}x{H} -s {SPP} -m {M}"
                               f"{' + env ' + env_desc if env_desc else ''}{' RR on' if args.rr else ''}"
                               f"{' unidirectional PathTracer' if use_pt else ''}"
                               f"{' (BASELINE configs[1])' if default_workload else ''} "
                               + ("for the whole frame, row bands per GPU + RCCL sum-reduce" if use_pt else
                                  "per GPU, sample-range shards + RCCL sum-reduce"),
                   "pipeline": ["auto (megakernel)", "megakernel", "wavefront"][args.pipeline],
                   "scene": args.scene, "width": W, "height": H, "spp_per_gpu": SPP,
                   "max_depth": M, "envmap": env_desc, "russian_roulette": args.rr,
                   "parallelism": f"samples x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                     "traffic": traffic, "kernel": "k_pt" if use_pt else "k_bdpt_sample",
                     "kernel_ms": round(kern_ms, 3),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "counts_per_launch": {"node_aabbs": st.node_visits, "tri_tests": st.tri_tests,
                                           "sph_tests": st.sph_tests, "hits": st.hits,
                                           "closest_rays": st.closest_rays,
                                           "shadow_rays": st.shadow_rays}},
    }
    if use_pt:
        out["config"]["integrator"] = "PathTracer (pathtracer.cpp:47-340)"
        out["config"]["parallelism"] = f"row bands x{world}"
        out["scaling"] = "strong"
    if world == 1 and not args.no_parity and not use_pt:
        out["parity"] = parity_check(scene, seed, rr=args.rr)
    if world == 1 and not args.no_cpu_baseline and not use_pt:
        thr = min(16, os.cpu_count() or 1)
        dae = args.scene if args.scene.endswith(".dae") else os.path.join(REPO, "scenes", args.scene + ".dae")
        port = cpu_baseline(scene, args.scene, threads=thr, rr=args.rr)
        # the reference cannot run the environment light / roulette under BDPT: port only
        ref = (None if (args.envmap or args.rr)
               else cpu_baseline_reference(dae, os.path.basename(args.scene), threads=thr))
        out["cpu_baseline"] = ref if ref is not None else port
        if ref is not None:   # the oracle port's fp64 path, same host, for comparison
            out["cpu_baseline"]["port"] = {"value": port["value"], "cores": port["cores"], "sample": port["sample"]}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
