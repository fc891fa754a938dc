#!/usr/bin/env python3
"""Benchmark of the BDPT hot path on MI355X (BASELINE.json metric: Msamples/s at m=5, plus
per-pixel RMSE vs the CPU path at a matched seed).

Default workload (N=1, and the fixed render split across ranks for N>1): the north-star target,
CBlucy 1920x1080 -s 128 -m 5. dae/sky/CBlucy.dae is absent from the reference checkout
(.MISSING_LARGE_BLOBS), so the scene is its stand-in scenes/CBlucy_standin.dae (SURVEY.md §8d:
CBbunny's box, light and camera, the bunny subdivided 1->4 to 114,304 triangles; written by
tools/gen_standin.py), loaded through the product loader (bdpt_dae_load, the reference CLI's
ColladaParser + Application::load path). One "step" = one full 1920x1080 frame of 128 samples per
pixel (265.4 M pixel-samples) through the C-ABI (libbdpt_amd.so, k_bdpt_sample).
Other BASELINE configs: --workload c2 | c3 | c4 | c5 (c5's ennis.exr is an LFS pointer in the
reference: a synthetic sky of the same role stands in, tools/envmap.py).

Multi-GPU, strong scaling by default: the step's fixed render (the workload's spp of every pixel)
is split by sample range — rank r renders global sample indices [s*spp + r*spp/N,
s*spp + (r+1)*spp/N) of step s (sample keys are global, so the image does not depend on N up to
fp32 summation order) — and the W*H*3 fp32 frames are summed inside the timed region (splats land
anywhere, so a tile gather would not do). Two launch forms (plan_launch):
* `python bench.py --gpus N` (no launcher): N contexts in this process on devices 0..N-1 (or
  --devices), rendered concurrently, summed by the C-ABI's RCCL reduce (bdpt_reduce_frames, the
  CLI's -g N) into context 0's frames; `rccl_ranks` = the communicator's ranks (distinct devices);
* under torchrun (WORLD_SIZE set, must equal --gpus): one rank per GPU, bdpt_amd.ShardedRender's
  all-reduce of the sample frame; --dist-backend picks RCCL ("nccl", the default) or gloo (the
  same all_reduce of the device tensor; two ranks can then share one GPU, --devices 0,0, as
  tests/test_gpu_multirank.py runs it).
--scaling weak gives every rank the full spp instead. value = pixel-samples of all ranks /
max-over-ranks wall time. A named workload refuses to run with a product knob set in the
environment (PRODUCT_KNOBS); every BDPT_* variable is recorded in config.env.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "bidirectional-pathtracing_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "Msamples/sec (spp×pixels/s) at m=5; per-pixel RMSE vs CPU at matched seed"
STANDIN = "scenes/CBlucy_standin.dae"
# name: (scene, W, H, spp, max_depth, envmap, russian roulette, what it is)
WORKLOADS = {
    "ns": (STANDIN, 1920, 1080, 128, 5, None, False,
           "north star: CBlucy (stand-in) 1920x1080 -s 128 -m 5"),
    "c2": ("scenes/CBspheres.dae", 480, 360, 128, 5, None, False, "BASELINE configs[1]: CBspheres 480x360 -s 128 -m 5"),
    "c3": (STANDIN, 800, 600, 128, 5, None, False, "BASELINE configs[2]: CBlucy (stand-in) 800x600 -s 128 -m 5"),
    "c4": ("scenes/CBgems.dae", 1920, 1080, 256, 7, None, False, "BASELINE configs[3]: CBgems 1920x1080 -s 256 -m 7"),
    "c5": (STANDIN, 1920, 1080, 1024, 8, "synth:1024x512", True,
           "BASELINE configs[4]: CBlucy (stand-in) + env (synthetic sky for ennis.exr) 1920x1080 -s 1024 -m 8 RR"),
}
HBM_PEAK_GBPS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BYTES_NODE, BYTES_TRI, BYTES_SPH, BYTES_HIT = 32, 36, 16, 40
# environment-light table reads (bdpt_stats v6): a sampled direction reads 2 guide
# cells + 2 CDF entries per axis (marginal, row), the texel pdf and 4 texels; a radiance lookup 4
# texels; a pdf lookup one texel pdf
BYTES_ENV_SAMPLE, BYTES_ENV_LOOKUP, BYTES_ENV_PDF = 76, 48, 4


from bdpt_amd import rank_sample_range  # noqa: E402  (the multi-GPU split lives in the product module)


def algorithmic_bytes(st) -> int:
    return (BYTES_NODE * st.node_visits + BYTES_TRI * st.tri_tests + BYTES_SPH * st.sph_tests
            + BYTES_HIT * st.hits + env_bytes(st))


def env_bytes(st) -> int:
    return (BYTES_ENV_SAMPLE * st.env_samples + BYTES_ENV_LOOKUP * st.env_lookups
            + BYTES_ENV_PDF * st.env_pdf_lookups)


# What the kernel's loads actually request (bdpt_core.h): a 4-wide node is 7 float4 (112 B) for 4
# children = 28 B per child AABB (LDS modes 0 / 2), a 2-wide node 4 float4 for 2 = 32 B (modes 1 /
# 3); a primitive test loads its whole 48-B record (3 float4, software-pipelined); a closest hit
# its 48-B shading record.
FETCH_NODE_CHILD = {0: 28, 1: 32, 2: 28, 3: 32}
FETCH_PRIM, FETCH_HIT = 48, 48


def fetched_bytes(st) -> int:
    return (FETCH_NODE_CHILD.get(st.lds_mode, 32) * st.node_visits + FETCH_PRIM * (st.tri_tests + st.sph_tests)
            + FETCH_HIT * st.hits + env_bytes(st))


def global_memory_bytes(st) -> int:
    """The algorithmic bytes minus what the kernel read from the CU's LDS copy of the scene (the
    BFS treelet in LDS mode 2; the whole scene in modes 1 / 3): the part that has to come through
    the L2 / HBM path."""
    lm = st.lds_mode
    nodes = st.node_visits - st.lds_node_visits
    prims = 0 if lm in (1, 3) else BYTES_TRI * st.tri_tests + BYTES_SPH * st.sph_tests
    hits = 0 if lm == 3 else BYTES_HIT * st.hits
    return BYTES_NODE * nodes + prims + hits + env_bytes(st)


def ensure_standin(path: str) -> None:
    """scenes/CBlucy_standin.dae is generated (deterministic, 4 MB) rather than committed."""
    if os.path.basename(path) == os.path.basename(STANDIN) and not os.path.exists(path):
        subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_standin.py"),
                        os.path.join(REPO, "scenes", "CBbunny.dae"), path], check=True)


def cpu_baseline(scene, name: str, W: int, H: int, SPP: int, M: int, threads: int, budget_s: float = 12.0,
                 rr: bool = False) -> dict:
    """The oracle's fp64 reference-semantics path (mode COUNTER64: the reference's arithmetic,
    multi-threaded like the reference's -t N) timed on this host on a bounded sample of the same
    workload (full frame, a few spp)."""
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


def host_cores() -> dict:
    """The host CPUs this process may run on: nproc (os.cpu_count(), the whole node), the
    affinity mask, and the cgroup CPU quota where one is set (a GPU box's share of its node).
    `usable` = the smallest of them: the thread count the CPU baselines run at."""
    n = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return {"nproc": n, "affinity": aff, "cgroup_quota": quota, "usable": min(x for x in (n, aff, quota) if x)}


def progress(msg: str) -> None:
    """a progress line on stderr (the JSON line alone goes to stdout)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def ref_driver_render(dae: str, W: int, H: int, spp: int, M: int, threads: int, timeout: float = 900):
    """Seconds of the reference's own "Rendering... 100%! (Xs)" report (tiles + its per-tile
    whole-frame tonemap, raytraced_renderer.cpp:595-620,654-682; its timer starts after
    build_accel), or None."""
    import re
    import tempfile
    progress(f"reference CPU path: {os.path.basename(dae)} {W}x{H} s{spp} m{M} -t {threads}")
    with tempfile.TemporaryDirectory() as td:
        try:
            r = subprocess.run([REF_DRIVER, "-s", str(spp), "-t", str(threads), "-m", str(M), "-r", str(W), str(H),
                                "-f", os.path.join(td, "ref.png"), os.path.abspath(dae)],
                               capture_output=True, text=True, timeout=timeout, cwd=td)
        except subprocess.TimeoutExpired:
            progress(f"reference CPU path at -t {threads}: over {timeout:.0f} s, not counted")
            return None
    m = re.findall(r"Rendering\.\.\. 100%! \(([0-9.]+)s\)", r.stdout)
    return float(m[-1]) if r.returncode == 0 and m else None


def cpu_baseline_reference(dae: str, name: str, W: int, H: int, M: int, threads: int, cores: dict,
                           min_spp: int = 4):
    """The reference's own `-t N` CPU path: oracle/_ref/ref_driver (built by __graft_entry__.build()
    from the reference's sources: RaytracedRenderer + BidirectionalPathTracer, reference flags)
    rendering the same scene and resolution. The headline figure is a render of `min_spp` spp,
    where the reference's per-tile whole-frame tonemap (raytraced_renderer.cpp:619, image.h:194-209:
    2,040 tiles x 2.07 Mpx at 1080p, independent of spp) weighs a quarter of what it does at 1 spp;
    the 1-spp figure is reported beside it. None when the binary is not present."""
    if not os.path.exists(REF_DRIVER) or not os.path.exists(dae):
        return None
    t1 = ref_driver_render(dae, W, H, 1, M, threads)
    if t1 is None:
        return None
    tn = ref_driver_render(dae, W, H, min_spp, M, threads)
    if tn is None:
        return None
    # also at -t nproc (os.cpu_count(), the whole node) when the box's CPU quota is smaller: the
    # faster of the two is the baseline, both are reported
    runs, slow = {threads: tn}, {}
    if cores["nproc"] > threads:
        cap = max(60.0, 2.0 * tn)
        tp = ref_driver_render(dae, W, H, min_spp, M, cores["nproc"], timeout=cap)
        if tp is not None:
            runs[cores["nproc"]] = tp
        else:
            slow[str(cores["nproc"])] = {"seconds": None, "note": f"stopped after {cap:.0f} s wall (over 2x -t {threads})"}
    best = min(runs, key=runs.get)
    tn = runs[best]
    return {"value": W * H * min_spp / tn / 1e6, "unit": "Msamples/s", "cores": best, "kind": "reference",
            "host": cores,
            "threads_tried": {**{str(t): {"seconds": round(s_, 2), "value": round(W * H * min_spp / s_ / 1e6, 5)}
                                 for t, s_ in runs.items()}, **slow},
            "sample": f"{name} {W}x{H}, {min_spp} spp, m={M}: the reference's RaytracedRenderer + "
                      f"BidirectionalPathTracer (oracle/_ref/ref_driver, -O3 -mavx2), the faster of -t "
                      f"{' / -t '.join([str(t) for t in runs] + list(slow))} (node nproc {cores['nproc']}, usable "
                      f"{cores['usable']}): -t {best}, {tn:.1f} s of rendering",
            "spp1": {"value": round(W * H / t1 / 1e6, 5), "seconds": round(t1, 2),
                     "note": "1 spp: the per-tile whole-frame tonemap is a larger share of this time"}}


def parity_check(scene, W: int, H: int, M: int, seed: int, rr: bool = False, threads: int = 16) -> dict:
    """The per-pixel quality half of the metric, on the workload's full frame at the same seed,
    samples 0 and 1 rendered as two 1-spp frames:
    * rmse: the GPU's 2-spp sample buffer vs oracle COUNTER32 (mode 2: the device's fp32 semantics,
      tolerance 1e-4);
    * vs_fp64: the GPU vs oracle COUNTER64 (mode 1: the reference's fp64 arithmetic, same random
      numbers): per-pixel RMSE, the Monte Carlo noise of the same image, their ratio, and the
      shares of samples that took another path (fp32 flips) / agree to 1e-5, against the fp32
      tolerance stated in DESIGN.md §3 (tests/_parity.py)."""
    import numpy as np
    import bdpt_amd as B
    from _parity import TOL_AGREE, TOL_DIVERGED, TOL_NOISE_RATIO, fp64_agreement
    from _util import MODE_C32, MODE_C64, oracle_render
    S = 2
    pt = B.BidirectionalPathTracer(scene, W, H, 1, M, seed=seed, russian_roulette=rr)
    ge, gs = [], []
    for k in range(S):
        pt.clear()
        pt.raytrace_tiles([], k, 1)
        ge.append(pt.read_frame(B.FRAME_EYE).astype(np.float64))
        gs.append(pt.read_frame(B.FRAME_SAMPLE).astype(np.float64))
    pt.close()
    o32 = [oracle_render(scene, W, H, 1, M, MODE_C32, seed=seed, s0=k, count=1, threads=threads, rr=rr)
           for k in range(S)]
    o64 = [oracle_render(scene, W, H, 1, M, MODE_C64, seed=seed, s0=k, count=1, threads=threads, rr=rr)
           for k in range(S)]
    g = np.mean(gs, axis=0)
    ref = np.mean([o[0] for o in o32], axis=0)
    agr = fp64_agreement(ge, gs, [o[1] for o in o64], [o[0] for o in o64])
    agr = {k: (round(v, 8) if isinstance(v, float) else v) for k, v in agr.items()}
    agr["tolerance"] = {"diverged_frac_max": TOL_DIVERGED, "rmse_over_noise_max": TOL_NOISE_RATIO,
                        "agree_1e-5_frac_min": TOL_AGREE}
    agr["cpu"] = "oracle COUNTER64 (the reference's fp64 arithmetic, same counter RNG)"
    return {"rmse": float(np.sqrt(np.mean((g - ref) ** 2))), "spp": S, "frame": f"{W}x{H}",
            "tolerance": 1e-4, "cpu": "oracle COUNTER32 (fp32 device semantics)",
            "rmse_vs_fp64": agr["rmse_vs_fp64"], "diverged_frac_vs_fp64": agr["diverged_frac"],
            "vs_fp64": agr}


def load_traffic(workload: str, kernel_ms: float):
    """HBM-side bytes of one launch of this workload from the committed PMC passes
    (profiles/traffic_<workload>.json: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc runs of
    tools/prof_render.py, reduced by tools/pmc_traffic.py). Counters cannot be collected inside the
    timed process (rocprofv3 wraps the whole program), so the file records which run it came from."""
    path = os.path.join(REPO, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        rec = json.load(f)
    b = rec.get("hbm_bytes_per_launch")
    if not b:
        return None, None
    gbps = b / (kernel_ms * 1e-3) / 1e9
    pms = rec.get("kernel_ms")
    info = {"source": os.path.relpath(path, REPO), "read_bytes": rec.get("hbm_read_bytes"),
            "write_bytes": rec.get("hbm_write_bytes"),
            "gbps_at_this_kernel_ms": round(gbps, 2), "frac_at_this_kernel_ms": round(gbps / HBM_PEAK_GBPS, 5),
            "pmc_kernel_ms": pms}
    if pms:   # the bytes over the duration of the dispatch they were counted on (same rocprofv3 run)
        info["pmc_gbps"] = round(b / (pms * 1e-3) / 1e9, 2)
        info["pmc_frac"] = round(b / (pms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5)
    return b, info


# Run-time switches of the product library that change its tree or its kernel (bdpt_hip.hip
# bdpt_create, bdpt_scene.cpp build_host_scene): a named (headline) workload refuses to run with any
# of them set, so the line always states the product configuration; every BDPT_* variable that is
# set goes into config.env.
PRODUCT_KNOBS = ("BDPT_LDS_MODE", "BDPT_NTOP_MAX", "BDPT_BLOCK_MAJOR", "BDPT_XCD_GROUPS",
                 "BDPT_BVH", "BDPT_SAH_LEAF", "BDPT_SAH_CT", "BDPT_SAH_BINS", "BDPT_SBVH",
                 "BDPT_SBVH_BUDGET")


def knob_env(environ) -> dict:
    """every BDPT_* variable of the environment (recorded in config.env)"""
    return {k: environ[k] for k in sorted(environ) if k.startswith("BDPT_")}


def check_knobs(environ, named: bool) -> None:
    """A named workload is the product configuration: refuse if a product knob is set."""
    bad = [k for k in PRODUCT_KNOBS if k in environ]
    if named and bad:
        raise SystemExit(f"bench.py: {', '.join(f'{k}={environ[k]}' for k in bad)} set: these change the "
                         f"product's tree / kernel, so a named workload (the headline) refuses to run; unset "
                         f"them, or give an explicit --scene / --width / ... configuration to measure a variant")


def plan_launch(gpus: int, world_size_env, devices_arg, ndev: int) -> dict:
    """How `bench.py --gpus N` runs, decided before anything touches a GPU:
    * "torchrun": WORLD_SIZE is set (one process per GPU under torch.distributed.run); it must
      equal --gpus;
    * "single": no WORLD_SIZE and --gpus 1: one context;
    * "inprocess": no WORLD_SIZE and --gpus N > 1: N contexts in this process on devices
      0..N-1 (or --devices), their sample ranges rendered concurrently and the frames summed by
      the C-ABI's RCCL reduce (bdpt_reduce_frames) inside the timed region.
    Raises SystemExit (non-zero) on a mismatch: too few visible devices, a --devices list of the
    wrong length, or WORLD_SIZE != --gpus."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} < 1")
    devmap = [int(x) for x in devices_arg.split(",")] if devices_arg else None
    if devmap is not None and any(d < 0 for d in devmap):
        raise SystemExit(f"bench.py: negative device in --devices {devices_arg}")
    if world_size_env is not None:
        world = int(world_size_env)
        if world != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} (torchrun) but --gpus {gpus}: they must agree")
        return {"mode": "torchrun", "world": world, "devmap": devmap}
    if devmap is not None and len(devmap) != gpus:
        raise SystemExit(f"bench.py: --devices lists {len(devmap)} devices for --gpus {gpus}")
    devices = devmap or list(range(gpus))
    if max(devices) >= ndev:
        raise SystemExit(f"bench.py: --gpus {gpus} needs device {max(devices)}, but only {ndev} visible")
    return {"mode": "single" if gpus == 1 else "inprocess", "world": gpus, "devices": devices}


class Timed:
    """what a timed region measured: wall seconds (max over ranks), rank 0's mean launch ms, and
    per-rank rows (elapsed s, kernel ms, pixel-samples per step, device)"""

    def __init__(self, elapsed, kern_ms, rows, world):
        self.elapsed, self.kern_ms, self.rows, self.world = elapsed, kern_ms, rows, world

    @property
    def samples_per_step(self) -> float:
        return sum(r[2] for r in self.rows)


def run_torchrun_or_single(args, B, scene, W, H, SPP, M, rr, seed, plan, use_pt, scaling):
    """One context per process: the plain N=1 path (no WORLD_SIZE) or one rank under torchrun
    (bdpt_amd.ShardedRender: this rank's sample range, bdpt_copy_frame, one all-reduce)."""
    import numpy as np
    import torch
    world = plan["world"]
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if plan["mode"] == "torchrun":
        devmap = plan["devmap"]
        gpu = devmap[rank % len(devmap)] if devmap else local
    else:
        gpu = plan["devices"][0]
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    # under torchrun (WORLD_SIZE set) the process group is made at every world size, 1 included, so
    # the RCCL all-reduce of the frame runs on one GPU exactly as it does on eight
    if plan["mode"] == "torchrun":
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    stream = torch.cuda.Stream(dev)          # a real stream: handle 0 would mean "ctx's own"
    torch.cuda.set_stream(stream)
    band = [(0, H * rank // world, W, H * (rank + 1) // world - H * rank // world)]
    t_create = time.perf_counter()
    if use_pt:   # whole pixels: each rank renders its row band with all SPP samples
        pt = B.PathTracer(scene, W, H, SPP, M, seed=seed, device=dev.index, max_tolerance=0.0)
    else:
        # sample weight 1/ns_aa: strong = the workload's spp, weak = the N-GPU image of N*spp
        pt = B.BidirectionalPathTracer(scene, W, H, SPP if scaling == "strong" else SPP * world, M, seed=seed,
                                       device=dev.index, pipeline=args.pipeline, russian_roulette=rr)
    pt.set_stream(stream.cuda_stream)
    t_create = time.perf_counter() - t_create
    frame = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
    # the multi-GPU path (bdpt_amd.ShardedRender): this rank's sample range (or, for the
    # PathTracer, its row band), the sample frame copied into `frame`, one all-reduce of `frame`
    sh = B.ShardedRender(pt, frame, rank, world, SPP, scaling, dist)

    def render(k: int):
        if use_pt:
            pt.raytrace_tiles(band, 0, SPP)
        else:
            sh.render(k)

    for k in range(args.warmup):
        render(k)
        sh.reduce()
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
        sh.reduce()                                 # bdpt_copy_frame + all_reduce over the ranks
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rank_samples = int(pt.read_sample_counts().astype(np.int64)[band[0][1]:band[0][1] + band[0][3]].sum()) \
        if use_pt else W * H * sh.samples(0)
    rows = sh.gather_floats([elapsed, kern_ms, float(rank_samples), float(gpu)])
    if args.dump_frame and rank == 0:
        np.save(args.dump_frame, frame.cpu().numpy().reshape(H, W, 3))
    pt.close()
    t = Timed(max(r[0] for r in rows), kern_ms, rows, world)
    t.rank, t.dist, t.dev, t.t_create = rank, dist, dev, t_create
    t.rccl_ranks = None
    t.label = ("" if dist is None else " + RCCL all-reduce" if args.dist_backend == "nccl" else " + gloo all-reduce")
    t.backend = args.dist_backend if dist is not None else None
    return t


def run_inprocess(args, B, scene, W, H, SPP, M, rr, seed, plan, use_pt, scaling):
    """N contexts in this one process (no launcher), one per device of plan["devices"] (the
    CLI's -g N form, pathtracer_cli.cpp): per step every context clears its frames and renders its
    sample range (or, for the PathTracer, its row band) on a stream of its device — the launches
    are asynchronous, so the devices render concurrently — then ONE bdpt_reduce_frames (RCCL
    ncclReduce over the distinct devices; contexts sharing a device are summed on it first) puts the
    whole frame into context 0's. The clear keeps every step's reduced frame equal to one render
    of that step's samples. Reference: raytraced_renderer.cpp:323-327 (the N worker threads this
    replaces), bidirection.cpp:457-466 (why a whole-frame sum)."""
    import numpy as np
    import torch
    devices = plan["devices"]
    N = len(devices)
    torch.cuda.set_device(devices[0])
    streams = [torch.cuda.Stream(torch.device("cuda", d)) for d in devices]
    t_create = time.perf_counter()
    pts = []
    for r, d in enumerate(devices):
        if use_pt:
            p = B.PathTracer(scene, W, H, SPP, M, seed=seed, device=d, max_tolerance=0.0)
        else:
            p = B.BidirectionalPathTracer(scene, W, H, SPP if scaling == "strong" else SPP * N, M, seed=seed,
                                          device=d, pipeline=args.pipeline, russian_roulette=rr)
        p.set_stream(streams[r].cuda_stream)
        pts.append(p)
    red = B.FrameReducer(pts)
    t_create = time.perf_counter() - t_create
    bands = [(0, H * r // N, W, H * (r + 1) // N - H * r // N) for r in range(N)]

    def sync_all():
        for d in devices:
            torch.cuda.synchronize(d)

    evs = []

    def step(k: int, timed: bool):
        for r, p in enumerate(pts):
            p.clear()
            if timed:
                with torch.cuda.device(devices[r]):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(streams[r])
            if use_pt:
                p.raytrace_tiles([bands[r]], 0, SPP)
            else:
                base, n = B.rank_sample_range(k, r, N, SPP, scaling)
                if n > 0:
                    p.raytrace_tiles([], base, n)
            if timed:
                with torch.cuda.device(devices[r]):
                    e1.record(streams[r])
                evs.append((r, e0, e1))
        red.reduce(0)                               # RCCL: every device's frames into context 0's

    for k in range(args.warmup):
        step(k, False)
    sync_all()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, True)
    sync_all()
    elapsed = time.perf_counter() - t0
    kms = [float(np.mean([a.elapsed_time(b) for r_, a, b in evs if r_ == r])) for r in range(N)]
    if use_pt:
        samples = [int(p.read_sample_counts().astype(np.int64)[b[1]:b[1] + b[3]].sum()) for p, b in zip(pts, bands)]
        # context 0 holds the reduced counts: its own band is its own samples (the others' bands
        # were zero in it before the reduce and are summed in after)
    else:
        samples = [W * H * B.rank_sample_range(0, r, N, SPP, scaling)[1] for r in range(N)]
    if args.dump_frame:
        np.save(args.dump_frame, pts[0].read_frame(B.FRAME_SAMPLE))
    rccl_ranks = red.ranks
    red.close()
    for p in pts:
        p.close()
    rows = [[elapsed, kms[r], float(samples[r]), float(devices[r])] for r in range(N)]
    t = Timed(elapsed, kms[0], rows, N)
    t.rank, t.dist, t.dev, t.t_create = 0, None, torch.device("cuda", devices[0]), t_create
    t.rccl_ranks = rccl_ranks
    t.label = f" + RCCL reduce (bdpt_reduce_frames: {N} contexts in one process, {rccl_ranks} RCCL rank(s))"
    t.backend = "rccl (bdpt_reduce_frames, one process)"
    return t


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs: under torchrun it must equal WORLD_SIZE; without a launcher, N > 1 runs N "
                         "contexts in this process (devices 0..N-1 or --devices) with the RCCL frame reduce")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="ns",
                    help="ns = the north-star target (default); c2..c5 = BASELINE.json configs[1..4]")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: the workload's fixed render split across ranks (default); "
                         "weak: every rank renders the full spp")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend under torchrun: nccl (= RCCL on ROCm, the default) or "
                         "gloo (same all_reduce of the device frame; lets two ranks share one GPU in tests)")
    ap.add_argument("--devices", default=None,
                    help="device of each rank / context, comma-separated (default: LOCAL_RANK under "
                         "torchrun, 0..N-1 in one process), e.g. 0,0")
    ap.add_argument("--dump-frame", default=None,
                    help="rank 0 saves the last step's reduced sample frame (.npy, H x W x 3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--scene", default=None, help="override: a .dae path")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--max-depth", type=int, default=None)
    ap.add_argument("--pipeline", type=int, choices=[0, 1], default=0, help="0 auto = 1 megakernel")
    ap.add_argument("--envmap", default=None,
                    help="environment light (DESIGN.md §9): an .exr path, or synth:WxH for the "
                         "synthetic sky of tools/envmap.py (the reference's exr/*.exr are LFS pointers)")
    ap.add_argument("--rr", action="store_true", help="Russian roulette on both subpaths")
    ap.add_argument("--integrator", choices=["bdpt", "pt"], default="bdpt",
                    help="bdpt (the reference's BidirectionalPathTracer, the headline) or pt (its "
                         "unidirectional PathTracer, DESIGN.md §10; adaptive sampling off: every "
                         "pixel takes all spp; ranks split the frame into row bands)")
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    scene_path = args.scene or os.path.join(REPO, wl[0])
    W = args.width or wl[1]
    H = args.height or wl[2]
    SPP = args.spp or wl[3]
    M = args.max_depth if args.max_depth is not None else wl[4]
    envmap = args.envmap if args.envmap is not None else wl[5]
    rr = args.rr or wl[6]
    named = (args.scene is None and args.width is None and args.height is None and args.spp is None
             and args.max_depth is None and args.envmap is None and not args.rr)
    check_knobs(os.environ, named)
    knobs = knob_env(os.environ)

    import numpy as np
    import torch
    import bdpt_amd as B

    # decided before any GPU call (device_count does not initialise HIP on this image)
    plan = plan_launch(args.gpus, os.environ.get("WORLD_SIZE"), args.devices,
                       0 if "WORLD_SIZE" in os.environ else torch.cuda.device_count())
    ensure_standin(scene_path)

    t_load = time.perf_counter()
    scene = B.load_dae(scene_path, W, H)      # bdpt_dae_load: the CLI's scene path
    t_load = time.perf_counter() - t_load
    env_desc = None
    if envmap:
        if envmap.startswith("synth:"):
            sys.path.insert(0, os.path.join(REPO, "tools"))
            from envmap import synth_envmap
            ew, eh = (int(v) for v in envmap[6:].split("x"))
            scene.set_envmap(synth_envmap(ew, eh))
            env_desc = f"synthetic sky {ew}x{eh} (tools/envmap.py)"
        else:
            scene.set_envmap(B.load_exr(envmap))
            env_desc = os.path.basename(envmap)
    seed = 5489
    use_pt = args.integrator == "pt"
    scaling = "strong" if use_pt else args.scaling
    run = run_inprocess if plan["mode"] == "inprocess" else run_torchrun_or_single
    t = run(args, B, scene, W, H, SPP, M, rr, seed, plan, use_pt, scaling)
    world, rank, dist, dev, rows = t.world, t.rank, t.dist, t.dev, t.rows
    kern_ms, elapsed = t.kern_ms, t.elapsed
    samples_per_step = t.samples_per_step

    # algorithmic bytes of rank 0's launch: in-kernel counters on a separate, untimed launch of
    # the same work (counting perturbs timing), SURVEY.md §8d.
    band = [(0, H * rank // world, W, H * (rank + 1) // world - H * rank // world)]
    if use_pt:
        ps = B.PathTracer(scene, W, H, SPP, M, seed=seed, device=dev.index, max_tolerance=0.0,
                          collect_stats=True)
        ps.raytrace_tiles(band, 0, SPP)
    else:
        ps = B.BidirectionalPathTracer(scene, W, H, SPP, M, seed=seed, device=dev.index,
                                       collect_stats=True, pipeline=args.pipeline, russian_roulette=rr)
        b0, n0 = rank_sample_range(0, rank, world, SPP, scaling)
        ps.raytrace_tiles([], b0, max(1, n0))
    st = ps.stats()
    ps.close()
    bytes_launch = algorithmic_bytes(st)
    gmem_launch = global_memory_bytes(st)
    fetched_launch = fetched_bytes(st)
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    value = samples_per_step * args.steps / elapsed / 1e6
    traffic, traffic_info = (None, None)
    if world == 1 and named and not use_pt and args.pipeline == 0:
        traffic, traffic_info = load_traffic(args.workload, kern_ms)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return 0
    wname = wl[7] if named else (f"{os.path.basename(scene_path)} {W}x{H} -s {SPP} -m {M}"
                                 f"{' + env ' + env_desc if env_desc else ''}{' RR on' if rr else ''}")
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: fixed-seed renders (Philox counter RNG) of {os.path.basename(scene_path)} "
                f"loaded by the product's .dae loader (bdpt_dae_load)"
                + ("; CBlucy.dae is absent from the reference, its stand-in (tools/gen_standin.py, "
                   "114,304 triangles) is rendered" if os.path.basename(scene_path) == os.path.basename(STANDIN) else ""),
        "config": {"workload": wname
                   + (" unidirectional PathTracer" if use_pt else "")
                   + (", whole frame per step split across GPUs" if scaling == "strong" else ", full spp per GPU")
                   + (" (row bands)" if use_pt else " (sample ranges)")
                   + t.label,
                   "workload_key": args.workload if named else "custom",
                   "pipeline": ["auto (megakernel)", "megakernel"][args.pipeline],
                   "scene": os.path.relpath(scene_path, REPO), "width": W, "height": H, "spp": SPP,
                   "max_depth": M, "envmap": env_desc, "russian_roulette": rr,
                   "parallelism": f"{'row bands' if use_pt else 'sample ranges'} x{world}",
                   "launch": plan["mode"],
                   "env": knobs,
                   "host_setup_s": {"dae_load": round(t_load, 3), "bdpt_create": round(t.t_create, 3)}},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                     "traffic": traffic, "kernel": "k_pt" if use_pt else "k_bdpt_sample",
                     "kernel_ms": round(kern_ms, 3),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "note": "achieved / frac = SURVEY §8d algorithmic scene bytes (its convention: 32 B/child "
                             "AABB, 36 B/triangle test, 16 B/sphere test, 40 B/closest hit; environment light: "
                             "76 B/sampled direction, 48 B/radiance lookup, 4 B/pdf lookup) / launch time (HIP "
                             "events on the ctx stream); fetched_* = the bytes the loads request (28 B/child of a "
                             "4-wide node, 32 B/child of a 2-wide one, 48 B/primitive record, 48 B/shading "
                             "record); gmem_* = the §8d bytes minus the scene reads served from the CU's LDS "
                             "copy (the part that goes through L2 / HBM); traffic = measured HBM-side bytes "
                             "(PMC: 2 x FETCH_SIZE + WRITE_SIZE, FETCH_SIZE counting half the bytes of every "
                             "read width this kernel uses, tools/fetch_calib.hip; traffic_pmc.pmc_frac over the "
                             "dispatch they were counted on)",
                     "fetched_bytes_per_launch": fetched_launch,
                     "frac_fetched_bytes": round(fetched_launch / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                     "gmem_bytes_per_launch": gmem_launch,
                     "gmem_achieved": round(gmem_launch / (kern_ms * 1e-3) / 1e9, 2),
                     "gmem_frac": round(gmem_launch / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                     "lds_mode": st.lds_mode,
                     "counts_per_launch": {"samples": st.samples, "node_aabbs": st.node_visits,
                                           "node_aabbs_from_lds": st.lds_node_visits,
                                           "tri_tests": st.tri_tests,
                                           "sph_tests": st.sph_tests, "hits": st.hits,
                                           "closest_rays": st.closest_rays,
                                           "shadow_rays": st.shadow_rays,
                                           "env_samples": st.env_samples, "env_lookups": st.env_lookups,
                                           "env_pdf_lookups": st.env_pdf_lookups}},
    }
    if traffic_info:
        out["roofline"]["traffic_pmc"] = traffic_info
    if t.rccl_ranks is not None:
        out["rccl_ranks"] = t.rccl_ranks
    if world > 1 or dist is not None:
        out["per_rank"] = {"elapsed_s": [round(r[0], 4) for r in rows],
                           "kernel_ms": [round(r[1], 3) for r in rows],
                           "samples_per_step": [int(r[2]) for r in rows], "device": [int(r[3]) for r in rows],
                           "backend": t.backend}
    if use_pt:
        out["config"]["integrator"] = "PathTracer (pathtracer.cpp:47-340)"
    cores = host_cores()
    thr = cores["usable"]
    progress(f"timed {args.steps} steps: {value:.1f} Msamples/s")
    if world == 1 and not args.no_parity and not use_pt:
        progress("parity leg: GPU vs oracle modes 2 and 1")
        out["parity"] = parity_check(scene, W, H, M, seed, rr=rr, threads=thr)
    if world == 1 and not args.no_cpu_baseline and not use_pt:
        progress("CPU baseline: oracle port")
        port = cpu_baseline(scene, os.path.basename(scene_path), W, H, SPP, M, threads=thr, rr=rr)
        # the reference cannot run the environment light / roulette under BDPT: port only
        ref = (None if (env_desc or rr)
               else cpu_baseline_reference(scene_path, os.path.basename(scene_path), W, H, M, threads=thr,
                                           cores=cores))
        out["cpu_baseline"] = ref if ref is not None else port
        if ref is not None:   # the oracle port's fp64 path, same host, for comparison
            out["cpu_baseline"]["port"] = {"value": port["value"], "cores": port["cores"], "sample": port["sample"]}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
