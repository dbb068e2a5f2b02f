#!/usr/bin/env python3
"""Benchmark: Msplats/s of the full frame (preprocess -> depth sort -> scan ->
duplicate -> bin sort -> ranges -> composite [-> exchange -> gather]) on
BASELINE.json's headline workload: 6M-splat scene @ 1920x1080, SH degree 3
(configs[2]; a seeded synthetic scene with 3DGS statistics — no garden .ply
exists offline).  Inputs are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Multi-GPU is weak scaling: every rank holds its own 6M-splat shard of a
(6M x N)-splat scene and owns 1/N of the tile rows; value = all splats / frame
time (max over ranks).  Prints one JSON line on rank 0.

At N=1 the line also carries
  roofline      the slowest stage's algorithmic bytes / its average kernel
                time; for preprocess / composite that time comes from HIP
                events carried in the kernels' own dispatch packets over the
                K timed frames (stage_timing 2: no extra packets, no syncs);
                the full per-stage table ("stages") comes from a few extra
                untimed frames with an event between every stage
                and `traffic`: its HBM bytes per launch from two rocprofv3
                PMC passes (FETCH_SIZE, WRITE_SIZE) run as child processes
                (FETCH_SIZE doubled: gfx950 tallies 128-B reads at 64 B,
                MI355X_MICROARCH.md §HBM); null if rocprofv3 is unavailable
  cpu_baseline  the CPU oracle (oracle/gs_oracle.c, OpenMP) on the same
                scene and camera, repeated for >= --cpu-seconds
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 78.6     # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz lane-ops/s (fp32 non-FMA)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--splats", type=int, default=6_000_000, help="splats per GPU")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--sh", type=int, default=3)
    ap.add_argument("--mode", default="tile")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=0, help="splats in the CPU baseline sample (0 = all)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum CPU baseline duration")
    ap.add_argument("--traffic", type=int, default=1, help="measure roofline.traffic with rocprofv3 PMC (N=1)")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="N=1: 2 = a frame's projection/sort overlaps the previous frame's composite")
    ap.add_argument("--scheme", default="rows", choices=["rows", "slabs"],
                    help="N>1: bin-row ownership (bit-exact, default) or depth slabs + RGBA reduce (DESIGN.md §6b)")
    return ap.parse_args()


def stage_summary(stats_list):
    keys = ["preprocess", "depth_sort", "scan", "duplicate", "sort", "ranges", "composite"]
    out = {}
    for k in keys:
        ms = float(np.mean([s[f"ms_{k}"] for s in stats_list]))
        by = float(np.mean([s[f"bytes_{k}"] for s in stats_list]))
        out[k] = {"ms": ms, "bytes": by, "gbs": by / (ms * 1e6) if ms > 0 else 0.0}
    ex = float(np.mean([s["ms_exchange"] for s in stats_list]))
    if ex > 0:  # multi-GPU: count + pack + all_to_all (not a kernel roofline)
        out["exchange"] = {"ms": ex, "bytes": 0.0, "gbs": 0.0}
    return out


def cpu_baseline(scene, view, proj, w, h, sh, sample, seconds):
    from oracle import oracle_py as O

    n = scene.n if sample <= 0 else min(sample, scene.n)
    sub = scene if n == scene.n else scene.subset(slice(0, n))
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    O.render(sub.subset(slice(0, min(n, 20000))), view, proj, w, h, sh_degree=sh, nthreads=threads)  # warm
    frames, t0 = 0, time.perf_counter()
    while True:
        O.render(sub, view, proj, w, h, sh_degree=sh, nthreads=threads)
        frames += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or frames >= 50:
            break
    return {"value": round(n * frames / dt / 1e6, 3), "unit": "Msplats/s", "cores": threads, "kind": "port",
            "sample": f"{frames} x one {w}x{h} SH{sh} frame of {n} splats of the same scene and camera "
                      f"(oracle/gs_oracle.c, OpenMP, {threads} threads), {dt:.1f} s"}


STAGE_KERNEL = {"preprocess": "preprocess_kernel", "depth_sort": "rts_pass_kernel<3>", "scan": "scan_reduce_kernel",
                "duplicate": "scan_duplicate_kernel", "sort": "rts_pass_kernel<1>", "ranges": "rts_pass_kernel<1>",
                "composite": "composite_kernel"}


def pmc_traffic(args, kernel):
    """HBM bytes per launch of `kernel`: two rocprofv3 --pmc passes over a
    short run of this benchmark in child processes (counters and traces are
    never combined; each pass its own process)."""
    import csv
    import shutil
    import subprocess
    import tempfile

    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    bench = [sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--cpu-baseline", "0",
             "--traffic", "0", "--no-stage-timing", "--splats", str(args.splats), "--width", str(args.width),
             "--height", str(args.height), "--sh", str(args.sh), "--mode", args.mode, "--seed", str(args.seed)]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    kb = {}
    with tempfile.TemporaryDirectory(dir=env["TMPDIR"]) as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = Path(td) / ctr
            cmd = [exe, "--kernel-trace", "--pmc", ctr, "-d", str(out), "-o", "run", "--output-format", "csv",
                   "--"] + bench
            try:
                p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300, env=env,
                                   cwd=str(ROOT))
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 {ctr} timed out"
            if p.returncode != 0:
                return None, f"rocprofv3 {ctr} exited {p.returncode}"
            vals = []
            for f in out.rglob("*counter_collection.csv"):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"no {ctr} samples for {kernel}"
            kb[ctr] = sum(vals) / len(vals)
    return 1024.0 * (2.0 * kb["FETCH_SIZE"] + kb["WRITE_SIZE"]), None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a 1-GPU box (never set by the driver): every rank on
    # device 0, collectives over gloo staged through host memory.
    backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
    if os.environ.get("GS_BENCH_SAME_DEVICE") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera

    W, H = args.width, args.height
    # each rank generates its own shard (distinct seeds): weak scaling
    scene = S.synthetic_scene(args.splats, seed=args.seed + 1000 * rank, sh_degree=args.sh, aspect=W / H)
    cam = default_camera(W, H)
    view, proj = cam.getViewMatrix(), cam.getProjectionMatrix()
    timing = 0 if args.no_stage_timing else 2  # timed frames: dispatch-packet events only
    opts = Options(mode=args.mode, sh_degree=args.sh, crop=False, stage_timing=timing,
                   frames_in_flight=args.frames_in_flight if world == 1 else 1)

    if world == 1:
        r = InstancedSplatRenderer(scene, opts)
        r.initialize(local)
        out = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        step = lambda: r.render(view, proj, W, H, out=out)
        rh = r
    else:
        from gaussian_splat_amd.distributed import HipShardBackend, HipSlabBackend, ShardedRenderer, SlabRenderer

        if args.scheme == "slabs":
            be = HipSlabBackend(scene, rank, world, rank * args.splats, opts, local)
            sr = SlabRenderer(be, rank, world)
        else:
            be = HipShardBackend(scene, rank, world, rank * args.splats, opts, local)
            sr = ShardedRenderer(be, rank, world)
        step = lambda: sr.render(view, proj, W, H, gather=True)
        rh = be.r

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1e3 / args.steps
    total_splats = args.splats * world
    value = total_splats / (ms * 1e-3) / 1e6

    s0 = rh.last_stats()
    # the order the timed frames built their bin lists in (the default picks
    # it per frame from the previous frame's pair count)
    binning = {1: "depth-first", 2: "bin-first"}.get(int(s0.get("binning", 0)), "?")
    timed = {}
    pipelined = world == 1 and args.frames_in_flight >= 2
    if timing == 2:  # kernel times of the timed frames (last <= 64)
        pre, comp = rh.kernel_times(args.steps)
        timed = {"preprocess": float(np.mean(pre)), "composite": float(np.mean(comp))} if len(pre) else {}
    # pipelined frames overlap the composite of frame k with the projection of
    # frame k+1, so their kernel durations include the co-running kernel: the
    # roofline takes the standalone kernels from extra unpipelined frames,
    # timed by the same dispatch-packet events
    standalone = {}
    if timing == 2 and pipelined:
        rh.set_frames_in_flight(1)
        n_sa = min(max(args.steps, 3), 10)
        for _ in range(n_sa):
            step()
        torch.cuda.synchronize()
        pre, comp = rh.kernel_times(n_sa)
        standalone = {"preprocess": float(np.mean(pre)), "composite": float(np.mean(comp))} if len(pre) else {}
        rh.set_frames_in_flight(args.frames_in_flight)
    # full stage breakdown: extra untimed frames, an event between every stage
    st = {}
    if not args.no_stage_timing:
        rh.set_stage_timing(1)
        stats = []
        for _ in range(min(max(args.steps, 3), 10)):
            step()
            stats.append(rh.last_stats())
        st = stage_summary(stats)

    line = None
    if rank == 0:
        rl = None
        if st:
            dom = max((k for k in st if k != "exchange"), key=lambda k: st[k]["ms"])
            d = st[dom]
            kms, src = d["ms"], "stage events, extra untimed frames"
            if pipelined and dom in standalone:
                kms = standalone[dom]
                src = f"dispatch-packet events, {n_sa} extra unpipelined frames (standalone kernel)"
            elif pipelined:
                src = "stage events, extra untimed unpipelined frames (standalone kernel)"
            elif dom in timed:
                kms, src = timed[dom], f"dispatch-packet events, {min(args.steps, 64)} timed frames"
            gbs = d["bytes"] / (kms * 1e6)
            rl = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None, "kernel": dom,
                  "kernel_ms": round(kms, 4), "bytes": int(d["bytes"]), "timing": src}
        line = {
            "metric": "Msplats/sec (6M-splat scene @1080p, SH3, full frame)",
            "value": round(value, 2), "unit": "Msplats/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded 3DGS-statistics scene; no garden .ply offline)",
            "config": {"workload": f"{args.splats} splats/GPU @ {W}x{H}, SH{args.sh}, {args.mode} contract",
                       "global_splats": total_splats, "width": W, "height": H, "sh_degree": args.sh,
                       "parallelism": (f"splat-shard x{world}, 32-px bin-row ownership, all_to_all + gather, {backend}"
                                       if args.scheme == "rows" else
                                       f"splat-shard x{world}, depth slabs, all_to_all + T all_gather + RGBA "
                                       f"reduce, {backend}") if world > 1 else
                                      ("single GPU, 2 frames in flight (projection/sort of frame k+1 under the "
                                       "composite of frame k)" if args.frames_in_flight == 2 else "single GPU"),
                       "pairs": int(s0["pairs"]), "visible": int(s0["visible"]), "binning": binning},
            "roofline": rl,
            "stages": {k: {kk: round(vv, 4) for kk, vv in v.items()} for k, v in st.items()},
            "timed_kernel_ms": {k: round(v, 4) for k, v in timed.items()},
            "standalone_kernel_ms": {k: round(v, 4) for k, v in standalone.items()},
            "timed_kernel_note": ("timed frames, preprocess of frame k+1 co-running with the composite of frame k"
                                  if pipelined else "timed frames"),
        }
        if world == 1 and rl is not None and args.traffic:
            kern = STAGE_KERNEL[rl["kernel"]]
            if rl["kernel"] == "depth_sort" and binning == "bin-first":
                kern = "bin_depth_sort_kernel"
            traffic, why = pmc_traffic(args, kern)
            rl["traffic"] = round(traffic) if traffic is not None else None
            if why:
                rl["traffic_note"] = why
        if world == 1 and args.cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene, view, proj, W, H, args.sh, args.cpu_sample,
                                                args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
