#!/usr/bin/env python3
"""Benchmark: Msplats/s of the full frame (preprocess -> sort/binning ->
composite [-> exchange -> gather / reduce]) and the frame's achieved HBM GB/s,
on BASELINE.json's workloads, inputs resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W --config 1080p|4k|50m|1m]

Workloads (seeded synthetic scenes with 3DGS statistics; the garden .ply
does not exist offline):
  1080p (default)  BASELINE config 3: 6M-splat scene @1920x1080, SH degree 3
  4k               BASELINE config 4: the same scene @3840x2160
  50m              BASELINE config 5: 50M-splat stress scene @3840x2160, SH 0
  1m               BASELINE config 2: 1M splats @1920x1080, SH 0

Multi-GPU is STRONG scaling over one global scene; value = global splats /
frame time (max over ranks).  Two launchers:
  group  (`--gpus N` outside torchrun, the default there): ONE process drives
         all N GPUs through the C-ABI group (gs_create_sharded_from_handle,
         RCCL over xGMI: csrc/host/group.cpp)
  ranks  (the driver's torchrun line, or --launcher ranks, which starts it):
         one process per GPU, torch.distributed over RCCL (distributed.py);
         WORLD_SIZE must equal --gpus
Both time the two exact multi-GPU schemes (bit-identical to one GPU's frame)
over the same K frames and report both in `schemes`:
  rows   the north star's splat-index sharding: rank r holds the shard
         [r*N/g, (r+1)*N/g) of the global scene (generated chunk-wise, so a
         rank builds only its shard); 32-px bin-row ownership, all-to-all of
         the projected records, band gather.  Two frames in flight by default
         (--pipeline-rows 1): frame k's all-to-all under frame k-1's render
  bands  SURVEY §8(e)'s fallback: the scene REPLICATED on every rank, each
         renders its own bin rows, band gather; no exchange
The headline rule (stated identically in DESIGN.md §6 and README):
`value` is the rows scheme's whenever rows is at least as fast as bands at
that world size; otherwise it is bands', named as the replicated scheme in
`config.parallelism` and `scheme_choice`.  Rows are link-bound at 2 ranks
(about half of every rank's records cross the one xGMI link between them).
The north star's depth slabs + transmittance all_gather + RGBA reduce
(--scheme slabs / both) do NOT meet its 1e-4 tolerance (pixels at the 0.99
break) and are not part of the default run.

At N=1 the line also carries
  roofline      the dominant kernel's algorithmic bytes / its standalone
                duration (HIP events in its own dispatch packet, extra
                unpipelined frames), and `kernels`: preprocess and composite
                (the north star's kernel) always, each with its HBM fraction
                (composite bytes from the records its workgroups actually
                fetched, early-out included), PMC traffic (rocprofv3
                FETCH_SIZE x 2 + WRITE_SIZE per launch, MI355X_MICROARCH.md
                §HBM) and VALU-issue fraction (SQ_INSTS_VALU x 2 cycles per
                wave64 instruction over 1024 SIMDs at 2.4 GHz)
  settled       the same K frames timed again after 60 more frames (clock
                ramp), beside the value
  orbit         the same K frames on an orbiting camera (--orbit-probe), beside
                the value: the default still camera is depth cuts' best case
  cpu_baseline  the CPU oracle (oracle/gs_oracle.c, OpenMP) on the same scene
                and camera on all host threads, and on 1 thread over a
                bounded subset (cpu_baseline_1core)
Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
SIMDS = 1024                 # 256 CUs x 4 SIMD-32
CLOCK_HZ = 2.4e9             # peak engine clock
VALU_ISSUE_CYC = 2           # cycles per wave64 VALU instruction per SIMD, waves interleaved (MI355X_MICROARCH.md:54)

CONFIGS = {
    "1080p": dict(splats=6_000_000, width=1920, height=1080, sh=3, seed=2,
                  label="BASELINE config 3: 6M-splat scene @1920x1080, SH3"),
    "4k": dict(splats=6_000_000, width=3840, height=2160, sh=3, seed=2,
               label="BASELINE config 4: 6M-splat scene @3840x2160, SH3"),
    "50m": dict(splats=50_000_000, width=3840, height=2160, sh=0, seed=4,
                label="BASELINE config 5: 50M-splat stress scene @3840x2160, SH0"),
    "1m": dict(splats=1_000_000, width=1920, height=1080, sh=0, seed=1,
               label="BASELINE config 2: 1M-splat scene @1920x1080, SH0"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle", type=int, default=0,
                    help="untimed frames before the warmup (0 = the warmup alone, as the driver runs it)")
    ap.add_argument("--settled-probe", type=int, default=60,
                    help="after the timed region: this many more untimed frames, then the same K frames timed "
                         "again, reported beside the value as 'settled' (0 = skip)")
    ap.add_argument("--config", default="1080p", choices=sorted(CONFIGS))
    ap.add_argument("--splats", type=int, default=0, help="global splats (0 = the config's)")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--sh", type=int, default=-1)
    ap.add_argument("--seed", type=int, default=-1)
    ap.add_argument("--profile", default="uniform", choices=["uniform", "heavy"],
                    help="scale distribution: uniform 3DGS statistics or the heavy-tailed stress variant")
    ap.add_argument("--camera", default="fixed", choices=["fixed", "orbit"],
                    help="fixed: the reference app's camera every frame; orbit (N=1): a new view every frame, "
                         "the eye turning 0.01 rad about the target per frame (splats leave and enter the view)")
    ap.add_argument("--mode", default="tile")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="minimum CPU baseline duration")
    ap.add_argument("--pmc", type=int, default=1, help="N=1: rocprofv3 PMC passes (traffic, VALU instructions)")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="N=1: 2 = a frame's projection/sort overlaps the previous frame's composite")
    ap.add_argument("--scheme", default="all", choices=["rows", "slabs", "bands", "both", "all"],
                    help="N>1: all = rows (splat-sharded) + bands (replicated), both exact; value = rows' when it is "
                         "at least as fast as bands, else bands'; slabs = depth slabs + RGBA reduce (approximate, "
                         "outside the 1e-4 tolerance); both = rows + slabs")
    ap.add_argument("--pipeline-rows", type=int, default=1,
                    help="N>1: 1 = rows frames pipelined (frame k's all-to-all under frame k-1's render, a second "
                         "communicator set); 0 = one frame at a time")
    ap.add_argument("--launcher", default="group", choices=["group", "ranks"],
                    help="--gpus N outside torchrun: group = one process drives every GPU (gs_create_sharded, "
                         "RCCL); ranks = one process per GPU (torch.distributed.run, the driver's launch line)")
    ap.add_argument("--orbit-probe", type=int, default=1,
                    help="N=1, fixed camera: after the settled probe, time the same K frames once more with an "
                         "orbiting camera (a new view every frame) and report them as 'orbit' (0 = skip)")
    ap.add_argument("--comm-timeout", type=float, default=120.0,
                    help="N>1: seconds before a rendezvous or collective that a peer never joins fails")
    a = ap.parse_args()
    c = CONFIGS[a.config]
    a.splats = a.splats or c["splats"]
    a.width = a.width or c["width"]
    a.height = a.height or c["height"]
    a.sh = c["sh"] if a.sh < 0 else a.sh
    a.seed = c["seed"] if a.seed < 0 else a.seed
    a.label = c["label"] if (a.splats, a.width, a.height, a.sh) == (c["splats"], c["width"], c["height"], c["sh"]) \
        else f"{a.splats} splats @{a.width}x{a.height}, SH{a.sh}"
    return a


def spawn_ranks(args) -> int:
    """--gpus N outside torchrun: one rank process per GPU (the parent never
    touches a GPU), the driver's own launch line; returns their exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd)


def headline(schemes, order):
    """The headline scheme (README, this module's docstring):
    rows, the north star's splat-index sharding, whenever it is at least as
    fast as the replicated-scene bands at this world size; else bands."""
    exact = [k for k in ("rows", "bands") if k in schemes]
    if not exact:
        return order[0], exact
    if "rows" in exact and ("bands" not in exact or schemes["rows"]["ms"] <= schemes["bands"]["ms"]):
        return "rows", exact
    return "bands", exact


def scheme_choice(head, exact, world):
    if len(exact) < 2:
        return head
    return (f"{head}: rows (splat-sharded) is the headline whenever it is at least as fast as bands (the scene "
            f"replicated on every rank); at world size {world} {head} was "
            + ("(rows at most bands' time)" if head == "rows" else "faster (rows are link-bound at few ranks)")
            + "; both timed over the same frames, reported in schemes, bit-identical to the 1-GPU frame")


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


def cpu_baseline(scene, view, proj, w, h, sh, threads, seconds, max_frames=50):
    from oracle import oracle_py as O

    O.render(scene.subset(slice(0, min(scene.n, 20000))), view, proj, w, h, sh_degree=sh, nthreads=threads)  # warm
    frames, t0 = 0, time.perf_counter()
    while True:
        O.render(scene, view, proj, w, h, sh_degree=sh, nthreads=threads)
        frames += 1
        dt = time.perf_counter() - t0
        if dt >= seconds or frames >= max_frames:
            break
    return {"value": round(scene.n * frames / dt / 1e6, 3), "unit": "Msplats/s", "cores": threads, "kind": "port",
            "sample": f"{frames} x one {w}x{h} SH{sh} frame of {scene.n} splats of the same scene and camera "
                      f"(oracle/gs_oracle.c, OpenMP, {threads} thread{'s' if threads > 1 else ''}), {dt:.1f} s"}


KERNEL_NAME = {"preprocess": "preprocess_kernel", "composite": "composite_"}  # (composite_kernel, composite_strip_kernel)
# (depth-cut frames: the composite's pass 2 over the fallback lists is a separate, usually empty
# launch; the dispatch-packet events and the PMC means are the front lists' pass)
KERNEL_EXCLUDE = {"composite": ", 2>"}


def pmc_passes(args):
    """Per-launch PMC means of the preprocess and composite kernels: one
    rocprofv3 --kernel-trace --pmc child process per counter group (counters
    never combined with traces of other domains)."""
    import csv
    import shutil
    import tempfile

    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    bench = [sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--settle", "0", "--cpu-baseline", "0",
             "--pmc", "0", "--orbit-probe", "0", "--no-stage-timing", "--frames-in-flight", "1", "--splats", str(args.splats),
             "--width", str(args.width), "--height", str(args.height), "--sh", str(args.sh), "--mode", args.mode,
             "--seed", str(args.seed), "--profile", args.profile]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    out = {k: {} for k in KERNEL_NAME}
    with tempfile.TemporaryDirectory(dir=env["TMPDIR"]) as td:
        for grp in (["FETCH_SIZE"], ["WRITE_SIZE"], ["SQ_INSTS_VALU", "SQ_WAVES"]):
            d = Path(td) / grp[0]
            cmd = [exe, "--kernel-trace", "--pmc", *grp, "-d", str(d), "-o", "run", "--output-format", "csv",
                   "--"] + bench
            try:
                p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300, env=env,
                                   cwd=str(ROOT))
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 {grp} timed out"
            if p.returncode != 0:
                return None, f"rocprofv3 {grp} exited {p.returncode}"
            vals = {(k, c): [] for k in KERNEL_NAME for c in grp}
            for f in d.rglob("*counter_collection.csv"):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        for k, kn in KERNEL_NAME.items():
                            name = row.get("Kernel_Name", "")
                            if k in KERNEL_EXCLUDE and KERNEL_EXCLUDE[k] in name:
                                continue
                            if kn in name and row.get("Counter_Name") in grp:
                                vals[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
            for (k, c), v in vals.items():
                if v:
                    out[k][c] = sum(v) / len(v)
    for k, cs in out.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:  # KB; FETCH_SIZE counts 128-B reads at 64 B on gfx950
            cs["traffic"] = 1024.0 * (2.0 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"])
    return out, None


def kernel_entry(ms, nbytes, pmc):
    e = {"ms": round(ms, 4), "bytes": int(nbytes), "hbm_gbs": round(nbytes / (ms * 1e6), 1) if ms > 0 else 0.0,
         "hbm_frac": round(nbytes / (ms * 1e6) / HBM_PEAK_GBS, 4) if ms > 0 else 0.0, "traffic": None}
    if pmc:
        if "traffic" in pmc:
            e["traffic"] = int(pmc["traffic"])
        if "SQ_INSTS_VALU" in pmc and ms > 0:
            e["valu_insts"] = int(pmc["SQ_INSTS_VALU"])
            e["valu_issue_frac"] = round(pmc["SQ_INSTS_VALU"] * VALU_ISSUE_CYC / (SIMDS * CLOCK_HZ * ms * 1e-3), 4)
    return e


def group_main(args):
    """`--gpus N` outside torchrun: ONE process drives all N GPUs through the
    C-ABI group (gs_create_sharded_from_handle / gs_create_replicated_from_
    handle, csrc/host/group.cpp), collectives over RCCL (xGMI) when every rank
    has its own device.  GS_BENCH_SAME_DEVICE=1 (a one-GPU rehearsal, never set
    by the driver) puts every rank on device 0: peer copies, or the test RCCL
    stub when GS_RCCL_LIB names it."""
    import torch

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, ShardedGroup, default_camera

    N, W, H, G = args.splats, args.width, args.height, args.gpus
    same = os.environ.get("GS_BENCH_SAME_DEVICE") == "1"
    devices = [0] * G if same else list(range(G))
    if not same and torch.cuda.device_count() < G:
        sys.exit(f"bench.py: --gpus {G} but {torch.cuda.device_count()} devices")
    transport = ("rccl" if os.environ.get("GS_RCCL_LIB") else "copy") if same else "auto"
    scene = S.activate(S.synthetic_raw(N, seed=args.seed, aspect=W / H, rest=args.sh > 0, profile=args.profile),
                       args.sh)
    cam = default_camera(W, H)
    view, proj = cam.getViewMatrix(), cam.getProjectionMatrix()
    src = InstancedSplatRenderer(scene, Options(mode=args.mode, sh_degree=args.sh, crop=False))
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    pipe = bool(args.pipeline_rows) and args.frames_in_flight >= 2

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    def timed(step, steps, warmup, drain=None):
        for _ in range(args.settle + warmup):
            step()
        if drain is not None:
            drain()
        sync_all()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if drain is not None:  # (pipelined rows: the last frame finishes inside the timed region)
            drain()
        sync_all()
        return (time.perf_counter() - t0) * 1e3 / steps

    schemes, groups = {}, {}
    order = {"both": ["rows"], "all": ["bands", "rows"]}.get(args.scheme, [args.scheme])
    for sch in order:
        if sch == "slabs":
            continue  # (the approximate scheme: torch.distributed launcher only)
        g = ShardedGroup(src, G, replicated=(sch == "bands"))
        g.initialize(devices, transport)
        drain = None
        if sch == "rows" and pipe:
            g.set_frames_in_flight(2)
            step = (lambda g_=g: g_.render_pipelined(view, proj, W, H, out=out))
            drain = (lambda g_=g: g_.flush(W, H, out=out))
        else:
            step = (lambda g_=g: g_.render(view, proj, W, H, out=out))
        schemes[sch] = {"ms": timed(step, args.steps, args.warmup, drain), "step": step, "drain": drain,
                        "transport": g.transport}
        groups[sch] = g
    head, exact = headline(schemes, order)
    ms = schemes[head]["ms"]
    settled_line = None
    if args.settled_probe > 0:
        for _ in range(args.settled_probe):
            schemes[head]["step"]()
        settled_line = {"extra_frames": args.settled_probe,
                        "ms_per_step": round(timed(schemes[head]["step"], args.steps, 0, schemes[head]["drain"]), 4),
                        "note": "the same frames timed again after the value's run and these extra untimed frames"}
    s0 = groups[head].last_stats(0)
    tr = schemes[head]["transport"]
    par = (f"rows: {G} GPUs from one process (gs_create_sharded), splat-index shards of one global scene, 32-px "
           f"bin-row ownership, all-to-all of projected records + band gather ({tr}"
           + ("; 2 frames in flight: a frame's all-to-all under the previous frame's render" if pipe else "") + ")"
           if head == "rows" else
           f"bands: {G} GPUs from one process (gs_create_replicated), the scene REPLICATED on every rank (not "
           f"splat-sharded), each renders its 32-px bin rows, band gather ({tr})")
    line = {
        "metric": "Msplats/sec + achieved HBM GB/s (6M-splat scene @1080p, SH3, full frame)"
        if args.config == "1080p" else f"Msplats/sec + achieved HBM GB/s ({args.label})",
        "value": round(N / (ms * 1e-3) / 1e6, 2), "unit": "Msplats/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "settle": {"frames": args.settle, "note": "untimed frames before the warmup (--settle), per timed scheme"},
        "settled": settled_line, "orbit": None, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic (seeded 3DGS-statistics scene, {args.profile} scales; no garden .ply offline)",
        "hbm_gbs": None,
        "config": {"workload": args.label, "global_splats": N, "width": W, "height": H, "sh_degree": args.sh,
                   "parallelism": par, "launcher": "group (one process, csrc/host/group.cpp)",
                   "devices": devices, "pairs": int(s0["pairs"]), "visible": int(s0["visible"])},
        "comm": {"backend": tr, "ranks": G},
        "schemes": {k: {"ms_per_step": round(v["ms"], 4), "value": round(N / (v["ms"] * 1e-3) / 1e6, 2),
                        "transport": v["transport"]} for k, v in schemes.items()},
        "scheme_choice": scheme_choice(head, exact, G),
    }
    if same:
        line["rehearsal"] = ("every rank on device 0 (GS_BENCH_SAME_DEVICE): the protocol, not xGMI; "
                             + ("RCCL entry points from GS_RCCL_LIB" if transport == "rccl" else "peer copies"))
    print(json.dumps(line), flush=True)
    for g in groups.values():
        g.close()


def main():
    args = parse()
    if args.camera == "orbit" and args.gpus > 1:
        sys.exit("bench.py: --camera orbit is a single-GPU workload")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        if args.launcher == "group":
            return group_main(args)
        sys.exit(spawn_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    # Rehearsal knobs for a 1-GPU box (never set by the driver): every rank on
    # device 0, collectives over gloo staged through host memory.
    backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
    if os.environ.get("GS_BENCH_SAME_DEVICE") == "1":
        local = 0
    if world > 1:
        from gaussian_splat_amd.distributed import init_ranks

        torch.cuda.set_device(local)
        # bounded: a rank that never joins or stops answering makes the others
        # exit non-zero after --comm-timeout seconds instead of hanging
        init_ranks(backend, args.comm_timeout, device=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera
    from gaussian_splat_amd.distributed import shard_bounds

    W, H, N = args.width, args.height, args.splats
    b, e = shard_bounds(N, world, rank)
    # this rank's shard of the global scene (generated chunk-wise: the same
    # splats whichever rank builds them)
    scene = S.activate(S.synthetic_raw(N, seed=args.seed, aspect=W / H, rest=args.sh > 0, profile=args.profile,
                                       start=b, stop=e), args.sh)
    cam = default_camera(W, H)
    view, proj = cam.getViewMatrix(), cam.getProjectionMatrix()
    # kernel times come from dispatch-packet events on extra frames after the
    # timed region; the timed frames carry none (the events cost ~0.5 % of a
    # frame: 0.7356-0.7394 against 0.7416-0.7428 ms)
    timing = 0 if args.no_stage_timing else 2
    opts = Options(mode=args.mode, sh_degree=args.sh, crop=False, stage_timing=0,
                   frames_in_flight=args.frames_in_flight if world == 1 else 1)

    settled = {"frames": 0, "ms": 0.0}

    def timed(step, steps, warmup, settle=None, drain=None):
        # --settle: untimed frames before the warmup (default none, the
        # driver's --warmup governs).  Every rank runs the same count, so
        # collectives stay matched.
        settle = args.settle if settle is None else settle
        t_s = time.perf_counter()
        for _ in range(settle):
            step()
        torch.cuda.synchronize()
        settled["frames"] += settle
        settled["ms"] += (time.perf_counter() - t_s) * 1e3
        for _ in range(warmup):
            step()
        if drain is not None:
            drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        if drain is not None:  # (pipelined row frames: the last frame finishes inside the timed region)
            drain()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt * 1e3 / steps

    def settled_probe(step, steps, drain=None):
        # The value is the driver's protocol (its --warmup only).  The GPU
        # leaves idle clocks over the first ~40 frames (5-frame blocks 0.89 ->
        # 0.78 ms at 1080p, tools/warm_probe.py), so the same K
        # frames are timed once more after --settled-probe further frames and
        # reported beside it, never as the value.
        if args.settled_probe <= 0:
            return None
        for _ in range(args.settled_probe):
            step()
        return {"extra_frames": args.settled_probe, "ms_per_step": round(timed(step, steps, 0, settle=0, drain=drain), 4),
                "note": "the same frames timed again after the value's run and these extra untimed frames"}

    schemes = {}
    orbit_line = None
    if world == 1:
        r = InstancedSplatRenderer(scene, opts)
        r.initialize(local)
        out = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        if args.camera == "orbit":
            views = []
            for _ in range(720):  # (cycled: 7.2 rad of orbit)
                views.append(cam.getViewMatrix())
                cam.orbit(0.01)
            frame = [0]

            def step():
                r.render(views[frame[0] % len(views)], proj, W, H, out=out)
                frame[0] += 1
        else:
            step = lambda: r.render(view, proj, W, H, out=out)
        rh = r
        drain = None
        ms = timed(step, args.steps, args.warmup)
        s_timed = r.last_stats()  # (the timed frames' lists, before the probes below move the camera)
        settled_line = settled_probe(step, args.steps)
        if args.camera == "fixed" and args.orbit_probe:
            # camera sensitivity: the default camera is the
            # best case for depth cuts (cuts taken two frames back are exact),
            # so the same K frames are timed once more on an orbiting camera;
            # beside the value, never as it.  Afterwards the fixed camera's
            # frames (kernel and stage timing below) run again.
            ocam = default_camera(W, H)
            oviews = []
            for _ in range(args.warmup + args.steps):
                ocam.orbit(0.01)
                oviews.append(ocam.getViewMatrix())
            of = [0]

            def ostep():
                r.render(oviews[of[0] % len(oviews)], proj, W, H, out=out)
                of[0] += 1

            oms = timed(ostep, args.steps, args.warmup, settle=0)
            os_ = r.last_stats()
            orbit_line = {"ms_per_step": round(oms, 4), "value": round(N / (oms * 1e-3) / 1e6, 2),
                          "warmup": args.warmup, "steps": args.steps, "pairs": int(os_["pairs"]),
                          "pairs_sorted": int(os_.get("pairs_sorted", os_["pairs"])),
                          "open_tiles": int(os_.get("open_tiles", 0)), "cut_dilate": int(os_.get("cut_dilate", 0)),
                          "binning": {1: "depth-first", 2: "bin-first"}.get(int(os_.get("binning", 0)), "?"),
                          "note": "the same K frames on an orbiting camera (0.01 rad per frame about the target), "
                                  "after the settled probe, with their own warmup; reported beside the value"}
            # back to the fixed camera for the kernel and stage timing, for as
            # many frames as the orbit's cut dilation takes to decay (one bin of
            # radius per 8 frames without an open quadrant, per buffer set)
            for _ in range(args.warmup + 2 * 8 * 5):
                step()
    else:
        from gaussian_splat_amd.distributed import (BandRenderer, HipBandBackend, HipShardBackend, HipSlabBackend,
                                                    ShardedRenderer, SlabRenderer)

        # (bands first: no exchange; rows on process groups of their own, so
        # the default group only times)
        order = {"both": ["rows", "slabs"], "all": ["bands", "rows"]}.get(args.scheme, [args.scheme])
        for sch in order:
            if sch == "bands":  # the whole scene on every rank
                full = S.activate(S.synthetic_raw(N, seed=args.seed, aspect=W / H, rest=args.sh > 0,
                                                  profile=args.profile), args.sh)
                # (no exchange between the frame's stages: two frames in flight as at N=1)
                import dataclasses
                be = HipBandBackend(full, rank, world,
                                    dataclasses.replace(opts, frames_in_flight=args.frames_in_flight), local)
                sr = BandRenderer(be, rank, world)
            elif sch == "slabs":
                be = HipSlabBackend(scene, rank, world, b, opts, local)
                sr = SlabRenderer(be, rank, world)
            else:
                be = HipShardBackend(scene, rank, world, b, opts, local)
                # two frames in flight: frame k's record exchange (its own
                # communicator) overlaps frame k-1's render and gather
                pipe = args.frames_in_flight >= 2 and bool(args.pipeline_rows)
                sr = ShardedRenderer(be, rank, world, group=dist.new_group(backend=backend), pipeline=pipe,
                                     exchange_group=dist.new_group(backend=backend) if pipe else None)
            stp = (lambda s_=sr: s_.render(view, proj, W, H, gather=True))
            drn = getattr(sr, "flush", None) if getattr(sr, "pipeline", False) else None
            schemes[sch] = {"ms": timed(stp, args.steps, args.warmup, drain=drn), "handle": be.r, "step": stp,
                            "drain": drn}
        head, exact = headline(schemes, order)
        ms, rh, step = schemes[head]["ms"], schemes[head]["handle"], schemes[head]["step"]
        drain = schemes[head]["drain"]
        settled_line = settled_probe(step, args.steps, drain=drain)
    value = N / (ms * 1e-3) / 1e6

    s0 = s_timed if world == 1 else rh.last_stats()
    binning = {1: "depth-first", 2: "bin-first"}.get(int(s0.get("binning", 0)), "?")
    pipelined = world == 1 and args.frames_in_flight >= 2
    timed_k, n_co = {}, min(max(args.steps, 3), 64)
    if timing == 2:  # kernel times of frames run as the timed ones were (pipelined), after them
        rh.set_stage_timing(2)
        for _ in range(n_co):
            step()
        torch.cuda.synchronize()
        pre, comp = rh.kernel_times(n_co)
        timed_k = {"preprocess": float(np.mean(pre)), "composite": float(np.mean(comp))} if len(pre) else {}
    # standalone kernels (the roofline's timing): extra unpipelined frames
    # timed by the same dispatch-packet events
    standalone, n_sa = {}, min(max(args.steps, 3), 10)
    if timing == 2:
        if pipelined:
            rh.set_frames_in_flight(1)
        for _ in range(n_sa):
            step()
        torch.cuda.synchronize()
        pre, comp = rh.kernel_times(n_sa)
        standalone = {"preprocess": float(np.mean(pre)), "composite": float(np.mean(comp))} if len(pre) else {}
        sa_stats = rh.last_stats()  # (records the composite fetched in such a frame)
        if pipelined:
            rh.set_frames_in_flight(args.frames_in_flight)
    # full stage breakdown: extra untimed frames, an event between every stage
    st = {}
    if not args.no_stage_timing:
        rh.set_stage_timing(1)
        stats = []
        for _ in range(n_sa):
            step()
            stats.append(rh.last_stats())
        st = stage_summary(stats)
        rh.set_stage_timing(timing)
    if drain is not None:  # (pipelined row frames: every rank finishes the frame in flight)
        drain()

    line = None
    if rank == 0:
        frame_bytes = sum(v["bytes"] for k, v in st.items() if k != "exchange") if st else 0.0
        line = {
            "metric": "Msplats/sec + achieved HBM GB/s (6M-splat scene @1080p, SH3, full frame)"
            if args.config == "1080p" else f"Msplats/sec + achieved HBM GB/s ({args.label})",
            "value": round(value, 2), "unit": "Msplats/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "settle": {"frames": settled["frames"], "ms": round(settled["ms"], 1),
                       "note": "untimed frames before the warmup (--settle), per timed scheme"},
            "settled": settled_line,
            "orbit": orbit_line,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic (seeded 3DGS-statistics scene, {args.profile} scales; no garden .ply offline)"
                    + ("; orbiting camera, a new view every frame" if args.camera == "orbit" else ""),
            "hbm_gbs": round(frame_bytes / (ms * 1e6), 1) if frame_bytes else None,
            "config": {"workload": args.label, "global_splats": N, "width": W, "height": H, "sh_degree": args.sh,
                       "parallelism": ((f"rows: {world} ranks, splat-index shards of one global scene, 32-px bin-row "
                                        f"ownership, all_to_all of projected records + band gather ({backend}, world "
                                        f"{world}" + ("; 2 frames in flight: a frame's exchange under the previous "
                                                      "frame's render" if drain is not None else "") + ")")
                                       if head == "rows" else
                                       (f"bands: {world} ranks, the scene REPLICATED on every rank (not splat-sharded), "
                                        f"each renders its 32-px bin rows, band gather ({backend}, world {world})")
                                       if head == "bands" else
                                       (f"slabs: {world} ranks, splat-index shards, depth slabs + RGBA reduce "
                                        f"(approximate; {backend}, world {world})"))
                       if world > 1 else
                       ("single GPU, 2 frames in flight (projection/sort of frame k+1 under the composite of frame k)"
                        if args.frames_in_flight == 2 else "single GPU"),
                       "pairs": int(s0["pairs"]), "visible": int(s0["visible"]), "binning": binning,
                       "depth_cuts": bool(s0.get("cut_frame", 0)), "pairs_sorted": int(s0.get("pairs_sorted", s0["pairs"])),
                       "open_tiles": int(s0.get("open_tiles", 0)), "cut_dilate": int(s0.get("cut_dilate", 0))},
            "stages": {k: {kk: round(vv, 4) for kk, vv in v.items()} for k, v in st.items()},
            "timed_kernel_ms": {k: round(v, 4) for k, v in timed_k.items()},
            "timed_kernel_note": (f"dispatch-packet events on {n_co} frames run as the timed ones, after them "
                                  "(the timed frames carry no events)") if timed_k else None,
            "standalone_kernel_ms": {k: round(v, 4) for k, v in standalone.items()},
        }
        if world > 1:
            line["comm"] = {"backend": dist.get_backend(), "ranks": dist.get_world_size()}
            line["schemes"] = {k: {"ms_per_step": round(v["ms"], 4), "value": round(N / (v["ms"] * 1e-3) / 1e6, 2)}
                               for k, v in schemes.items()}
            line["scheme_choice"] = scheme_choice(head, exact, world)
            if "slabs" in line["schemes"]:
                line["schemes"]["slabs"]["note"] = ("depth slabs + transmittance all_gather + RGBA reduce "
                                                    "(approximate, outside the 1e-4 tolerance: reassociated transmittance product)")
        if st and standalone:
            pmc, why = (pmc_passes(args) if (world == 1 and args.pmc) else (None, "pmc off"))
            kern = {}
            for k in ("preprocess", "composite"):
                nbytes = sa_stats[f"bytes_{k}"]
                kern[k] = kernel_entry(standalone[k], nbytes, (pmc or {}).get(k))
            kern["composite"]["records_fetched"] = int(sa_stats["records_fetched"])
            kern["composite"]["pairs"] = int(sa_stats["pairs"])
            dom = max(kern, key=lambda k: kern[k]["ms"])
            d = kern[dom]
            line["roofline"] = {"bound": "hbm", "achieved": d["hbm_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": d["hbm_frac"], "traffic": d["traffic"], "kernel": dom, "kernel_ms": d["ms"],
                                "bytes": d["bytes"], "valu_issue_frac": d.get("valu_issue_frac"),
                                "timing": f"dispatch-packet events, {n_sa} extra unpipelined frames "
                                          "(standalone kernel)",
                                "kernels": kern}
            if why:
                line["roofline"]["pmc_note"] = why
        if world == 1 and args.cpu_baseline:
            threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
            line["cpu_baseline"] = cpu_baseline(scene, view, proj, W, H, args.sh, threads, args.cpu_seconds)
            sub = scene.subset(slice(0, min(scene.n, max(scene.n // 8, 1))))
            line["cpu_baseline_1core"] = cpu_baseline(sub, view, proj, W, H, args.sh, 1, args.cpu_seconds,
                                                      max_frames=20)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
