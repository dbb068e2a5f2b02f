#!/usr/bin/env python3
"""Per-rank compute of the splat-sharded row scheme on one GPU (virtual
ranks): for world g, rank r projects its splat-index shard
[r*N/g, (r+1)*N/g) and packs the exchange records (gs_shard_project), then
renders the records every rank sent it into its owned 32-px bin rows
(gs_shard_render).  Both are timed per rank (mean of K frames after warm-up,
one frame in flight), with the bytes each rank sends and receives and the
band it contributes to the gather.

The exchange and the gather are not run over links here (one GPU): their
per-rank bytes are recorded, and `link_model_ms` prices them at the xGMI
rate the task states (7 links per GPU, ~153.6 GB/s each, taken as 76.8 GB/s
per direction): the all_to_all sends each peer its records over a dedicated
link, the gather brings every band into rank 0 over its own link.  That
model is labelled as such; the measured numbers are project_ms/render_ms.

  python tools/rows_probe.py [--splats 6000000] [--worlds 1,2,4,8] [--width 1920 --height 1080 --sh 3]
  (config 5: --splats 50000000 --width 3840 --height 2160 --sh 0)
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

ap = argparse.ArgumentParser()
ap.add_argument("--splats", type=int, default=6_000_000)
ap.add_argument("--worlds", default="1,2,4,8")
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--sh", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--stages", type=int, default=0, help="world size whose per-rank render stage times to print")
ap.add_argument("--link-gbs", type=float, default=76.8, help="modelled xGMI rate per link and direction")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera  # noqa: E402
from gaussian_splat_amd.distributed import HipShardBackend, band_rows, shard_bounds, virtual_exchange  # noqa: E402

W, H = a.width, a.height
sc = S.synthetic_scene(a.splats, seed=a.seed, sh_degree=a.sh, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
opt = Options(sh_degree=a.sh, crop=False, frames_in_flight=1)


def timed(fn, k):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / k


res = {}
for g in [int(x) for x in a.worlds.split(",")]:
    if g == 1:  # the single-GPU frame, one frame in flight (the rows' per-rank pipeline depth)
        r = InstancedSplatRenderer(sc, opt)
        r.initialize(0)
        out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
        ms = timed(lambda: r.render(V, P, W, H, out=out), a.frames)
        r.set_frames_in_flight(2)  # (the bench's single-GPU frame: two in flight)
        ms2 = timed(lambda: r.render(V, P, W, H, out=out), a.frames)
        res[1] = {"frame_ms": round(ms, 4), "frame_ms_2_in_flight": round(ms2, 4),
                  "pairs": int(r.last_stats()["pairs"])}
        print(f"[rows_probe] world 1: {ms:.4f} ms (2 in flight: {ms2:.4f})", file=sys.stderr, flush=True)
        del r, out
        torch.cuda.empty_cache()
        continue
    bes = []
    for rk in range(g):
        b, e = shard_bounds(sc.n, g, rk)
        bes.append(HipShardBackend(sc.subset(slice(b, e)), rk, g, b, opt, 0))
    xb = bes[0].xbytes

    def frame(times=None):
        """One frame of every rank in the multi-process order: all projects,
        the exchange by slicing, all renders; per-call times when asked."""
        sends = []
        for be in bes:
            t = time.perf_counter()
            sends.append(be.project(V, P, W, H))  # (waits for its counts: host read)
            torch.cuda.synchronize()
            if times is not None:
                times["p"][be.rank].append((time.perf_counter() - t) * 1e3)
        recvs, nrecs = [], []
        for dst, (recv, nrec) in enumerate(virtual_exchange(sends, bes[0].xregions, g)):
            nrecs.append(nrec)
            recvs.append(recv if nrec else bes[dst].empty(xb))
        torch.cuda.synchronize()
        for be, rv, m in zip(bes, recvs, nrecs):
            t = time.perf_counter()
            be.render(rv, m, W, H)
            torch.cuda.synchronize()
            if times is not None:
                times["r"][be.rank].append((time.perf_counter() - t) * 1e3)
        return sends, recvs, nrecs

    for _ in range(3):
        frame()
    times = {"p": [[] for _ in range(g)], "r": [[] for _ in range(g)]}
    for _ in range(a.frames):
        sends, recvs, nrecs = frame(times)
    proj_ms = [float(np.median(x)) for x in times["p"]]
    render_ms = [float(np.median(x)) for x in times["r"]]
    pairs = [int(be.r.last_stats()["pairs"]) for be in bes]
    # a rank's pipelined compute as ShardedRenderer(pipeline=True) queues it
    # on its own stream: projection k+1, then the render of frame k, back to
    # back, with the render's composite on a second stream beside the next
    # projection (gs_shard_render_split; the exchange and the gather on their
    # own streams and links are not run here); the received records of the
    # last frame reused
    pipe_ms = []
    if g > 1:
        cs, ccs = torch.cuda.Stream(), torch.cuda.Stream()
        held = [rv.clone() for rv in recvs]
        torch.cuda.synchronize()
        for be, rv, m in zip(bes, held, nrecs):
            def step(k, be=be, rv=rv, m=m):
                with torch.cuda.stream(cs):
                    be.project(V, P, W, H, slot=k & 1)
                    be.render(rv, m, W, H, composite_stream=ccs)
            for k in range(10):
                step(k)
            torch.cuda.synchronize()
            runs = []  # (the median of three runs: the first frames of a rank can hit allocator growth)
            for _ in range(3):
                t = time.perf_counter()
                for k in range(a.frames):
                    step(k)
                torch.cuda.synchronize()
                runs.append((time.perf_counter() - t) * 1e3 / a.frames)
            pipe_ms.append(float(np.median(runs)))
        del held
    # bytes: records to every other rank (all_to_all) and the band to rank 0 (gather)
    sent = [sum(c for d, c in enumerate(sends[r][1]) if d != r) * xb for r in range(g)]
    max_peer = [max([c for d, c in enumerate(sends[r][1]) if d != r] or [0]) * xb for r in range(g)]
    band_bytes = band_rows(H, g) * W * 16
    link = a.link_gbs * 1e6  # bytes per ms
    model = [proj_ms[r] + max_peer[r] / link + render_ms[r] + (band_bytes / link if r else 0.0) for r in range(g)]
    # two frames in flight (ShardedRenderer(pipeline=True)): frame k's record
    # exchange runs while the rank renders and gathers frame k-1 and projects
    # frame k+1, and the rank computes on its own stream, so neither the
    # exchange nor its band's transfer to rank 0 (waited for on the caller's
    # stream) holds up its next frame: a rank's period is the longer of its
    # compute and its busiest link (to rank 0: the largest per-peer exchange
    # plus the band; rank 0 takes the bands over separate links)
    pipe = [max(pipe_ms[r] if pipe_ms else proj_ms[r] + render_ms[r], (max_peer[r] + (band_bytes if r else 0)) / link,
                band_bytes / link) for r in range(g)]
    res[g] = {"project_ms": [round(x, 4) for x in proj_ms], "render_ms": [round(x, 4) for x in render_ms],
              "compute_max_ms": round(max(p + q for p, q in zip(proj_ms, render_ms)), 4),
              "pipelined_compute_ms": [round(x, 4) for x in pipe_ms],
              "records_received": nrecs, "pairs": pairs, "bytes_sent": sent, "bytes_max_peer": max_peer,
              "band_bytes": band_bytes,
              "link_model_ms": round(max(model), 4), "pipelined_model_ms": round(max(pipe), 4)}
    print(f"[rows_probe] world {g}: compute max {res[g]['compute_max_ms']:.4f} ms  project "
          f"{[round(x, 3) for x in proj_ms]}  render {[round(x, 3) for x in render_ms]}  sent MB "
          f"{[round(x / 1e6, 1) for x in sent]}  pipelined compute {[round(x, 3) for x in pipe_ms]}  "
          f"link model {res[g]['link_model_ms']:.4f} ms  pipelined "
          f"{res[g]['pipelined_model_ms']:.4f} ms", file=sys.stderr, flush=True)
    if g == a.stages:
        for be, rv, m in zip(bes, recvs, nrecs):
            be.r.set_stage_timing(1)
            for _ in range(3):
                be.project(V, P, W, H)
                be.render(rv, m, W, H)
            st = be.r.last_stats()
            print(f"[rows_probe] world {g} rank {be.rank}: " + " ".join(
                f"{k[3:]}={st[k]:.4f}" for k in st if k.startswith("ms_")) + f" binning={st.get('binning')}",
                file=sys.stderr, flush=True)
    del bes, sends, recvs
    torch.cuda.empty_cache()
print(json.dumps({"splats": a.splats, "frame": [W, H], "sh_degree": a.sh,
                  "scheme": "rows (splat-index shards, bin-row ownership; virtual ranks on one GPU)",
                  "note": ("per-rank gs_shard_project (preprocess + pack, includes its host read of the counts) and "
                           "gs_shard_render (unpack + bin/sort + composite of the owned rows), one frame in flight; "
                           f"exchange and gather bytes recorded, priced by link_model_ms at {a.link_gbs} GB/s per "
                           "link and direction (a model, not a measurement); pipelined_model_ms: two frames in "
                           "flight, the rank on its own compute stream: max(pipelined_compute (projection k+1 and "
                           "render k back to back, the composite on a second stream), largest per-peer exchange + "
                           "band)"),
                  "worlds": res}))
