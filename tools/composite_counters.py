#!/usr/bin/env python3
"""Composite work counters on the bench workload (debug build):

  python tools/build_variant.py cnt -DGS_COMPOSITE_COUNTERS
  GSPLAT_LIB=ab/cnt.so python tools/composite_counters.py [--splats N]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("--splats", type=int, default=6_000_000)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--sh", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
args = ap.parse_args()

import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd._lib import lib  # noqa: E402
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera  # noqa: E402

W, H = args.width, args.height
scene = S.synthetic_scene(args.splats, seed=args.seed, sh_degree=args.sh, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
r = InstancedSplatRenderer(scene, Options(mode="tile", sh_degree=args.sh, crop=False))
r.initialize(0)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
if hasattr(lib(), "gs_debug_composite_timers"):  # -DGS_COMPOSITE_TIMERS build: phase cycles per wave
    f = lib().gs_debug_composite_timers
    f.argtypes = [C.POINTER(C.c_uint64)]
    buf = (C.c_uint64 * 8)()
    for _ in range(2):
        r.render(V, P, W, H, out=out)
        torch.cuda.synchronize()
        f(buf)
    c = list(buf)
    nw = max(c[7], 1)
    tot = c[6] / nw
    names = ["barrier_count", "staging", "barrier2", "compaction", "walk", "loop tail/prefetch issue"]
    for n, v in zip(names, c[:6]):
        print(f"{n:>26}: {v / nw:10.0f} cyc/wave  {100 * v / nw / tot:5.1f} %")
    print(f"{'wave lifetime':>26}: {tot:10.0f} cyc/wave ({nw} waves)")
    sys.exit(0)
f = lib().gs_debug_composite_counters
f.argtypes = [C.POINTER(C.c_uint64)]
buf = (C.c_uint64 * 20)()
r.render(V, P, W, H, out=out)
torch.cuda.synchronize()
f(buf)
r.render(V, P, W, H, out=out)
torch.cuda.synchronize()
f(buf)
c = list(buf)
st = r.last_stats()
waves, wg = c[0], c[0] // 4
names = ["waves", "batch-max exact 4x4-group walks", "batch-max per-lane walks", "bodies", "bodies w/ covered lane", "wg-batches", "list entries",
         "covered open lanes", "open lanes", "covered lanes", "sum max 4x4-group walks", "sum max 8x4-half walks",
         "sum max lane walks", "sum lane walks", "batch-max rect 4x4-group walks", "batch-max ellipse 4x4-group walks"]
for n, v in zip(names, c):
    print(f"{n:>24}: {v}")
print(f"pairs {st['pairs']}  list/bin {st['pairs'] / (st['tiles']):.0f}")
print(f"per wave: halves {c[1] / waves:.1f}  quarters {c[2] / waves:.1f}  bodies {c[3] / waves:.1f}  "
      f"covered-bodies {c[4] / waves:.1f}  lanes/covered-body {c[7] / max(c[4], 1):.1f}")
print(f"per body: open lanes {c[8] / max(c[3], 1):.1f}  covered lanes {c[9] / max(c[3], 1):.1f}  "
      f"covered+open {c[7] / max(c[3], 1):.1f}")
print(f"per wave walk steps: now {c[3] / waves:.1f}  4x4 groups {c[10] / waves:.1f}  8x4 halves {c[11] / waves:.1f}  "
      f"per-lane max {c[12] / waves:.1f}  per-lane mean {c[13] / waves / 64:.1f}")
print(f"per wave, summed per-batch maxima: exact 4x4 groups {c[1] / waves:.1f}  per-lane {c[2] / waves:.1f}  "
      f"rect 4x4 groups {c[14] / waves:.1f}  ellipse 4x4 groups {c[15] / waves:.1f}")
print(f"staged records {c[16]}  reaching the tile {c[17]} ({c[17] / max(c[16], 1):.3f})  "
      f"per wg: staged {c[16] / wg:.0f}  reaching {c[17] / wg:.0f}")
print(f"per wg: batches {c[5] / wg:.2f}  list {c[6] / wg:.0f}  batches if no exit {c[6] / wg / 256:.2f}")
tf = lib().gs_debug_composite_tile_fetch
tf.argtypes = [C.POINTER(C.c_uint32), C.c_uint]
nt = int(st["tiles"]) * 4
arr = (C.c_uint32 * nt)()
tf(arr, nt)
import numpy as np  # noqa: E402
f = np.frombuffer(arr, dtype=np.uint32).reshape(-1, 4).astype(np.int64)
print(f"records fetched: per tile (sum) {f.sum()}  per bin if a bin's tiles shared one fetch (sum of max) "
      f"{f.max(axis=1).sum()}  ratio {f.max(axis=1).sum() / max(f.sum(), 1):.3f}")
