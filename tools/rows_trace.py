#!/usr/bin/env python3
"""Kernel timeline of one virtual rank's row-scheme frame (run under
rocprofv3 --kernel-trace): world g virtual ranks on one GPU, frames in the
multi-process order; prints the kernels of the last frame of rank `--rank`
(project, then render) with their gaps.

  rocprofv3 --kernel-trace -d out -o run --output-format csv -- python tools/rows_trace.py
  python tools/rows_trace.py --analyze out/.../run_kernel_trace.csv
"""
import argparse
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--splats", type=int, default=6_000_000)
ap.add_argument("--analyze", default="")
a = ap.parse_args()

if a.analyze:
    rows = sorted(csv.DictReader(open(a.analyze)), key=lambda r: int(r["Start_Timestamp"]))
    # the last frame: from the last preprocess of rank 0 on (each rank: preprocess, count, scan, copy, pack)
    pre = [i for i, r in enumerate(rows) if "preprocess_kernel" in r["Kernel_Name"]]
    start = pre[-a.world]
    t0 = int(rows[start]["Start_Timestamp"])
    prev = t0
    for r in rows[start:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gs::", "")[:46]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:6.1f}  {name}")
        prev = e
    sys.exit(0)

import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd.api import Options, default_camera  # noqa: E402
from gaussian_splat_amd.distributed import HipShardBackend, shard_bounds, virtual_exchange  # noqa: E402

W, H = 1920, 1080
sc = S.synthetic_scene(a.splats, seed=2, sh_degree=3, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
opt = Options(sh_degree=3, crop=False, frames_in_flight=1)
g = a.world
bes = [HipShardBackend(sc.subset(slice(*shard_bounds(sc.n, g, r))), r, g, shard_bounds(sc.n, g, r)[0], opt, 0)
       for r in range(g)]
for _ in range(5):
    sends = [be.project(V, P, W, H) for be in bes]
    for dst, (recv, nrec) in enumerate(virtual_exchange(sends, bes[0].xregions, g)):
        bes[dst].render(recv if nrec else bes[dst].empty(bes[dst].xbytes), nrec, W, H)
    torch.cuda.synchronize()
print("done")
