#!/usr/bin/env python3
"""One rank's pipelined period in the row scheme, on one GPU:
rank r of a world of g virtual ranks projects its splat shard (frame k+1) and
renders the records it received (frame k) back to back on its stream, as
ShardedRenderer(pipeline=True) queues them, with the render's composite on the
same stream (gs_shard_render) or on a second one (gs_shard_render_split, the
next projection beside it).  The records are exchanged once, by slicing
(tools/rows_probe.py), then reused every frame; the exchange and the gather
are not run (they are on their own streams and links).  Prints one JSON line:
ms per frame both ways, per rank.

  python tools/rank_pipe_probe.py [--world 8] [--ranks 0,3] [--splats 6000000 --width 1920 --height 1080 --sh 3]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

ap = argparse.ArgumentParser()
ap.add_argument("--splats", type=int, default=6_000_000)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--ranks", default="0,3")
ap.add_argument("--frames", type=int, default=30)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--sh", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
a = ap.parse_args()

import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd.api import Options, default_camera  # noqa: E402
from gaussian_splat_amd.distributed import HipShardBackend, shard_bounds, virtual_exchange  # noqa: E402

W, H, g = a.width, a.height, a.world
sc = S.synthetic_scene(a.splats, seed=a.seed, sh_degree=a.sh, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
opt = Options(sh_degree=a.sh, crop=False, frames_in_flight=1)
bes = []
for rk in range(g):
    b, e = shard_bounds(sc.n, g, rk)
    bes.append(HipShardBackend(sc.subset(slice(b, e)), rk, g, b, opt, 0))
sends = [be.project(V, P, W, H) for be in bes]
recvs = [(rv.clone() if n else bes[d].empty(bes[0].xbytes), n)
         for d, (rv, n) in enumerate(virtual_exchange(sends, bes[0].xregions, g))]
torch.cuda.synchronize()
del sends
cs, ccs = torch.cuda.Stream(), torch.cuda.Stream()
res = {"world": g, "splats": a.splats, "frame": [W, H], "ranks": {}}
for r in [int(x) for x in a.ranks.split(",")]:
    be, (rv, n) = bes[r], recvs[r]
    out = {}
    for mode in ("one_stream", "split"):
        def frame(k):
            with torch.cuda.stream(cs):
                be.project(V, P, W, H, slot=k & 1)
                be.render(rv, n, W, H, **({"composite_stream": ccs} if mode == "split" else {}))
        for k in range(5):
            frame(k)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(a.frames):
            frame(k)
        torch.cuda.synchronize()
        out[mode] = round((time.perf_counter() - t) * 1e3 / a.frames, 4)
    res["ranks"][r] = out
    print(f"[rank_pipe_probe] world {g} rank {r}: {out}", file=sys.stderr, flush=True)
print(json.dumps(res), flush=True)
