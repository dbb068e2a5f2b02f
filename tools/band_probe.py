#!/usr/bin/env python3
"""Per-rank compute of the replicated-scene band scheme on one GPU (virtual
ranks): for world g, each rank's gs_band_render time over the whole scene
(mean of K frames after warm-up), and the slowest rank, the compute part of a
g-GPU frame.  The band gather is not run over links here (one GPU): its bytes
per rank are recorded and `gather_link_ms` prices the largest band at the
modelled xGMI rate (one link per sender into rank 0, as rows_probe.py);
`period_model_ms` = max(slowest rank, gather link), the gather of frame k
overlapping frame k+1's render.

  python tools/band_probe.py [--splats 6000000] [--worlds 1,2,4,8] [--width 1920 --height 1080 --sh 3]
  (config 5: --splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4)
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
ap.add_argument("--fif", type=int, default=2, help="frames in flight per rank")
ap.add_argument("--stages", type=int, default=0, help="world size whose per-rank stage times to print (0: off)")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--sh", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--link-gbs", type=float, default=76.8, help="modelled xGMI rate per link and direction")
a = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd.api import Options, default_camera  # noqa: E402
from gaussian_splat_amd.distributed import HipBandBackend  # noqa: E402

W, H = a.width, a.height
sc = S.synthetic_scene(a.splats, seed=a.seed, sh_degree=a.sh, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
opt = Options(sh_degree=a.sh, crop=False, frames_in_flight=a.fif)
res = {}
for g in [int(x) for x in a.worlds.split(",")]:
    per = []
    for r in range(g):
        be = HipBandBackend(sc, r, g, opt, 0)
        for _ in range(10):  # (a new handle: its cuts, buffers and binning choice settle first)
            be.render(V, P, W, H)
        torch.cuda.synchronize()
        runs = []  # (the median of three runs)
        for _ in range(3):
            t = time.perf_counter()
            for _ in range(a.frames):
                be.render(V, P, W, H)
            torch.cuda.synchronize()
            runs.append((time.perf_counter() - t) * 1e3 / a.frames)
        per.append(float(np.median(runs)))
        st = be.r.last_stats()
        del be
        torch.cuda.empty_cache()
    band_rows = -(-((H + 31) // 32) // g)  # 32-px bin rows of the largest band
    band_bytes = min(band_rows * 32, H) * W * 16
    link = band_bytes / (a.link_gbs * 1e6) if g > 1 else 0.0
    res[g] = {"ms_per_rank": [round(x, 4) for x in per], "max_ms": round(max(per), 4),
              "pairs_last_rank": int(st["pairs"]), "band_bytes_max": band_bytes,
              "gather_link_ms": round(link, 4), "period_model_ms": round(max(max(per), link), 4)}
    print(f"[band_probe] world {g}: max {max(per):.4f} ms  ranks {[round(x, 3) for x in per]}", file=sys.stderr,
          flush=True)
if a.stages:
    from dataclasses import replace
    for r in range(a.stages):
        be = HipBandBackend(sc, r, a.stages, replace(opt, stage_timing=1, frames_in_flight=1), 0)
        for _ in range(5):
            be.render(V, P, W, H)
        torch.cuda.synchronize()
        st = be.r.last_stats()
        print(f"[band_probe] world {a.stages} rank {r}: " + " ".join(
            f"{k[3:]}={st[k]:.4f}" for k in st if k.startswith("ms_")), file=sys.stderr, flush=True)
        del be
print(json.dumps({"splats": a.splats, "frame": [W, H], "sh_degree": a.sh, "seed": a.seed,
                  "scheme": "bands (virtual ranks, one GPU)",
                  "note": f"per-rank gs_band_render, {a.fif} frame(s) in flight; the gather is modelled "
                          f"(gather_link_ms: the largest band over one {a.link_gbs} GB/s link), not run",
                  "worlds": res}))
