#!/usr/bin/env python3
"""Per-frame binning-order log over a camera path.

Renders K frames of the bench scene with every stage timed (an event between
stages, one frame in flight so each frame's stats are its own) and prints, per
frame, the binning order the model picked, P, the pairs the front lists kept,
and the duplicate / sort / composite stage times; then the same with the
order forced each way, so the model's choice can be checked frame by frame.

  python tools/binning_probe.py [--profile heavy] [--camera orbit] [--frames 40]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splats", type=int, default=6_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--sh", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--profile", default="heavy", choices=["uniform", "heavy"])
    ap.add_argument("--camera", default="orbit", choices=["fixed", "orbit"])
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    import numpy as np
    import torch

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera

    W, H = a.width, a.height
    sc = S.activate(S.synthetic_raw(a.splats, seed=a.seed, aspect=W / H, rest=a.sh > 0, profile=a.profile), a.sh)
    cam = default_camera(W, H)
    proj = cam.getProjectionMatrix()
    views = []
    for _ in range(a.frames):
        views.append(cam.getViewMatrix())
        if a.camera == "orbit":
            cam.orbit(0.01)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    report = {"config": vars(a), "runs": {}}
    for binning in ("default", "bin_first", "depth_first"):
        r = InstancedSplatRenderer(sc, Options(sh_degree=a.sh, crop=False, stage_timing=1, binning=binning,
                                               frames_in_flight=1))
        r.initialize(0)
        rows = []
        for k, V in enumerate(views):
            r.render(V, proj, W, H, out=out)
            torch.cuda.synchronize()
            st = r.last_stats()
            rows.append({"frame": k, "binning": {1: "depth", 2: "bin"}.get(int(st["binning"]), "?"),
                         "pairs": int(st["pairs"]), "sorted": int(st["pairs_sorted"]),
                         "open": int(st["open_tiles"]), "dup": round(st["ms_duplicate"], 4),
                         "depth_sort": round(st["ms_depth_sort"], 4), "sort": round(st["ms_sort"], 4),
                         "composite": round(st["ms_composite"], 4), "total": round(st["ms_total"], 4)})
        r.close()
        del r
        torch.cuda.synchronize()
        tot = [x["total"] for x in rows[2:]]
        report["runs"][binning] = {"frames": rows, "mean_total_ms": float(np.mean(tot)),
                                   "bin_first_frames": sum(x["binning"] == "bin" for x in rows)}
        print(f"{binning:12s} mean total {np.mean(tot):.4f} ms  bin-first frames "
              f"{report['runs'][binning]['bin_first_frames']}/{len(rows)}", flush=True)
        if binning == "default":
            for x in rows:
                print("  ", json.dumps(x), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
