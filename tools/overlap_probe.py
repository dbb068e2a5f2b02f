#!/usr/bin/env python3
"""How much a third frame in flight could gain: two renderer handles on the
same scene, each pipelined (frames_in_flight 2) on its own composite stream,
rendering alternate frames, so one handle's projection can run under the other
handle's chain (scan .. per-bin sort).  Prints one JSON line: ms per frame of
one handle alone and of the two alternating (the same camera, the same frames).

  python tools/overlap_probe.py [--config 1080p|4k|50m] [--steps 40] [--warmup 60]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

CONFIGS = {"1080p": (6_000_000, 1920, 1080, 3), "4k": (6_000_000, 3840, 2160, 3), "50m": (50_000_000, 3840, 2160, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1080p", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera

    N, W, H, sh = CONFIGS[args.config]
    scene = S.activate(S.synthetic_raw(N, seed=0, aspect=W / H, rest=sh > 0), sh)
    cam = default_camera(W, H)
    view, proj = cam.getViewMatrix(), cam.getProjectionMatrix()
    rs, outs, streams = [], [], []
    for _ in range(2):
        r = InstancedSplatRenderer(scene, Options(sh_degree=sh, crop=False, stage_timing=0, frames_in_flight=2))
        r.initialize(0)
        rs.append(r)
        outs.append(torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0"))
        streams.append(torch.cuda.Stream())
    del scene

    def run(k, which):
        for i in range(k):
            j = which[i % len(which)]
            rs[j].render(view, proj, W, H, out=outs[j], stream=streams[j].cuda_stream)

    def timed(which):
        run(args.warmup, which)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps, which)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / args.steps

    res = {"config": args.config, "steps": args.steps, "one": [], "two": []}
    for _ in range(args.rounds):
        res["one"].append(round(timed([0]), 4))
        res["two"].append(round(timed([0, 1]), 4))
    a = torch.equal(outs[0], outs[1])
    res["same_image"] = bool(a)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
