#!/usr/bin/env python3
"""Per-workgroup timeline of the strip composite (debug build only).

Build:  python tools/build_variant.py trace -DGS_COMPOSITE_TRACE
Run:    GSPLAT_LIB=ab/trace.so python tools/composite_trace.py [--frames 5]

Renders the bench frame unpipelined, reads each strip workgroup's start/end
(s_memrealtime, 100 MHz), bin-pair slot and fetched records of the last
frame's front-list composite (gs_debug_composite_trace), and prints the
kernel span, the workgroup-duration distribution, the resident-workgroup
count over time (occupancy: 8 per CU = 2048 slots) and the ramp / drain.
"""
from __future__ import annotations

import argparse
import ctypes as C
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
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd._lib import lib
    from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera

    W, H = a.width, a.height
    sc = S.activate(S.synthetic_raw(a.splats, seed=a.seed, aspect=W / H, rest=a.sh > 0), a.sh)
    cam = default_camera(W, H)
    V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
    r = InstancedSplatRenderer(sc, Options(sh_degree=a.sh, crop=False, frames_in_flight=1))
    r.initialize(0)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    for _ in range(a.frames):
        r.render(V, P, W, H, out=out)
    torch.cuda.synchronize()
    L = lib()
    f = L.gs_debug_composite_trace
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int]
    tiles = (W + 31) // 32 * ((H + 31) // 32)
    nwg = 2 * tiles
    buf = np.zeros(4 * 65536, dtype=np.uint64)
    assert f(buf.ctypes.data, buf.size) == 0
    t = buf[: 4 * nwg].reshape(nwg, 4).astype(np.int64)
    t0, t1 = t[:, 0], t[:, 1]
    base = t0.min()
    s, e = (t0 - base) * 10.0 / 1000.0, (t1 - base) * 10.0 / 1000.0  # us (100 MHz ticks)
    dur = e - s
    span = e.max()
    grid = np.linspace(0, span, 200)
    resident = np.array([np.count_nonzero((s <= x) & (e > x)) for x in grid])
    full = 2048
    occ = float(np.trapz(resident, grid) / (span * full))
    last_start = float(s.max())
    rep = {"workgroups": int(nwg), "span_us": round(float(span), 2),
           "dur_us": {"mean": round(float(dur.mean()), 2), "p10": round(float(np.percentile(dur, 10)), 2),
                      "p50": round(float(np.percentile(dur, 50)), 2), "p90": round(float(np.percentile(dur, 90)), 2),
                      "max": round(float(dur.max()), 2)},
           "mean_resident_frac": round(occ, 3),
           "last_start_us": round(last_start, 2),
           "drain_us": round(float(span - last_start), 2),
           "time_to_full_us": round(float(grid[np.argmax(resident >= 0.95 * resident.max())]), 2),
           "max_resident": int(resident.max()),
           "dur_vs_fetched_corr": round(float(np.corrcoef(dur, t[:, 3])[0, 1]), 3),
           "by_dispatch_order": [round(float(dur[i:i + nwg // 10].mean()), 2) for i in range(0, nwg, nwg // 10)],
           "resident_curve": [int(x) for x in resident[::10]]}
    print(json.dumps(rep, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
