#!/usr/bin/env python3
"""Per-wave start/end trace of the composite on the bench workload (debug build):

  python tools/build_variant.py tr -DGS_COMPOSITE_TRACE
  GSPLAT_LIB=ab/tr.so python tools/composite_trace.py [--splats N]

Reports the kernel span, each XCD's span and wave-time, and the resident-wave
profile over time (how long the launch runs below full occupancy: the tail).
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ap = argparse.ArgumentParser()
ap.add_argument("--splats", type=int, default=6_000_000)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--sh", type=int, default=3)
ap.add_argument("--seed", type=int, default=2)
ap.add_argument("--save", default="")
args = ap.parse_args()

import torch  # noqa: E402

from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd._lib import lib  # noqa: E402
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera  # noqa: E402

W, H = args.width, args.height
scene = S.synthetic_scene(args.splats, seed=args.seed, sh_degree=args.sh, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
r = InstancedSplatRenderer(scene, Options(mode="tile", sh_degree=args.sh, crop=False, frames_in_flight=1))
r.initialize(0)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
f = lib().gs_debug_composite_trace
f.argtypes = [C.c_void_p, C.c_uint]
nw = 16 * ((W + 31) // 32) * ((H + 31) // 32)  # 4 tiles per 32x32 bin, 4 waves per tile
buf = np.zeros((nw, 4), dtype=np.uint32)
for _ in range(3):
    r.render(V, P, W, H, out=out)
    torch.cuda.synchronize()
f(buf.ctypes.data, nw)
t0 = buf[:, 0].astype(np.int64)
t1 = buf[:, 1].astype(np.int64)
base = t0.min()
t0 -= base
t1 -= base
xcc = buf[:, 3] & 0xF
hw = buf[:, 2]
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 0x7
span = t1.max()
print(f"waves {nw}  kernel span {span * 10 / 1000:.1f} us (first start -> last end, 10-ns ticks)")
print(f"wave lifetime mean {np.mean(t1 - t0) * 10 / 1000:.1f} us  p50 {np.median(t1 - t0) * 10 / 1000:.1f}  "
      f"p99 {np.percentile(t1 - t0, 99) * 10 / 1000:.1f}  max {(t1 - t0).max() * 10 / 1000:.1f}")
for x in range(8):
    m = xcc == x
    if not m.any():
        continue
    print(f"XCD {x}: waves {m.sum():5d}  start {t0[m].min() * 10 / 1000:6.1f}  end {t1[m].max() * 10 / 1000:6.1f} us  "
          f"wave-us {np.sum(t1[m] - t0[m]) * 10 / 1000:9.0f}  CUs {len(set(zip(se[m].tolist(), cu[m].tolist())))}")
# resident waves over time (1-us bins)
grid = np.arange(0, span + 100, 100)
res = np.zeros(len(grid))
for a, b in zip(t0, t1):
    res[a // 100:(b // 100) + 1] += 1
peak = res.max()
print(f"resident waves: peak {peak:.0f}")
for frac in (0.9, 0.75, 0.5, 0.25):
    below = np.nonzero(res >= frac * peak)[0]
    last = below.max() if len(below) else 0
    print(f"  last us with >= {int(frac * 100)} % of peak resident: {last}  (tail {len(grid) - 1 - last} us)")
print("profile (resident waves per 10 us):", " ".join(f"{int(v)}" for v in res[::10]))
if args.save:
    np.save(args.save, buf)
