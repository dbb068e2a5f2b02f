"""How the pipelined frame time settles after start-up: blocks of B frames timed
back to back (synchronised between blocks), from the first frame on."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gaussian_splat_amd import scene as S  # noqa: E402
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera  # noqa: E402

B, NB = int(sys.argv[1]) if len(sys.argv) > 1 else 5, int(sys.argv[2]) if len(sys.argv) > 2 else 30
W, H, N = 1920, 1080, 6_000_000
scene = S.activate(S.synthetic_raw(N, seed=2, aspect=W / H, rest=True), 3)
cam = default_camera(W, H)
view, proj = cam.getViewMatrix(), cam.getProjectionMatrix()
r = InstancedSplatRenderer(scene, Options(mode="tile", sh_degree=3, crop=False, stage_timing=0, frames_in_flight=2))
r.initialize(0)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
torch.cuda.synchronize()
for b in range(NB):
    t0 = time.perf_counter()
    for _ in range(B):
        r.render(view, proj, W, H, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / B
    st = r.last_stats()
    print(f"block {b:2d} frames {b * B:3d}-{b * B + B - 1:3d}: {ms:.4f} ms/frame  front {st['front_only']} "
          f"dilate {st['cut_dilate']} binning {st['binning']} sorted {st['pairs_sorted']}", flush=True)
