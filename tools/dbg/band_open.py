"""Debug: per-frame state of a replicated-scene band render (world 2, rank 0/1, still camera)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch
from gaussian_splat_amd import scene as S
from gaussian_splat_amd.api import Options, default_camera
from gaussian_splat_amd.distributed import HipBandBackend
W, H = 1920, 1080
sc = S.synthetic_scene(6_000_000, seed=2, sh_degree=3, aspect=W / H)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
for fif in (2, 1):
    for r in (0, 1):
        be = HipBandBackend(sc, r, 2, Options(sh_degree=3, crop=False, frames_in_flight=fif), 0)
        for k in range(12):
            be.render(V, P, W, H)
            torch.cuda.synchronize()
            st = be.r.last_stats()
            if k in (0, 1, 2, 5, 11):
                print(f"fif {fif} rank {r} frame {k}: open {st['open_tiles']} front {st['front_only']} dilate {st['cut_dilate']} "
                      f"cut {st['cut_frame']} pairs {st['pairs']} sorted {st['pairs_sorted']} binning {st['binning']}", flush=True)
        del be
        torch.cuda.empty_cache()
