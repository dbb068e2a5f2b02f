#!/usr/bin/env python3
"""Bin list sizes of the bench frame (bin-first), to size the per-bin sort."""
import numpy as np, sys
sys.path.insert(0, ".")
from gaussian_splat_amd import scene as S
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera
W, H = 1920, 1080
sc = S.synthetic_scene(6_000_000, seed=1000, sh_degree=3, aspect=W / H)
cam = default_camera(W, H)
r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False, binning="bin_first"))
r.initialize(0)
r.render_host(cam.getViewMatrix(), cam.getProjectionMatrix(), W, H)
keys, vals = r.sorted_pairs()
bins = np.bincount(keys.astype(np.int64), minlength=60 * 34)
nz = bins[bins > 0]
print("bins", len(bins), "nonzero", len(nz), "P", bins.sum())
print("mean", nz.mean(), "pcts", np.percentile(nz, [0, 10, 25, 50, 75, 90, 99, 100]))
print("over 8192:", (bins > 8192).sum(), "pairs in them", bins[bins > 8192].sum())
srt = np.sort(bins)[::-1]
print("top 20", srt[:20])
