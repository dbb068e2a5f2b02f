import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from gaussian_splat_amd import scene as S
from gaussian_splat_amd.api import InstancedSplatRenderer, Options, default_camera
from gaussian_splat_amd.distributed import render_virtual_shards, HipShardBackend, shard_bounds
W, H = 1920, 1080
for n in (200_000, 6_000_000):
    sc = S.synthetic_scene(n, seed=2, sh_degree=3, aspect=W / H)
    cam = default_camera(W, H); V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
    r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False)); r.initialize(0)
    ref = r.render(V, P, W, H).cpu().numpy()
    fr = render_virtual_shards(sc, 2, V, P, W, H, sh_degree=3)
    d = np.abs(fr - ref)
    print(n, "maxdiff", d.max(), "rows differing", np.nonzero(d.max(axis=(1, 2)) > 0)[0][[0, -1]] if d.max() > 0 else None,
          "alpha top/bottom", ref[:540, :, 3].mean(), ref[540:, :, 3].mean(), fr[:540, :, 3].mean(), fr[540:, :, 3].mean(), flush=True)
