import sys, numpy as np
sys.path.insert(0, ".")
from gaussian_splat_amd import scene as S, InstancedSplatRenderer, Options
from gaussian_splat_amd.api import default_camera
sc = S.activate(S.synthetic_raw(10000, seed=0, aspect=1.0), 0)
cam = default_camera(256, 256)
r = InstancedSplatRenderer(sc, Options(mode="tile", sh_degree=0, crop=True)); r.initialize(0)
print("init ok", flush=True)
img = r.render_host(cam.getViewMatrix(), cam.getProjectionMatrix(), 256, 256)
print("render ok", img.mean(), flush=True)
