import sys
sys.path.insert(0, ".")
from gaussian_splat_amd import scene as S
from gaussian_splat_amd import InstancedSplatRenderer, Options, default_camera
w, h = 640, 360
sc = S.synthetic_scene(200000, seed=91, aspect=w / h)
cam = default_camera(w, h)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
for b in ("depth_first", "bin_first"):
    r = InstancedSplatRenderer(sc, Options(binning=b))
    r.initialize(0)
    for k in range(2):
        img = r.render_host(V, P, w, h)
        st = r.last_stats()
        print(b, k, "fetched", st["records_fetched"], "4P", 4 * st["pairs"], "alpha>0.99 share", float((img[..., 3] >= 0.99).mean()))
