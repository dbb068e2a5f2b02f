"""Debug probe: the zoom-out retry scenario of test_front_only_retry_after_zoom_out, per frame:
differing words against the whole-list frame, pairs, front_only (GSPLAT_LIB selects the variant)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
from gaussian_splat_amd import InstancedSplatRenderer, Options, scene as S
from gaussian_splat_amd.api import default_camera

W, H = 800, 450
sc = S.activate(S.synthetic_raw(300000, seed=23, aspect=W / H, rest=False), 0)
views = []
for d in (2.2,) * 5 + (6.0,) * 4 + (4.0,) * 3:
    cam = default_camera(W, H)
    cam.setDistance(d)
    views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
ref = InstancedSplatRenderer(sc, Options(crop=False, binning="bin_first", depth_split=False))
ref.initialize(0)
refs = [ref.render_host(V, P, W, H) for V, P in views]
r = InstancedSplatRenderer(sc, Options(crop=False, binning="bin_first", depth_split=True, frames_in_flight=1))
r.initialize(0)
for k, (V, P) in enumerate(views):
    o = r.render_host(V, P, W, H)
    st = r.last_stats()
    bits = int(np.count_nonzero(o.view(np.uint32) != refs[k].view(np.uint32)))
    print(k, "bits", bits, "pairs", st["pairs"], "front", st["front_only"], "sorted", st["pairs_sorted"],
          "open", st["open_tiles"], flush=True)
