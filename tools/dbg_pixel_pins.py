"""Debug: device vs oracle vs float64 pin for each k_pin splat (GPU)."""
import json, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import pixel_pins as PX
from oracle import oracle_py as O
from gaussian_splat_amd import InstancedSplatRenderer, Options
KP = json.loads((ROOT / "tests/golden/known_answers.json").read_text())["k_pins"]
W, H = KP["width"], KP["height"]
for name, pin in sorted(PX.alpha_pins().items()):
    sp = next(s for s in KP["splats"] if s["name"] == name)
    cam = KP["cameras"][sp["camera"]]
    V, P = np.array(cam["view"], np.float32), np.array(cam["proj"], np.float32)
    sc = PX.pin_scene(sp)
    for binning in ("depth_first", "bin_first"):
        r = InstancedSplatRenderer(sc, Options(binning=binning, crop=False)); r.initialize(0)
        img = r.render_host(V, P, W, H)
        ref, _ = O.render(sc, V, P, W, H)
        d = np.abs(img - ref).max(axis=-1)
        rec, dk, nt = r.project_host(V, P, W, H)
        orec, odk, ont = O.project(sc, V, P, W, H)
        same = rec.tobytes() == orec.tobytes()
        ys, xs = np.nonzero(d)
        print(name, binning, "max|dev-ora|", float(d.max()), "ndiff", len(ys), "rec bitexact", same,
              "first", list(zip(xs[:5].tolist(), ys[:5].tolist())), "rect", hex(int(rec[0]['rect_lo'])), hex(int(rec[0]['rect_hi'])),
              hex(int(orec[0]['rect_lo'])), hex(int(orec[0]['rect_hi'])), flush=True)
