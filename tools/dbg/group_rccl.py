#!/usr/bin/env python3
"""Debug: the C-ABI group over the real RCCL on this one-GPU box.
  python tools/dbg/group_rccl.py WORLD SCHEME [pipe]
WORLD ranks all on device 0; prints the frames' differing words against the
1-GPU frame."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402

from conftest import orbit_views  # noqa: E402
from gaussian_splat_amd import InstancedSplatRenderer, Options, ShardedGroup  # noqa: E402
from gaussian_splat_amd import scene as S  # noqa: E402

world, scheme = int(sys.argv[1]), sys.argv[2]
pipe = len(sys.argv) > 3 and sys.argv[3] == "pipe"
t0 = time.time()
W, H = 640, 400
sc = S.activate(S.synthetic_raw(60000, seed=111, aspect=W / H, rest=True), 3)
r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False))
r.initialize(0)
g = ShardedGroup(r, world, replicated=scheme == "bands")
print(f"[group_rccl {time.time() - t0:6.2f}s] initialize world {world} {scheme}", flush=True)
g.initialize([0] * world, "rccl")
print(f"[group_rccl {time.time() - t0:6.2f}s] transport {g.transport}", flush=True)
if scheme != "bands":
    g.set_scheme(scheme)
for k, (V, P) in enumerate(orbit_views(W, H, 3)):
    a = g.render_host(V, P, W, H)
    ref = r.render_host(V, P, W, H)
    print(f"[group_rccl {time.time() - t0:6.2f}s] frame {k} differing words",
          int(np.count_nonzero(a.view(np.uint32) != ref.view(np.uint32))), flush=True)
g.close()
print("done", flush=True)
