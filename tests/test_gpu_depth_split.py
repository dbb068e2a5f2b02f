"""Two-slab frames (gs_options.depth_split = 1): bin-first frames
built and composited in two depth slabs, the second slab's pairs emitted and
sorted only for the bins the first slab's composite left open.  The per-pixel
operation sequence is the one-slab sequence of tile.metal:239-266 (the first
slab holds every pair below the depth-key cut, so it precedes the rest in S1
order), so the image must be bit-identical to the one-slab frame and to the
oracle, whatever the cut.

Covered: dense scenes (most bins close in the first slab), sparse ones
(every bin stays open), the live-50 rule, SH3, tiny / ragged frames, two
frames in flight over a camera path with growing pair counts, and the cut
pushed to both extremes (GS_DEPTH_SPLIT_FRAC is read once per process, so
the extremes run in child processes)."""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import orbit_views

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _scene(n, seed, sh, aspect, scale=1.0):
    from gaussian_splat_amd import scene as S
    sc = S.activate(S.synthetic_raw(n, seed=seed, aspect=aspect, rest=sh > 0), sh)
    sc.scale *= np.float32(scale)
    return sc


def _pair(sc, **kw):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    out = []
    for split in (True, False):
        r = InstancedSplatRenderer(sc, Options(binning="bin_first", crop=False, depth_split=split, **kw))
        r.initialize(0)
        out.append(r)
    return out


def _bits(a, b):
    return int(np.count_nonzero(np.asarray(a).view(np.uint32) != np.asarray(b).view(np.uint32)))


@pytest.mark.parametrize("n,w,h,mode,sh,scale", [
    (300000, 640, 360, "tile", 0, 1.0),    # dense: most bins close in the first slab
    (300000, 640, 360, "live50", 0, 1.0),
    (120000, 960, 540, "tile", 3, 1.5),
    (8000, 640, 360, "tile", 0, 0.5),      # sparse: nothing saturates, every bin stays open
    (40000, 17, 9, "tile", 0, 1.0),        # ragged single-bin frame
    (5000, 1, 1, "live50", 0, 1.0),
    (200000, 1920, 1080, "tile", 0, 3.0),  # large splats, long lists (> 8192 per bin)
])
def test_two_slab_bitexact(built, n, w, h, mode, sh, scale):
    from oracle import oracle_py as O
    sc = _scene(n, 131 + n % 7, sh, w / h, scale)
    two, one = _pair(sc, mode=mode, sh_degree=sh)
    for V, P in orbit_views(w, h, 2):
        a = two.render_host(V, P, w, h)
        b = one.render_host(V, P, w, h)
        assert _bits(a, b) == 0
        st, so = two.last_stats(), one.last_stats()
        assert st["two_slab"] == 1 and so["two_slab"] == 0
        assert st["pairs"] == so["pairs"] and st["pairs_sorted"] <= st["pairs"]
        assert 0 <= st["open_tiles"] <= 4 * st["tiles"]
        ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode)
        assert _bits(a, ref) == 0
    print(f"{n} @{w}x{h} {mode}: pairs {st['pairs']} sorted {st['pairs_sorted']} open tiles {st['open_tiles']} "
          f"cut {st['depth_cut']:#x}")


def test_two_slab_dense_scene_saves_pairs(built):
    """On the bench-like dense scene most bins close in the first slab: the
    frame sorts well under the one-slab pair count."""
    # the bench scene's coverage per pixel (6M splats @1080p) at a quarter of
    # the pixels: 1.5M splats of twice the size @960x540
    sc = _scene(1_500_000, 5, 0, 16 / 9, scale=2.0)
    two, one = _pair(sc)
    V, P = orbit_views(960, 540, 1)[0]
    assert _bits(two.render_host(V, P, 960, 540), one.render_host(V, P, 960, 540)) == 0
    st = two.last_stats()
    assert st["pairs_sorted"] < 0.8 * st["pairs"], st
    assert st["open_tiles"] < 2 * st["tiles"], st  # fewer than half of the 16x16 tiles stay open


def test_two_slab_pipelined_camera_path(built):
    """Two frames in flight: the second slab's lists are built on the
    composite stream while the side stream projects the next frame into the
    other buffer set (rects, cut and scratch per set).  A camera path whose
    pair count grows makes the first frames re-queue with larger buffers."""
    import torch

    from gaussian_splat_amd import InstancedSplatRenderer, Options, default_camera
    W, H = 800, 450
    sc = _scene(250000, 17, 3, W / H)
    views = []
    for d in (6.0, 4.0, 2.5, 5.0, 3.0):
        cam = default_camera(W, H)
        cam.setDistance(d)
        cam.orbit(0.2 * d, 0.05)
        views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    ref = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False, binning="bin_first", depth_split=False))
    ref.initialize(0)
    refs = [ref.render_host(V, P, W, H) for V, P in views]
    r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False, binning="bin_first", frames_in_flight=2,
                                           depth_split=True))
    r.initialize(0)
    outs = [r.render(V, P, W, H) for V, P in views for _ in range(2)]
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert _bits(o.cpu().numpy(), refs[k // 2]) == 0, k
    assert r.last_stats()["two_slab"] == 1


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from test_gpu_depth_split import _scene, _pair, _bits
from conftest import orbit_views
sc = _scene(200000, 9, 0, 16 / 9)
two, one = _pair(sc)
V, P = orbit_views(640, 360, 1)[0]
a = two.render_host(V, P, 640, 360); b = one.render_host(V, P, 640, 360)
st = two.last_stats()
assert st["two_slab"] == 1 and _bits(a, b) == 0, (st, _bits(a, b))
print("ok", st["pairs"], st["pairs_sorted"], st["open_tiles"], hex(st["depth_cut"]))
"""


@pytest.mark.parametrize("frac", ["0.0", "0.999", "0.6"])
def test_two_slab_cut_extremes(built, frac):
    """The cut at the front (the first slab holds the farthest bucket only),
    at the back (nearly everything in the first slab) and in between: the
    same image every time."""
    env = dict(os.environ, GS_DEPTH_SPLIT_FRAC=frac)
    code = _CHILD.format(root=str(ROOT), tests=str(ROOT / "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    print(frac, p.stdout.strip())
