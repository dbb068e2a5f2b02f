"""Depth-cut frames (gs_options.depth_split = 1).

A frame's lists (bin-first or depth-first binning) hold only the pairs whose depth key lies at or
ahead of their bin's cut (S1 order, tile.metal:239-249), the key at which
the bin's tiles finished in the set's previous frame, plus a margin.  A tile
those lists leave open keeps its per-pixel state and finishes with the rest
of its bin's pairs (the fallback lists).  Whatever the cuts, each pixel sees
the full list's operation sequence (tile.metal:251-266 / 50layer.metal:
208-222), so every frame must be bit-identical to the whole-list frame and
to the oracle.

Covered: static and moving cameras (the cuts then lag the view), camera
jumps that leave many tiles open, sparse scenes that never saturate, the
live-50 rule, SH3, BGRA8 output, one and two frames in flight, resolution
changes, lists over 8192 pairs, and a zero margin (GS_CUT_MARGIN, read once
per process, so in a child process)."""
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


def _pair(sc, binning="bin_first", **kw):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    out = []
    for cut in (True, False):
        r = InstancedSplatRenderer(sc, Options(binning=binning, crop=False, depth_split=cut, **kw))
        r.initialize(0)
        out.append(r)
    return out


def _bits(a, b):
    return int(np.count_nonzero(np.asarray(a).view(np.uint32) != np.asarray(b).view(np.uint32)))


def _path(w, h, kind, n):
    """Camera path: 'still' (one view), 'orbit' (small steps, the cuts lag
    by a frame), 'jump' (large turns and zooms: stale cuts everywhere)."""
    from gaussian_splat_amd.api import default_camera
    views = []
    for k in range(n):
        cam = default_camera(w, h)
        if kind == "orbit":
            cam.orbit(0.02 * k, 0.005 * k)
        elif kind == "jump":
            cam.setDistance((6.0, 2.5, 4.0, 1.8, 5.0, 3.0)[k % 6])
            cam.orbit(0.9 * k, 0.15 * (k % 3))
        views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    return views


@pytest.mark.parametrize("n,w,h,mode,sh,scale,path,binning", [
    (300000, 640, 360, "tile", 0, 1.0, "still", "bin_first"),
    (300000, 640, 360, "tile", 0, 1.0, "orbit", "bin_first"),
    (300000, 640, 360, "live50", 0, 1.0, "jump", "bin_first"),
    (120000, 960, 540, "tile", 3, 1.5, "jump", "bin_first"),
    (8000, 640, 360, "tile", 0, 0.5, "orbit", "bin_first"),      # sparse: nothing saturates, no list is cut
    (40000, 17, 9, "tile", 0, 1.0, "jump", "bin_first"),         # ragged single-bin frame
    (5000, 1, 1, "live50", 0, 1.0, "orbit", "bin_first"),
    (200000, 1920, 1080, "tile", 0, 3.0, "jump", "bin_first"),   # large splats, long lists (> 8192 per bin)
    # depth-first binning (4K and 50M frames): the pair keys carry the sorted depth keys
    (300000, 640, 360, "tile", 0, 1.0, "orbit", "depth_first"),
    (300000, 640, 360, "live50", 0, 1.0, "jump", "depth_first"),
    (120000, 960, 540, "tile", 3, 1.5, "jump", "depth_first"),
    (40000, 17, 9, "tile", 0, 1.0, "jump", "depth_first"),
    (200000, 1920, 1080, "tile", 0, 3.0, "jump", "depth_first"),
])
def test_depth_cuts_bitexact(built, n, w, h, mode, sh, scale, path, binning):
    from oracle import oracle_py as O
    sc = _scene(n, 131 + n % 7, sh, w / h, scale)
    cut, whole = _pair(sc, binning=binning, mode=mode, sh_degree=sh)
    opened = 0
    for k, (V, P) in enumerate(_path(w, h, path, 6)):
        a = cut.render_host(V, P, w, h)
        b = whole.render_host(V, P, w, h)
        assert _bits(a, b) == 0, k
        st, so = cut.last_stats(), whole.last_stats()
        assert st["cut_frame"] == 1 and so["cut_frame"] == 0
        # (front lists: dkey <= cut; fallback lists: a subset of the rest)
        assert st["pairs"] == so["pairs"] and st["pairs_sorted"] <= st["pairs"]
        assert 0 <= st["open_tiles"] <= 16 * st["tiles"]  # (8x8 quadrants left open)
        opened += st["open_tiles"]
        if k in (0, 5):
            ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode)
            assert _bits(a, ref) == 0, k
    print(f"{n} @{w}x{h} {mode} {path} {binning}: pairs {st['pairs']} sorted {st['pairs_sorted']} "
          f"open tiles (sum) {opened}")


@pytest.mark.parametrize("binning", ["bin_first", "depth_first"])
def test_depth_cuts_still_camera_saves_pairs(built, binning):
    """The bench-like dense scene under a still camera: from the third frame
    on, the lists hold a fraction of the pairs and no tile is left open."""
    # the bench scene's coverage per pixel (6M splats @1080p) at a quarter of
    # the pixels: 1.5M splats of twice the size @960x540
    sc = _scene(1_500_000, 5, 0, 16 / 9, scale=2.0)
    cut, whole = _pair(sc, binning=binning)
    V, P = orbit_views(960, 540, 1)[0]
    ref = whole.render_host(V, P, 960, 540)
    for k in range(4):
        assert _bits(cut.render_host(V, P, 960, 540), ref) == 0, k
    st = cut.last_stats()
    assert st["pairs_sorted"] < 0.6 * st["pairs"], st
    assert st["open_tiles"] == 0, st
    # bin-first frames with cuts write only their front pairs
    assert st["front_only"] == (1 if binning == "bin_first" else 0), st


@pytest.mark.parametrize("binning", ["bin_first", "depth_first"])
def test_depth_cuts_jump_opens_tiles(built, binning):
    """One frame in flight: each frame uses the previous frame's cuts.  A
    view that moves the scene nearer after a still stretch leaves tiles open
    (their saturation lies behind the old cuts); the fallback lists finish
    them, bit for bit."""
    from gaussian_splat_amd.api import default_camera
    W, H = 640, 360
    sc = _scene(400000, 23, 0, W / H, scale=1.2)
    cut, whole = _pair(sc, binning=binning)
    far = default_camera(W, H)
    far.setDistance(7.0)
    near = default_camera(W, H)
    near.setDistance(2.0)
    near.orbit(0.4, 0.1)
    opened = front_opened = 0
    for cam in (far, far, far, near, near, far, near):
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        assert _bits(cut.render_host(V, P, W, H), whole.render_host(V, P, W, H)) == 0
        st = cut.last_stats()
        opened += st["open_tiles"]
        # (a front-only frame that leaves tiles open: the fallback pairs were
        # regenerated from the splats' rects, launch_fallback_pairs)
        front_opened += st["open_tiles"] if st["front_only"] else 0
    assert opened > 0
    if binning == "bin_first":
        assert front_opened > 0


def test_depth_cuts_bgra8_and_resolution_change(built):
    """BGRA8 output in depth-cut frames (the open tiles' states live in their
    own buffer), and a resolution change (the cuts start over)."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    sc = _scene(250000, 31, 0, 16 / 9)
    cut, whole = _pair(sc)
    for (w, h) in ((640, 360), (640, 360), (800, 450), (800, 450), (640, 360), (640, 360)):
        for V, P in _path(w, h, "orbit", 2):
            assert _bits(cut.render_bgra8_host(V, P, w, h), whole.render_bgra8_host(V, P, w, h)) == 0
            assert _bits(cut.render_host(V, P, w, h), whole.render_host(V, P, w, h)) == 0


@pytest.mark.parametrize("binning", ["bin_first", "depth_first"])
def test_depth_cuts_pipelined_camera_path(built, binning):
    """Two frames in flight: a frame's cuts come from the frame before last
    (its buffer set); its fallback lists are built on the composite stream
    while the side stream projects the next frame into the other set (rects,
    open flags, cut tables per set).  A camera path whose pair count grows
    makes the first frames re-queue with larger buffers."""
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
    r = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False, binning=binning, frames_in_flight=2,
                                           depth_split=True))
    r.initialize(0)
    outs = [r.render(V, P, W, H).clone() for V, P in views for _ in range(3)]
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert _bits(o.cpu().numpy(), refs[k // 3]) == 0, k
    assert r.last_stats()["cut_frame"] == 1


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from test_gpu_depth_split import _scene, _pair, _bits, _path
sc = _scene(200000, 9, 0, 16 / 9)
cut, whole = _pair(sc)
opened = 0
for V, P in _path(640, 360, "orbit", 8):
    a = cut.render_host(V, P, 640, 360); b = whole.render_host(V, P, 640, 360)
    st = cut.last_stats()
    assert st["cut_frame"] == 1 and _bits(a, b) == 0, (st, _bits(a, b))
    opened += st["open_tiles"]
print("ok", st["pairs"], st["pairs_sorted"], opened)
"""


@pytest.mark.parametrize("margin", ["0", "1000"])
def test_depth_cuts_margin_extremes(built, margin):
    """No margin (the cuts sit on the last record each tile staged, so a
    moving camera opens tiles every frame) and a wide one: the same image
    every time."""
    env = dict(os.environ, GS_CUT_MARGIN=margin)
    code = _CHILD.format(root=str(ROOT), tests=str(ROOT / "tests"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    print(margin, p.stdout.strip())


@pytest.mark.parametrize("world,w,h,binning,path,table", [
    (2, 640, 360, "bin_first", "orbit", None),
    (3, 640, 360, "depth_first", "jump", None),
    (4, 960, 540, "default", "orbit", "interleaved"),
    (2, 640, 360, "bin_first", "jump", "switch"),   # the owner table changes mid-path: cuts start over
    (3, 100, 40, "bin_first", "orbit", None),       # two bin rows, three ranks: one owns none
    (2, 960, 540, "depth_first", "still", None),    # dense, still: the cuts save pairs on every rank
    (3, 960, 540, "bin_first", "still", "interleaved"),
])
def test_depth_cuts_virtual_ranks(built, world, w, h, binning, path, table):
    """Rank renders of the row scheme carry the depth cuts of
    their owned bins from frame to frame (quadrant records and cuts indexed by
    global bin, pixel states by global pixel; another rank's bins get no
    fallback): every assembled frame is bit-identical to the single-GPU
    whole-list frame."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd.distributed import VirtualShards
    dense = path == "still"  # (the bench scene's coverage per pixel, as in the still-camera test above)
    sc = _scene(1_500_000 if dense else 300000, 41 + world, 0, w / h, scale=2.0 if dense else 1.3)
    ref = InstancedSplatRenderer(sc, Options(crop=False, depth_split=False))
    ref.initialize(0)
    R = (h + 31) // 32
    inter = np.array([r % world for r in range(R)], np.uint8)
    vs = VirtualShards(sc, world, Options(crop=False, depth_split=True, binning=binning), 0,
                       inter if table == "interleaved" else None)
    saved = [0] * world
    for k, (V, P) in enumerate(_path(w, h, path, 4 if dense else 6)):
        if table == "switch" and k == 3:
            vs.set_rows(inter)
        a = vs.render(V, P, w, h).cpu().numpy()
        assert _bits(a, ref.render_host(V, P, w, h)) == 0, k
        for be in vs.backends:
            st = be.r.last_stats()
            assert (st["cut_frame"] == 1 or st["pairs"] == 0) and st["pairs_sorted"] <= st["pairs"], (k, be.rank, st)
            saved[be.rank] = st["pairs"] - st["pairs_sorted"]
    if dense:  # (the last frame)
        assert min(saved) > 0, saved


def test_binning_model_heavy_orbit_picks_bin_first(built):
    """on a heavy-tailed scene under an orbiting camera the
    binning-order model (renderer.cpp bin_first_order) must pick bin-first
    once it has seen a frame: the index-order duplicate emits
    wave-cooperatively (scan.hip coop_emit), so large splats no longer make it
    slower than the depth sort (round 5, profiles/r05/binning_heavy_orbit.json:
    0.92 against 1.05 ms a frame at 6M splats).  Every frame stays
    bit-identical to the forced depth-first frame."""
    import torch

    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd.api import default_camera
    W, H = 1280, 720
    sc = S.activate(S.synthetic_raw(1_500_000, seed=9, aspect=W / H, rest=True, profile="heavy"), 3)
    cam = default_camera(W, H)
    P = cam.getProjectionMatrix()
    auto = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False))
    auto.initialize(0)
    ref = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=False, binning="depth_first"))
    ref.initialize(0)
    picks = []
    for k in range(8):
        V = cam.getViewMatrix()
        cam.orbit(0.01)
        a = auto.render_host(V, P, W, H)
        picks.append(int(auto.last_stats()["binning"]))
        b = ref.render_host(V, P, W, H)
        assert int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32))) == 0, k
    torch.cuda.synchronize()
    assert picks[0] == 1, picks  # (the first frame at a resolution: depth-first, P unknown)
    assert all(p == 2 for p in picks[1:]), picks  # (2 = bin-first)


@pytest.mark.parametrize("w,h,n,scale", [(4128, 4128, 400000, 1.2), (1920, 1080, 1500000, 2.0)])
def test_depth_cuts_cut_table_sizes(built, w, h, n, scale):
    """The duplicate marks the pairs behind their cut from an LDS copy of the
    cut table when the frame has at most kDupCutBins (16,384) bins; a larger
    frame (129 x 129 bins) keeps the sort's own gather of cut[bin].  Both,
    with a jump that opens quadrants (the fallback filter masks the mark off),
    equal whole lists bit for bit."""
    from gaussian_splat_amd.api import default_camera
    sc = _scene(n, 41, 0, w / h, scale=scale)
    cut, whole = _pair(sc, binning="bin_first")
    far = default_camera(w, h)
    far.setDistance(7.0)
    near = default_camera(w, h)
    near.setDistance(2.5)
    near.orbit(0.3, 0.1)
    opened = sorted_lt = 0
    for cam in (far, far, far, near, near, far):
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        assert _bits(cut.render_host(V, P, w, h), whole.render_host(V, P, w, h)) == 0
        st = cut.last_stats()
        opened += st["open_tiles"]
        sorted_lt += int(st["pairs_sorted"] < st["pairs"])
    assert sorted_lt > 0 and opened > 0


@pytest.mark.parametrize("fif,scale", [(1, 1.0), (2, 1.0), (1, 3.0), (2, 3.0)])
def test_front_only_retry_after_zoom_out(built, fif, scale):
    """Front-only frames (a still camera with cuts: each duplicate block finds
    its offsets by look-back, the totals run beside it) whose pair count then
    outgrows the buffers: a zoom-out after several still frames brings the
    whole scene into view, so the frame's pairs (x2.7) exceed the capacity
    sized by the last frame's, so its lists
    are queued again with larger buffers (look-back statuses cleared again),
    and the frames after it re-grow their cuts.  Every frame is bit-identical
    to the whole-list frame.  (scale 3: saturated tiles, so the cuts keep
    part of the lists and the fallback lists run where a quadrant opens.)
    Round 6 found the re-queued front-only frame wrong before its bin ranges
    were emptied again (the no-op frame's tail regenerates fallback lists from
    the rects and writes their ranges)."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd.api import default_camera
    import torch

    W, H = 800, 450
    sc = _scene(300000, 23, 0, W / H, scale)
    views = []
    for d in (2.2,) * 5 + (6.0,) * 4 + (4.0,) * 3:
        cam = default_camera(W, H)
        cam.setDistance(d)
        views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    ref = InstancedSplatRenderer(sc, Options(crop=False, binning="bin_first", depth_split=False))
    ref.initialize(0)
    refs = [ref.render_host(V, P, W, H) for V, P in views]
    r = InstancedSplatRenderer(sc, Options(crop=False, binning="bin_first", depth_split=True, frames_in_flight=fif))
    r.initialize(0)
    pairs, fronts, outs = [], [], []
    for V, P in views:
        if fif == 2:
            outs.append(r.render(V, P, W, H).clone())
        else:
            outs.append(r.render_host(V, P, W, H))
        st = r.last_stats()
        pairs.append(st["pairs"])
        fronts.append(st["front_only"])
    if fif == 2:
        torch.cuda.synchronize()
        outs = [o.cpu().numpy() for o in outs]
    for k, o in enumerate(outs):
        assert _bits(o, refs[k]) == 0, (k, pairs, fronts)
    assert sum(fronts[1:5]) >= 3, fronts                      # the still frames emitted their front pairs only
    grew = [k for k in range(1, len(pairs)) if pairs[k] > 1.2 * pairs[k - 1]]
    assert grew and any(fronts[k] for k in grew), (pairs, fronts)  # a front-only frame outgrew the buffers
