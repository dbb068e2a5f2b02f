"""GPU parity: the HIP pipeline (through the C-ABI) against the CPU oracle.

Bar: per-splat records, depth keys and tile counts are
bit-identical; sorted (key, value) pairs are identical to a stable sort of
the oracle's pairs; framebuffers agree within the north-star 1e-4 L-inf per
channel and are in fact expected bit-identical (the fp32 contract fixes every
op).  Sizes are ones the oracle finishes in seconds.
"""
import numpy as np
import pytest

from conftest import check_slab_frame, orbit_views

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north star: per-channel L-inf vs the reference semantics


def _scene(n, seed, sh, aspect=1.0):
    from gaussian_splat_amd import scene as S
    return S.activate(S.synthetic_raw(n, seed=seed, aspect=aspect), sh)


def _renderer(scene, sh=0, mode="tile", crop=True):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    r = InstancedSplatRenderer(scene, Options(mode=mode, sh_degree=sh, crop=crop))
    r.initialize(0)
    return r


def _compare(img, ref):
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    linf = float(diff.max()) if diff.size else 0.0
    nbit = int(np.count_nonzero(img.view(np.uint32) != ref.view(np.uint32)))
    return linf, nbit


def _rect_bin_pairs(rec, dk, nt, W):
    """(bin, dkey, splat) for every 32x32 bin of every visible splat's rect
    (the superset the bin lists are drawn from), and the set of (bin, splat)
    pairs whose splat surely covers a pixel centre of the bin (float64,
    threshold shrunk by 1e-4: must be present)."""
    bx = (W + 31) // 32
    qmax = 9.21034037197618 * (1.0 - 1e-4)
    pairs, must = [], set()
    for i in np.nonzero(nt)[0]:
        lo, hi = int(rec["rect_lo"][i]), int(rec["rect_hi"][i])
        x0, y0, x1, y1 = lo & 0xFFFF, lo >> 16, hi & 0xFFFF, hi >> 16
        r = rec[i]
        for by in range(y0 >> 5, (y1 >> 5) + 1):
            for b in range(x0 >> 5, (x1 >> 5) + 1):
                key = by * bx + b
                pairs.append((key, int(dk[i]), int(i)))
                px = np.arange(max(b * 32, x0), min(b * 32 + 31, x1) + 1) + 0.5
                py = np.arange(max(by * 32, y0), min(by * 32 + 31, y1) + 1) + 0.5
                dx = px[None, :] - float(r["cx"])
                dy = float(r["cy"]) - py[:, None]
                u = dy * float(r["ay"]) + dx * float(r["ax"])
                v = dy * float(r["by"]) + dx * float(r["bx"])
                if np.any((u * u + v * v <= qmax) & (np.maximum(np.abs(u), np.abs(v)) <= 3.0 * (1 - 1e-5))):
                    must.add((key, int(i)))
    return pairs, must


@pytest.mark.parametrize("sh", [0, 1, 2, 3])
def test_records_bitexact(built, sh):
    from oracle import oracle_py as O
    sc = _scene(20000, seed=3 + sh, sh=sh, aspect=16 / 9)
    r = _renderer(sc, sh=sh)
    for V, P in orbit_views(640, 360):
        rec, dk, nt = r.project_host(V, P, 640, 360)
        orec, odk, ont = O.project(sc, V, P, 640, 360, sh_degree=sh)
        np.testing.assert_array_equal(nt, ont)
        vis = ont > 0
        assert vis.sum() > 1000
        np.testing.assert_array_equal(dk[vis], odk[vis])
        np.testing.assert_array_equal(rec[vis].view(np.uint32).reshape(-1, 12), orec[vis].view(np.uint32).reshape(-1, 12))


def test_render_config1_bitexact(built, default_cam_256):
    """Config 1: 10k-splat synthetic scene, 256x256, reference default camera."""
    from oracle import oracle_py as O
    V, P = default_cam_256
    sc = _scene(10000, 0, 0)
    r = _renderer(sc)
    img = r.render_host(V, P, 256, 256)
    ref, st = O.render(sc, V, P, 256, 256)
    linf, nbit = _compare(img, ref)
    assert linf <= TOL
    assert nbit == 0, f"{nbit} channel values differ bitwise (L-inf {linf})"
    stats = r.last_stats()
    rec, dk, nt = O.project(sc, V, P, 256, 256)
    pairs, must = _rect_bin_pairs(rec, dk, nt, 256)
    # (splat, 32x32 bin) pairs: the rect's bins minus those the ellipse misses
    assert len(must) <= stats["pairs"] <= len(pairs)
    assert st["pairs"] >= stats["pairs"]
    assert stats["visible"] == int((nt > 0).sum())


@pytest.mark.parametrize("sh,mode", [(0, "tile"), (3, "tile"), (0, "live50"), (3, "live50")])
def test_render_1080p_parity(built, sh, mode):
    from oracle import oracle_py as O
    sc = _scene(150000, 11 + sh, sh, aspect=16 / 9)
    r = _renderer(sc, sh=sh, mode=mode)
    for V, P in orbit_views(1920, 1080, 2):
        img = r.render_host(V, P, 1920, 1080)
        ref, _ = O.render(sc, V, P, 1920, 1080, sh_degree=sh, mode=mode)
        linf, nbit = _compare(img, ref)
        assert linf <= TOL
        assert nbit == 0, f"{nbit} differing values, L-inf {linf}"


@pytest.mark.parametrize("n,w,h,sh,mode,cap,grow", [(10000, 256, 256, 0, "tile", 32, 4.0),
                                                     (20000, 640, 360, 0, "live50", 50, 4.0),
                                                     (150000, 1920, 1080, 3, "tile", 32, 1.0),
                                                     (40000, 640, 360, 0, "live50", 8, 1.0)])
def test_render_cap_parity(built, n, w, h, sh, mode, cap, grow):
    """cap mode: first `cap` covering fragments per pixel
    in arrival order, then S1 order and the mode's composite.  Splats are
    grown so that per-pixel lists overflow the cap."""
    from oracle import oracle_py as O
    sc = _scene(n, 21 + sh, sh, aspect=w / h)
    sc.scale *= grow
    r = _renderer(sc, sh=sh, mode=mode)
    r.set_cap(cap)
    V, P = orbit_views(w, h, 1)[0]
    img = r.render_host(V, P, w, h)
    ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode, cap=cap)
    linf, nbit = _compare(img, ref)
    assert linf <= TOL
    assert nbit == 0, f"{nbit} differing values, L-inf {linf}"
    uncapped, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode)
    assert np.count_nonzero(uncapped.view(np.uint32) != ref.view(np.uint32)) > 0  # the cap is exercised
    r.set_cap(0)
    again = r.render_host(V, P, w, h)
    np.testing.assert_array_equal(again.view(np.uint32), uncapped.view(np.uint32))


@pytest.mark.parametrize("n,w,h,sh,mode", [(10000, 256, 256, 0, "tile"), (150000, 1920, 1080, 3, "live50")])
def test_render_bgra8(built, n, w, h, sh, mode):
    """BGRA8Unorm output converted inside the composite == the oracle frame
    converted by the oracle, byte for byte; device and host paths agree."""
    import torch
    from oracle import oracle_py as O
    sc = _scene(n, 41 + sh, sh, aspect=w / h)
    r = _renderer(sc, sh=sh, mode=mode)
    V, P = orbit_views(w, h, 1)[0]
    got = r.render_bgra8_host(V, P, w, h)
    ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode=mode)
    np.testing.assert_array_equal(got, O.to_bgra8(ref))
    assert got[..., 3].any() and got[..., 2].any()
    dev = r.render_bgra8(V, P, w, h)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), got)
    np.testing.assert_array_equal(O.to_bgra8(r.render_host(V, P, w, h)), got)


@pytest.mark.parametrize("n,w,h,sh", [(10000, 256, 256, 0), (60000, 640, 400, 3)])
def test_render_mlab_bitexact(built, n, w, h, sh):
    """MLAB k-buffer mode (gaussian_splat.metal:201-361): index-ordered bin
    lists, half k-buffer in registers, resolve; bit-identical to the oracle's
    half-emulated k-buffer."""
    from oracle import oracle_py as O
    sc = _scene(n, seed=61, sh=sh, aspect=w / h)
    r = _renderer(sc, sh=sh, mode="mlab")
    for V, P in orbit_views(w, h, 2):
        img = r.render_host(V, P, w, h)
        ref, _ = O.render(sc, V, P, w, h, sh_degree=sh, mode="mlab")
        assert _compare(img, ref) == (0.0, 0)
        assert img[..., 3].max() > 0.5


def test_mlab_virtual_shards_bitexact(built):
    """MLAB through the row multi-GPU scheme: arrival order survives the exchange."""
    from gaussian_splat_amd import distributed as D
    W, H = 640, 400
    sc = _scene(40000, 67, 0, aspect=W / H)
    V, P = orbit_views(W, H, 1)[0]
    ref = _renderer(sc, sh=0, mode="mlab", crop=False).render_host(V, P, W, H)
    img = D.render_virtual_shards(sc, 3, V, P, W, H, sh_degree=0, mode="mlab")
    assert _compare(img, ref) == (0.0, 0)


@pytest.mark.parametrize("w,h", [(640, 360), (1920, 1080)])
def test_render_anisotropic_bitexact(built, w, h):
    """Needles, discs and sub-pixel splats at random orientations: the
    composite's 8x8-cell exclusion mask (computed in preprocess) must never
    drop a covered pixel, so the frame stays bit-exact."""
    from oracle import oracle_py as O
    sc = _scene(60000, 61, 0, aspect=w / h)
    rng = np.random.default_rng(61)
    kind = rng.integers(0, 3, sc.n)
    s = sc.scale.copy()
    s[kind == 0] *= np.array([30.0, 0.02, 0.02], np.float32)   # needles
    s[kind == 1] *= np.array([8.0, 8.0, 0.01], np.float32)     # discs
    s[kind == 2] *= 0.05                                         # tiny
    sc.scale[:] = s
    r = _renderer(sc)
    for V, P in orbit_views(w, h, 2):
        img = r.render_host(V, P, w, h)
        ref, _ = O.render(sc, V, P, w, h)
        assert _compare(img, ref) == (0.0, 0)


def test_stage_timing_modes(built):
    """Timing never changes the image; stage_timing 2 reports per-frame
    preprocess/composite kernel times from the dispatch-packet events (ring
    of 64 frames), stage_timing 1 the full stage breakdown."""
    import torch
    sc = _scene(30000, seed=17, sh=1, aspect=16 / 9)
    r = _renderer(sc, sh=1)
    V, P = orbit_views(640, 360)[0]
    ref = r.render_host(V, P, 640, 360)
    out = torch.empty((360, 640, 4), dtype=torch.float32, device="cuda:0")
    for mode in (2, 1, 0):
        r.set_stage_timing(mode)
        for _ in range(3 if mode != 2 else 70):
            r.render(V, P, 640, 360, out=out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        st = r.last_stats()
        pre, comp = r.kernel_times(100)
        if mode == 2:
            assert len(pre) == 64 and np.all(pre > 0) and np.all(comp > 0)
            assert st["ms_preprocess"] > 0 and st["ms_composite"] > 0 and st["ms_total"] >= st["ms_composite"]
            assert st["ms_sort"] == 0
        else:
            assert len(pre) == 0
        if mode == 1:
            assert all(st[f"ms_{k}"] > 0 for k in ("preprocess", "depth_sort", "scan", "duplicate", "sort",
                                                   "composite"))


def test_frames_in_flight_empty_frames_user_stream(built):
    """frames_in_flight 2 on a user (non-null) stream, with empty frames (camera
    facing away, no pairs) between normal ones: every output equals the
    single-stream render, and the empty frames are the clear colour."""
    import torch
    from gaussian_splat_amd.api import default_camera
    W, H = 480, 270
    sc = _scene(30000, seed=72, sh=1, aspect=W / H)
    views = orbit_views(W, H, 2)
    cam = default_camera(W, H)
    cam.setTarget(2 * cam.position - cam.target)  # the scene is behind the camera
    views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    r1 = _renderer(sc, sh=1)
    refs = [r1.render_host(V, P, W, H) for V, P in views]
    assert r1.last_stats()["pairs"] == 0
    r2 = _renderer(sc, sh=1)
    r2.set_frames_in_flight(2)
    seq = [0, 2, 1, 2, 2, 0, 1]
    stream = torch.cuda.Stream()
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in seq]
    with torch.cuda.stream(stream):
        for k, v in enumerate(seq):
            r2.render(*views[v], W, H, out=outs[k], stream=stream.cuda_stream)
    stream.synchronize()
    for k, v in enumerate(seq):
        assert _compare(outs[k].cpu().numpy(), refs[v]) == (0.0, 0), k
    assert not np.any(refs[2][..., 3])  # nothing drawn


def test_frames_in_flight_bitexact(built):
    """frames_in_flight 2: a frame's projection/sort runs on the handle's side
    stream while the previous frame composites; every output equals the
    single-stream render, across camera changes, both output formats and an
    interleaved gs_project_host (which must wait for the pipelined composite)."""
    import torch
    W, H = 640, 360
    sc = _scene(80000, seed=71, sh=2, aspect=W / H)
    views = orbit_views(W, H, 3)
    r1 = _renderer(sc, sh=2)
    refs = [r1.render_host(V, P, W, H) for V, P in views]
    r2 = _renderer(sc, sh=2)
    r2.set_frames_in_flight(2)
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(7)]
    seq = [0, 1, 2, 2, 0, 1, 0]
    for k, v in enumerate(seq):
        r2.render(*views[v], W, H, out=outs[k])
        if k == 3:
            rec, dk, nt = r2.project_host(*views[1], W, H)
    bg = r2.render_bgra8(*views[2], W, H)
    torch.cuda.synchronize()
    for k, v in enumerate(seq):
        assert _compare(outs[k].cpu().numpy(), refs[v]) == (0.0, 0), k
    from oracle import oracle_py as O
    np.testing.assert_array_equal(bg.cpu().numpy(), O.to_bgra8(refs[2]))
    rec1, dk1, nt1 = r1.project_host(*views[1], W, H)
    vis = nt1 > 0  # records of culled splats are not written (undefined)
    np.testing.assert_array_equal(nt, nt1)
    np.testing.assert_array_equal(dk, dk1)
    np.testing.assert_array_equal(rec[vis].view(np.uint8), rec1[vis].view(np.uint8))


def test_render_device_out_matches_host(built):
    import torch
    sc = _scene(30000, 5, 0, aspect=4 / 3)
    r = _renderer(sc)
    V, P = orbit_views(800, 600, 1)[0]
    host = r.render_host(V, P, 800, 600)
    dev = r.render(V, P, 800, 600)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy().view(np.uint32), host.view(np.uint32))
    again = r.render(V, P, 800, 600).cpu().numpy()
    np.testing.assert_array_equal(again.view(np.uint32), host.view(np.uint32))  # deterministic


@pytest.mark.parametrize("n,huge", [(40000, 0), (4096, 0), (6001, 300), (2048 * 3 + 1, 7)])
def test_sorted_pairs_match_stable_sort(built, n, huge):
    """Bin lists == a stable sort of the depth-ordered pairs by bin, over the
    rect's bins minus those the splat's ellipse misses (bin-exclusion mask):
    never a bin outside the rect, always every bin with a covered pixel
    centre.  Covers sizes around block boundaries and splats blown up to
    cover much of the frame."""
    from oracle import oracle_py as O
    W, H = 512, 384
    sc = _scene(n, 9, 0, aspect=W / H)
    if huge:
        idx = np.random.default_rng(n).choice(n, huge, replace=False)
        sc.scale[idx] *= 40.0
    r = _renderer(sc)
    V, P = orbit_views(W, H, 1)[0]
    r.render_host(V, P, W, H)
    keys, vals = r.sorted_pairs()
    rec, dk, nt = O.project(sc, V, P, W, H)
    pairs, must = _rect_bin_pairs(rec, dk, nt, W)
    got = set(zip(keys.tolist(), vals.tolist()))
    assert len(got) == len(keys)                                  # no duplicates
    assert got <= {(k, i) for k, _, i in pairs}                   # only bins of the rect
    assert must <= got                                            # every surely covered bin
    ek = np.array([(k << 15) | d for k, d, i in pairs if (k, i) in got], np.uint64)
    ev = np.array([i for k, d, i in pairs if (k, i) in got], np.uint32)
    order = np.argsort(ek, kind="stable")  # (bin, dkey), ties by splat index
    np.testing.assert_array_equal(keys.astype(np.uint64), ek[order] >> np.uint64(15))  # bin id
    np.testing.assert_array_equal(vals, ev[order])


@pytest.mark.parametrize("n,w,h,mode,cap,wall,zr", [
    (40000, 64, 64, "tile", 0, 0, (1, 9)),       # 8193..16384 pairs per bin (12-bit key span: 6+6)
    (100000, 64, 64, "tile", 0, 0, (1, 9)),      # > 16384: global-memory path
    (100000, 64, 64, "live50", 32, 0, (1, 9)),
    (30000, 512, 384, "tile", 0, 0, (1, 9)),     # <= 8192
    (30000, 512, 384, "tile", 0, 0, (4, 4.2)),   # key span < 256: one pass
    (30000, 512, 384, "live50", 0, 0, (0.3, 9)), # 13-bit span: 8+7
    (30000, 512, 384, "tile", 0, 1, (1, 9)),     # half the splats at one depth
    (12000, 64, 64, "tile", 0, 2, (1, 9))])      # all at one depth (span 0 or 1)
def test_bin_first_equals_depth_first(built, n, w, h, mode, cap, wall, zr):
    """Bin-first order (bin lists in arrival order, then a stable per-bin
    depth sort, bin_depth_sort.hip) builds exactly the depth-first order's
    bin lists and image in every list size class and every key-span path,
    and matches the oracle."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    from oracle import oracle_py as O
    sc = S.activate(S.synthetic_raw(n, seed=21, aspect=w / h, zrange=zr), 0)
    V, P = orbit_views(w, h, 1)[0]
    if wall:  # splats on a plane at view depth 5 (one or two half-depth keys)
        rng = np.random.default_rng(5)
        eye, fwd = np.array([0.0, 2.0, 5.0]), -np.array([0.0, 2.0, 5.0]) / np.sqrt(29.0)
        right = np.cross(fwd, [0.0, -1.0, 0.0]); right /= np.linalg.norm(right)
        up = np.cross(right, fwd)
        k = n // 2 if wall == 1 else n
        a, b = rng.uniform(-1.5, 1.5, (2, k))
        sc.pos[:k] = (eye + 5.0 * fwd + a[:, None] * right + b[:, None] * up).astype(np.float32)
    out = {}
    for b in ("depth_first", "bin_first"):
        r = InstancedSplatRenderer(sc, Options(mode=mode, cap=cap, binning=b, depth_split=False))  # (one-slab lists)
        r.initialize(0)
        img = r.render_host(V, P, w, h)
        keys, vals = r.sorted_pairs()
        out[b] = (img, keys, vals, r.last_stats()["pairs"])
    img0, k0, v0, p0 = out["depth_first"]
    img1, k1, v1, p1 = out["bin_first"]
    assert p0 == p1
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_array_equal(v1, v0)
    assert _compare(img1, img0) == (0.0, 0)
    per_bin = np.bincount(k0, minlength=((w + 31) // 32) * ((h + 31) // 32))
    assert per_bin.max() > (16384 if n == 100000 else 8192 if n == 40000 else 0)
    ref, _ = O.render(sc, V, P, w, h, mode=mode, cap=cap)
    linf, nbit = _compare(img1, ref)
    assert linf <= TOL and nbit == 0, (linf, nbit)


def test_bin_sort_size_classes(built):
    """A frame of 4096 bins (2048 x 2048), where the per-bin sort runs in two
    size classes (bin_depth_sort.hip: lists of <= 4096 pairs in 256-lane
    workgroups, longer ones in 512-lane workgroups or through global memory),
    with lists in every class: two clusters of splats over a uniform scene.
    Bin-first equals depth-first (keys, vals, image) and the oracle."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    from oracle import oracle_py as O
    w = h = 2048
    sc = S.activate(S.synthetic_raw(200000, seed=21, aspect=1.0, zrange=(1, 9)), 0)
    rng = np.random.default_rng(7)
    eye = np.array([0.0, 2.0, 5.0])
    fwd = -eye / np.linalg.norm(eye)
    right = np.cross(fwd, [0.0, -1.0, 0.0])
    right /= np.linalg.norm(right)
    up = np.cross(right, fwd)
    o = 0
    for k, sig, (ox, oy) in ((60000, 0.15, (0.0, 0.0)), (60000, 0.015, (0.8, 0.5))):
        a, b = rng.normal(0, sig, (2, k))
        d = rng.uniform(3.0, 6.0, k)
        sc.pos[o:o + k] = (eye + d[:, None] * fwd + (a + ox)[:, None] * right + (b + oy)[:, None] * up).astype(np.float32)
        o += k
    V, P = orbit_views(w, h, 1)[0]
    out = {}
    for b in ("depth_first", "bin_first"):
        r = InstancedSplatRenderer(sc, Options(binning=b, depth_split=False))
        r.initialize(0)
        img = r.render_host(V, P, w, h)
        keys, vals = r.sorted_pairs()
        out[b] = (img, keys, vals)
    img0, k0, v0 = out["depth_first"]
    img1, k1, v1 = out["bin_first"]
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_array_equal(v1, v0)
    assert _compare(img1, img0) == (0.0, 0)
    per_bin = np.bincount(k0, minlength=64 * 64)
    assert per_bin.size == 4096 and (per_bin > 8192).any() and ((per_bin > 4096) & (per_bin <= 8192)).any()
    assert ((per_bin > 1) & (per_bin <= 4096)).sum() > 3000
    ref, _ = O.render(sc, V, P, w, h)
    linf, nbit = _compare(img1, ref)
    assert linf <= TOL and nbit == 0, (linf, nbit)


def test_bin_first_frame_sequences(built):
    """Sequences of bin-first frames (repeats, camera and resolution
    switches, pipelined frames with host-output frames in between, which
    switch pipelining off and on) all equal the depth-first renders."""
    import torch
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    sc = _scene(60000, 33, 1, aspect=16 / 9)
    seq = [(640, 360, 0), (640, 360, 0), (640, 360, 1), (800, 450, 2), (640, 360, 1), (800, 450, 0)]
    refr = InstancedSplatRenderer(sc, Options(sh_degree=1, binning="depth_first"))
    refr.initialize(0)
    refs = [refr.render_host(*orbit_views(w, h, 3)[v], w, h) for w, h, v in seq]
    for fif in (1, 2):
        r = InstancedSplatRenderer(sc, Options(sh_degree=1, binning="bin_first", frames_in_flight=fif))
        r.initialize(0)
        outs = []
        for w, h, v in seq:
            outs.append(r.render(*orbit_views(w, h, 3)[v], w, h))
            if v == 2:  # a host-output frame in between (never pipelined)
                assert _compare(r.render_host(*orbit_views(w, h, 3)[v], w, h), refs[len(outs) - 1]) == (0.0, 0)
        torch.cuda.synchronize()
        for k, o in enumerate(outs):
            assert _compare(o.cpu().numpy(), refs[k]) == (0.0, 0), (fif, k)
        assert r.last_stats()["binning"] == 2


@pytest.mark.parametrize("binning", ["depth_first", "bin_first"])
def test_pair_count_growth(built, binning):
    """The duplicate and the bin sort are queued before the host sees the
    frame's pair count, sized by the last frame's: frames whose count grows
    (camera moving in, P several times the last) take the re-queue path and
    still equal a fresh renderer's frame, pipelined or not."""
    import torch
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd.api import default_camera
    sc = _scene(50000, 41, 0, aspect=16 / 9)
    W, H = 640, 360
    views = []
    for d in (2.0, 3.0, 12.0, 6.0, 2.0):  # P grows over the first four frames here
        cam = default_camera(W, H)
        cam.setDistance(d)
        views.append((cam.getViewMatrix(), cam.getProjectionMatrix()))
    refs, pairs = [], []
    for v in views:  # a fresh renderer per frame: its first frame always re-queues
        fr = InstancedSplatRenderer(sc, Options(sh_degree=0, binning=binning))
        fr.initialize(0)
        refs.append(fr.render_host(*v, W, H))
        pairs.append(fr.last_stats()["pairs"])
    # each growth step exceeds the last frame's capacity (P + 1/8 slack)
    assert pairs[1] > 1.3 * pairs[0] and pairs[2] > 1.3 * pairs[1] and pairs[3] > pairs[2], pairs
    for fif in (1, 2):
        r = InstancedSplatRenderer(sc, Options(sh_degree=0, binning=binning, frames_in_flight=fif))
        r.initialize(0)
        outs = [r.render(*v, W, H) for v in views]
        torch.cuda.synchronize()
        for k, o in enumerate(outs):
            assert _compare(o.cpu().numpy(), refs[k]) == (0.0, 0), (fif, k)
        assert r.last_stats()["pairs"] == pairs[-1]


def test_large_splats_bin_first(built):
    """One duplicate block (4096 splats in index order) of large splats among
    small ones: the block's pairs span more sort tiles than its LDS digit
    counts cover, so the first sort pass's counts also go through the
    global-atomic path (the average per block keeps the fused counts on).
    Bin-first frames, first and repeated, equal the depth-first frame."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    W, H = 960, 540
    v, p = orbit_views(W, H, 1)[0]

    def frame(raw, binning, repeat=1):
        r = InstancedSplatRenderer(S.activate(raw, 0), Options(sh_degree=0, binning=binning))
        r.initialize(0)
        for _ in range(repeat):
            img = r.render_host(v, p, W, H)
        return img, r.last_stats()["pairs"]

    base = S.synthetic_raw(40960, seed=77, aspect=16 / 9)
    _, p0 = frame(base, "depth_first")
    raw = S.synthetic_raw(40960, seed=77, aspect=16 / 9)
    raw.log_scale[8192:12288] += np.float32(np.log(14.0))
    ref, p1 = frame(raw, "depth_first")
    assert p1 - p0 > 4 * 6144, (p0, p1)            # the large block's extra pairs: > 4 sort tiles
    assert p1 / 10 <= 3 * 6144, p1                 # average per block: fused counts stay on
    img, pb = frame(raw, "bin_first", repeat=2)    # (frame 2: P known, no re-queue)
    assert pb == p1
    assert _compare(img, ref) == (0.0, 0)


@pytest.mark.parametrize("n,bits", [(0, 8), (1, 8), (4095, 13), (4096, 16), (4097, 20), (100000, 28),
                                    (1 << 20, 32), (3_000_001, 30)])
def test_radix_sort(built, n, bits):
    import torch
    from gaussian_splat_amd import radix_sort_pairs
    rng = np.random.default_rng(n + bits)
    hi = (1 << bits) if bits < 32 else (1 << 32)
    k = rng.integers(0, min(hi, 1 << 12) if n > 1000 and bits > 12 and n % 2 else hi, n, dtype=np.uint64).astype(np.uint32)
    v = np.arange(n, dtype=np.uint32)
    kt = torch.from_numpy(k.view(np.int32)).cuda()
    vt = torch.from_numpy(v.view(np.int32)).cuda()
    radix_sort_pairs(kt, vt, bits)
    torch.cuda.synchronize()
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(kt.cpu().numpy().view(np.uint32), k[order])
    np.testing.assert_array_equal(vt.cpu().numpy().view(np.uint32), v[order])


def test_empty_and_culled(built):
    from gaussian_splat_amd import scene as S
    sc = _scene(5000, 2, 0)
    sc.pos[:] = np.array([0.0, 2.0, 9.0], np.float32)  # behind the eye at (0,2,5)
    sc.pos[:, 2] = 4.999
    r = _renderer(sc)
    V, P = orbit_views(128, 128, 1)[0]
    img = r.render_host(V, P, 128, 128)
    assert not img.any()
    assert r.last_stats()["pairs"] == 0
    assert r.last_stats()["visible"] == 0
    empty = S.Scene(np.zeros((0, 3)), np.zeros((0, 4)), np.zeros((0, 3)), np.zeros(0), np.zeros((0, 3)))
    r0 = _renderer(empty)
    assert r0.getPointCount() == 0
    assert not r0.render_host(V, P, 64, 48).any()


def test_ply_dropin_path(built, tmp_path):
    """gs_create(.ply) == oracle PLY restatement -> crop -> render."""
    from gaussian_splat_amd import scene as S
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from oracle import oracle_py as O
    raw = S.synthetic_raw(8000, seed=21, aspect=1.0)
    raw.pos[::7, 0] += np.float32(5.5)  # push every 7th splat outside the crop cube
    raw.pos[3::11, 2] -= np.float32(5.0)
    p = S.write_ply(tmp_path / "s.ply", raw)
    r = InstancedSplatRenderer(str(p), Options())
    r.initialize(0)
    ok, pts = O.ply_load(p)
    keep = O.crop(pts)
    assert r.getPointCount() == len(keep) < 8000
    from gaussian_splat_amd.api import Scene
    sc = Scene.from_points(pts[keep])
    V, P = orbit_views(256, 256, 1)[0]
    img = r.render_host(V, P, 256, 256)
    ref, _ = O.render(sc, V, P, 256, 256)
    assert _compare(img, ref) == (0.0, 0)


@pytest.mark.parametrize("world,cap,table", [(2, 0, None), (3, 0, None), (3, 32, None), (4, 0, "interleaved")])
def test_virtual_shards_bitexact(built, world, cap, table):
    """K virtual ranks on one GPU through gs_shard_project/gs_shard_render
    reassemble the single-GPU frame bit for bit (SURVEY §8e verification);
    with a fragment cap, arrival order survives the exchange."""
    from gaussian_splat_amd import distributed as D
    W, H = 640, 400
    sc = _scene(60000, 31, 3, aspect=W / H)
    if cap:
        sc.scale *= 3.0
    full = _renderer(sc, sh=3)
    full.set_cap(cap)
    V, P = orbit_views(W, H, 1)[0]
    ref = full.render_host(V, P, W, H)
    owner = None
    if table == "interleaved":  # a custom gs_shard_set_rows table
        owner = (np.arange((H + 31) // 32) % world).astype(np.uint8)[::-1].copy()
    img = D.render_virtual_shards(sc, world, V, P, W, H, sh_degree=3, cap=cap, owner=owner)
    assert _compare(img, ref) == (0.0, 0)


@pytest.mark.parametrize("world,mode,sh", [(2, "tile", 3), (4, "tile", 0), (3, "live50", 0)])
def test_virtual_slabs(built, world, mode, sh):
    """Depth-slab scheme with K virtual ranks on one GPU:
    every slab's transmittance and (C, delta alpha) contributions are
    bit-identical to the oracle's slab passes on the same splats, and the
    summed frame is within the north star's 1e-4 of the 1-GPU frame (the
    transmittance product reassociates the A / T recurrence)."""
    from oracle import oracle_py as O
    from gaussian_splat_amd import distributed as D
    W, H = 640, 400
    sc = _scene(60000, 41, sh, aspect=W / H)
    V, P = orbit_views(W, H, 2)[1]
    full = _renderer(sc, sh=sh, mode=mode, crop=False)
    ref = full.render_host(V, P, W, H)
    frame, bounds, t_all, contrib, _ = D.render_virtual_slabs(sc, world, V, P, W, H, sh_degree=sh, mode=mode,
                                                              parts=True)
    rec, dk, nt = O.project(sc, V, P, W, H, sh_degree=sh)
    vis = nt > 0
    slab = np.searchsorted(bounds[1:-1].astype(np.int64), dk.astype(np.int64), side="right")
    assert len(set(slab[vis].tolist())) == world  # every slab holds splats
    ot = np.stack([O.composite_slab(rec[vis & (slab == d)], dk[vis & (slab == d)], W, H, 1, mode=mode)
                   for d in range(world)])
    np.testing.assert_array_equal(t_all.view(np.uint32), ot.view(np.uint32))
    for d in range(world):
        oc = O.composite_slab(rec[vis & (slab == d)], dk[vis & (slab == d)], W, H, 2, rank=d, t_all=ot, mode=mode)
        np.testing.assert_array_equal(contrib[d].view(np.uint32), oc.view(np.uint32))
    check_slab_frame(frame, ref)


def _rank_worker(rank, world, port, q, scheme="rows"):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import torch
    import torch.distributed as dist
    from gaussian_splat_amd import Options, scene as S
    from gaussian_splat_amd.distributed import (HipShardBackend, HipSlabBackend, ShardedRenderer, SlabRenderer,
                                                shard_bounds)
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from conftest import orbit_views
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        W, H = 800, 600
        sc = S.activate(S.synthetic_raw(60000, seed=51, aspect=W / H), 3)
        b, e = shard_bounds(sc.n, world, rank)
        Backend, Renderer = (HipSlabBackend, SlabRenderer) if scheme == "slabs" else (HipShardBackend, ShardedRenderer)
        be = Backend(sc.subset(slice(b, e)), rank, world, b, Options(sh_degree=3, crop=False), 0)
        if scheme == "pipe":  # two frames in flight, the rank on its own stream, a camera path
            sr = ShardedRenderer(be, rank, world, pipeline=True, exchange_group=dist.new_group(backend="gloo"),
                                 own_stream=True)
            frames = [sr.render(V, P, W, H) for V, P in orbit_views(W, H, 4)] + [sr.flush()]
            if rank == 0:
                torch.cuda.synchronize()
                q.put([None if f is None else f.cpu().numpy() for f in frames])
        else:
            V, P = orbit_views(W, H, 1)[0]
            frame = Renderer(be, rank, world).render(V, P, W, H)
            if rank == 0:
                torch.cuda.synchronize()
                q.put(frame.cpu().numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _rccl_exchange_worker(port, q):
    """(test_rccl_exchange_world1) puts ("ok", checks) or ("err", traceback)."""
    import traceback
    try:
        import sys
        from pathlib import Path
        sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
        import torch
        import torch.distributed as dist
        from gaussian_splat_amd.distributed import exchange_regions, exchange_start, init_ranks
        torch.cuda.set_device(0)
        init_ranks("nccl", 60, device=torch.device("cuda:0"), init_method=f"tcp://127.0.0.1:{port}", rank=0,
                   world_size=1)
        regions = exchange_regions()
        checks = []
        g = torch.Generator().manual_seed(5)
        for n in (1000, 0):
            send = torch.randint(0, 256, (max(1, n * sum(regions)),), generator=g, dtype=torch.uint8).cuda()
            recv, got = exchange_start(send, [n], regions, 1, None).wait()
            torch.cuda.synchronize()
            checks.append((n, got, recv.device.type, bool(torch.equal(recv[: n * sum(regions)], send[: n * sum(regions)]))))
        dist.destroy_process_group()
        q.put(("ok", checks))
    except Exception:  # (reported to the parent instead of leaving it waiting)
        q.put(("err", traceback.format_exc()))


def test_rccl_exchange_world1(built):
    """The rows scheme's record exchange (exchange_start: the counts, then one
    all_to_all_single per exchange region, asynchronous, on device buffers)
    through torch.distributed over the real RCCL, the driver's backend, with
    the one rank this box has (every record to itself; shard frames need a
    second rank, gs_shard_project refuses a world of one).  The received
    regions equal the sent ones; an empty send is received as empty."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_exchange_worker, args=(port, q))
    p.start()
    status, res = q.get(timeout=180)
    p.join(timeout=60)
    assert status == "ok", res
    assert p.exitcode == 0
    assert res == [(1000, 1000, "cuda", True), (0, 0, "cuda", True)]


@pytest.mark.parametrize("scheme", ["rows", "slabs", "pipe"])
def test_multiprocess_ranks_bitexact(built, scheme):
    """Two rank processes on the GPU through the product multi-GPU path
    (rows: gs_shard_project -> all_to_all -> gs_shard_render -> gather;
    slabs: gs_slab_project -> all_reduce -> gs_slab_pack -> all_to_all ->
    gs_slab_render -> all_gather -> gs_slab_composite -> reduce), collectives
    over gloo staged through host memory (one GPU here).  Rows: the frame
    equals the single-GPU render bit for bit; slabs: within 1e-4.  pipe: rows
    with two frames in flight and each rank computing on its own stream, over
    a camera path (every frame one call late, bit for bit)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q, scheme)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from gaussian_splat_amd import scene as S
    W, H = 800, 600
    sc = S.activate(S.synthetic_raw(60000, seed=51, aspect=W / H), 3)
    r = _renderer(sc, sh=3, crop=False)
    if scheme == "pipe":
        assert got[0] is None and len(got) == 5
        for k, (V, P) in enumerate(orbit_views(W, H, 4)):
            assert _compare(got[k + 1], r.render_host(V, P, W, H)) == (0.0, 0), k
        return
    V, P = orbit_views(W, H, 1)[0]
    ref = r.render_host(V, P, W, H)
    if scheme == "rows":
        assert _compare(got, ref) == (0.0, 0)
    else:
        check_slab_frame(got, ref)
