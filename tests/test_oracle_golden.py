"""Pin the oracle (CPU) against the golden vectors before trusting it.

- PLY I1: every fixture in tests/golden/ply is compared with the output the
  reference's OWN src/ply_loader.cpp produced for it (tools/make_golden.py via
  oracle/_ref), bit for bit; plus a live cross-check against oracle/_ref when
  that library is present.
- C1 / K1-K6 / S1 / A1: hand-derived known answers (tests/golden/known_answers.json),
  computed in float64 from the cited reference lines.  The Metal shaders
  cannot be built here, so these are the pins ("parity unpinned" by
  execution).
"""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle_py as O

GOLD = Path(__file__).resolve().parent / "golden"
KA = json.loads((GOLD / "known_answers.json").read_text())
MANIFEST = json.loads((GOLD / "ply" / "manifest.json").read_text())


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_ply_matches_reference_fixture(name):
    ok, pts = O.ply_load(GOLD / "ply" / f"{name}.ply")
    ref = np.load(GOLD / "ply" / f"{name}.ref.npy", allow_pickle=False)
    assert ok == MANIFEST[name]["ok"]
    assert pts.shape[0] == MANIFEST[name]["n"] == ref.shape[0]
    np.testing.assert_array_equal(pts.view(np.uint32), ref.view(np.uint32))


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_ply_matches_live_reference(tmp_path):
    from gaussian_splat_amd import scene as S
    for seed, ascii in ((1, False), (2, True), (3, False)):
        raw = S.synthetic_raw(500 if not ascii else 30, seed=seed, aspect=1.3)
        raw.f_dc[::4] = 0
        p = S.write_ply(tmp_path / f"r{seed}.ply", raw, ascii=ascii)
        ok1, a = O.ref_ply_load(p)
        ok2, b = O.ply_load(p)
        assert ok1 == ok2
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_crop_restatement():
    pts = np.load(GOLD / "ply" / "binary_62prop.ref.npy")
    keep = O.crop(pts, 5.0)
    ref = np.nonzero(np.all(np.abs(pts[:, :3]) < 5.0, axis=1))[0]
    np.testing.assert_array_equal(keep, ref)
    assert 0 < len(keep) < len(pts)


def test_camera_known_answers():
    V = O.look_at([0, 2, 5], [0, 0, 0], [0, -1, 0])
    np.testing.assert_allclose(V, np.array(KA["default_view"]), rtol=0, atol=2e-7)
    np.testing.assert_allclose(V[1, :3], [0, -0.9284767, 0.3713907], atol=1e-7)  # SURVEY §8c pin
    P = O.perspective(45.0, np.float32(1920) / np.float32(1080), 0.1, 1000.0)
    np.testing.assert_allclose(P, np.array(KA["proj_1080p"]), rtol=1e-6, atol=1e-7)
    assert abs(P[0, 0] * 960 - KA["fx_1080p"]) < 1e-3
    assert abs(P[0, 0] * 960 - 1303.675) < 1e-3
    VP = O.mat4_mul(P, V)
    np.testing.assert_allclose(VP, P.astype(np.float64) @ V.astype(np.float64), rtol=1e-6, atol=1e-6)


def test_isotropic_splat_record():
    """K1-K6 on a splat whose projection is hand-computable."""
    from gaussian_splat_amd.api import Scene
    k = KA["iso_splat"]
    sc = Scene(pos=np.array([k["pos"]]), rot=np.array([k["rot"]]), scale=np.array([k["scale"]]),
               opacity=np.array([0.8]), color=np.array([[0.1, 0.2, 0.3]]))
    V = O.look_at([0, 2, 5], [0, 0, 0], [0, -1, 0])
    P = O.perspective(45.0, 1.0, 0.1, 1000.0)
    rec, dk, nt = O.project(sc, V, P, 256, 256)
    r = rec[0]
    for f in ("cx", "cy", "ax", "ay", "bx", "by"):
        assert abs(float(r[f]) - k[f]) <= 2e-5 * max(1.0, abs(k[f])), f
    x0, y0, x1, y1 = k["rect"]
    assert int(r["rect_lo"]) == x0 | (y0 << 16) and int(r["rect_hi"]) == x1 | (y1 << 16)
    assert nt[0] == k["ntiles"]
    assert dk[0] == 0x7C00 - int(np.float16(k["zf"]).view(np.uint16))


@pytest.mark.parametrize("case", sorted(KA["composite"]))
@pytest.mark.parametrize("mode", ["tile", "live50"])
def test_composite_known_answers(case, mode):
    c = KA["composite"][case]
    out = O.composite_list(np.array(c["frags"], np.float32).reshape(-1, 5), mode=mode, cap=c.get("cap", 0))
    np.testing.assert_allclose(out, c[mode], rtol=0, atol=2e-7)


@pytest.mark.parametrize("case", sorted(KA["composite"]))
def test_composite_known_answers_aform(case):
    """The T-form contract against the reference's own A-form
    (tile.metal:252-263: sa = alpha (1 - A), A += sa, break at A >= 0.99),
    derived in float64 and float32 (tools/make_golden.py).  Where both forms
    break after the same record the answers agree to rounding; where the break
    flips, A reaches 0.99 within 1e-5 at that test (a straddle, the 0.99 edge
    of tests/pixel_pins.py), and the case is named."""
    c = KA["composite"][case]
    out = O.composite_list(np.array(c["frags"], np.float32).reshape(-1, 5), mode="tile", cap=c.get("cap", 0))
    if not c["straddle"]:
        assert c["n_tform"] == c["n_aform64"] == c["n_aform32"]
        np.testing.assert_allclose(out, c["tile_aform64"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out, c["tile_aform32"], rtol=0, atol=2.5e-7)
    else:
        assert case == "saturate_edge", "an unexpected break flip between the T-form and the A-form"
        assert abs(c["straddle_A"] - 0.99) < 1e-5
        # the A-form stops one record earlier; that record's weight is what separates them
        assert c["n_tform"] == c["n_aform64"] + 1


def test_survey_depth_order_finding():
    """descending distance -> the farthest (green) ends on top."""
    out = O.composite_list(np.array(KA["composite"]["survey_rgb"]["frags"], np.float32), "tile")
    np.testing.assert_allclose(out, [0.125, 0.5, 0.25, 0.875], atol=1e-7)


def test_half_bits():
    for v, bits in KA["half_bits"].items():
        assert O.f16_bits(float(v)) == bits, v
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(1e-4, 2000, 20000), rng.uniform(1e-7, 1e-4, 2000)]).astype(np.float32)
    got = np.array([O.f16_bits(float(x)) for x in xs], np.uint16)
    np.testing.assert_array_equal(got, xs.astype(np.float16).view(np.uint16))


def test_expf_accuracy():
    xs = np.linspace(-4.7, 0.0, 20001, dtype=np.float32)
    got = np.array([O.expf(float(x)) for x in xs], np.float64)
    rel = np.abs(got / np.exp(xs.astype(np.float64)) - 1)
    assert rel.max() < 5e-7
    assert O.expf(0.0) == 1.0
    qs = np.linspace(0.0, 9.2104, 20001, dtype=np.float32)
    g = np.array([O.gauss(float(q)) for q in qs], np.float64)
    assert np.abs(g / np.exp(-0.5 * qs.astype(np.float64)) - 1).max() < 5e-7
    assert O.gauss(0.0) == 1.0
    # the composite's gaussian on the scaled conic: 2^-q' = exp(-q/2), q' = q log2(e)/2
    qs = np.linspace(0.0, 6.6439, 40001, dtype=np.float32)
    g2 = np.array([O.gauss2(float(q)) for q in qs], np.float64)
    assert np.abs(g2 / np.exp2(-qs.astype(np.float64)) - 1).max() < 2e-7
    assert O.gauss2(0.0) == 1.0 and O.gauss2(1.0) == 0.5 and O.gauss2(6.0) == 2.0 ** -6


def test_oracle_render_invariants():
    """Frame-level invariants of the contract on config 1."""
    from gaussian_splat_amd import scene as S
    sc = S.synthetic_scene(10000, seed=0, aspect=1.0)
    V = O.look_at([0, 2, 5], [0, 0, 0], [0, -1, 0])
    P = O.perspective(45.0, 1.0, 0.1, 1000.0)
    img, st = O.render(sc, V, P, 256, 256)
    a = img[..., 3]
    assert (a >= 0).all() and (a <= 1.0 + 1e-6).all()
    assert (img[..., :3] <= a[..., None] + 1e-6).all()  # premultiplied: C <= A when rgb <= 1
    assert st["visible"] == 10000 and st["pairs"] > 10000
    img2, _ = O.render(sc, V, P, 256, 256, nthreads=1)
    np.testing.assert_array_equal(img.view(np.uint32), img2.view(np.uint32))  # thread-count independent


def test_bgra8_conversion():
    """BGRA8Unorm output: clamp, x255, round half to even,
    bytes B, G, R, A.  Parity unpinned (Metal's conversion cannot run here);
    pinned to that published rule."""
    from oracle import oracle_py as O
    special = np.array([[1.0, 0.0, 0.0, 1.0], [0.5, -1.0, 2.0, np.nan], [0.0, 0.25, 0.75, 0.999]], np.float32)
    got = O.to_bgra8(special.reshape(1, 3, 4))[0]
    np.testing.assert_array_equal(got[0], [0, 0, 255, 255])          # pure red -> B=0, G=0, R=255
    np.testing.assert_array_equal(got[1], [255, 0, 128, 0])           # 127.5 -> 128 (even), clamp, NaN -> 0
    rng = np.random.default_rng(5)
    x = rng.uniform(-0.1, 1.1, (64, 48, 4)).astype(np.float32)
    x[0, :, :] = (np.arange(48 * 4, dtype=np.float32).reshape(48, 4) + 0.5) / np.float32(255)  # near-ties
    y = np.rint(np.clip(x, 0, 1) * np.float32(255)).astype(np.uint8)
    np.testing.assert_array_equal(O.to_bgra8(x), y[..., [2, 1, 0, 3]])


def _pin_scene(sp, **kw):
    from gaussian_splat_amd.api import Scene
    return Scene(pos=np.array([sp["pos"]]), rot=np.array([sp["rot"]]), scale=np.array([sp["scale"]]),
                 opacity=np.array([0.7]), color=np.array([[0.2, 0.4, 0.6]]), **kw)


@pytest.mark.parametrize("name", [s["name"] for s in KA["k_pins"]["splats"]])
def test_projection_pins(name):
    """K1-K5 (tile.metal:40-157): the oracle's fp32 record and intermediates
    against a float64 restatement written straight from the shader lines
    (tools/make_golden.py ref64_vertex): rotated anisotropic off-axis splats
    (the J z-column sign, :122-123, changes b), both eigen fallbacks and a
    0 < |b| <= 1e-8 one (:77-81), the near / far clip and a splat behind the
    eye.  Relative tolerance 2e-5 (fp32 rounding of well-conditioned cases)."""
    kp = KA["k_pins"]
    sp = next(s for s in kp["splats"] if s["name"] == name)
    cam = kp["cameras"][sp["camera"]]
    V, P = np.array(cam["view"], np.float32), np.array(cam["proj"], np.float32)
    rec, dbg = O.project_debug(_pin_scene(sp), V, P, kp["width"], kp["height"])
    e = sp["expect"]
    assert bool(dbg["visible"][0]) == e["visible"], (name, e.get("cull"))
    assert abs(float(dbg["zf"][0]) - e["zf"]) <= 2e-5 * max(1.0, abs(e["zf"]))
    if not e["visible"]:  # culled before the covariance (the oracle stops there)
        return
    scale = max(abs(e["a"]), abs(e["c"]))
    for k in ("a", "b", "c"):
        assert abs(float(dbg[k][0]) - e[k]) <= 2e-5 * scale, (k, float(dbg[k][0]), e[k])
    for k in ("r1", "r2"):
        assert abs(float(dbg[k][0]) - e[k]) <= 2e-5 * e[k], k
    np.testing.assert_allclose([dbg["e1x"][0], dbg["e1y"][0]], e["e1"], rtol=0, atol=2e-5)
    r = rec[0]
    for k in ("cx", "cy"):
        assert abs(float(r[k]) - e[k]) <= 2e-5 * max(1.0, abs(e[k])), k
    na, nb = np.hypot(e["ax"], e["ay"]), np.hypot(e["bx"], e["by"])
    np.testing.assert_allclose([r["ax"], r["ay"]], [e["ax"], e["ay"]], rtol=0, atol=2e-5 * na)
    np.testing.assert_allclose([r["bx"], r["by"]], [e["bx"], e["by"]], rtol=0, atol=2e-5 * nb)
    assert int(dbg["dkey"][0]) == 0x7C00 - int(np.float16(np.float32(e["zf"])).view(np.uint16))


def test_sh_basis_pins():
    """N2 (no reference counterpart): SH degree 1-3 colours of the oracle
    against the published 3DGS basis evaluated in float64 (make_golden.py
    ref64_sh), including clamped channels."""
    kp = KA["k_pins"]
    cam = kp["cameras"]["default"]
    V, P = np.array(cam["view"], np.float32), np.array(cam["proj"], np.float32)
    from gaussian_splat_amd.api import Scene
    for c in kp["sh"]:
        sc = Scene(pos=np.array([c["pos"]]), rot=np.array([[1.0, 0.2, -0.1, 0.3]]), scale=np.array([[0.02] * 3]),
                   opacity=np.array([0.5]), color=np.array([c["f_dc"]]), sh_rest=np.array([c["f_rest"]]))
        rec, dbg = O.project_debug(sc, V, P, kp["width"], kp["height"], sh_degree=c["deg"])
        assert dbg["visible"][0]
        np.testing.assert_allclose([rec[0]["r"], rec[0]["g"], rec[0]["b"]], c["rgb"], rtol=2e-5, atol=2e-6)


# ---- K6 + F1 per pixel (tests/pixel_pins.py; tools/make_golden.py --pixels) ----
import pixel_pins as PX  # noqa: E402


@pytest.mark.parametrize("name", sorted(PX.alpha_pins()))
def test_pixel_alpha_pins(name):
    """K6 (quad coverage) + F1 (gaussian, 0.01 cutoff, alpha) of one splat at
    every pixel of its quad's box, the oracle against the float64 raster
    restatement (edge functions + barycentric uv, tile.metal:142-156,185-197):
    within 1e-6 off the straddling centres, which are counted."""
    pin = PX.alpha_pins()[name]
    kp = KA["k_pins"]
    sp = next(s for s in kp["splats"] if s["name"] == name)
    cam = kp["cameras"][sp["camera"]]
    V, P = np.array(cam["view"], np.float32), np.array(cam["proj"], np.float32)
    img, _ = O.render(PX.pin_scene(sp), V, P, kp["width"], kp["height"])
    worst, nst, nflip = PX.check_alpha(img, pin)
    print(f"{name}: max |alpha - pin| {worst:.3g}, {nst} straddling centres ({nflip} differ)")


@pytest.mark.parametrize("name", PX.frame_names())
def test_pixel_frames(name):
    """Small frames of overlapping rotated splats (needles, dense stacks that
    saturate, half-depth ties) against the float64 tile-rule image: within
    1e-4 per channel off the straddle mask."""
    fx = PX.load_frame(name)
    img, _ = O.render(PX.frame_scene(fx), fx["view"], fx["proj"], int(fx["width"]), int(fx["height"]))
    worst, nst, nflip = PX.check_frame(img, fx)
    assert img[..., 3].max() > 0.9
    print(f"{name}: max error {worst:.3g}, {nst} straddling pixels ({nflip} beyond 1e-4)")


@pytest.mark.parametrize("name", sorted(PX.alpha_pins()))
def test_pixel_alpha_given_record(name):
    """K6 + F1 alone: the float64 raster restatement evaluated at the oracle's
    own fp32 record (centre, conic, opacity taken exactly) against the
    oracle's frame, within 1e-6 off the straddling centres."""
    kp = KA["k_pins"]
    sp = next(s for s in kp["splats"] if s["name"] == name)
    cam = kp["cameras"][sp["camera"]]
    V, P = np.array(cam["view"], np.float32), np.array(cam["proj"], np.float32)
    sc = PX.pin_scene(sp)
    W, H = kp["width"], kp["height"]
    rec, dbg = O.project_debug(sc, V, P, W, H)
    x0, y0, al, st = PX.record_alpha(rec[0], float(dbg["zf"][0]), W, H)
    img, _ = O.render(sc, V, P, W, H)
    worst, nst, nflip = PX.check_alpha(img, {"x0": x0, "y0": y0, "alpha": al, "straddle": st}, tol=PX.ALPHA_TOL)
    print(f"{name}: max |alpha - pin(record)| {worst:.3g}, {nst} straddling centres ({nflip} differ)")
