"""CPU tests of the scene ingest: gs_create's direct
binary PLY -> HBM-plane path (mmap, parallel conversion, scene_io.cpp) must
hold exactly the floats of the reference path PLYLoader::load -> PointData ->
crop (src/ply_loader.cpp:88-146, instanced_splat_renderer.mm:359-388), here
read back with gs_get_scene.  Expected values: the reference's own loader
outputs (tests/golden/ply/*.ref.npy, made by oracle/_ref) and, for large
files, the oracle restatement (oracle/gs_oracle.c ora_ply_load)."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle_py as O

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden" / "ply"
MANIFEST = json.loads((GOLD / "manifest.json").read_text())


def raw_columns(path):
    """(names, n, float32 payload [n, nprops]) of a binary PLY as the
    reference reads it (every property 4 B, properties of all elements)."""
    data = Path(path).read_bytes()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    names, n = [], 0
    for line in data[:end].decode().splitlines():
        t = line.split()
        if t[:2] == ["element", "vertex"]:
            n = int(t[2])
        elif t and t[0] == "property":
            names.append(t[2])
    want = n * len(names) * 4
    body = data[end:end + want]
    # a short payload reads as zeros past its end (one zeroed chunk buffer,
    # ply_loader.cpp:89-95, for files under 10000 vertices)
    body = body[:len(body) // 4 * 4] + bytes(want - len(body) // 4 * 4)
    cols = np.frombuffer(body, "<f4").reshape(n, len(names))
    return names, n, cols


def expected(points, path, sh, crop, r=5.0):
    """gs_scene_soa arrays from PointData (+ raw f_dc for SH > 0), cropped."""
    p = np.asarray(points, np.float32).reshape(-1, 62)
    keep = np.all(np.abs(p[:, 0:3]) < r, axis=1) if crop else np.ones(len(p), bool)
    col = p[:, 6:9]
    if sh > 0:
        names, n, cols = raw_columns(path)
        col = np.zeros((n, 3), np.float32)
        for c in range(3):  # the last column of that name wins, as in load()
            idx = [j for j, nm in enumerate(names) if nm == f"f_dc_{c}"]
            if idx:
                col[:, c] = cols[:, idx[-1]]
    rest = p[:, 17:62].copy()
    k = {0: 0, 1: 3, 2: 8, 3: 15}[sh]
    mask = np.zeros(45, bool)
    for ch in range(3):
        mask[ch * 15:ch * 15 + k] = True
    rest[:, ~mask] = 0
    return dict(pos=p[keep, 0:3], rot=p[keep, 13:17], scale=p[keep, 10:13], opacity=p[keep, 9], color=col[keep],
                sh_rest=rest[keep])


def check_scene(sc, exp):
    for f, v in exp.items():
        got = getattr(sc, f)
        assert got.shape == v.shape, f
        np.testing.assert_array_equal(got.view(np.uint32), np.ascontiguousarray(v).view(np.uint32), err_msg=f)


@pytest.mark.parametrize("crop", [True, False])
@pytest.mark.parametrize("sh", [0, 3])
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_gs_create_matches_reference_loader(built, name, sh, crop):
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options
    path = GOLD / f"{name}.ply"
    if not MANIFEST[name]["ok"]:
        with pytest.raises(GsError):
            InstancedSplatRenderer(path, Options(sh_degree=sh, crop=crop))
        return
    if sh > 0 and (name.startswith("ascii") or "truncated" in name):
        pytest.skip("raw f_dc of ASCII / truncated files: PLYLoader path, covered by test_host")
    r = InstancedSplatRenderer(path, Options(sh_degree=sh, crop=crop))
    ref = np.load(GOLD / f"{name}.ref.npy", allow_pickle=False)
    check_scene(r.scene(), expected(ref, path, sh, crop))


@pytest.mark.parametrize("sh", [0, 1, 2, 3])
def test_gs_create_large_parallel_crop(built, tmp_path, sh):
    """>= 64k vertices (chunked conversion on every load thread), a tenth of
    them outside the crop box, some all-zero f_dc (the skip quirk)."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    raw = S.synthetic_raw(90001, seed=11, aspect=1.3, rest=True)
    raw.pos[::10] *= 3.0
    raw.f_dc[::7] = 0
    p = S.write_ply(tmp_path / "big.ply", raw)
    ok, pts = O.ply_load(p)
    assert ok
    r = InstancedSplatRenderer(p, Options(sh_degree=sh, crop=True))
    exp = expected(pts, p, sh, True)
    assert r.getPointCount() == len(exp["pos"]) < 90001
    check_scene(r.scene(), exp)


def test_soa_and_points_paths_crop_identically(built):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    raw = S.synthetic_raw(70000, seed=3, rest=True)
    raw.pos[1::9] *= 4.0
    sc = S.activate(raw, 3)
    a = InstancedSplatRenderer(sc, Options(sh_degree=3, crop=True)).scene()
    keep = np.all(np.abs(sc.pos) < 5.0, axis=1)
    check_scene(a, dict(pos=sc.pos[keep], rot=sc.rot[keep], scale=sc.scale[keep], opacity=sc.opacity[keep],
                        color=sc.color[keep], sh_rest=sc.sh_rest[keep]))


def test_subset_handles(built):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd import scene as S
    sc = S.synthetic_scene(5000, seed=8, sh_degree=2)
    r = InstancedSplatRenderer(sc, Options(sh_degree=2, crop=False))
    full = r.scene()
    for b, e in ((0, 5000), (0, 0), (1234, 4321), (4999, 5000)):
        sub = r.subset(b, e).scene()
        for f in ("pos", "rot", "scale", "opacity", "color", "sh_rest"):
            np.testing.assert_array_equal(getattr(sub, f), getattr(full, f)[b:e])
    from gaussian_splat_amd import GsError
    with pytest.raises(GsError):
        r.subset(10, 5001)


def test_sharded_group_host_side(built):
    """gs_create_sharded_from_handle splits the scene without a GPU; rendering
    needs gs_group_initialize (a device)."""
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options, ShardedGroup
    from gaussian_splat_amd import scene as S
    sc = S.synthetic_scene(1001, seed=2)
    r = InstancedSplatRenderer(sc, Options(crop=False))
    g = ShardedGroup(r, 3)
    assert g.size == 3 and g.getPointCount() == 1001 and g.transport == "none"
    with pytest.raises(GsError):
        g.render_host(np.eye(4), np.eye(4), 16, 16)
    with pytest.raises(GsError):
        ShardedGroup(r, 0)


def test_group_timeout_env_is_validated(built, monkeypatch):
    """GS_COMM_TIMEOUT_MS: a value that is not a positive integer
    is rejected by gs_group_initialize instead of becoming a 1 ms bound; the
    check runs before any device is touched, so it holds on the CPU."""
    from gaussian_splat_amd import GsError, InstancedSplatRenderer, Options, ShardedGroup
    from gaussian_splat_amd import _lib
    from gaussian_splat_amd import scene as S
    r = InstancedSplatRenderer(S.synthetic_scene(64, seed=3), Options(crop=False))
    for bad in ("abc", "10ms", "0", "-5", ""):
        monkeypatch.setenv("GS_COMM_TIMEOUT_MS", bad)
        g = ShardedGroup(r, 2)
        with pytest.raises(GsError):
            g.initialize([0, 0], transport="copy")
        assert "GS_COMM_TIMEOUT_MS" in _lib.last_error()
    # an explicit gs_group_set_timeout wins over the environment
    monkeypatch.setenv("GS_COMM_TIMEOUT_MS", "abc")
    g = ShardedGroup(r, 2)
    g.set_timeout(5000)
    with pytest.raises(GsError):
        g.initialize([0, 0], transport="copy")  # (no device here)
    assert "GS_COMM_TIMEOUT_MS" not in _lib.last_error()
