"""The C++ drop-in: tests/cpp/dropin_app.cpp is the
reference's own call sequence (src/main.mm:55-58, 69-72, 179, 192-198) --
TrackballCamera, InstancedSplatRenderer(plyPath), initialize(&device),
render(commandBuffer, drawable, view, proj, w, h) -- compiled with hipcc
against include/gsplat/*.h and libgsplat.so, no Python in the loop.  The
GPU tests run it as a separate process and compare its framebuffer with the
oracle's restatement of PLYLoader::load -> crop -> render, bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

APP = ROOT / "tests" / "cpp" / "dropin_app"


@pytest.fixture(scope="module")
def app(built):
    from gaussian_splat_amd import build
    return build.build_dropin_app()


def test_dropin_app_links(app):
    """The program is built and resolves libgsplat.so through its rpath; with
    no arguments it prints its usage before touching a GPU."""
    ldd = subprocess.run(["ldd", str(app)], capture_output=True, text=True, check=True).stdout
    line = [l for l in ldd.splitlines() if "libgsplat.so" in l]
    assert line and "not found" not in line[0], ldd
    r = subprocess.run([str(app)], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def _scene_ply(tmp_path, n, seed):
    from gaussian_splat_amd import scene as S
    raw = S.synthetic_raw(n, seed=seed, aspect=16 / 9, rest=False)
    raw.pos[::53, 0] += np.float32(7.0)  # some outside the crop cube (instanced_splat_renderer.mm:382-386)
    raw.f_dc[::17] = 0.0                 # the all-zero DC quirk (ply_loader.cpp:133)
    return S.write_ply(tmp_path / "scene.ply", raw)


def _run_app(app, ply, w, h, out, frames=1, bgra8=False):
    cmd = [str(app), str(ply), str(w), str(h), str(out), str(frames)] + (["bgra8"] if bgra8 else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=dict(os.environ))
    assert r.returncode == 0, r.stderr
    npts = int(r.stdout.split()[1])
    buf = np.fromfile(out, dtype=np.uint8)
    # column-major float[16] (simd_float4x4 layout) -> the matrix itself
    V = buf[:64].view(np.float32).reshape(4, 4).T.copy()
    P = buf[64:128].view(np.float32).reshape(4, 4).T.copy()
    return npts, V, P, buf[128:]


def _oracle_frame(ply, V, P, w, h):
    from gaussian_splat_amd.api import Scene
    from oracle import oracle_py as O
    ok, pts = O.ply_load(ply)
    keep = O.crop(pts)
    assert ok
    ref, _ = O.render(Scene.from_points(pts[keep]), V, P, w, h)
    return len(keep), ref


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,frames", [(20000, 256, 256, 1), (150000, 1280, 720, 3)])
def test_dropin_app_matches_oracle(app, tmp_path, n, w, h, frames):
    """fp32 RGBA drawable: same point count as the oracle's load + crop, the
    camera's matrices equal the reference defaults (SURVEY §8c pin), and the
    frame is bit-identical to the oracle's."""
    from gaussian_splat_amd.api import default_camera
    ply = _scene_ply(tmp_path, n, seed=71)
    npts, V, P, px = _run_app(app, ply, w, h, tmp_path / "out.bin", frames)
    cam = default_camera(w, h)
    np.testing.assert_array_equal(V, cam.getViewMatrix())
    np.testing.assert_array_equal(P, cam.getProjectionMatrix())
    nref, ref = _oracle_frame(ply, V, P, w, h)
    assert npts == nref
    img = px.view(np.float32).reshape(h, w, 4)
    assert int(np.count_nonzero(img.view(np.uint32) != ref.view(np.uint32))) == 0
    assert img[..., 3].max() > 0.5


@pytest.mark.gpu
def test_dropin_app_bgra8(app, tmp_path):
    """renderBGRA8: the drawable's BGRA8Unorm bytes (metal_renderer.mm:58)
    equal the oracle frame's conversion byte for byte."""
    from oracle import oracle_py as O
    w, h = 640, 360
    ply = _scene_ply(tmp_path, 40000, seed=72)
    _, V, P, px = _run_app(app, ply, w, h, tmp_path / "out.bin", frames=2, bgra8=True)
    _, ref = _oracle_frame(ply, V, P, w, h)
    np.testing.assert_array_equal(px.reshape(h, w, 4), O.to_bgra8(ref))


@pytest.mark.gpu
def test_dropin_app_missing_file(app, tmp_path):
    """The ctor keeps the reference's silent behaviour on a missing file
    (instanced_splat_renderer.mm:346-349); initialize() then fails and the
    program reports it instead of rendering."""
    r = subprocess.run([str(app), str(tmp_path / "nope.ply"), "64", "64", str(tmp_path / "o.bin")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "initialize" in r.stderr
