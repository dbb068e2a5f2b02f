"""GPU tests of the replicated-scene band scheme (gs_band_render, SURVEY
§8(e) fallback): every rank holds the whole scene and renders
only its owned bin rows; here the ranks are virtual (handles on one GPU).

Bar: the assembled bands are bit-identical to the 1-GPU frame, with the
default contiguous ownership (rects clipped to the band) and with a custom,
non-contiguous owner table (no clipping), for ranks owning no rows, and for
world 1 (the band is the frame)."""
import numpy as np
import pytest

from conftest import orbit_views

pytestmark = pytest.mark.gpu


def _scene(n, seed, sh, aspect, heavy=False):
    from gaussian_splat_amd import scene as S
    return S.activate(S.synthetic_raw(n, seed=seed, aspect=aspect, rest=sh > 0,
                                      profile="heavy" if heavy else "uniform"), sh)


def _bands(sc, opt, world, V, P, W, H, owner=None):
    import torch

    from gaussian_splat_amd.distributed import HipBandBackend, assemble
    bands = []
    for r in range(world):
        be = HipBandBackend(sc, r, world, opt, 0, owner=owner)
        bands.append(be.render(V, P, W, H))
        torch.cuda.synchronize()
    if world == 1:
        return bands[0][:H].cpu().numpy()
    return assemble(bands, W, H, world, owner).cpu().numpy()


@pytest.mark.parametrize("world,mode,sh,W,H", [(2, "tile", 3, 640, 400), (3, "live50", 0, 640, 400),
                                               (4, "tile", 3, 1920, 1080), (1, "tile", 0, 256, 256)])
def test_band_frames_bitexact(built, world, mode, sh, W, H):
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    n = 200000 if W > 1000 else 60000
    sc = _scene(n, 91 + world, sh, W / H)
    opt = Options(mode=mode, sh_degree=sh, crop=False)
    r = InstancedSplatRenderer(sc, opt)
    r.initialize(0)
    for V, P in orbit_views(W, H, 2):
        ref = r.render_host(V, P, W, H)
        got = _bands(sc, opt, world, V, P, W, H)
        assert int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))) == 0


def test_band_custom_owner_and_idle_rank(built):
    """Interleaved (non-contiguous) rows: no band clipping, the owner table
    alone selects the pairs; a rank that owns no row leaves an empty band."""
    from gaussian_splat_amd import InstancedSplatRenderer, Options
    W, H = 512, 320  # 10 bin rows
    sc = _scene(50000, 97, 0, W / H, heavy=True)
    opt = Options(crop=False)
    r = InstancedSplatRenderer(sc, opt)
    r.initialize(0)
    V, P = orbit_views(W, H, 1)[0]
    ref = r.render_host(V, P, W, H)
    owner = np.array([0, 2, 0, 2, 2, 0, 0, 2, 0, 2], np.uint8)  # rank 1 owns nothing
    got = _bands(sc, opt, 3, V, P, W, H, owner=owner)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("world,binning,path", [(2, "bin_first", "orbit"), (3, "bin_first", "jump"),
                                                 (2, "depth_first", "orbit")])
def test_band_frames_depth_cuts_bitexact(built, world, binning, path):
    """Contiguous bands over a camera path: a clipped band bins without its
    owner table (gs_handle::band_local), so from a buffer set's second frame
    on its lists carry depth cuts, the bin-first duplicate marks the pairs
    behind them, and open quadrants finish from the fallback lists.  Every
    frame of every rank equals the 1-GPU frame bit for bit."""
    import torch

    from gaussian_splat_amd import InstancedSplatRenderer, Options
    from gaussian_splat_amd.api import default_camera
    from gaussian_splat_amd.distributed import HipBandBackend, assemble
    W, H = 640, 384
    sc = _scene(700000, 71 + world, 0, W / H)
    sc.scale *= np.float32(2.0)  # (the bench scene's coverage per pixel: the lists saturate)
    opt = Options(crop=False, binning=binning)
    ref_r = InstancedSplatRenderer(sc, opt)
    ref_r.initialize(0)
    ranks = [HipBandBackend(sc, r, world, opt, 0) for r in range(world)]
    cut_frames = sorted_lt_pairs = opened = ref_lt = 0
    for k in range(8):
        cam = default_camera(W, H)
        if path == "orbit":
            cam.orbit(0.02 * k, 0.005 * k)
        else:  # still, then a jump that leaves quadrants open behind the old cuts
            cam.orbit(0.0 if k < 5 else 0.5, 0.0 if k < 5 else 0.1)
        V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
        ref = ref_r.render_host(V, P, W, H)
        rs = ref_r.last_stats()
        ref_lt += int(rs["pairs_sorted"] < rs["pairs"])
        bands = [be.render(V, P, W, H) for be in ranks]
        torch.cuda.synchronize()
        got = assemble(bands, W, H, world).cpu().numpy()
        assert int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32))) == 0, f"frame {k}"
        for be in ranks:
            st = be.r.last_stats()
            cut_frames += int(st["cut_frame"])
            sorted_lt_pairs += int(st["pairs_sorted"] < st["pairs"])
            opened += int(st["open_tiles"])
    assert cut_frames >= world * 4, cut_frames  # (each rank: frames 3..8 have cuts)
    assert ref_lt > 0  # (the scene saturates: the 1-GPU cuts drop pairs)
    assert sorted_lt_pairs > 0
    if path == "jump":
        assert opened > 0
